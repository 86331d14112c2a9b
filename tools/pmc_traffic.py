"""Turns a tools/profile_round.sh run into the committed profile files.

  python tools/pmc_traffic.py gpurun_out/prof_r03 r03

Per profiled workload W (c3, c4):
  profiles/<round>_kernel_stats_<W>.csv  rocprofv3 --kernel-trace --stats
  profiles/<round>_bench_<W>.json        the bench line of the same run
  profiles/<round>_pmc_<W>.csv           per-dispatch FETCH_SIZE / WRITE_SIZE of the last step
  profiles/<round>_sq_<W>.csv            per-kernel SQ counters (wave cycles, waits, VALU)
  profiles/pmc_traffic[_W].json          HBM bytes per bench-stage launch (read by bench.py for
                                         roofline.traffic_carried; c3 -> pmc_traffic.json)
and for the bench-only workloads (c2, c5) the bench line and kernel stats.

HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide
coalesced streaming read, so it is doubled; WRITE_SIZE is exact.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# kernel symbol (rocprofv3 -T) -> bench stage (pdp_hip.h PDP_STAGE_*)
STAGE_OF = {"k_histogram_tiles": "histogram", "k_bucket_pass": "onesweep_first", "k_sort_first": "onesweep_first",
            "k_filter": "filter", "k_thin": "buckets", "k_lean": "buckets", "k_segments": "buckets",
            "k_segments_big": "buckets", "k4_fill_ranges": "buckets", "k_pair_pass": "pair_pass",
            "k_pair_pass12_first": "pair_pass", "k_pair_pass12": "pair_pass", "k4_offsets": "pair_pass", "k4_set_counter": "pair_pass", "k4_reduce": "reduce",
            "k4_zero_shared": "reduce", "k4_finalize": "reduce", "k_release": "release",
            "k_unpack_counts": "buckets", "k_subruns": "survivor_group", "k_grp_count": "survivor_group", "k_group": "survivor_group",
            "k_bucket_pass8": "onesweep_first"}
# kernels of a records radix sort (the survivor sort after k_filter, or a pid-sort pass >= 1)
# (round 5's device-sized survivor sort is k_onesweep_dev + k_status_clear: missing here until round 6, which
# under-booked the c3 survivor sort at 1.09 GB against 6.21 GB measured)
SORT = {"k_histogram", "k_onesweep", "k_onesweep_dev", "k_status_clear", "k_tile_counts", "k_offsets",
        "k_tile_chunk_sums", "k_tile_chunk_scan", "k_tile_bases"}


def stage_of(name):
    """Bench stage of a kernel outside SORT; kernels no stage claims are booked as "other" (so step_bytes
    counts every byte of the step)."""
    if name in STAGE_OF:
        return STAGE_OF[name]
    if name.startswith("k_pair_pass"):
        return "pair_pass"
    if name.startswith("k4_"):
        return "reduce"
    if name.startswith(("k_thin", "k_lean", "k_segments", "k_ranges")):
        return "buckets"
    return "other"


def kname(s):
    s = s.replace("void ", "").replace("(anonymous namespace)::", "")
    return s.split("(")[0].split("<")[0].strip()


def dispatches(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    for r in rows:
        r["Kernel_Name"] = kname(r["Kernel_Name"])
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def last_step(rows):
    """Dispatches of the last pipeline step (from the last k_histogram_tiles to k_release)."""
    starts = [i for i, r in enumerate(rows) if r["Kernel_Name"] == "k_histogram_tiles"]
    out = rows[starts[-1]:] if starts else rows
    end = next((i for i, r in enumerate(out) if r["Kernel_Name"] == "k_release"), len(out) - 1)
    return out[:end + 1]


def stage_bytes(rows, scale):
    """Bytes per launch of each bench stage: every stage is one ProfScope per
    step (its kernels summed), except onesweep_rest and tile_counts (one per
    pid-sort pass >= 1: averaged)."""
    tot, n_rest, n_tc, filtered = collections.defaultdict(float), 0, 0, False
    for r in rows:
        name = r["Kernel_Name"]
        b = float(r["Counter_Value"]) * 1024.0 * scale
        filtered |= name == "k_filter"
        if name in SORT and filtered:
            tot["survivor_sort"] += b
        elif name == "k_onesweep":
            tot["onesweep_rest"] += b
            n_rest += 1
        elif name in ("k_tile_counts", "k_tile_chunk_sums", "k_tile_chunk_scan", "k_tile_bases"):
            tot["tile_counts"] += b
            n_tc += name == "k_tile_counts"
        else:
            tot[stage_of(name)] += b
    if n_rest:
        tot["onesweep_rest"] /= n_rest
    if n_tc:
        tot["tile_counts"] /= n_tc
    return dict(tot)


def sq_summary(src_dir, out_csv):
    """Per-kernel sums of the SQ pass (all dispatches of the run)."""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.Counter()
    for p in glob.glob(os.path.join(src_dir, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(p)):
            k = kname(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Dispatch_Id"] not in seen:
                seen.add(r["Dispatch_Id"])
                calls[k] += 1
    names = sorted({c for v in agg.values() for c in v})
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches"] + names)
        for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
            w.writerow([k, calls[k]] + [f"{v.get(c, 0):.0f}" for c in names])
    return agg


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    for w in ("c3", "c4", "c2", "c5", "c3v"):
        kt = os.path.join(src, f"kt_{w}", "run_kernel_stats.csv")
        if os.path.exists(kt):
            shutil.copy(kt, os.path.join(prof, f"{rnd}_kernel_stats_{w}.csv"))
        b = os.path.join(src, f"bench_{w}.out")
        if os.path.exists(b) and os.path.getsize(b):
            line = open(b).read().strip().splitlines()[-1]
            with open(os.path.join(prof, f"{rnd}_bench_{w}.json"), "w") as f:
                f.write(line + "\n")
        sq = os.path.join(src, f"sq_{w}")
        if os.path.isdir(sq):
            sq_summary(sq, os.path.join(prof, f"{rnd}_sq_{w}.csv"))
        fp = os.path.join(src, f"pmc_{w}_FETCH_SIZE", "run_counter_collection.csv")
        wp = os.path.join(src, f"pmc_{w}_WRITE_SIZE", "run_counter_collection.csv")
        if not (os.path.exists(fp) and os.path.exists(wp)):
            continue
        bench = json.loads(open(os.path.join(src, f"pmc_{w}_FETCH_SIZE.out")).read().strip().splitlines()[-1])
        fetch = last_step(dispatches(fp, "FETCH_SIZE"))
        write = last_step(dispatches(wp, "WRITE_SIZE"))
        with open(os.path.join(prof, f"{rnd}_pmc_{w}.csv"), "w", newline="") as f:
            wr_ = csv.writer(f)
            wr_.writerow(["kernel", "counter", "value_KiB", "lds_bytes", "vgprs", "scratch"])
            for rows, c in ((fetch, "FETCH_SIZE"), (write, "WRITE_SIZE")):
                for r in rows:
                    wr_.writerow([r["Kernel_Name"], c, r["Counter_Value"], r.get("LDS_Block_Size"),
                                  r.get("VGPR_Count") or r.get("Arch_VGPR_Count"), r.get("Scratch_Size")])
        rd, wb = stage_bytes(fetch, 2.0), stage_bytes(write, 1.0)
        out = {
            "round": rnd,
            "workload": w,
            "config_rows": bench["config"]["rows_per_gpu"],
            "note": "HBM bytes per launch = 2 x FETCH_SIZE KiB x 1024 (gfx950 half-count) + WRITE_SIZE KiB x 1024; "
                    "separate rocprofv3 --pmc passes (tools/profile_round.sh)",
            "read_bytes_per_launch": rd,
            "write_bytes_per_launch": wb,
            "bytes_per_launch": {k: rd.get(k, 0.0) + wb.get(k, 0.0) for k in sorted(set(rd) | set(wb))},
            # every dispatch of the step (stages with several launches -- pid-sort passes -- counted each time)
            "step_bytes": sum(float(r["Counter_Value"]) * 2048.0 for r in fetch) +
                          sum(float(r["Counter_Value"]) * 1024.0 for r in write),
        }
        name = "pmc_traffic.json" if w == "c3" else f"pmc_traffic_{w}.json"
        json.dump(out, open(os.path.join(prof, name), "w"), indent=1)
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
