"""Turns a tools/profile_round.sh run into the committed profile files.

  python tools/pmc_traffic.py gpurun_out/prof_r01 r01

Writes profiles/<round>_kernel_stats.csv (rocprofv3 --kernel-trace --stats),
profiles/<round>_bench.json (the bench line of the same run),
profiles/<round>_pmc.csv (per-dispatch FETCH_SIZE / WRITE_SIZE of our
kernels) and profiles/pmc_traffic.json (HBM bytes per launch of each bench
stage, read by bench.py for roofline.traffic).

HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide
coalesced streaming read, so it is doubled; WRITE_SIZE is exact.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAGE_OF = {"k_histogram": "histogram", "k_segments": "buckets", "k_lean": "buckets", "k_release": "release",
            "k_histogram_tiles": "histogram", "k_tile_counts": "tile_counts", "k_filter": "filter",
            "k_thin": "buckets", "k_segments_big": "buckets"}
# kernels of the radix sort of the L0 pre-filter's survivors (after k_filter)
SURVIVOR_SORT = {"k_histogram", "k_onesweep", "k_tile_counts", "k_offsets", "k_tile_chunk_sums", "k_tile_chunk_scan",
                 "k_tile_bases"}


def dispatches(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def last_step(rows):
    """Dispatches of the last pipeline step (from the last k_histogram on)."""
    starts = [i for i, r in enumerate(rows) if r["Kernel_Name"] == "k_histogram_tiles"]
    if not starts:
        starts = [i for i, r in enumerate(rows) if r["Kernel_Name"] == "k_histogram"]
    out = rows[starts[-1]:]
    end = next((i for i, r in enumerate(out) if r["Kernel_Name"] == "k_release"), len(out) - 1)
    return out[:end + 1]


def stage_bytes(rows, scale):
    res, seen_sweep, filtered = {}, 0, False
    for r in rows:
        name = r["Kernel_Name"]
        b = float(r["Counter_Value"]) * 1024.0 * scale
        filtered |= name == "k_filter"
        if filtered and name in SURVIVOR_SORT:
            res.setdefault("survivor_sort", [0.0])[0] += b  # all kernels of the sort, one launch of the stage
            continue
        if name == "k_onesweep":
            st = "onesweep_first" if seen_sweep == 0 else "onesweep_rest"
            seen_sweep += 1
        else:
            st = STAGE_OF.get(name)
        if st is None:
            continue
        res.setdefault(st, []).append(b)
    return {k: sum(v) / len(v) for k, v in res.items()}


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), os.path.join(prof, f"{rnd}_kernel_stats.csv"))
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(prof, f"{rnd}_bench.json"))
    bench = json.loads(open(os.path.join(src, "pmc_FETCH_SIZE.json")).read().strip().splitlines()[-1])
    fetch = last_step(dispatches(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE"))
    write = last_step(dispatches(os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE"))
    with open(os.path.join(prof, f"{rnd}_pmc.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "counter", "value_KiB", "lds_bytes", "vgprs", "scratch"])
        for rows, c in ((fetch, "FETCH_SIZE"), (write, "WRITE_SIZE")):
            for r in rows:
                w.writerow([r["Kernel_Name"], c, r["Counter_Value"], r["LDS_Block_Size"], r["VGPR_Count"],
                            r["Scratch_Size"]])
    rd, wr = stage_bytes(fetch, 2.0), stage_bytes(write, 1.0)
    out = {
        "round": rnd,
        "config_rows": bench["config"]["rows_per_gpu"],
        "note": "HBM bytes per launch = 2 x FETCH_SIZE KiB x 1024 (gfx950 half-count) + WRITE_SIZE KiB x 1024; "
                "separate rocprofv3 --pmc passes (tools/profile_round.sh)",
        "read_bytes_per_launch": rd,
        "write_bytes_per_launch": wr,
        "bytes_per_launch": {k: rd.get(k, 0.0) + wr.get(k, 0.0) for k in sorted(set(rd) | set(wr))},
    }
    json.dump(out, open(os.path.join(prof, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
