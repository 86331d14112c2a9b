"""Benchmark: DP COUNT+SUM+MEAN with contribution bounding and private partition
selection (BASELINE.json metric) on synthetic Zipf(1.1)-keyed rows.

  python bench.py [--gpus N --steps K --warmup W]

One "step" = one pass of the hot path over one batch: pdp_bound_accumulate
(histogram + radix passes + LDS bucket bounding + K4 per-partition reduction)
[+ RCCL reduce-scatter of the per-partition accumulators when N > 1] +
pdp_release (truncated-geometric selection + Laplace noise).  Inputs (int64
pid, int64 pk, f64 value) are generated on device before timing and stay
resident.

Scaling.  c3 is BASELINE.json's headline "1B rows/1M partitions" across the
node: with --gpus N every rank processes 1e9/N rows of 1e7/N privacy ids of
its own (pid-sharded input, strong scaling; the N=1 line is the whole 1e9
rows on one GPU).  --weak keeps --rows rows per rank instead.  c4 is one
GPU's share of the 8-GPU stress config (4e9 rows total, 5e8 per GPU): weak
at every N.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
GUIDE_COPY_GBS = 6290.0  # MI355X_MICROARCH.md:36, measured device copy

# Per-GPU shapes of BASELINE.json configs (SURVEY.md 8(d) "Synthetic inputs").
# c3 is the headline: COUNT+SUM+MEAN, private selection, 1e9 rows / 1e6 Zipf partitions.
# c2: COUNT+SUM over 1e5 PUBLIC partitions (no selection), 1e8 rows, 1e6 uniform pids.
# c4: high-cardinality stress, one GPU's shard of 4e9 rows / 5e7 Zipf partitions, L0=32.
# `strong`: --rows / --pids are node totals split over the ranks (c3 = 1e9 rows across the node).
WORKLOADS = {
    "c3": dict(rows=1e9, partitions=1e6, pids=1e7, zipf=1.1, l0=4, linf=2, public=False, metrics="mean",
               cpu_sample=1.2e7, strong=True),  # CPU baseline rows per host core (~10 s of CPU work)
    # c3v: BASELINE configs[2] as written -- the c3 shape with MEAN + VARIANCE (+ COUNT + SUM): K2 also writes
    # the y slot array and K4 runs a second (y) reduction
    "c3v": dict(rows=1e9, partitions=1e6, pids=1e7, zipf=1.1, l0=4, linf=2, public=False, metrics="variance",
                cpu_sample=1.2e7, strong=True),
    "c2": dict(rows=1e8, partitions=1e5, pids=1e6, zipf=0.0, l0=8, linf=4, public=True, metrics="count_sum",
               cpu_sample=1.2e7),
    "c4": dict(rows=5e8, partitions=5e7, pids=1.25e7, zipf=1.1, l0=32, linf=4, public=False, metrics="mean",
               cpu_sample=5e5),  # the oracle's O(P) release dominates at P=5e7
    # c5: UtilityAnalysisEngine.analyze with 64 configurations (L0 x Linf) over 1e8 rows: per-partition
    # COUNT / SUM / PRIVACY_ID_COUNT error metrics + truncated-geometric keep probability
    # (pdp_utility_analysis); cpu_sample = total rows of the CPU baseline.
    "c5": dict(rows=1e8, partitions=1e5, pids=1e6, zipf=1.1, l0=0, linf=0, public=False, metrics="analysis",
               cpu_sample=2e5),
}
SWEEP = [(l0, linf) for l0 in (1, 2, 4, 8, 16, 32, 64, 128) for linf in range(1, 9)]
SWEEP_SUM_BOUNDS = (0.0, 20.0)  # min/max_sum_per_partition of every c5 configuration
# fp64 operations k_ana_metrics spends per (pair, configuration) with SUM + COUNT + PRIVACY_ID_COUNT
# (pdp_analysis.inc): q 1, q(1-q) 2, SumCombiner terms 11, CountCombiner 10,
# PrivacyIdCountCombiner 4, selection moments 7
ANALYSIS_FLOP_PER_PAIR_CONFIG = 35
FP64_SPEC_TFLOPS = 78.6  # MI355X fp64 vector peak (AMD spec; MI355X_MICROARCH.md lists none)


def analysis_oracle_cfgs(eps_sel=0.25, delta_sel=1e-6):
    """c5 configurations for the CPU baseline (pdp_analysis_oracle)."""
    import pdp_analysis_oracle as ao
    lo, hi = SWEEP_SUM_BOUNDS
    return [ao.AnalysisConfig(l0, linf, lo, hi, "truncated_geometric", eps_sel, delta_sel) for l0, linf in SWEEP]


def pmc_traffic(stage, rows, workload="c3"):
    """HBM bytes per launch of `stage` from profiles/pmc_traffic[_<workload>].json
    (written by tools/pmc_traffic.py from the separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of tools/profile_round.sh) when that profile
    was taken on this same workload size; (None, None) otherwise."""
    name = "pmc_traffic.json" if workload == "c3" else f"pmc_traffic_{workload}.json"
    try:
        with open(os.path.join(ROOT, "profiles", name)) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    if d.get("config_rows") != rows or stage not in d.get("bytes_per_launch", {}):
        return None, None
    return d["bytes_per_launch"][stage], d.get("round")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--workload", choices=sorted(WORKLOADS), default="c3",
                   help="c3 = headline (BASELINE.json metric); c2 / c4 = the other single-GPU-sized configs")
    p.add_argument("--rows", type=float, default=None, help="rows per GPU")
    p.add_argument("--partitions", type=float, default=None)
    p.add_argument("--pids", type=float, default=None, help="privacy ids per GPU")
    p.add_argument("--zipf", type=float, default=None)
    p.add_argument("--l0", type=int, default=None)
    p.add_argument("--linf", type=int, default=None)
    p.add_argument("--cpu-sample", type=float, default=None, help="rows of the CPU baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-profile", action="store_true")
    p.add_argument("--seed", type=int, default=20250204)
    p.add_argument("--debug-flags", type=int, default=0, help="kernel ablation flags (experiments only)")
    p.add_argument("--debug-flags2", type=int, default=0, help="second debug-flag word (A/B of alternative forms)")
    p.add_argument("--weak", action="store_true", help="c3: --rows / --pids per rank instead of node totals")
    p.add_argument("--graph", action="store_true",
                   help="capture one step (accumulate + release) in a hipGraph once and replay it in the timed "
                        "loop (every kernel still runs every step); one GPU only")
    p.add_argument("--share", type=int, default=0,
                   help="one GPU runs the LAST rank's share of an N-GPU strong-scaling step (rows and privacy ids "
                        "/ N, global ids via pid_base, no collective): the per-rank compute of SCALE, not SCALE")
    args = p.parse_args()
    for k, v in WORKLOADS[args.workload].items():
        if k != "strong" and getattr(args, k, None) is None:
            setattr(args, k, v)
    args.strong = bool(WORKLOADS[args.workload].get("strong")) and not args.weak
    return args


def stage_bytes(stage, n_in, n_kept, P, nfields, survivors=0, survivor_passes=0, k4=None, y_slots=False,
                grouped=False):
    """Algorithmic bytes of one launch of each kernel (Roofline).
    With the L0 pre-filter (survivors > 0): K0 reads the privacy ids only, the
    first pass is the bucket pass (+ a 4-B tag per row), k_filter reads the
    tags twice (sketch, count) and moves the survivors' records, and the
    survivor sort and K2 see the survivors only.  K4
    (k4 = (slots, pairs, passes)): K2 also writes one 16-B slot per sorted row,
    the first pair pass reads the slots and writes the pairs, later passes
    read + write the pairs, the reduction reads the pairs and writes
    row_count / count / x (8 B each) per partition.  VARIANCE (y_slots): K2
    writes a second slot array and K4 runs once more on it (same bytes per
    pair-pass / reduce launch)."""
    sorted_rows = survivors if survivors else n_kept
    slots, pairs, kpasses = k4 or (0, 0, 0)
    return {
        "histogram": (8 if survivors else 16) * n_in,  # read int64 pid (+ int64 pk)
        # read 3 columns, write 16-B records (+ the pre-filter's 4-B tags)
        "onesweep_first": (24 + 16 + (4 if survivors else 0)) * n_in,
        "onesweep_rest": 32 * n_kept,  # read + write 16-B records
        # tags twice (sketch, count) + keep bytes written and read; per survivor its 16-B record read and written
        "filter": 8.5 * n_kept + 32 * survivors,
        # histogram read + per look-back pass (read + write) after the first grouping step, which k_filter
        # does while compacting (round 6); with the LDS grouping (survivor_group) there is no such pass
        "survivor_sort": survivors * (16 + 32 * max(survivor_passes - 1 - (1 if grouped else 0), 0)),
        "survivor_group": 32 * survivors,
        "buckets": 16 * sorted_rows + (32 if y_slots else 16) * slots,  # read 16-B records once (+ K4: write the pair slots)
        "pair_pass": 16 * slots + 16 * pairs + 32 * pairs * max(kpasses - 1, 0),
        "reduce": 16 * pairs + 24 * P,
        "release": P * (3 * 8 + 1 + 8 * nfields),
        # c5: read the input columns once; read the (pk, privacy id, count, sum) pairs once and write
        # C x P x (3 metrics x 5 + keep probability) doubles
        "analysis_pairs": 24 * n_in,
        "analysis_metrics": 20 * n_kept + P * len(SWEEP) * (5 * 3 + 1) * 8,
    }.get(stage)


def copy_peak_gbs(torch, lib=None, nbytes=8 << 30, iters=5):
    """Achievable HBM ceiling on this box (read + write bytes / time of a
    device-to-device copy of `nbytes`), the measured counterpart of the 8 TB/s
    spec peak: with `lib`, libpdp_hip's 16-B-per-lane
    streaming kernel (pdp_stream_copy, the float4 shape MI355X_MICROARCH.md
    measures at 6.29 TB/s); else torch's copy_."""
    import ctypes
    src = torch.empty(nbytes // 8, dtype=torch.int64, device="cuda")
    dst = torch.empty_like(src)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def copy():
        if lib is None:
            dst.copy_(src)
        elif lib.pdp_stream_copy(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), nbytes, stream):
            raise RuntimeError("pdp_stream_copy failed")

    copy()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        copy()
    b.record()
    torch.cuda.synchronize()
    gbs = 2 * nbytes * iters / (a.elapsed_time(b) * 1e-3) / 1e9
    del src, dst
    torch.cuda.empty_cache()
    return round(gbs, 1)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


_SHM = {}  # fork-shared sample buffers of the CPU baseline workers


def _cpu_gen(task):
    """Worker: rows [lo, hi) of the synthetic sample into the shared buffers."""
    import numpy as np
    import pdp_oracle as o
    lo, hi, U, P, seed, zipf = task
    pid, pk, val = o.synth_rows(hi - lo, U, P, seed=seed, zipf_s=zipf, row_offset=lo)
    _SHM["pid"][lo:hi] = pid
    _SHM["pk"][lo:hi] = pk
    _SHM["val"][lo:hi] = val
    return hi - lo


def _cpu_bound(task):
    """Worker: bound + accumulate the rows of privacy-id shard w (pid % W == w);
    returns the touched partitions' accumulators (sparse)."""
    import numpy as np
    import pdp_oracle as o
    w, W, P, l0, linf, seed = task
    pid, pk, val = _SHM["pid"], _SHM["pk"], _SHM["val"]
    mine = (pid % W) == w
    acc = o.bound_and_accumulate(pid[mine], pk[mine], val[mine], P, o.BoundParams(l0, linf, 0.0, 10.0), "hash",
                                 seed=seed)
    idx = np.flatnonzero(acc.row_count)
    return idx, acc.row_count[idx], acc.count[idx], acc.sum[idx], acc.nsum[idx], acc.nsumsq[idx]


def _cpu_analysis(task):
    """Worker: per-partition metrics of a slice of the c5 configurations."""
    import pdp_analysis_oracle as ao
    lo, hi, P = task
    ao.per_partition(*_SHM["pairs"], P, analysis_oracle_cfgs()[lo:hi], ["sum", "count", "privacy_id_count"])
    return hi - lo


def cpu_baseline_analysis(args, P, W):
    """c5 on the host: oracle pre-aggregation of the sample, then the 64
    configurations split over W processes (pdp_analysis_oracle.py)."""
    import multiprocessing as mp

    import pdp_analysis_oracle as ao
    import pdp_oracle as o
    m = int(args.cpu_sample)
    U = max(1, int(args.pids * m / args.rows))
    pid, pk, val = o.synth_rows(m, U, P, seed=args.seed, zipf_s=args.zipf)
    t0 = time.perf_counter()
    _SHM["pairs"] = ao.preaggregate(pid, pk, val)
    ctx = mp.get_context("fork")
    with ctx.Pool(W) as pool:
        step = (len(SWEEP) + W - 1) // W
        pool.map(_cpu_analysis, [(i, min(i + step, len(SWEEP)), P) for i in range(0, len(SWEEP), step)])
    dt = time.perf_counter() - t0
    del _SHM["pairs"]
    return {"value": m / dt, "unit": "rows/s", "cores": W, "kind": "port", "plan_item": 3,
            "host_cpus_visible": os.cpu_count(), "cpu_model": _cpu_model(),
            "sample": f"c5: {m} rows, {U} privacy ids, {P} Zipf({args.zipf}) partitions, {len(SWEEP)} "
                      f"configurations; numpy restatement (oracle/pdp_analysis_oracle.py): pre-aggregation on one "
                      f"process, configurations split over {W}; {dt:.1f} s"}


def cpu_baseline(args, P):
    """BASELINE.md CPU plan item 3: the numpy restatement (oracle/pdp_oracle.py)
    on the host cores of this box, privacy ids sharded over a process pool
    (the reference's LocalBackend is single-threaded and cannot travel here).
    Runs before the GPU is initialised (fork pool).  The sample is generated
    in parallel outside the timed region; timed: shard + bound + accumulate
    per worker, merge, selection + noise."""
    import mmap
    import multiprocessing as mp

    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pdp_oracle as o  # checker / baseline only
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    W = max(1, min(16, cores))  # the GPU box's CPU share is 16 cores per GPU
    if WORKLOADS[args.workload]["metrics"] == "analysis":
        return cpu_baseline_analysis(args, P, W)
    m = int(args.cpu_sample) * W
    U = max(1, int(args.pids * m / args.rows))
    for name, dt in (("pid", np.int64), ("pk", np.int64), ("val", np.float64)):
        _SHM[name] = np.frombuffer(mmap.mmap(-1, max(8 * m, 8)), dtype=dt, count=m)
    ctx = mp.get_context("fork")
    metrics = WORKLOADS[args.workload]["metrics"]
    with ctx.Pool(W) as pool:
        bounds = np.linspace(0, m, W + 1).astype(np.int64)
        pool.map(_cpu_gen, [(int(bounds[i]), int(bounds[i + 1]), U, P, args.seed, args.zipf) for i in range(W)])
        t0 = time.perf_counter()
        parts = pool.map(_cpu_bound, [(w, W, P, args.l0, args.linf, 1) for w in range(W)])
        rc, cnt, sm, ns, nq = (np.zeros(P, np.int64), np.zeros(P, np.int64), np.zeros(P), np.zeros(P), np.zeros(P))
        for idx, a, b, c, d, e in parts:
            rc[idx] += a
            cnt[idx] += b
            sm[idx] += c
            ns[idx] += d
            nq[idx] += e
        acc = o.Accumulators(rc, cnt, sm, ns, nq)
        bp = o.BoundParams(args.l0, args.linf, 0.0, 10.0)
        if WORKLOADS[args.workload]["public"]:
            spec = o.ReleaseSpec(("count", "sum"), "laplace", {"count": (0.5, 0.0), "sum": (0.5, 0.0)}, None)
        elif metrics == "variance":
            spec = o.ReleaseSpec(("variance", "mean", "count", "sum"), "laplace", {"variance": (0.5, 0.0)},
                                 "truncated_geometric", (0.5, 1e-6))
        else:
            spec = o.ReleaseSpec(("mean", "count", "sum"), "laplace", {"mean": (0.5, 0.0)}, "truncated_geometric",
                                 (0.5, 1e-6))
        if metrics != "count":
            o.release(acc, bp, spec, seed=2)
        dt = time.perf_counter() - t0
    for k in list(_SHM):
        del _SHM[k]
    return {"value": m / dt, "unit": "rows/s", "cores": W, "kind": "port", "plan_item": 3,
            "host_cpus_visible": os.cpu_count(), "cpu_model": _cpu_model(),
            "sample": f"{args.workload}: {m} rows ({int(args.cpu_sample)} per core), {U} privacy ids, {P} "
                      f"{'public uniform' if WORKLOADS[args.workload]['public'] else f'Zipf({args.zipf})'} "
                      f"partitions, L0={args.l0}, Linf={args.linf}; numpy restatement (oracle/pdp_oracle.py), "
                      f"privacy ids sharded over {W} processes, merge + selection + noise on one; {dt:.1f} s"}


def launch_ranks(args):
    """`--gpus N` without a torch.distributed launcher: start N rank processes
    (one per GPU, LOCAL_RANK = rank) from this parent, which never touches the
    GPU, and return the worst exit code.  Rank 0 prints the JSON line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    return max(abs(p.wait()) for p in procs)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cpu = None
    if rank == 0 and world_size == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, int(args.partitions))  # before the GPU is initialised (fork pool)

    import torch
    import torch.distributed as dist

    from pipelinedp_amd import native
    from pipelinedp_amd.distributed import World
    from pipelinedp_amd.executor import BoundConfig, HipExecutor, ReleaseConfig

    torch.cuda.set_device(local)
    world = None
    if world_size > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = World(rank, world_size)

    # --share N: this single GPU plays rank N-1 of an N-GPU strong-scaling run (ids rebased, hashed globally)
    split = args.share if args.share > 1 and world_size == 1 else world_size
    vrank = split - 1 if args.share > 1 and world_size == 1 else rank
    n = int(args.rows // split) if args.strong else int(args.rows)
    P = int(args.partitions)
    U = int(args.pids // split) if args.strong else int(args.pids)
    ex = HipExecutor(local)
    pid, pk, val = ex.generate(n, U, P, seed=args.seed, zipf_s=args.zipf, lo=0.0, hi=10.0, row_offset=vrank * n)
    # Multi-GPU: rank r's rows carry its own privacy ids (global id = r * U + local id), so every privacy id
    # lives on one rank (pid-sharded input); the sort uses the dense local ids.
    public = WORKLOADS[args.workload]["public"]
    count_sum = WORKLOADS[args.workload]["metrics"] == "count_sum"
    sweep = WORKLOADS[args.workload]["metrics"] == "analysis"
    variance = WORKLOADS[args.workload]["metrics"] == "variance"
    mask = native.METRIC_COUNT | native.METRIC_SUM | (0 if count_sum else native.METRIC_MEAN)
    if variance:
        mask |= native.METRIC_VARIANCE
    if sweep:
        # UtilityAnalysisOptions(eps=1, delta=1e-6), metrics COUNT+SUM+PRIVACY_ID_COUNT, private selection:
        # NaiveBudgetAccountant gives the GENERIC mechanism eps 1/4 and all of delta
        mask = native.METRIC_COUNT | native.METRIC_SUM | native.METRIC_PRIVACY_ID_COUNT
        ana_cfgs = [native.AnalysisConfig(l0, linf, SWEEP_SUM_BOUNDS[0], SWEEP_SUM_BOUNDS[1],
                                          native.SELECTION_TRUNCATED_GEOMETRIC, 0, 0.25, 1e-6) for l0, linf in SWEEP]
    # rank r's privacy ids are global ids r * U + local id: the sampling hashes the global id (pid_base, ABI 3),
    # so an N-GPU step bounds exactly what one process over the concatenated rows would
    bounds = BoundConfig(mask, args.l0, args.linf, 0.0, 10.0, sampling_seed=args.seed + 1,
                         debug_flags=args.debug_flags, debug_flags2=args.debug_flags2,
                         pid_base=vrank * U if split > 1 else 0)
    # NaiveBudgetAccountant(eps=1, delta=1e-6): MeanCombiner (Laplace) eps 0.5, selection eps 0.5 delta 1e-6
    eps = [0.0] * 6
    delta = [0.0] * 6
    if count_sum:  # public partitions: the whole budget goes to COUNT and SUM (weights 1:1)
        eps[native.MECH_COUNT] = eps[native.MECH_SUM] = 0.5
    elif variance:
        eps[native.MECH_VARIANCE] = 0.5
    else:
        eps[native.MECH_MEAN] = 0.5
    if not public:
        eps[native.MECH_SELECTION], delta[native.MECH_SELECTION] = 0.5, 1e-6
    selection = native.SELECTION_NONE if public else native.SELECTION_TRUNCATED_GEOMETRIC
    rel = ReleaseConfig(mask, native.NOISE_LAPLACE, selection, eps, delta, 1, True, noise_seed=args.seed + 2)
    fields = native.metric_fields(mask)

    # Stream-ordered steps: the accumulate enqueues without waiting for the stream (PDP_BOUND_ASYNC; its
    # status is checked once the timed loop has drained), so consecutive steps run back to back on the GPU
    # and the host enqueues the next step while the current one runs.  Per-step times: hipEvents.
    def step():
        if sweep:
            metrics, prob, pids = ex.analyze(pid, pk, val, U, P, mask, ana_cfgs)
            return (pids > 0,)
        if world is not None:
            return world.aggregate_async(ex, pid, pk, val, U, P, bounds, rel, gather=False)
        acc = ex.accumulate(pid, pk, val, U, P, bounds, sync=False)
        return ex.release(acc, rel, bounds)

    def check_status():
        if world is not None and not sweep:
            world.check_async_status(ex, "cuda")  # every rank's status, before any result is trusted
        if not sweep:
            st_code = ex.status()
            if st_code:
                raise RuntimeError(f"accumulate status {st_code}: {native.lib().pdp_last_error().decode()}")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    check_status()
    st = ex.stats()
    run = step
    graph_res = None
    if args.graph:
        # one step captured once (tests/test_gpu_stream_order.py: replay == eager bit for bit); the release's
        # selection table is built before the capture (pdp_prepare_release)
        if world is not None or sweep:
            raise SystemExit("--graph: one GPU, aggregate workloads only")
        ex.prepare_release(rel, bounds)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            graph_res = step()
        graph.replay()
        torch.cuda.synchronize()
        check_status()

        def run():
            graph.replay()
            return graph_res
    rows_after_public_filter = int(st.kept_rows_in)
    surv = int(st.filter_rows)  # rows that survive the L0 pre-filter (0: it did not run)
    surv_passes = int(st.sort_passes) - 1 if surv else 0
    k4 = (int(st.k4_slots), int(st.k4_pairs), int(st.k4_passes)) if st.k4_slots else None
    if not args.no_profile and not args.graph:
        ex.profile(True)
        ex.profile_read(reset=True)
    if world is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    ev[0].record()
    for i in range(args.steps):
        res = run()
        ev[i + 1].record()  # per-step stamps for the median (no host wait inside the timed loop)
    torch.cuda.synchronize()
    if world is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    check_status()
    if world is not None:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kept_parts = int(res[0].sum().item())

    roofline = None
    stages = {}
    if not args.no_profile and args.graph:
        # replays record no per-stage events: the stage times come from as many eager profiled steps, run after
        # the graph-timed loop
        ex.profile(True)
        ex.profile_read(reset=True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        check_status()
    if not args.no_profile:
        prof = ex.profile_read(reset=True)
        ex.profile(False)
        for s, (ms, cnt) in prof.items():
            if cnt:
                stages[s] = {"ms_per_launch": ms / cnt, "launches_per_step": cnt / args.steps}
        if sweep and "analysis_select" in stages and "analysis_metrics" in stages:
            # the select launches run inside the metrics stage: report k_ana_metrics on its own
            m, sel = stages["analysis_metrics"], stages["analysis_select"]
            m["ms_per_launch"] = (m["ms_per_launch"] * m["launches_per_step"] -
                                  sel["ms_per_launch"] * sel["launches_per_step"]) / m["launches_per_step"]
        dom = max(stages, key=lambda s: stages[s]["ms_per_launch"] * stages[s]["launches_per_step"])
        nb = (P + world_size - 1) // world_size if world else P
        b = stage_bytes(dom, n, rows_after_public_filter, nb, len(fields), surv, surv_passes, k4, variance,
                        "survivor_group" in stages)
        ach = b / (stages[dom]["ms_per_launch"] * 1e-3) / 1e9
        traffic, prof_round = pmc_traffic(dom, n, args.workload) if not sweep else (None, None)
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": None,
                    "traffic_note": "HBM bytes need separate rocprofv3 --pmc passes (FETCH_SIZE x2 on gfx950 + "
                                    "WRITE_SIZE); not measurable inside this run",
                    "traffic_carried": None if traffic is None else {
                        "bytes_per_launch": traffic, "round": prof_round, "source": "profiles/pmc_traffic.json",
                        "label": "CARRIED from the committed PMC profile of this workload size "
                                 "(tools/profile_round.sh), not measured in this run"},
                    "algorithmic_bytes_per_launch": b,
                    **({"bound_note": "c5 kernels are fp64-VALU bound (per-(pair, configuration) SumMetrics terms, "
                                      "Poisson-binomial pmf per partition); the HBM fraction is reported for "
                                      "completeness only"} if sweep else {}),
                    "ms_per_launch_source": "hipEvents on the launch stream, averaged over the timed steps" +
                                            (" (--graph: over as many eager profiled steps after the graph-timed "
                                             "loop)" if args.graph else "")}
        if sweep:
            # fp64-VALU bound: FLOP/s of k_ana_metrics against the box's measured fp64 FMA rate
            import ctypes
            tf = ctypes.c_double(0.0)
            native.check(native.lib().pdp_fp64_probe(ctypes.byref(tf), ex.stream_handle), "pdp_fp64_probe")
            flops = rows_after_public_filter * len(SWEEP) * ANALYSIS_FLOP_PER_PAIR_CONFIG
            ms = stages["analysis_metrics"]["ms_per_launch"]
            ach = flops / (ms * 1e-3) / 1e12
            roofline = {"bound": "fp64", "kernel": "analysis_metrics (k_ana_metrics)", "achieved": round(ach, 2),
                        "peak": round(tf.value, 1), "unit": "TFLOP/s", "frac": round(ach / tf.value, 4),
                        "peak_note": "pdp_fp64_probe: fp64 FMA chains on this box (2 FLOP per FMA); AMD spec "
                                     f"{FP64_SPEC_TFLOPS} TFLOP/s",
                        "frac_of_spec": round(ach / FP64_SPEC_TFLOPS, 4),
                        "algorithmic_flops_per_launch": flops,
                        "flops_note": f"{ANALYSIS_FLOP_PER_PAIR_CONFIG} fp64 operations per (pair, configuration) "
                                      f"x {rows_after_public_filter} pairs x {len(SWEEP)} configurations",
                        "traffic": None,
                        "ms_per_launch_source": "hipEvents on the launch stream (analysis_metrics minus the nested "
                                                "analysis_select), averaged over the timed steps"}
        for s in stages:
            bs = stage_bytes(s, n, rows_after_public_filter, nb, len(fields), surv, surv_passes, k4, variance,
                             "survivor_group" in stages)
            if bs:
                stages[s]["achieved_GBs"] = round(bs / (stages[s]["ms_per_launch"] * 1e-3) / 1e9, 1)

    # bounding statistics of one more (untimed) run: rows and (pid, pk) pairs kept
    kept = {}
    if not sweep:
        acc = ex.accumulate(pid, pk, val, U, P, bounds)
        kept = {"rows_kept_after_bounding": int(acc.count.sum().item()) if acc.count is not None else None,
                "pairs_kept_after_bounding": int(acc.row_count.sum().item())}
        del acc

    rows_per_s = n * world_size * args.steps / elapsed  # (--share: one rank's rows, this GPU alone)
    step_s = sorted(ev[i].elapsed_time(ev[i + 1]) * 1e-3 for i in range(args.steps))
    med = step_s[len(step_s) // 2] if len(step_s) % 2 else 0.5 * (step_s[len(step_s) // 2 - 1] + step_s[len(step_s) // 2])
    copy_gbs = copy_peak_gbs(torch, native.lib()) if rank == 0 and not args.no_profile else None
    if roofline is not None:
        roofline["copy_peak_measured"] = copy_gbs
        roofline["copy_peak_note"] = ("pdp_stream_copy: non-temporal 16-B-per-lane streaming copy of 8 GiB (8 loads "
                                      "in flight per lane, 32768 workgroups), (read + write) bytes / time -- the best "
                                      "of the copy shapes tools/copy_probe.py sweeps (plain / nt loads and stores, "
                                      "2048-32768 workgroups: 4.7-5.6 TB/s; a read-only stream reaches 7.1 TB/s, "
                                      "profiles/r04_copy_probe.json); the achievable ceiling of a read+write kernel "
                                      "next to the 8 TB/s spec peak")
        if copy_gbs and roofline.get("unit") == "GB/s":
            roofline["frac_of_copy"] = round(roofline["achieved"] / copy_gbs, 4)
        if roofline.get("unit") == "GB/s":
            # the guide's measured device copy (the stricter ceiling than this build's own probe)
            roofline["guide_copy"] = GUIDE_COPY_GBS
            roofline["frac_of_guide_copy"] = round(roofline["achieved"] / GUIDE_COPY_GBS, 4)
            roofline["guide_copy_note"] = "device-to-device copy measured by /opt/skills/guides/MI355X_MICROARCH.md:36"

    if rank == 0:
        e2e = rows_per_s * 24 / 1e9
        line = {
            "metric": "input rows/sec (node) for DP COUNT+SUM+MEAN, 1B rows/1M partitions; % HBM peak",
            "value": rows_per_s, "unit": "rows/s", "n_gpus": world_size, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "ms_per_step_median": med * 1e3, "value_median_step": n * world_size / med,
            "median_note": "median of the per-step hipEvent times on rank 0 (BASELINE.md: median); value = K steps / "
                           "total wall time between the synchronised brackets",
            "host_waits_per_step": int(ex.stats().host_waits) if not sweep else None,
            "scaling": "strong" if args.strong else "weak", "vs_baseline": None, "dtype": "f64",
            "launch": "hipGraph replay of one captured step" if args.graph else "eager stream-ordered launches",
            **({"rank_share": {"of_gpus": split, "rank": vrank, "pid_base": vrank * U,
                               "label": "ONE GPU running one rank's share of an N-GPU strong-scaling c3 step "
                                        "(rows and privacy ids / N, all partitions; no collective) -- not SCALE"}}
               if split > 1 and world_size == 1 else {}),
            "data": "synthetic (on-device Philox generator, oracle/pdp_oracle.py:synth_rows)",
            "config": {"workload": (f"c5: UtilityAnalysisEngine.analyze, {len(SWEEP)} configurations "
                                    f"(L0 1..128 x Linf 1..8, sum bounds {SWEEP_SUM_BOUNDS}), COUNT+SUM+PRIVACY_ID_COUNT "
                                    f"per-partition error metrics + truncated-geometric keep probability, "
                                    f"{n:.2e} rows/GPU, {U:.1e} privacy ids, {P:.1e} Zipf({args.zipf}) partitions; "
                                    f"value = input rows/s for the whole analysis") if sweep else
                                   f"{args.workload}: DP {'COUNT+SUM' if count_sum else 'COUNT+SUM+MEAN+VARIANCE' if variance else 'COUNT+SUM+MEAN'}, "
                                   f"{n * world_size:.2e} rows on {world_size} GPU(s) ({n:.2e} rows/GPU), "
                                   f"{U:.1e} privacy ids/GPU, {P:.1e} "
                                   f"{'public uniform' if public else f'Zipf({args.zipf})'} partitions, "
                                   f"L0={args.l0}, Linf={args.linf}, [0,10], Laplace, "
                                   f"{'no selection (public partitions)' if public else 'truncated-geometric selection'}"
                                   f", eps=1 delta=1e-6",
                       "rows_total": n * world_size, "rows_per_gpu": n, "partitions": P, "privacy_ids_per_gpu": U,
                       **({"c4_node_shape": "4e9 rows / 5e7 partitions over 8 GPUs = 5e8 rows per GPU (this line: "
                                            f"{world_size} GPU(s) x 5e8)"} if args.workload == "c4" else {}),
                       "parallelism": f"pid-sharded x{world_size}" + (" + RCCL reduce-scatter" if world else "")},
            "roofline": roofline,
            "roofline_e2e": {"definition": "rows/s x 24 B/row (int64 pid + int64 pk + f64 value read once) / "
                                           "8 TB/s (BASELINE.md:61-64)",
                             "bytes_per_row": 24, "achieved": round(e2e, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": round(e2e / PEAK_HBM_GBS, 4)},
            "cpu_baseline": cpu,
            "reference_cpu_carried": {"value": 66.1e3, "unit": "rows/s", "cores": 1, "plan_item": 1,
                                      "kind": "reference LocalBackend (stubbed PyDP: identity noise, keep-all)",
                                      "where": "measured in the build container, NOT on this box (the reference "
                                               "never ships here); carried from BASELINE.md:28",
                                      "config": "COUNT+SUM+MEAN, 1e6 rows, 1e5 users, 17,770 Zipf(1.1) partitions, "
                                                "L0=2, Linf=1"},
            "fp64_sums": "K4: per-partition sums accumulate in 64-bit fixed point (exact integer adds of each pair "
                         "record's rint(x * 2^F), F = 62 - ceil(log2 max|x|)), so counts, sums and keep decisions are "
                         "identical bit for bit run to run and for any grid (pdp_reduce.inc)",
            "kernels": stages, "rows_after_public_filter": rows_after_public_filter,
            "l0_prefilter_survivors": surv, **kept,
            "k4_pair_slots": k4[0] if k4 else None, "k4_pairs": k4[1] if k4 else None,
            "k4_passes": k4[2] if k4 else None,
            "kept_partitions_rank0": kept_parts,
            "sort_passes": int(st.sort_passes), "bucket_low_bits": int(st.bucket_low_bits),
            "fallback_rows": int(st.fallback_rows),
        }
        if st.sweep_tiles:
            line["sweep_cycles_per_tile"] = {k: round(st.sweep_cycles[i] / st.sweep_tiles)
                                             for i, k in enumerate(("load", "rank", "lookback", "scatter"))}
        print(json.dumps(line), flush=True)
    if world is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
