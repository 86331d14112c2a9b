"""The multi-GPU path (World.aggregate: [privacy-id shuffle by all-to-all,]
rank-local bound+accumulate, RCCL reduce-scatter of the [P] accumulators,
owner-side release, all-gather) on the nccl (= RCCL) backend with real
device tensors and the HIP library.  One GPU box => world size 1, so these
check the collective calls (dtypes, shapes, layouts, splits) on RCCL; the
world-size-2 data flow is covered by the gloo tests (tests/test_distributed.py).
Must equal the single-process path bit-exactly: the shuffle and the
reduce-scatter of one rank are the identity, K4 sums are exact, and Philox
noise is keyed by the global partition id."""
import socket

import numpy as np
import pytest

import pdp_oracle as o

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def rccl():
    import torch
    import torch.distributed as dist
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("shuffle", [False, True])
def test_world_aggregate_on_rccl_matches_single_process(rccl, shuffle):
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.distributed import World
    from pipelinedp_amd.executor import BoundConfig, HipExecutor, ReleaseConfig

    ex = HipExecutor(0)
    n, U, P = 50000, 900, 777
    pid, pk, val = o.synth_rows(n, U, P, seed=21, zipf_s=1.1)
    d = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    mask = native.METRIC_COUNT | native.METRIC_SUM | native.METRIC_MEAN | native.METRIC_PRIVACY_ID_COUNT
    bounds = BoundConfig(mask, 3, 2, 0.0, 10.0, sampling_seed=5)
    eps = [0.0] * native.NUM_MECH
    delta = [0.0] * native.NUM_MECH
    eps[native.MECH_MEAN], eps[native.MECH_PRIVACY_ID_COUNT] = 0.4, 0.3
    eps[native.MECH_SELECTION], delta[native.MECH_SELECTION] = 0.3, 1e-5
    rel = ReleaseConfig(mask, native.NOISE_LAPLACE, native.SELECTION_TRUNCATED_GEOMETRIC, eps, delta,
                        noise_seed=9)
    world = World(0, 1)
    k1, m1, f1 = world.aggregate(ex, d(pid), d(pk), d(val), U, P, bounds, rel, gather=True, shuffle=shuffle)
    acc = ex.accumulate(d(pid), d(pk), d(val), U, P, bounds)
    k2, m2, f2 = ex.release(acc, rel, bounds)
    torch.cuda.synchronize()
    assert f1 == f2
    np.testing.assert_array_equal(k1.cpu().numpy(), k2[:P].cpu().numpy())
    kept = k2[:P].bool().cpu().numpy()
    a, b = m1.cpu().numpy()[:, kept], m2[:, :P].cpu().numpy()[:, kept]
    np.testing.assert_array_equal(a, b)


def test_shuffle_by_privacy_id_on_rccl_keeps_rows(rccl):
    """World.shuffle_by_privacy_id at world size 1: pdp_shard_rows + the
    all_to_all_single calls return every row, in input order."""
    import torch
    from pipelinedp_amd.distributed import World
    from pipelinedp_amd.executor import HipExecutor
    ex = HipExecutor(0)
    pid, pk, val = o.synth_rows(20000, 700, 300, seed=3)
    d = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    a, b, c = World(0, 1).shuffle_by_privacy_id(ex, d(pid), d(pk), d(val))
    np.testing.assert_array_equal(a.cpu().numpy(), pid)
    np.testing.assert_array_equal(b.cpu().numpy(), pk)
    np.testing.assert_array_equal(c.cpu().numpy(), val)


def test_dp_engine_with_world_on_rccl_matches_single_process(rccl):
    """DPEngine(HipBackend(world=World(0, 1))) on host rows with string keys:
    the cross-rank key dictionaries, num_partitions agreement, privacy-id
    shuffle, reduce-scatter, owner release and all-gather on RCCL, through
    the public API; equal to HipBackend() without a world."""
    import pipelinedp_amd as pdp
    from pipelinedp_amd.distributed import World
    pid, pk, val = o.synth_rows(8000, 400, 60, seed=23, zipf_s=1.1)
    rows = [(f"user{a}", f"movie{b}", float(v)) for a, b, v in zip(pid, pk, val)]

    def run(world):
        backend = pdp.HipBackend(world=world, sampling_seed=5, noise_seed=9)
        acct = pdp.NaiveBudgetAccountant(total_epsilon=10, total_delta=1e-3)
        engine = pdp.DPEngine(acct, backend)
        params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.MEAN,
                                              pdp.Metrics.PRIVACY_ID_COUNT],
                                     max_partitions_contributed=3, max_contributions_per_partition=2,
                                     min_value=0.0, max_value=10.0)
        ex = pdp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                                value_extractor=lambda r: r[2])
        res = engine.aggregate(rows, params, ex)
        acct.compute_budgets()
        return sorted((k, tuple(t)) for k, t in res)

    want = run(None)
    got = run(World(0, 1))
    assert len(want) > 5
    assert [k for k, _ in got] == [k for k, _ in want]
    for (_, g), (_, w) in zip(got, want):
        np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("world_size", [2, 3, 8])
@pytest.mark.parametrize("metrics", ["mean_var", "sum_clip", "sum_partition_bounds", "enforced", "count_only",
                                     "pid_count_only"])
def test_partials_over_emulated_ranks_equal_one_gpu_bitwise(world_size, metrics):
    """The multi-GPU merge without a process group: the rows are split by
    shard_of(pid) into world_size shards, each shard runs
    pdp_bound_accumulate_partials on this GPU, the int64 partials are summed
    (what the RCCL SUM reduce-scatter does, in any order), and
    pdp_finalize_partials converts once.  Counts AND fp64 sums equal one
    pdp_bound_accumulate over all rows bit for bit (K4's fixed point is an
    integer sum), for MEAN + VARIANCE (x and y runs), clipped SUM and SUM with
    per-partition sum bounds; a NaN value makes its partition's sums NaN on
    both paths.  Also contribution_bounds_already_enforced (k_enforced -> K4
    with L_inf = 1) and the COUNT-only / PRIVACY_ID_COUNT-only masks, whose
    partials carry no x / nan rows (Partials.fields_for)."""
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.distributed import shard_of
    from pipelinedp_amd.executor import BoundConfig, HipExecutor, Partials
    ex = HipExecutor(0)
    n, U, P = 120000, 3000, 1500
    pid, pk, val = o.synth_rows(n, U, P, seed=31, zipf_s=1.1, value_lo=-5, value_hi=15)
    # one more privacy id with a single NaN row in partition 5: always kept
    pid, pk, val = np.append(pid, U), np.append(pk, 5), np.append(val, np.nan)
    U += 1
    M = native
    if metrics == "mean_var":
        cfg = BoundConfig(M.METRIC_COUNT | M.METRIC_MEAN | M.METRIC_VARIANCE | M.METRIC_PRIVACY_ID_COUNT, 3, 4,
                          0.0, 10.0, sampling_seed=12)
    elif metrics == "sum_clip":
        cfg = BoundConfig(M.METRIC_COUNT | M.METRIC_SUM, 4, 3, -2.0, 12.0, sampling_seed=12)
    elif metrics == "sum_partition_bounds":
        cfg = BoundConfig(M.METRIC_SUM, 5, 2, None, None, -3.0, 25.0, sampling_seed=12)
    elif metrics == "enforced":
        cfg = BoundConfig(M.METRIC_COUNT | M.METRIC_SUM | M.METRIC_MEAN, 3, 2, 0.0, 10.0,
                          bounds_already_enforced=True, sampling_seed=12)
    elif metrics == "count_only":
        cfg = BoundConfig(M.METRIC_COUNT, 3, 2, sampling_seed=12)
    else:
        cfg = BoundConfig(M.METRIC_PRIVACY_ID_COUNT, 2, 1, sampling_seed=12)
    if metrics in ("count_only", "pid_count_only"):
        assert "x_hi" not in Partials.fields_for(cfg.metrics_mask)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    one = ex.accumulate(d(pid), d(pk), d(val), U, P, cfg)
    shard = shard_of(pid, world_size)
    total = None
    for r in range(world_size):
        m = shard == r
        parts = ex.accumulate_partials(d(pid[m]), d(pk[m]), d(val[m]), U, P, cfg)
        total = parts.data.clone() if total is None else total + parts.data
    acc = ex.finalize_partials(Partials(total, parts.fields, P), cfg)
    torch.cuda.synchronize()
    for name in ("row_count", "count"):
        a, b = getattr(one, name), getattr(acc, name)
        assert (a is None) == (b is None)
        if a is not None:
            assert torch.equal(a, b), name
    for name in ("x", "y"):
        a, b = getattr(one, name), getattr(acc, name)
        assert (a is None) == (b is None)
        if a is not None:
            np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy(), err_msg=name)
    if one.x is not None:
        assert bool(torch.isnan(one.x[5])) and int(torch.isnan(one.x).sum()) == 1


def test_partials_with_an_empty_rank_equal_one_gpu_bitwise():
    """A rank with no rows (possible for small inputs or skewed shards) exports all-zero partials;
    adding them changes nothing: the merge over [rows of rank 0 | no rows] equals one
    pdp_bound_accumulate bit for bit, and an all-empty merge finalises to zero accumulators."""
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.executor import BoundConfig, HipExecutor, Partials
    ex = HipExecutor(0)
    n, U, P = 50000, 2000, 900
    pid, pk, val = o.synth_rows(n, U, P, seed=41, zipf_s=1.1, value_lo=-2, value_hi=9)
    M = native
    cfg = BoundConfig(M.METRIC_COUNT | M.METRIC_MEAN | M.METRIC_VARIANCE, 3, 2, 0.0, 8.0, sampling_seed=5)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    one = ex.accumulate(d(pid), d(pk), d(val), U, P, cfg)
    full = ex.accumulate_partials(d(pid), d(pk), d(val), U, P, cfg)
    e = np.zeros(0, np.int64)
    empty = ex.accumulate_partials(d(e), d(e), d(np.zeros(0)), U, P, cfg)
    torch.cuda.synchronize()
    assert int(empty.data.abs().sum()) == 0
    acc = ex.finalize_partials(Partials(full.data + empty.data, full.fields, P), cfg)
    zero = ex.finalize_partials(Partials(empty.data.clone(), empty.fields, P), cfg)
    torch.cuda.synchronize()
    for name in ("row_count", "count", "x", "y"):
        a, b = getattr(one, name), getattr(acc, name)
        np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy(), err_msg=name)
        assert float(getattr(zero, name).abs().sum()) == 0.0, name


def test_analysis_of_no_rows():
    """An empty input through the utility analysis: every partition has no privacy ids, the keep
    probability is 0 and the metrics are the empty accumulators'."""
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.executor import HipExecutor
    ex = HipExecutor(0)
    e = np.zeros(0, np.int64)
    cfg = native.AnalysisConfig(2, 1, 0.0, 5.0, native.SELECTION_TRUNCATED_GEOMETRIC, 0, 1.0, 1e-5)
    mask = native.METRIC_SUM | native.METRIC_COUNT | native.METRIC_PRIVACY_ID_COUNT
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    m, prob, pids = ex.analyze(d(e), d(e), d(np.zeros(0)), 10, 7, mask, [cfg])
    torch.cuda.synchronize()
    assert float(prob.abs().sum()) == 0.0
    assert int(pids.sum()) == 0
    assert float(m.abs().sum()) == 0.0


def test_rebased_rank_ids_with_pid_base_equal_global_ids_and_filter():
    """ABI 3 pid_base: ranks owning contiguous ranges of global privacy ids
    (the host-rows path, World.exchange_by_key_hash) pass them rebased to
    [0, U_rank) with pid_base = the range start.  The sampling hashes
    pid_base + pid, so the merged partials equal one pdp_bound_accumulate over
    the global ids bit for bit -- and the L0 pre-filter, sized by U_rank, runs on
    every rank (with the global U it would not: 5e6 rows per rank < 4 L0 U = 6.4e6)."""
    import dataclasses

    import torch
    from pipelinedp_amd import native as M
    from pipelinedp_amd.executor import BoundConfig, HipExecutor, Partials
    ex = HipExecutor(0)
    n, P, W = 40_000_000, 100_000, 8  # 5e6 rows per rank: above the filter's 2^22-row minimum
    U = n // 100
    pid, pk, val = ex.generate(n, U, P, seed=77, zipf_s=1.1, lo=-2.0, hi=12.0)  # on-device generator
    cfg = BoundConfig(M.METRIC_COUNT | M.METRIC_SUM | M.METRIC_MEAN | M.METRIC_PRIVACY_ID_COUNT, 4, 2, 0.0, 10.0,
                      sampling_seed=21)
    one = ex.accumulate(pid, pk, val, U, P, cfg)
    torch.cuda.synchronize()
    bounds = [r * U // W for r in range(W + 1)]
    total = None
    for r in range(W):
        m = (pid >= bounds[r]) & (pid < bounds[r + 1])
        n_r, U_r = int(m.sum()), bounds[r + 1] - bounds[r]
        assert (1 << 22) <= n_r < 4 * 4 * U and n_r >= 4 * 4 * U_r  # the filter rule, global U vs rank U
        rc = dataclasses.replace(cfg, pid_base=bounds[r])
        parts = ex.accumulate_partials((pid[m] - bounds[r]).contiguous(), pk[m].contiguous(), val[m].contiguous(),
                                       U_r, P, rc)
        torch.cuda.synchronize()
        assert ex.stats().filter_rows > 0, r
        total = parts.data.clone() if total is None else total + parts.data
    acc = ex.finalize_partials(Partials(total, parts.fields, P), cfg)
    torch.cuda.synchronize()
    assert torch.equal(one.row_count, acc.row_count) and torch.equal(one.count, acc.count)
    np.testing.assert_array_equal(one.x.cpu().numpy(), acc.x.cpu().numpy())
