"""GPU parity at BASELINE.json's full sizes, through size-independent properties.

The CPU oracle cannot run 1e9 rows in test time, so at full size the HIP path
(through the C ABI) is checked against invariants computed independently with
plain torch ops on the same device-resident inputs:

* non-binding bounds (every pid has <= L0 partitions and every pair <= Linf rows,
  asserted on the data): count == bincount(pk) and privacy-id count == distinct
  pids per pk, bit-exact; sum == index_add of the values, |d| <= 1e-9 * (sum of
  |terms| + 1) (fp64, summation order differs) -- the reference's
  `combine_accumulators_per_key` (`pipeline_backend.py:528-538`) with nothing
  sampled away;
* binding bounds (the headline config, c3 shape): each pid keeps exactly
  min(#partitions, L0) partitions (`contribution_bounders.py:90-92`), so
  sum(privacy-id count) == sum_pid min(npk, L0) bit-exact; per pk
  row_count <= count <= min(Linf * row_count, rows of pk)
  (`contribution_bounders.py:74-76`); |sum(clip - mid)| <= count * (b - a) / 2;
* the L0 pre-filter (on by default at this shape): a second run with the
  filter disabled gives identical counts and privacy-id counts, sums to 1e-9.
"""
import pytest

pytestmark = pytest.mark.gpu

MASK_COUNT, MASK_SUM, MASK_MEAN, MASK_PID = 1, 2, 4, 16
NO_FILTER = 134217728  # debug flag: full pid sort, no L0 pre-filter


@pytest.fixture(scope="module")
def ex():
    from pipelinedp_amd.executor import HipExecutor
    return HipExecutor(0)


def _pairs(torch, pid, pk, P):
    """Distinct (pid, pk) pairs as sorted int64 keys pid*P + pk."""
    return torch.unique(pid * P + pk, sorted=True)


def test_non_binding_200m_rows_exact(ex):
    import torch
    from pipelinedp_amd.executor import BoundConfig
    n, U, P, L0, Linf = 200_000_000, 100_000_000, 100_000, 16, 16
    pid, pk, val = ex.generate(n, U, P, seed=0x5EED0002, zipf_s=0.0, lo=0.0, hi=10.0)
    keys = _pairs(torch, pid, pk, P)
    per_pid = torch.bincount(keys // P, minlength=U)
    assert int(per_pid.max()) <= L0
    _, mult = torch.unique_consecutive(torch.sort(pid * P + pk).values, return_counts=True)
    assert int(mult.max()) <= Linf
    del mult

    cfg = BoundConfig(MASK_COUNT | MASK_SUM | MASK_PID, L0, Linf, 0.0, 10.0, sampling_seed=9)
    acc = ex.accumulate(pid, pk, val, U, P, cfg)
    torch.cuda.synchronize()
    assert torch.equal(acc.count, torch.bincount(pk, minlength=P))
    assert torch.equal(acc.row_count, torch.bincount(keys % P, minlength=P))
    ref = torch.zeros(P, dtype=torch.float64, device=pid.device).index_add_(0, pk, val)
    absref = torch.zeros_like(ref).index_add_(0, pk, val.abs())
    assert bool(((acc.x - ref).abs() <= 1e-9 * (absref + 1.0)).all())


def test_headline_1b_rows_binding_invariants(ex):
    import torch
    from pipelinedp_amd.executor import BoundConfig
    n, U, P, L0, Linf, a, b = 1_000_000_000, 10_000_000, 1_000_000, 4, 2, 0.0, 10.0
    pid, pk, val = ex.generate(n, U, P, seed=20250204, zipf_s=1.1, lo=a, hi=b)
    mask = MASK_COUNT | MASK_SUM | MASK_MEAN | MASK_PID
    cfg = BoundConfig(mask, L0, Linf, a, b, sampling_seed=13)
    acc = ex.accumulate(pid, pk, val, U, P, cfg)
    torch.cuda.synchronize()
    assert 0 < ex.stats().filter_rows < n // 5  # the pre-filter ran: survivors only go through the pid sort
    rc, cnt, nsum = acc.row_count.clone(), acc.count.clone(), acc.x.clone()

    rows_pk = torch.bincount(pk, minlength=P)
    keys = _pairs(torch, pid, pk, P)
    del pid, val
    npk = torch.bincount(keys // P, minlength=U)
    assert int(rc.sum()) == int(npk.clamp(max=L0).sum())
    assert bool((rc <= torch.bincount(keys % P, minlength=P)).all())
    del keys, npk
    assert bool((cnt >= rc).all())
    assert bool((cnt <= torch.minimum(Linf * rc, rows_pk)).all())
    assert bool((nsum.abs() <= cnt.to(torch.float64) * (b - a) / 2 + 1e-6).all())

    pid, pk, val = ex.generate(n, U, P, seed=20250204, zipf_s=1.1, lo=a, hi=b)
    nofilter = BoundConfig(mask, L0, Linf, a, b, sampling_seed=13, debug_flags=NO_FILTER)
    acc2 = ex.accumulate(pid, pk, val, U, P, nofilter)
    torch.cuda.synchronize()
    assert ex.stats().filter_rows == 0
    assert torch.equal(acc2.row_count, rc)
    assert torch.equal(acc2.count, cnt)
    absmax = cnt.to(torch.float64) * (b - a) / 2
    assert bool(((acc2.x - nsum).abs() <= 1e-9 * (absmax + 1.0)).all())


def test_c3_release_selection_and_noise_full_size(ex):
    """pdp_release at the headline size (1e9 rows): noise-free means equal
    nsum / max(1, count) + mid (compute_dp_mean, dp_computations.py:353-397);
    with noise, the truncated-geometric keep count lies within 5 sigma of
    sum_p p(n_p) over the observed privacy-id counts (dp_engine.py:312-362)."""
    import math

    import numpy as np
    import torch

    import pdp_oracle as o
    from pipelinedp_amd import native
    from pipelinedp_amd.executor import BoundConfig, ReleaseConfig
    n, U, P, L0, Linf, a, b = 1_000_000_000, 10_000_000, 1_000_000, 4, 2, 0.0, 10.0
    pid, pk, val = ex.generate(n, U, P, seed=20250204, zipf_s=1.1, lo=a, hi=b)
    mask = MASK_COUNT | MASK_SUM | MASK_MEAN
    cfg = BoundConfig(mask, L0, Linf, a, b, sampling_seed=13)
    acc = ex.accumulate(pid, pk, val, U, P, cfg)
    del pid, pk, val
    eps = [0.0, 0.0, 0.5, 0.0, 0.0, 0.5]
    delta = [0.0] * 5 + [1e-6]
    off = ReleaseConfig(mask, native.NOISE_LAPLACE, native.SELECTION_TRUNCATED_GEOMETRIC, eps, delta, 1,
                        add_noise=False, noise_seed=3)
    keep0, out0, fields = ex.release(acc, off, cfg)
    torch.cuda.synchronize()
    assert fields == ["mean", "count", "sum"]
    cnt = acc.count.to(torch.float64)
    mean = acc.x / torch.clamp(cnt, min=1.0) + (a + (b - a) / 2)
    kept0 = keep0.bool()
    assert torch.equal(kept0, acc.row_count > 0)  # noise-free: keep iff p(n) > 0
    assert torch.equal(out0[1][kept0], cnt[kept0])
    assert bool(((out0[0] - mean).abs() <= 1e-12 * mean.abs().clamp(min=1.0))[kept0].all())
    assert bool(torch.isnan(out0[:, ~kept0]).all())  # dropped partitions: not in the result

    on = ReleaseConfig(mask, native.NOISE_LAPLACE, native.SELECTION_TRUNCATED_GEOMETRIC, eps, delta, 1,
                       add_noise=True, noise_seed=4)
    keep, out, _ = ex.release(acc, on, cfg)
    torch.cuda.synchronize()
    table = torch.tensor(o.truncated_geometric_table(0.5, 1e-6, L0), dtype=torch.float64, device=acc.count.device)
    rc = acc.row_count
    p = torch.where(rc < len(table), table[rc.clamp(max=len(table) - 1)], torch.ones_like(table[:1]))
    expect, var = float(p.sum()), float((p * (1 - p)).sum())
    kept = int(keep.sum())
    assert abs(kept - expect) <= 5 * math.sqrt(var) + 1, (kept, expect, var)
    # Laplace(b = L0 * Linf / eps_count) on the released counts of the kept partitions, b = 4 * 2 / 0.25
    kb = keep.bool()
    resid = (out[1][kb] - cnt[kb]).cpu().numpy()
    bscale = L0 * Linf / 0.25
    assert abs(np.mean(np.abs(resid)) - bscale) <= 5 * bscale / math.sqrt(len(resid))


def test_c3_variance_full_size(ex):
    """c3 as BASELINE.json configs[2] defines it: MEAN + VARIANCE (+ COUNT +
    SUM) at 1e9 rows, 1e7 privacy ids, 1e6 Zipf(1.1) partitions, L0 = 4,
    Linf = 2, [0, 10], truncated-geometric selection.  This runs the VARIANCE
    slot array and K4's second (y) run at full size.

    * the L0 pre-filter is exact: filtered == unfiltered bit for bit for
      row_count, count, x AND y (K4 sums in fixed point, so the record order
      of the two paths does not matter);
    * 0 <= y <= count * ((b - a) / 2)^2 (VarianceCombiner.create_accumulator,
      combiners.py:371-381: y = sum of (clip(v) - mid)^2);
    * noise-off release equals compute_dp_var's formulas on the accumulators
      (dp_computations.py:400-459 with _compute_mean_for_normalized_sum
      :310-345): mean_sq = y / max(1, count), var = mean_sq - (x / max(1,
      count))^2, mean = x / max(1, count) + mid, sum = mean * count."""
    import torch

    from pipelinedp_amd import native
    from pipelinedp_amd.executor import BoundConfig, ReleaseConfig
    n, U, P, L0, Linf, a, b = 1_000_000_000, 10_000_000, 1_000_000, 4, 2, 0.0, 10.0
    mask = MASK_COUNT | MASK_SUM | MASK_MEAN | native.METRIC_VARIANCE
    pid, pk, val = ex.generate(n, U, P, seed=20250204, zipf_s=1.1, lo=a, hi=b)
    cfg = BoundConfig(mask, L0, Linf, a, b, sampling_seed=13)
    acc = ex.accumulate(pid, pk, val, U, P, cfg)
    torch.cuda.synchronize()
    assert 0 < ex.stats().filter_rows < n // 5  # the pre-filter ran
    rc, cnt, x, y = acc.row_count.clone(), acc.count.clone(), acc.x.clone(), acc.y.clone()
    del acc
    nofilter = BoundConfig(mask, L0, Linf, a, b, sampling_seed=13, debug_flags=NO_FILTER)
    acc2 = ex.accumulate(pid, pk, val, U, P, nofilter)
    torch.cuda.synchronize()
    assert ex.stats().filter_rows == 0
    assert torch.equal(acc2.row_count, rc)
    assert torch.equal(acc2.count, cnt)
    assert torch.equal(acc2.x, x)
    assert torch.equal(acc2.y, y)
    del acc2, pid, pk, val

    half = (b - a) / 2
    cf = cnt.to(torch.float64)
    assert int(rc.sum()) > 0
    assert bool((y >= 0).all()) and bool((y <= cf * half * half * (1 + 1e-12) + 1e-9).all())
    assert bool((x.abs() <= cf * half + 1e-6).all())
    assert bool((x * x <= y * cf * (1 + 1e-9) + 1e-6).all())  # Cauchy-Schwarz on the kept terms

    eps = [0.0, 0.0, 0.0, 0.5, 0.0, 0.5]
    delta = [0.0] * 5 + [1e-6]
    from pipelinedp_amd.executor import Accumulators
    acc = Accumulators(torch, P, rc.device, mask)
    acc.row_count.copy_(rc)
    acc.count.copy_(cnt)
    acc.x.copy_(x)
    acc.y.copy_(y)
    off = ReleaseConfig(mask, native.NOISE_LAPLACE, native.SELECTION_TRUNCATED_GEOMETRIC, eps, delta, 1,
                        add_noise=False, noise_seed=3)
    keep, out, fields = ex.release(acc, off, cfg)
    torch.cuda.synchronize()
    assert sorted(fields) == ["count", "mean", "sum", "variance"]
    kb = keep.bool()
    assert torch.equal(kb, rc > 0)  # noise-free: keep iff p(n) > 0
    f = {name: out[i][kb] for i, name in enumerate(fields)}
    cf, x, y = cf[kb], x[kb], y[kb]
    den = cf.clamp(min=1.0)
    nmean = x / den
    var = y / den - nmean * nmean
    mean = nmean + (a + half)
    assert torch.equal(f["count"], cf)
    tol = lambda v: 1e-12 * v.abs().clamp(min=1.0)  # noqa: E731  (division order only)
    assert bool(((f["mean"] - mean).abs() <= tol(mean)).all())
    assert bool(((f["variance"] - var).abs() <= tol(var) + 1e-12 * half * half).all())
    assert bool(((f["sum"] - mean * cf).abs() <= tol(mean * cf)).all())


def test_c4_shard_binding_invariants(ex):
    """c4 shard (BASELINE configs[3] per GPU): 5e8 rows, 1.25e7 privacy ids,
    5e7 Zipf(1.1) partitions, L0=32, Linf=4 -- the LDS partition cache under
    real contention and k_unpack_counts over 5e7 partitions."""
    import torch
    from pipelinedp_amd.executor import BoundConfig
    n, U, P, L0, Linf, a, b = 500_000_000, 12_500_000, 50_000_000, 32, 4, 0.0, 10.0
    pid, pk, val = ex.generate(n, U, P, seed=0x5EED0004, zipf_s=1.1, lo=a, hi=b)
    cfg = BoundConfig(MASK_COUNT | MASK_SUM | MASK_MEAN | MASK_PID, L0, Linf, a, b, sampling_seed=21)
    acc = ex.accumulate(pid, pk, val, U, P, cfg)
    torch.cuda.synchronize()
    rc, cnt, nsum = acc.row_count, acc.count, acc.x
    rows_pk = torch.bincount(pk, minlength=P)
    keys = _pairs(torch, pid, pk, P)
    del pid, val
    npk = torch.bincount(keys // P, minlength=U)
    assert int(npk.max()) > L0  # binding
    assert int(rc.sum()) == int(npk.clamp(max=L0).sum())
    assert bool((rc <= torch.bincount(keys % P, minlength=P)).all())
    del keys, npk
    assert bool((cnt >= rc).all())
    assert bool((cnt <= torch.minimum(Linf * rc, rows_pk)).all())
    assert bool((nsum.abs() <= cnt.to(torch.float64) * (b - a) / 2 + 1e-6).all())


def test_c4_partitions_non_binding_exact(ex):
    """5e7 Zipf(1.1) partitions with non-binding bounds (L0=32 -> LDS cache on):
    count == bincount(pk), privacy-id count == distinct pids per pk (exact)."""
    import torch
    from pipelinedp_amd.executor import BoundConfig
    n, U, P, L0, Linf = 200_000_000, 100_000_000, 50_000_000, 32, 16
    pid, pk, val = ex.generate(n, U, P, seed=0x5EED0005, zipf_s=1.1, lo=0.0, hi=10.0)
    keys = _pairs(torch, pid, pk, P)
    assert int(torch.bincount(keys // P, minlength=U).max()) <= L0
    _, mult = torch.unique_consecutive(torch.sort(pid * P + pk).values, return_counts=True)
    assert int(mult.max()) <= Linf
    del mult
    cfg = BoundConfig(MASK_COUNT | MASK_SUM | MASK_PID, L0, Linf, 0.0, 10.0, sampling_seed=9)
    acc = ex.accumulate(pid, pk, val, U, P, cfg)
    torch.cuda.synchronize()
    assert torch.equal(acc.count, torch.bincount(pk, minlength=P))
    assert torch.equal(acc.row_count, torch.bincount(keys % P, minlength=P))
    # fp64 reference sums on the host: torch's device index_add_ serialises on
    # the Zipf head partition (same-address fp64 atomics)
    import numpy as np
    pkh, valh = pk.cpu().numpy(), val.cpu().numpy()
    ref = np.bincount(pkh, weights=valh, minlength=P)
    absref = np.bincount(pkh, weights=np.abs(valh), minlength=P)
    assert np.all(np.abs(acc.x.cpu().numpy() - ref) <= 1e-9 * (absref + 1.0))


def test_c5_utility_analysis_full_size(ex):
    """c5 (BASELINE configs[4]): UtilityAnalysisEngine over 1e8 rows, 1e6
    privacy ids, 1e5 Zipf(1.1) partitions, 64 (L0, Linf) configurations.
    Size-independent checks against plain torch / numpy on the same inputs
    (analysis/combiners.py:228-310, contribution_bounders.py:38-75):
    * per partition, for every configuration: COUNT.sum == rows of the
      partition and PRIVACY_ID_COUNT.sum == distinct privacy ids (exact),
      SUM.sum == the value sum (1e-9 relative);
    * COUNT.per_partition_error_max == sum over pairs of min(0, Linf - count)
      (exact), per_partition_error_min == 0 (counts >= 0);
    * expected cross-partition error <= 0 for COUNT, keep probability in
      [0, 1] and 0 exactly where the partition has no privacy id."""
    import numpy as np
    import torch
    from pipelinedp_amd import native
    n, U, P = 100_000_000, 1_000_000, 100_000
    sweep = [(l0, linf) for l0 in (1, 2, 4, 8, 16, 32, 64, 128) for linf in range(1, 9)]
    pid, pk, val = ex.generate(n, U, P, seed=0x5EED0005, zipf_s=1.1, lo=0.0, hi=10.0)
    cfgs = [native.AnalysisConfig(l0, linf, 0.0, 20.0, native.SELECTION_TRUNCATED_GEOMETRIC, 0, 0.25, 1e-6)
            for l0, linf in sweep]
    mask = native.METRIC_SUM | native.METRIC_COUNT | native.METRIC_PRIVACY_ID_COUNT
    metrics, prob, pids = ex.analyze(pid, pk, val, U, P, mask, cfgs)
    torch.cuda.synchronize()
    assert metrics.shape == (len(cfgs), 3, 5, P)

    rows_pk = torch.bincount(pk, minlength=P).to(torch.float64)
    keys, mult = torch.unique(pid * P + pk, sorted=True, return_counts=True)
    kpk = keys % P
    distinct = torch.bincount(kpk, minlength=P)
    assert torch.equal(pids, distinct)
    pkh, valh = pk.cpu().numpy(), val.cpu().numpy()
    vsum = np.bincount(pkh, weights=valh, minlength=P)
    vabs = np.bincount(pkh, weights=np.abs(valh), minlength=P)
    m = metrics.cpu().numpy()
    for c, (l0, linf) in enumerate(sweep):
        assert np.array_equal(m[c, 1, 0], rows_pk.cpu().numpy()), c
        assert np.array_equal(m[c, 2, 0], distinct.to(torch.float64).cpu().numpy()), c
        assert np.all(np.abs(m[c, 0, 0] - vsum) <= 1e-9 * (vabs + 1.0)), c
        assert np.all(m[c, 1, 1] == 0.0), c
        assert np.all(m[c, 1, 3] <= 0.0), c
    kpkh, multh = kpk.cpu().numpy(), mult.cpu().numpy()
    for linf in (1, 4, 8):
        c = sweep.index((1, linf))
        err_max = np.bincount(kpkh, weights=np.minimum(linf - multh, 0).astype(np.float64), minlength=P)
        assert np.array_equal(m[c, 1, 2], err_max), linf
    pr = prob.cpu().numpy()
    assert pr.shape == (len(cfgs), P)
    assert np.all((pr >= 0.0) & (pr <= 1.0 + 1e-12))
    assert np.all(pr[:, distinct.cpu().numpy() == 0] == 0.0)


def test_c2_public_partitions_full_size(ex):
    """c2 (BASELINE configs[1]) at full size: 1e8 rows, 1e6 uniform privacy
    ids, 2e5 partitions of which the 1e5 even ones are public, so half the rows
    really drop (_drop_not_public_partitions, dp_engine.py:283-297) before
    bounding; COUNT + SUM + PRIVACY_ID_COUNT, L0 = 8, Linf = 4, through the L0
    pre-filter.  Each privacy id keeps min(#public partitions, L0) partitions;
    per public partition row_count <= count <= min(Linf * row_count, rows);
    sums of values clipped to [0, 10] lie in [0, 10 * count]; the unfiltered
    path gives the same counts bit for bit."""
    import torch
    from pipelinedp_amd.executor import BoundConfig
    n, U, P2, L0, Linf, a, b = 100_000_000, 1_000_000, 200_000, 8, 4, 0.0, 10.0
    pid, pk2, val = ex.generate(n, U, P2, seed=0xC2, zipf_s=0.0, lo=-2.0, hi=12.0)
    pk = torch.where(pk2 % 2 == 0, pk2 // 2, torch.full_like(pk2, -1))  # public: even keys -> dense ids
    del pk2
    P = P2 // 2
    mask = MASK_COUNT | MASK_SUM | MASK_PID
    cfg = BoundConfig(mask, L0, Linf, a, b, sampling_seed=21)
    acc = ex.accumulate(pid, pk, val, U, P, cfg)
    torch.cuda.synchronize()
    st = ex.stats()
    assert st.kept_rows_in == int((pk >= 0).sum())
    assert 0 < st.filter_rows < st.kept_rows_in  # the pre-filter ran
    rc, cnt, sm = acc.row_count.clone(), acc.count.clone(), acc.x.clone()

    pub = pk >= 0
    ppid, ppk = pid[pub], pk[pub]
    rows_pk = torch.bincount(ppk, minlength=P)
    keys = _pairs(torch, ppid, ppk, P)
    del ppid, ppk, pub
    npk = torch.bincount(keys // P, minlength=U)
    assert int(rc.sum()) == int(npk.clamp(max=L0).sum())
    assert bool((rc <= torch.bincount(keys % P, minlength=P)).all())
    del keys, npk
    assert bool((cnt >= rc).all())
    assert bool((cnt <= torch.minimum(Linf * rc, rows_pk)).all())
    assert bool((sm >= -1e-9).all()) and bool((sm <= b * cnt.to(torch.float64) + 1e-6).all())

    nofilter = BoundConfig(mask, L0, Linf, a, b, sampling_seed=21, debug_flags=NO_FILTER)
    acc2 = ex.accumulate(pid, pk, val, U, P, nofilter)
    torch.cuda.synchronize()
    assert ex.stats().filter_rows == 0
    assert torch.equal(acc2.row_count, rc)
    assert torch.equal(acc2.count, cnt)
    assert bool(((acc2.x - sm).abs() <= 1e-9 * (b * cnt.to(torch.float64) + 1.0)).all())


def test_more_than_2_32_rows_k4_equals_two_halves(ex):
    """4.4e9 rows (> 2^32) in ONE call keep K4's fixed-point reduction (round
    4 fell back to fp64 atomics at >= 2^32 rows): privacy id = row // 16, each
    privacy id's 16 rows in 16 distinct partitions (pk = 7919 row mod P), so
    with L0 = 4 every privacy id keeps exactly 4 single-row pairs:
    sum(row_count) == sum(count) == 4 U.  Two privacy-id-disjoint halves
    (< 2^32 rows each) through pdp_bound_accumulate_partials, summed, give
    the same accumulators bit for bit -- the merge of pipeline_backend.py:528-538
    whatever the split.  COUNT + PRIVACY_ID_COUNT (no value column: 16 B/row,
    70 GB of input + ~160 GB of workspace)."""
    import torch
    from pipelinedp_amd.executor import BoundConfig
    n, P, L0, Linf = 4_400_000_000, 1_000_000, 4, 1
    U = n // 16
    assert n > (1 << 32) and (n // 2) < (1 << 32)
    dev = torch.device("cuda", 0)
    # built in slices: this torch build's elementwise kernels (arange, ...) fill only numel mod 2^32
    # elements of a tensor with more than 2^32 (round 5, tools/diag_big3.py)
    C = 1 << 30
    pid = torch.empty(n, dtype=torch.int64, device=dev)
    pk = torch.empty(n, dtype=torch.int64, device=dev)
    per_pk = torch.zeros(P, dtype=torch.int64, device=dev)
    for c0 in range(0, n, C):
        r = torch.arange(c0, min(n, c0 + C), dtype=torch.int64, device=dev)
        pid[c0:c0 + r.numel()] = r // 16
        pk[c0:c0 + r.numel()] = r.mul_(7919).remainder_(P)
        per_pk += torch.bincount(pk[c0:c0 + r.numel()], minlength=P)
        del r
    assert int(pid[-1]) == (n - 1) // 16 and int(pk[-1]) == (n - 1) * 7919 % P
    cfg = BoundConfig(MASK_COUNT | MASK_PID, L0, Linf, sampling_seed=5)
    acc = ex.accumulate(pid, pk, None, U, P, cfg)
    torch.cuda.synchronize()
    st = ex.stats()
    assert 0 < st.k4_pairs <= 4 * U and st.fallback_rows == 0  # (the hot-partition tables take some pairs)
    rc, cnt = acc.row_count.clone(), acc.count.clone()
    del acc
    assert int(rc.sum()) == 4 * U and int(cnt.sum()) == 4 * U
    assert torch.equal(rc, cnt)  # every kept pair is one row
    assert bool((rc <= per_pk).all())
    h = n // 2  # a multiple of 16: the halves share no privacy id
    total = None
    for lo in (0, h):
        parts = ex.accumulate_partials(pid[lo:lo + h], pk[lo:lo + h], None, U, P, cfg)
        total = parts.data.clone() if total is None else total + parts.data
        del parts
    torch.cuda.synchronize()
    assert torch.equal(total[0], rc) and torch.equal(total[1], cnt)
