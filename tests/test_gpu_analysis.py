"""Utility analysis on the MI355X (pdp_utility_analysis through the C ABI and
the host engine) against the reference UtilityAnalysisEngine goldens, the
reference tests' known answers (analysis/tests/utility_analysis_engine_test.py:
157-220, 222-302) and the numpy oracle on random multi-configuration inputs.

Tolerances: fp64 sums 1e-9 relative (summation order); keep probabilities
1e-9 relative (the Poisson-binomial recurrence runs in the same order as the
reference's, pdp_analysis.inc: k_ana_select)."""
import numpy as np
import pytest

import pdp_analysis_oracle as ao
import pdp_oracle as o
from analysis_util import CASES, check_case, run_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ex():
    from pipelinedp_amd.executor import HipExecutor
    return HipExecutor(0)


@pytest.mark.parametrize("name", CASES)
def test_gpu_engine_matches_reference_golden(name):
    import pipelinedp_amd as pdp
    d, got = run_case(name, pdp.HipBackend())
    check_case(d, got)


def test_gpu_reference_known_answers():
    import pipelinedp_amd as pdp
    _, got = run_case("reference_per_partition_errors", pdp.HipBackend())
    assert len(got) == 10
    for v in got.values():
        assert v[1].per_partition_error_max == -10
        assert v[1].expected_cross_partition_error == pytest.approx(-18.0, abs=1e-5)
        assert v[1].std_cross_partition_error == pytest.approx(1.89736, abs=1e-5)
        assert v[1].std_noise == pytest.approx(11.95312, abs=1e-5)


def _cfgs(rng, C, private, l0_choices=None):
    from pipelinedp_amd import native
    sel = [native.SELECTION_TRUNCATED_GEOMETRIC, native.SELECTION_LAPLACE, native.SELECTION_GAUSSIAN]
    out = []
    for c in range(C):
        a = native.AnalysisConfig()
        a.max_partitions_contributed = int(rng.integers(1, 40) if l0_choices is None else rng.choice(l0_choices))
        a.max_contributions_per_partition = int(rng.integers(1, 6))
        a.min_sum_per_partition = float(rng.uniform(-5, 1))
        a.max_sum_per_partition = float(a.min_sum_per_partition + rng.uniform(0.1, 8))
        if private:
            a.selection = sel[c % 3]
            a.selection_eps, a.selection_delta = 1.0, 1e-5
        out.append(a)
    return out


# grouped: at most 5 distinct L0 values, so the selection runs in
# k_ana_select_grouped (one pmf / CDF table per L0); otherwise (> 16 distinct
# L0 values at C = 64, 70) in k_ana_select<true / false>.
@pytest.mark.parametrize("private", [True, False])
@pytest.mark.parametrize("C,grouped", [(1, False), (64, False), (70, False), (64, True), (70, True)])
def test_analysis_matches_oracle_many_configs(ex, private, C, grouped):
    import torch
    from pipelinedp_amd import native
    rng = np.random.default_rng(C + 100 * private + 7 * grouped)
    n, U, P = 40000, 1500, 400
    pid, pk, val = o.synth_rows(n, U, P, seed=C, zipf_s=1.1)
    if not private:
        pk = np.where(pk % 7 == 3, -1, pk)  # non-public rows
    cfgs = _cfgs(rng, C, private, [1, 3, 8, 20, 39] if grouped else None)
    mask = native.METRIC_SUM | native.METRIC_COUNT | native.METRIC_PRIVACY_ID_COUNT
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    metrics, prob, pids = ex.analyze(t(pid), t(pk), t(val), U, P, mask, cfgs)
    torch.cuda.synchronize()
    pairs = ao.preaggregate(pid, pk, val)
    sel = {0: None, 1: "truncated_geometric", 2: "laplace", 3: "gaussian"}
    ocfgs = [ao.AnalysisConfig(c.max_partitions_contributed, c.max_contributions_per_partition,
                               c.min_sum_per_partition, c.max_sum_per_partition, sel[c.selection], c.selection_eps,
                               c.selection_delta) for c in cfgs]
    ref = ao.per_partition(*pairs, P, ocfgs, ["sum", "count", "privacy_id_count"], public=not private)
    m = metrics.cpu().numpy()
    for b, name in enumerate(["sum", "count", "privacy_id_count"]):
        np.testing.assert_allclose(m[:, b], ref[name], rtol=1e-9, atol=1e-8, err_msg=name)
    np.testing.assert_array_equal(pids.cpu().numpy(), np.bincount(pairs[0], minlength=P))
    if private:
        np.testing.assert_allclose(prob.cpu().numpy(), ref["prob_keep"], rtol=1e-9, atol=1e-12)
        assert (pids.cpu().numpy() > 100).any() and ((pids.cpu().numpy() > 0) & (pids.cpu().numpy() <= 100)).any()


def test_preaggregate_matches_oracle(ex):
    import torch
    n, U, P = 30000, 900, 300
    pid, pk, val = o.synth_rows(n, U, P, seed=5, zipf_s=1.1)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    for ns in (P, 120):
        gpk, gc, gs, gn = (a.cpu().numpy() for a in ex.preaggregate(t(pid), t(pk), t(val), U, P, ns))
        rpk, rc, rs, rn = ao.preaggregate(pid, pk, val, num_sampled=ns)
        key_g = np.lexsort((gc, gn, gpk))
        key_r = np.lexsort((rc, rn, rpk))
        np.testing.assert_array_equal(gpk[key_g], rpk[key_r])
        np.testing.assert_array_equal(gc[key_g], rc[key_r])
        np.testing.assert_array_equal(gn[key_g], rn[key_r])
        np.testing.assert_allclose(np.sort(gs), np.sort(rs), rtol=1e-12, atol=1e-12)
        assert gpk.max() < ns


@pytest.mark.parametrize("name", ["private_gaussian", "public_gaussian", "private_laplace"])
def test_gpu_perform_utility_analysis_matches_reference_golden(name):
    """perform_utility_analysis with pdp_utility_aggregate on the GPU against
    the reference goldens (Gaussian quantiles closed form: exact; Laplace:
    the reference's Monte-Carlo estimates by distribution, analysis_util)."""
    import pipelinedp_amd as pdp
    from analysis_util import check_aggregate
    from test_analysis import _agg_as_dicts, run_perform
    d, res = run_perform(name, pdp.HipBackend())
    check_aggregate(d, _agg_as_dicts(res), rtol=1e-8, atol=1e-9, quantile_sigmas=4.0)


@pytest.mark.parametrize("private", [True, False])
@pytest.mark.parametrize("laplace", [True, False])
def test_gpu_aggregate_errors_match_oracle(ex, private, laplace):
    """pdp_utility_aggregate against pdp_analysis_oracle.aggregate_accumulator
    on random multi-configuration per-partition metrics (1e-9 relative: the
    kernel's Newton quantiles and the oracle's bisection agree to ~1e-14)."""
    import torch
    from cpu_executor import CpuExecutor
    from pipelinedp_amd import native
    rng = np.random.default_rng(5 + private + 2 * laplace)
    n, U, P, C = 30000, 2000, 400, 7
    pid, pk, val = o.synth_rows(n, U, P, seed=13, zipf_s=1.2)
    cfgs = _cfgs(rng, C, private)
    mask = native.METRIC_SUM | native.METRIC_COUNT | native.METRIC_PRIVACY_ID_COUNT
    d = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    metrics, prob, pids = ex.analyze(d(pid), d(pk), d(val), U, P, mask, cfgs)
    std = [[float(rng.uniform(0.5, 20.0)) for _ in range(3)] for _ in range(C)]
    kinds = [native.NOISE_LAPLACE if (laplace or c % 2) else native.NOISE_GAUSSIAN for c in range(C)]
    q = [0.1, 0.5, 0.9, 0.99, 0.03]
    err, sel = ex.aggregate_errors(metrics, prob, pids, mask, std, kinds, q, private)
    cpu = CpuExecutor()
    err2, sel2 = cpu.aggregate_errors(metrics.cpu(), None if prob is None else prob.cpu(), pids.cpu(), mask, std, kinds,
                                      q, private)
    np.testing.assert_allclose(err.cpu().numpy(), err2.numpy(), rtol=1e-9, atol=1e-9)
    if private:
        np.testing.assert_allclose(sel.cpu().numpy(), sel2.numpy(), rtol=1e-12, atol=1e-9)
    again, _ = ex.aggregate_errors(metrics, prob, pids, mask, std, kinds, q, private)
    assert torch.equal(err, again)  # fixed-order reduction


@pytest.mark.parametrize("C,private", [(64, True), (70, False)])
def test_gpu_analysis_bitwise_deterministic(ex, C, private):
    """Per-partition utility metrics are identical bit for bit run to run
    (the reference merges accumulators in a fixed order, analysis/combiners.py:
    228-310): partitions cut by a chunk boundary are merged from per-chunk
    slots in chunk order (k_ana_fix), not with fp64 atomics.  Zipf(1.2) keys
    over 3e6 rows: head partitions span hundreds of 2048-pair chunks.  Also
    checked against the oracle (1e-9 relative)."""
    import torch
    from pipelinedp_amd import native
    rng = np.random.default_rng(5 + C)
    n, U, P = 3_000_000, 60_000, 2_000
    pid, pk, val = o.synth_rows(n, U, P, seed=77 + C, zipf_s=1.2, value_lo=-3, value_hi=9)
    cfgs = _cfgs(rng, C, private)
    mask = native.METRIC_SUM | native.METRIC_COUNT | native.METRIC_PRIVACY_ID_COUNT
    d = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    runs = []
    for _ in range(3):
        m, prob, pids = ex.analyze(d(pid), d(pk), d(val), U, P, mask, cfgs)
        torch.cuda.synchronize()
        runs.append((m.cpu().numpy(), None if prob is None else prob.cpu().numpy()))
    for m, prob in runs[1:]:
        np.testing.assert_array_equal(m, runs[0][0])
        if private:
            np.testing.assert_array_equal(prob, runs[0][1])
    sel = {native.SELECTION_NONE: None, native.SELECTION_TRUNCATED_GEOMETRIC: "truncated_geometric",
           native.SELECTION_LAPLACE: "laplace", native.SELECTION_GAUSSIAN: "gaussian"}
    ocfgs = [ao.AnalysisConfig(c.max_partitions_contributed, c.max_contributions_per_partition, c.min_sum_per_partition,
                               c.max_sum_per_partition, sel[c.selection], c.selection_eps, c.selection_delta)
             for c in cfgs[:4]]
    ref = ao.per_partition(*ao.preaggregate(pid, pk, val), P, ocfgs, ["sum", "count", "privacy_id_count"],
                           public=not private)
    for c in range(4):
        for b, name in enumerate(("sum", "count", "privacy_id_count")):
            want = ref[name][c]
            np.testing.assert_allclose(runs[0][0][c, b], want, rtol=1e-9, atol=1e-9 * (np.abs(want).max() + 1.0),
                                       err_msg=f"{c} {name}")


def test_analysis_after_aggregate_on_one_workspace(ex):
    """Workspace reuse across entry points: an aggregate (its look-back passes
    leave record bytes where the analysis layout keeps its look-back status
    words) and then a utility analysis on the same executor and workspace give
    the analysis result of a fresh executor, bit for bit.  Round 4 found the
    status region's clear keyed on the workspace base instead of the region's
    address: at full size the analysis sort met stale bytes that read as
    published status words and scattered out of range (next_epoch)."""
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.executor import BoundConfig, HipExecutor
    n, U, P = 4_000_000, 400_000, 2_000_000
    pid, pk, val = ex.generate(n, U, P, seed=91, zipf_s=0.0, lo=0.0, hi=10.0)
    mask = native.METRIC_COUNT | native.METRIC_SUM
    ex.accumulate(pid, pk, val, U, P, BoundConfig(mask, 32, 4, 0.0, 10.0, sampling_seed=3))
    torch.cuda.synchronize()
    rng = np.random.default_rng(12)
    na, Ua, Pa = 1_000_000, 50_000, 70_000
    apid, apk, aval = ex.generate(na, Ua, Pa, seed=92, zipf_s=1.1, lo=-3.0, hi=9.0)
    cfgs = _cfgs(rng, 8, True)
    amask = native.METRIC_SUM | native.METRIC_COUNT | native.METRIC_PRIVACY_ID_COUNT
    m1, p1, _ = ex.analyze(apid, apk, aval, Ua, Pa, amask, cfgs)
    fresh = HipExecutor(0)
    m2, p2, _ = fresh.analyze(apid, apk, aval, Ua, Pa, amask, cfgs)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(m1.cpu().numpy(), m2.cpu().numpy())
    np.testing.assert_array_equal(p1.cpu().numpy(), p2.cpu().numpy())


def test_analysis_sort_forms_bitwise_equal(ex):
    """The (pk, pid) sort by decoupled look-back (default) and reduce-then-scan
    (debug flag SORT_TILESCAN; its fused first pass still runs by look-back) give
    the same per-partition metrics bit for bit.  A round-4 build took the
    reduce-then-scan tile counts of the fused first pass from the unwritten
    record buffer."""
    import torch
    from pipelinedp_amd import native
    rng = np.random.default_rng(21)
    n, U, P = 600_000, 20_000, 3_000
    pid, pk, val = o.synth_rows(n, U, P, seed=23, zipf_s=1.1, value_lo=-2, value_hi=8)
    cfgs = _cfgs(rng, 16, True)
    mask = native.METRIC_SUM | native.METRIC_COUNT | native.METRIC_PRIVACY_ID_COUNT
    d = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    runs = []
    for form in (0, native.DEBUG_SORT_TILESCAN):
        ex.set_debug(form)
        try:
            m, prob, _ = ex.analyze(d(pid), d(pk), d(val), U, P, mask, cfgs)
            torch.cuda.synchronize()
        finally:
            ex.set_debug(0)
        runs.append((m.cpu().numpy(), prob.cpu().numpy()))
    np.testing.assert_array_equal(runs[0][0], runs[1][0])
    np.testing.assert_array_equal(runs[0][1], runs[1][1])


def test_analysis_npart_forms_bitwise_equal(ex):
    """n_partitions per privacy id from one atomic per pair (default) or from the bucketed LDS
    histogram of the sampled pairs' ids (default; the pairs of partitions that are
    not sampled keep their atomics; debug flag ANA_NPART_ATOMICS forces the atomics): identical
    metrics, keep probabilities and exported pairs,
    with all partitions sampled and with a third of them."""
    import torch
    from pipelinedp_amd import native
    rng = np.random.default_rng(41)
    n, U, P = 500_000, 70_000, 2_000
    pid, pk, val = o.synth_rows(n, U, P, seed=43, zipf_s=1.1, value_lo=-2, value_hi=8)
    cfgs = _cfgs(rng, 16, True)
    mask = native.METRIC_SUM | native.METRIC_COUNT | native.METRIC_PRIVACY_ID_COUNT
    d = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    for ns in (None, P // 3):
        runs = []
        for form in (native.DEBUG_ANA_NPART_ATOMICS, 0):
            ex.set_debug(form)
            try:
                m, prob, ids = ex.analyze(d(pid), d(pk), d(val), U, P, mask, cfgs, num_sampled_partitions=ns)
                pairs = ex.preaggregate(d(pid), d(pk), d(val), U, P, num_sampled_partitions=ns)
                torch.cuda.synchronize()
            finally:
                ex.set_debug(0)
            runs.append([m.cpu().numpy(), prob.cpu().numpy(), ids.cpu().numpy()] +
                        [t.cpu().numpy() for t in pairs])
        for a, b in zip(runs[0], runs[1]):
            np.testing.assert_array_equal(a, b)


def test_analysis_nonpublic_rows_dropped_and_out_of_range_rejected(ex):
    """The fused first sort pass packs rows itself (k_histogram<2> / k_ana_sort_first, as k_ana_pack
    did): rows of non-public partitions (pk < 0) are dropped -- the metrics equal those of the
    remaining rows bit for bit -- and a partition id >= P or a public row's privacy id >= U is an
    error, as in the aggregate path."""
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.native import NativeError
    rng = np.random.default_rng(31)
    n, U, P = 200_000, 5_000, 700
    pid, pk, val = o.synth_rows(n, U, P, seed=37, zipf_s=1.1, value_lo=-1, value_hi=6)
    drop = rng.random(n) < 0.3
    pk_np = pk.copy()
    pk_np[drop] = -1
    cfgs = _cfgs(rng, 8, True)
    mask = native.METRIC_SUM | native.METRIC_COUNT | native.METRIC_PRIVACY_ID_COUNT
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    m1, p1, _ = ex.analyze(d(pid), d(pk_np), d(val), U, P, mask, cfgs)
    keep = ~drop
    m2, p2, _ = ex.analyze(d(pid[keep]), d(pk[keep]), d(val[keep]), U, P, mask, cfgs)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(m1.cpu().numpy(), m2.cpu().numpy())
    np.testing.assert_array_equal(p1.cpu().numpy(), p2.cpu().numpy())
    bad_pk = pk.copy()
    bad_pk[123] = P
    with pytest.raises(NativeError, match="out of range"):
        ex.analyze(d(pid), d(bad_pk), d(val), U, P, mask, cfgs)
    bad_pid = pid.copy()
    bad_pid[456] = U
    with pytest.raises(NativeError, match="out of range"):
        ex.analyze(d(bad_pid), d(pk), d(val), U, P, mask, cfgs)
