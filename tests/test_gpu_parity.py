"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
reference golden vectors.

Tolerances: counts / privacy-id counts / keep decisions bit-exact.  fp64
sums bit-exact too (check_acc with the bounds): every K2 kernel and the
generic path sum a (pid, pk) group's kept rows in input order, as the oracle
does (np.bincount over the stably sorted rows) and as the reference's
per-group create_accumulator does (combiners.py:305-311, 364-373), and K4 adds
the pairs' rint(x 2^F) exactly, so GPU x / y == o.k4_finalize(o.k4_partials(
...)) bit for bit.  (Tolerance |d| <= 1e-9 (sum |terms| + 1) remains only for
the fp64-atomic forms: NO_K4 and the parameter sweep.)
Noisy outputs with identical Philox draws rel 1e-9 (libm ulps).
"""
import math

import numpy as np
import pytest

import pdp_oracle as o
from golden_util import aggregate_cases, encode_case, load

pytestmark = pytest.mark.gpu

MASK = {"count": 1, "sum": 2, "mean": 4, "variance": 8, "privacy_id_count": 16}


@pytest.fixture(scope="module")
def ex():
    from pipelinedp_amd.executor import HipExecutor
    return HipExecutor(0)


def _dev(a, torch):
    return None if a is None else torch.from_numpy(np.ascontiguousarray(a)).cuda()


BATCH_KERNEL = 4096  # debug flag: k_segments (register bitonic batches) instead of k_lean
NO_K4, K4_P16, K4_SOA, ODD_GRID = 1, 2, 4, 8  # debug flags (native.DEBUG_*): alternative forms


def run_gpu(ex, pid, pk, val, U, P, bp: o.BoundParams, mask, seed=3, fallback=False, debug_flags=0, debug_flags2=0):
    import torch
    from pipelinedp_amd.executor import BoundConfig
    cfg = BoundConfig(mask, bp.max_partitions_contributed, bp.max_contributions_per_partition, bp.min_value,
                      bp.max_value, bp.min_sum_per_partition, bp.max_sum_per_partition,
                      bp.contribution_bounds_already_enforced, seed, fallback, debug_flags, debug_flags2)
    acc = ex.accumulate(_dev(pid, torch), _dev(pk, torch), _dev(val, torch), U, P, cfg)
    torch.cuda.synchronize()
    g = lambda t: None if t is None else t.cpu().numpy()  # noqa: E731
    return cfg, acc, g(acc.row_count), g(acc.count), g(acc.x), g(acc.y)


def check_acc(ref, rc, cnt, x, y, mask, value=None, bp=None):
    np.testing.assert_array_equal(rc, ref.row_count)
    if cnt is not None:
        np.testing.assert_array_equal(cnt, ref.count)
    if bp is not None:
        # input-order pair sums + exact fixed-point merge: bit for bit (module docstring)
        kx, ky = o.k4_finalize(o.k4_partials(ref, len(rc), bp, mask), bp, mask)
        if x is not None and kx is not None:
            np.testing.assert_array_equal(x, kx)
        if y is not None and ky is not None:
            np.testing.assert_array_equal(y, ky)
    scale = 1e-9 * ((ref.count + 1) * (1.0 if value is None else max(1.0, float(np.abs(value).max())))**2) + 1e-9
    if mask & (4 | 8):
        assert np.all(np.abs(x - ref.nsum) <= scale)
        if mask & 8:
            assert np.all(np.abs(y - ref.nsumsq) <= scale)
    elif mask & 2:
        assert np.all(np.abs(x - ref.sum) <= scale)


CONFIGS = [
    # n, U, P, zipf, L0, Linf, vb, pb, mask
    (30000, 500, 200, 1.1, 3, 2, (0.0, 10.0), None, 1 | 2 | 4),
    (30000, 50, 1000, 0.0, 4, 1, (0.0, 10.0), None, 1 | 2 | 16),
    (50000, 4000, 3000, 1.3, 2, 3, (-2.0, 7.0), None, 1 | 2 | 4 | 8),
    (20000, 300, 100, 0.0, 5, 2, None, (-5.0, 40.0), 1 | 2),
    (20000, 20, 50, 0.0, 60, 60, None, None, 1 | 16),  # non-binding, big pid buckets
    (25000, 3, 7, 0.0, 2, 5, (1.0, 5.0), None, 1 | 2 | 4 | 16),  # pids with > 2048 rows -> generic path
    (5000, 5000, 1, 0.0, 1, 1, (0.0, 1.0), None, 1 | 2),  # one partition
    (4000, 1, 3000, 1.1, 7, 2, (0.0, 10.0), None, 1 | 4 | 16),  # one privacy id
    (60000, 400, 5000, 1.1, 4, 2, (0.0, 10.0), None, 1 | 2 | 4),  # ~150 rows / pid: lean + big-batch kernels
    (40000, 2000, 300, 1.3, 16, 1, (0.0, 5.0), None, 1 | 4 | 8 | 16),  # largest L0 of the lean kernel
    (30000, 1000, 3, 0.0, 2, 8, (0.0, 10.0), None, 1 | 2),  # groups of > 4 kept rows (wave-sum path)
    (40000, 500, 3000, 1.1, 32, 2, (0.0, 10.0), None, 1 | 2 | 4 | 16),  # c4-like L0=32, binding for some pids
    (30000, 250, 20000, 0.0, 64, 3, (-1.0, 9.0), None, 1 | 4 | 8 | 16),  # L0=64: every lane holds a kept group
    (30000, 250, 20000, 0.0, 65, 3, (0.0, 10.0), None, 1 | 2),  # L0 > 64: lean with two output slots per lane
    (30000, 200, 20000, 0.0, 128, 2, (0.0, 10.0), None, 1 | 4 | 16),  # largest L0 of the lean kernel
    (30000, 200, 20000, 0.0, 129, 2, (0.0, 10.0), None, 1 | 2 | 16),  # L0 > 128: batch kernel
    (40000, 400, 40, 1.1, 16, 2, (0.0, 10.0), None, 1 | 2 | 4 | 16),  # sorted K2 + second (L_inf) sort
    (20000, 400, 12, 0.0, 17, 3, (-1.0, 4.0), None, 1 | 4 | 8),  # sorted K2, every group over L_inf
    (12000, 200, 500, 1.1, 70, 1, (0.0, 10.0), None, 1 | 2 | 16),  # sorted K2 with two output slots
    (40000, 300, 500, 1.1, 3, 12, (0.0, 10.0), None, 1 | 2 | 4 | 8 | 16),  # pre-filter with L_inf > 8: k_lean
    (60000, 150, 2000, 1.2, 8, 8, (-1.0, 6.0), (-2.0, 30.0), 1 | 2),  # largest thin L0 / L_inf, sum bounds
    (30000, 2, 3, 0.0, 2, 4, (0.0, 10.0), None, 1 | 2 | 4 | 8 | 16),  # (pid, pk) groups of ~5000 rows: big-group kernel
]


LEAN_MIN_SEARCH = 1048576  # debug flag: k_lean ranks L0 by minimum searches also for L0 >= 16
NO_FILTER = 134217728  # debug flag: never use the L0 pre-filter
FORCE_FILTER = 268435456  # debug flag: L0 pre-filter whenever L0 <= 8 (small inputs too)
NO_THIN = 536870912  # debug flag: the pre-filter's survivors go through k_lean, not k_thin
FILTER_MAX_L0 = 8


@pytest.mark.parametrize("mode", ["lean", "lean_min_search", "batch", "fallback", "filter", "filter_lean",
                                  "filter_batch", "filter_fallback", "filter_rec8"])
@pytest.mark.parametrize("cfgi", range(len(CONFIGS)))
def test_bound_accumulate_matches_oracle(ex, cfgi, mode):
    """filter*: the L0 pre-filter forced on; filter_rec8: its bucket pass with 8-byte {pk, row index}
    records, k_filter gathering the survivors' values (round-6 experiment, debug2 FILTER_REC8)."""
    n, U, P, z, L0, Linf, vb, pb, mask = CONFIGS[cfgi]
    pid, pk, val = o.synth_rows(n, U, P, seed=100 + cfgi, zipf_s=z, value_lo=-5, value_hi=15)
    bp = o.BoundParams(L0, Linf, *(vb or (None, None)), *(pb or (None, None)))
    need_val = bool(mask & (2 | 4 | 8))
    _, _, rc, cnt, x, y = run_gpu(ex, pid, pk, val if need_val else None, U, P, bp, mask, seed=77 + cfgi,
                                  fallback=mode in ("fallback", "filter_fallback"),
                                  debug_flags={"batch": BATCH_KERNEL, "lean_min_search": LEAN_MIN_SEARCH,
                                               "filter": FORCE_FILTER, "filter_fallback": FORCE_FILTER,
                                               "filter_lean": FORCE_FILTER | NO_THIN, "filter_rec8": FORCE_FILTER,
                                               "filter_batch": FORCE_FILTER | BATCH_KERNEL}.get(mode, 0),
                                  debug_flags2=2 if mode == "filter_rec8" else 0)
    ref = o.bound_and_accumulate(pid, pk, val if need_val else None, P, bp, "hash", seed=77 + cfgi)
    check_acc(ref, rc, cnt, x, y, mask, val, bp)
    st = ex.stats()
    if cfgi == 5 and "fallback" not in mode:
        assert st.fallback_rows > 0  # huge privacy ids went through the generic path
    if mode.startswith("filter"):
        assert (st.filter_rows > 0) == (L0 <= FILTER_MAX_L0)  # the pre-filter ran (and kept rows)
        if L0 <= FILTER_MAX_L0:  # exactly the restated filter's survivors (pdp_oracle.prefilter_survivors)
            assert st.filter_rows == int(o.prefilter_survivors(pid, pk, 77 + cfgi, L0).sum())


@pytest.mark.parametrize("L0,Linf,z,rows_per_pid", [(1, 1, 1.1, 100), (2, 3, 0.0, 100), (4, 2, 1.1, 100),
                                                    (8, 4, 0.0, 100), (8, 1, 1.3, 100), (2, 2, 1.1, 14)])
def test_prefilter_matches_unfiltered_at_scale(ex, L0, Linf, z, rows_per_pid):
    """The L0 pre-filter (automatic at this size: 2^22 rows) against the same
    run with the filter disabled, and both against the oracle: counts and
    privacy-id counts bit-exact, sums to 1e-9; the survivors are a small
    share of the rows.  With 14 rows per pid, U ~ 3e5 > 2^16: privacy ids of
    different buckets share their low 16 bits, the survivor sort's key."""
    n, P = 1 << 22, 200000
    U = n // rows_per_pid
    pid, pk, val = o.synth_rows(n, U, P, seed=500 + L0, zipf_s=z, value_lo=-5, value_hi=15)
    bp = o.BoundParams(L0, Linf, 0.0, 10.0)
    mask = 1 | 2 | 4 | 16
    _, _, rc, cnt, x, _ = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=9)
    surv = ex.stats().filter_rows
    assert 0 < surv < (n // 2 if rows_per_pid >= 100 else n)
    assert surv == int(o.prefilter_survivors(pid, pk, 9, L0).sum())  # the restated filter, row for row
    _, _, rc2, cnt2, x2, _ = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=9, debug_flags=NO_FILTER)
    assert ex.stats().filter_rows == 0
    np.testing.assert_array_equal(rc, rc2)
    np.testing.assert_array_equal(cnt, cnt2)
    np.testing.assert_allclose(x, x2, rtol=1e-9, atol=1e-9)
    ref = o.bound_and_accumulate(pid, pk, val, P, bp, "hash", seed=9)
    check_acc(ref, rc, cnt, x, None, mask, val, bp)
    # the 8-byte bucket records (values gathered by row index, debug2 FILTER_REC8), the bucket pass
    # without its low-level-first order within a tile's bucket run (debug2 NO_CLASS_SPLIT) and K2's
    # 2048-row chunks (debug2 THIN_CHUNK_2048, the c3-sized choice): the same survivors and
    # accumulators, bit for bit
    for flags2 in (2, 16, 32):
        _, _, rc3, cnt3, x3, _ = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=9, debug_flags2=flags2)
        assert ex.stats().filter_rows == surv
        for a, b in ((rc, rc3), (cnt, cnt3), (x, x3)):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("U,P", [(1 << 14, 20), (1 << 18, 12)])
def test_prefilter_dense_survivor_batches(ex, U, P):
    """Few partitions per privacy id (P <= 20, L0 = 8): nearly every row survives the L0 pre-filter, so
    k_filter's compaction batches overflow its LDS stage (direct stores) and a wave's 2048 rows need
    several gather rounds (count pass first, round 6).  U = 2^14: 64 ids per bucket, the filter's digit
    order is the whole grouping; U = 2^18: 1024 ids per bucket, k_group finishes it.  Against the
    unfiltered path bit for bit and the oracle."""
    n = 1 << 22
    pid, pk, val = o.synth_rows(n, U, P, seed=700 + P, zipf_s=0.0, value_lo=-5, value_hi=15)
    bp = o.BoundParams(8, 3, 0.0, 10.0)
    mask = 1 | 2 | 4 | 16
    _, _, rc, cnt, x, _ = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=31, debug_flags=FORCE_FILTER)
    surv = ex.stats().filter_rows
    assert surv > n // 2  # dense: most rows survive
    assert surv == int(o.prefilter_survivors(pid, pk, 31, 8).sum())
    _, _, rc2, cnt2, x2, _ = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=31, debug_flags=NO_FILTER)
    for a, b in ((rc, rc2), (cnt, cnt2), (x, x2)):
        np.testing.assert_array_equal(a, b)
    ref = o.bound_and_accumulate(pid, pk, val, P, bp, "hash", seed=31)
    check_acc(ref, rc, cnt, x, None, mask, val, bp)


@pytest.mark.parametrize("flags2", [0, 16])
def test_prefilter_with_non_public_rows(ex, flags2):
    """The pre-filter's bucket pass places a non-public row (pk < 0) in its privacy id's bucket with a
    "dropped" tag (k_filter never keeps it) and orders each tile's bucket run by level class.  With 30 %
    of the rows non-public, the oracle's accumulators bit for bit (also without the class split:
    NO_CLASS_SPLIT)."""
    n, U, P = 1 << 21, 20000, 30000
    pid, pk, val = o.synth_rows(n, U, P, seed=41, zipf_s=1.1, value_lo=-5, value_hi=15)
    rng = np.random.default_rng(41)
    pk = np.where(rng.random(n) < 0.3, -1, pk)
    for L0, Linf in ((2, 2), (5, 3)):
        bp = o.BoundParams(L0, Linf, 0.0, 10.0)
        mask = 1 | 2 | 4 | 16
        _, _, rc, cnt, x, _ = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=23, debug_flags=FORCE_FILTER,
                                      debug_flags2=flags2)
        st = ex.stats()
        assert st.filter_rows > 0 and st.kept_rows_in == int((pk >= 0).sum())
        ref = o.bound_and_accumulate(pid, pk, val, P, bp, "hash", seed=23)
        check_acc(ref, rc, cnt, x, None, mask, val, bp)
        assert st.filter_rows == int(o.prefilter_survivors(pid, pk, 23, L0).sum())


@pytest.mark.parametrize("L0,Linf,rows_per_pid,zipf", [(1, 1, 4, 0.0), (2, 3, 6, 1.1), (4, 2, 5, 1.3),
                                                         (8, 4, 16, 0.0)])
def test_survivor_grouping_forms_bitwise_equal(ex, L0, Linf, rows_per_pid, zipf):
    """Privacy-id buckets wider than 256 ids (here U = 2^19: 2048 ids per bucket, 11 low bits) take two
    survivor-grouping steps: k_filter writes each bucket's survivors ordered by the low digit, then the
    LDS grouping of each (bucket, low digit) sub-run (k_group, round 6).  Against look-back passes on the
    remaining bits (debug2 NO_GROUP) and the device-side fallback that hands every sub-run to the
    look-back pass (debug2 GROUP_FALLBACK): identical accumulators, bit for bit, and the oracle's."""
    n, P = 1 << 21, 50000
    U = 1 << 19 if rows_per_pid < 16 else 1 << 17
    pid, pk, val = o.synth_rows(n, U, P, seed=600 + L0, zipf_s=zipf, value_lo=-5, value_hi=15)
    bp = o.BoundParams(L0, Linf, 0.0, 10.0)
    mask = 1 | 2 | 4 | 16
    runs = []
    for flags2 in (0, 4, 8):  # default, NO_GROUP, GROUP_FALLBACK
        _, _, rc, cnt, x, _ = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=13, debug_flags=FORCE_FILTER,
                                      debug_flags2=flags2)
        st = ex.stats()
        assert st.filter_rows > 0 and st.sort_passes == 3  # bucket pass + two grouping steps
        runs.append((rc, cnt, x))
    for other in runs[1:]:
        for a, b in zip(runs[0], other):
            np.testing.assert_array_equal(a, b)
    ref = o.bound_and_accumulate(pid, pk, val, P, bp, "hash", seed=13)
    check_acc(ref, runs[0][0], runs[0][1], runs[0][2], None, mask, val, bp)


def test_full_width_privacy_ids_and_wide_partition_ids(ex):
    """Privacy ids over the whole 32-bit domain (U = 2^32, including 0 and
    2^32 - 1: four radix passes) and partition ids near a 2^24 + 1 domain,
    binding bounds, against the oracle."""
    rng = np.random.default_rng(2024)
    U, P, n = 1 << 32, (1 << 24) + 1, 40000
    ids = np.unique(np.concatenate([[0, U - 1], rng.integers(0, U, 600)]))
    pid = rng.choice(ids, n).astype(np.int64)
    pid[:50] = U - 1
    pk = rng.choice(np.concatenate([[0, P - 1], rng.integers(0, P, 900)]), n).astype(np.int64)
    val = rng.uniform(-5, 15, n)
    bp = o.BoundParams(3, 2, 0.0, 10.0)
    for fallback in (False, True):
        _, _, rc, cnt, x, _ = run_gpu(ex, pid, pk, val, U, P, bp, 1 | 4 | 16, seed=31, fallback=fallback)
        ref = o.bound_and_accumulate(pid, pk, val, P, bp, "hash", seed=31)
        check_acc(ref, rc, cnt, x, None, 1 | 4 | 16, val, bp)
    assert ex.stats().sort_passes == 4


@pytest.mark.parametrize("U", [15_000_000, 20_000_000])
@pytest.mark.parametrize("L0,Linf", [(1, 1), (4, 2), (8, 3)])
def test_prefilter_half_sketch_wide_buckets(ex, L0, Linf, U):
    """U = 1.5e7 privacy ids: buckets of ~58,600 ids, wider than the LDS
    holds at 32 bits per id, so the filter uses 16-bit sketches (2 levels
    per octave).  U = 2e7: buckets of ~78,100 ids, 17 low bits -- the
    filter's digit order on the low byte, then look-back passes on bits 8-16
    (no LDS grouping).  20,000 ids spread over the whole range carry ~100
    rows each.  Survivors equal the restatement's; bounding equals the
    oracle."""
    rng = np.random.default_rng(11 + L0)
    P, n = 50_000, 1 << 21
    assert o.prefilter_sketch_bits(U) == 16
    ids = rng.choice(U, 20000, replace=False)
    pid = ids[rng.integers(0, len(ids), n)].astype(np.int64)
    pk = np.minimum(rng.zipf(1.3, n) - 1, P - 1).astype(np.int64)
    val = rng.uniform(-5, 15, n)
    bp = o.BoundParams(L0, Linf, 0.0, 10.0)
    mask = 1 | 2 | 4 | 16
    _, _, rc, cnt, x, _ = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=21, debug_flags=FORCE_FILTER)
    surv = ex.stats().filter_rows
    assert surv == int(o.prefilter_survivors(pid, pk, 21, L0, 16).sum())
    assert surv < n
    ref = o.bound_and_accumulate(pid, pk, val, P, bp, "hash", seed=21)
    check_acc(ref, rc, cnt, x, None, mask, val, bp)


@pytest.mark.parametrize("flags", [0, FORCE_FILTER])
def test_dropped_rows_and_public_partitions(ex, flags):
    n, U, P = 20000, 800, 400
    pid, pk, val = o.synth_rows(n, U, P, seed=9)
    pk = np.where(pk % 3 == 0, -1, pk)  # non-public rows dropped
    bp = o.BoundParams(3, 2, 0.0, 10.0)
    _, _, rc, cnt, x, _ = run_gpu(ex, pid, pk, val, U, P, bp, 1 | 2 | 16, debug_flags=flags)
    assert ex.stats().kept_rows_in == int((pk >= 0).sum())
    assert (ex.stats().filter_rows > 0) == bool(flags)
    ref = o.bound_and_accumulate(pid, pk, val, P, bp, "hash", seed=3)
    check_acc(ref, rc, cnt, x, None, 1 | 2 | 16, val, bp)
    assert rc[::3].sum() == 0
    pk_all = np.full(n, -1)
    _, _, rc, cnt, x, _ = run_gpu(ex, pid, pk_all, val, U, P, bp, 1 | 2, debug_flags=flags)
    assert rc.sum() == 0 and cnt.sum() == 0 and np.all(x == 0)
    assert ex.stats().kept_rows_in == 0


def test_empty_input(ex):
    bp = o.BoundParams(1, 1, 0.0, 1.0)
    e = np.zeros(0, np.int64)
    _, _, rc, cnt, x, _ = run_gpu(ex, e, e, np.zeros(0), 1, 5, bp, 1 | 2)
    assert rc.sum() == 0 and cnt.sum() == 0


@pytest.mark.parametrize("flags", [0, FORCE_FILTER])
def test_out_of_range_ids_raise(ex, flags):
    from pipelinedp_amd.native import NativeError
    bp = o.BoundParams(1, 1, 0.0, 1.0)
    pid = np.array([0, 1, 2], np.int64)
    pk = np.array([0, 5, 1], np.int64)
    with pytest.raises(NativeError, match="out of range"):
        run_gpu(ex, pid, pk, np.zeros(3), 3, 5, bp, 1, debug_flags=flags)
    with pytest.raises(NativeError, match="out of range"):
        run_gpu(ex, np.array([0, 3, 2], np.int64), np.array([0, 4, 1], np.int64), np.zeros(3), 3, 5, bp, 1,
                debug_flags=flags)


def test_already_enforced_matches_oracle(ex):
    n, P = 30000, 500
    _, pk, val = o.synth_rows(n, 10, P, seed=4, zipf_s=1.2)
    bp = o.BoundParams(3, 2, 0.0, 10.0, contribution_bounds_already_enforced=True)
    _, _, rc, cnt, x, _ = run_gpu(ex, None, pk, val, 1, P, bp, 1 | 2)
    ref = o.bound_and_accumulate(None, pk, val, P, bp)
    check_acc(ref, rc, cnt, x, None, 1 | 2, val, bp)


@pytest.mark.parametrize("flags", [0, FORCE_FILTER, NO_THIN | FORCE_FILTER, BATCH_KERNEL])
def test_determinism_of_counts_and_sums(ex, flags):
    """K4 (pdp_reduce.inc): counts AND fp64 sums are identical bit for bit run
    to run and whatever the K2 grid (the records reach the fixed-point
    accumulators in a different order), for every K2 kernel."""
    n, U, P = 200000, 5000, 2000
    pid, pk, val = o.synth_rows(n, U, P, seed=21, zipf_s=1.1)
    bp = o.BoundParams(4, 2, 0.0, 10.0)
    mask = 1 | 4 | 8 | 16
    r1 = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=5, debug_flags=flags)
    r2 = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=5, debug_flags=flags)
    r3 = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=5, debug_flags=flags | ODD_GRID)
    for r in (r2, r3):
        for i in (2, 3, 4, 5):
            np.testing.assert_array_equal(r1[i], r[i])
    ref = o.bound_and_accumulate(pid, pk, val, P, bp, "hash", seed=5)
    check_acc(ref, r1[2], r1[3], r1[4], r1[5], mask, val, bp)


@pytest.mark.parametrize("cfgi", [0, 2, 3, 5, 9, 11, 16, 20])
def test_k4_reduction_matches_atomic_path(ex, cfgi):
    """The K4 pair-record reduction against the round-2 fp64-atomic
    accumulation (debug flag NO_K4) on the same bounding: counts bit-exact, sums to
    1e-12 relative (only the summation differs)."""
    n, U, P, z, L0, Linf, vb, pb, mask = CONFIGS[cfgi]
    pid, pk, val = o.synth_rows(n, U, P, seed=100 + cfgi, zipf_s=z, value_lo=-5, value_hi=15)
    bp = o.BoundParams(L0, Linf, *(vb or (None, None)), *(pb or (None, None)))
    a = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=7)
    b = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=7, debug_flags=NO_K4)
    np.testing.assert_array_equal(a[2], b[2])
    if a[3] is not None:
        np.testing.assert_array_equal(a[3], b[3])
    for i in (4, 5):
        if a[i] is not None:
            np.testing.assert_allclose(a[i], b[i], rtol=1e-12, atol=1e-9)


def test_nan_values_propagate_to_their_partition(ex):
    """A NaN value reaches its partition's sum as NaN (np.clip / sum
    semantics of combiners.py:254-261, 305-311); other partitions are
    unaffected."""
    n, U, P = 20000, 400, 300
    pid, pk, val = o.synth_rows(n, U, P, seed=19)
    val = val.copy()
    bad = np.flatnonzero(pk == 7)
    val[bad] = np.nan
    bp = o.BoundParams(400, 400, 0.0, 10.0)  # non-binding: every row kept
    _, _, rc, cnt, x, _ = run_gpu(ex, pid, pk, val, U, P, bp, 1 | 2, seed=3)
    assert np.isnan(x[7])
    ok = np.arange(P) != 7
    np.testing.assert_allclose(x[ok], np.bincount(pk, np.clip(np.nan_to_num(val), 0, 10), P)[ok], rtol=1e-12)
    np.testing.assert_array_equal(cnt, np.bincount(pk, minlength=P))


# ---------------------------------------------------------------------------
# Release (selection + noise) against the oracle with the same Philox draws
# ---------------------------------------------------------------------------

RELEASES = [
    (("mean", "count", "sum", "privacy_id_count"), "laplace", "truncated_geometric"),
    (("variance", "mean", "count", "sum"), "gaussian", "truncated_geometric"),
    (("count", "sum"), "laplace", "laplace"),
    (("count", "privacy_id_count"), "gaussian", "gaussian"),
    (("sum",), "laplace", None),
    (("mean",), "gaussian", None),
]


@pytest.mark.parametrize("ri", range(len(RELEASES)))
def test_release_matches_oracle(ex, ri):
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.executor import ReleaseConfig
    metrics, kind, sel = RELEASES[ri]
    mask = sum(MASK[m] for m in metrics)
    n, U, P = 60000, 3000, 1500
    pid, pk, val = o.synth_rows(n, U, P, seed=31 + ri, zipf_s=1.1)
    bp = o.BoundParams(3, 2, -1.0, 6.0)
    cfg, acc, *_ = run_gpu(ex, pid, pk, val, U, P, bp, mask, seed=8)
    ref = o.bound_and_accumulate(pid, pk, val, P, bp, "hash", seed=8)
    budgets = {m: (0.3 + 0.1 * i, 1e-7 * (i + 1)) for i, m in enumerate(("count", "sum", "mean", "variance",
                                                                         "privacy_id_count"))}
    slot = {"count": 0, "sum": 1, "mean": 2, "variance": 3, "privacy_id_count": 4}
    eps = [0.0] * 6
    delta = [0.0] * 6
    for m, (e, d) in budgets.items():
        eps[slot[m]], delta[slot[m]] = e, d
    eps[5], delta[5] = 0.7, 1e-5
    selc = {None: 0, "truncated_geometric": 1, "laplace": 2, "gaussian": 3}[sel]
    rel = ReleaseConfig(mask, 0 if kind == "laplace" else 1, selc, eps, delta, 1, True, noise_seed=99 + ri)
    keep, out, fields = ex.release(acc, rel, cfg)
    torch.cuda.synchronize()
    spec = o.ReleaseSpec(metrics, kind, budgets, sel, (0.7, 1e-5), 1)
    k2, o2 = o.release(ref, bp, spec, seed=99 + ri)
    assert fields == o.metric_field_order(metrics)
    np.testing.assert_array_equal(keep.cpu().numpy().astype(bool), k2)
    outn = out.cpu().numpy()
    for i, f in enumerate(fields):
        np.testing.assert_allclose(outn[i], o2[f], rtol=1e-9, atol=1e-7, err_msg=f)


# ---------------------------------------------------------------------------
# Full DPEngine API against the reference golden vectors (noise disabled)
# ---------------------------------------------------------------------------


@pytest.mark.parametrize("fallback", [False, True])
@pytest.mark.parametrize("name", aggregate_cases())
def test_engine_matches_reference_golden(name, fallback):
    import pipelinedp_amd as pdp
    from test_host_api import _params_from_cfg
    d = load(name)
    cfg = d["meta"]["cfg"]
    acct = pdp.NaiveBudgetAccountant(total_epsilon=cfg.get("eps", 1.0), total_delta=cfg.get("delta", 1e-6))
    backend = pdp.HipBackend(sampling_seed=1, noise_seed=2, _unsafe_disable_noise_for_testing=True,
                             _debug_force_fallback=fallback)
    engine = pdp.DPEngine(acct, backend)
    enforced = cfg.get("already_enforced", False)
    has_val = len(d["value"]) > 0
    rows = list(zip(d["pid"].tolist() if len(d["pid"]) else [None] * len(d["pk"]), d["pk"].tolist(),
                    d["value"].tolist() if has_val else [None] * len(d["pk"])))
    ex = pdp.DataExtractors(privacy_id_extractor=None if enforced else (lambda r: r[0]),
                            partition_extractor=lambda r: r[1], value_extractor=lambda r: r[2])
    public = d["public"].tolist() if bool(d["has_public"]) else None
    res = engine.aggregate(rows, _params_from_cfg(cfg), ex, public)
    acct.compute_budgets()
    got = dict(list(res))
    exp_keys = d["out_keys"].tolist()
    assert sorted(got) == sorted(exp_keys)
    fields = d["meta"]["fields"]
    tol = _fp64_field_bounds(d, cfg, fields)
    for k, row in zip(exp_keys, d["out_vals"]):
        t = got[k]
        assert list(t._fields) == fields
        for f, e in zip(fields, row):
            g = getattr(t, f)
            if f in ("count", "privacy_id_count"):
                assert g == e, (k, f)
            else:
                assert abs(g - e) <= tol(k, f, dict(zip(fields, row))), (k, f, g, e, tol(k, f, dict(zip(fields, row))))


U53 = 2.0**-53


def _fp64_field_bounds(d, cfg, fields):
    """Per-(partition, field) bound of |GPU - reference| for the noise-free
    golden outputs: only the summation order differs (GPU: fixed-point pair
    merge of input-order pair sums; reference: fp64 sums in its own order,
    combiners.py:305-311,364-373), so for a sum of n terms
        |s_gpu - s_ref| <= E = 4 (n + 2) 2^-53 sum|terms|
    (both sides within (n + 2) u sum|t| of the exact sum, with a factor-2
    margin), and means / variances carry it through compute_dp_mean / _var's
    formulas (dp_computations.py:310-459) with a few ulps per operation.
    n and sum|terms| are taken over ALL input rows of the partition (the kept
    rows are a subset), so the bound holds whatever the bounding kept."""
    m = set(cfg["metrics"])
    keys = d["pk"]
    v = d["value"] if len(d["value"]) else np.zeros(len(keys))
    has_vb = "min_value" in cfg
    a, b = (cfg.get("min_value", 0.0), cfg.get("max_value", 0.0))
    mid = a + (b - a) / 2
    meanlike = bool(m & {"mean", "variance"})
    if meanlike:
        t = np.clip(v, a, b) - mid
    elif has_vb:
        t = np.clip(v, a, b)
    elif "min_sum_per_partition" in cfg:  # per-(pid, pk) sums clipped to [smin, smax]: |term| <= max(|smin|, |smax|)
        t = np.full(len(keys), max(abs(cfg["min_sum_per_partition"]), abs(cfg["max_sum_per_partition"])))
    else:
        t = v
    uk, inv = np.unique(keys, return_inverse=True)
    n_rows = np.bincount(inv, minlength=len(uk)).astype(np.float64)
    s1 = np.bincount(inv, weights=np.abs(t), minlength=len(uk))
    s2 = np.bincount(inv, weights=t * t, minlength=len(uk))
    where = {int(k): i for i, k in enumerate(uk)}

    def bound(key, f, exp):
        i = where.get(int(key))
        n, S1, S2 = (n_rows[i], s1[i], s2[i]) if i is not None else (0.0, 0.0, 0.0)
        ex = 4 * (n + 2) * U53 * S1
        ey = 4 * (n + 2) * U53 * S2
        c = max(float(exp.get("count", n)), 1.0)
        tiny = 1e-300
        if not meanlike:
            return ex + tiny  # sum
        mn = exp["mean"] - mid if "mean" in exp else 0.0
        e_mn = ex / c + 2 * U53 * abs(mn)
        e_mean = e_mn + 2 * U53 * (abs(mn) + abs(mid))
        if f == "mean":
            return e_mean + tiny
        if f == "sum":
            return c * e_mean + 2 * U53 * abs(exp.get("sum", 0.0)) + tiny
        if f == "variance":
            # dp_var = (nsumsq / c + mid of the squares interval) - mn^2 (compute_dp_var, compute_squares_interval)
            sa, sb = (0.0, max(a * a, b * b)) if a < 0 < b else (a * a, b * b)
            sq_mid = sa + (sb - sa) / 2 if sa != sb else 0.0
            msq = exp["variance"] + mn * mn
            e_msq = ey / c + 2 * U53 * (abs(msq) + 2 * abs(sq_mid))
            return e_msq + 2 * abs(mn) * e_mn + e_mn * e_mn + 4 * U53 * (abs(msq) + mn * mn) + tiny
        raise AssertionError(f)

    return bound


@pytest.mark.parametrize("fallback", [False, True])
@pytest.mark.parametrize("name", aggregate_cases())
def test_golden_inputs_accumulate_bitwise_vs_oracle(ex, name, fallback):
    """The golden cases' own inputs through pdp_bound_accumulate: counts and
    sums bit for bit against the oracle's accumulators merged in K4's fixed
    point (the oracle itself equals the reference's LocalBackend on these
    cases, tests/test_oracle.py; module docstring for the L_inf rule)."""
    d = load(name)
    cfg = d["meta"]["cfg"]
    pid, pk, keys = encode_case(d)
    enforced = cfg.get("already_enforced", False)
    bp = o.BoundParams(cfg["L0"], cfg["Linf"], cfg.get("min_value"), cfg.get("max_value"),
                       cfg.get("min_sum_per_partition"), cfg.get("max_sum_per_partition"), enforced)
    mask = 0
    for m in cfg["metrics"]:
        mask |= MASK[m]
    has_val = len(d["value"]) > 0
    val = d["value"].astype(np.float64) if has_val and mask & (2 | 4 | 8) else None
    P = max(len(keys), 1)
    U = int(pid.max()) + 1 if len(pid) else 1
    _, _, rc, cnt, x, y = run_gpu(ex, None if enforced else pid, pk, val, U, P, bp, mask, seed=19,
                                  fallback=fallback and not enforced)
    ref = o.bound_and_accumulate(None if enforced else pid, pk, val, P, bp, "hash", seed=19)
    check_acc(ref, rc, cnt, x, y, mask, val, bp)


def test_engine_columnar_device_input_and_select_partitions():
    import torch
    import pipelinedp_amd as pdp
    n, U, P = 50000, 2000, 300
    pid, pk, val = o.synth_rows(n, U, P, seed=12, zipf_s=1.1)
    acct = pdp.NaiveBudgetAccountant(total_epsilon=1e6, total_delta=1e-6)
    backend = pdp.HipBackend(sampling_seed=4, noise_seed=5)
    engine = pdp.DPEngine(acct, backend)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.MEAN], max_partitions_contributed=3,
                                 max_contributions_per_partition=2, min_value=0, max_value=10)
    data = pdp.ColumnarData(partition=torch.from_numpy(pk).cuda(), privacy_id=torch.from_numpy(pid).cuda(),
                            value=torch.from_numpy(val).cuda(), num_partitions=P, num_privacy_ids=U)
    res = engine.aggregate(data, params, None)
    sel = engine.select_partitions(data, pdp.SelectPartitionsParams(max_partitions_contributed=3), None)
    acct.compute_budgets()
    out = dict(res)
    ref = o.bound_and_accumulate(pid, pk, val, P, o.BoundParams(3, 2, 0.0, 10.0), "hash", seed=4)
    for k, t in out.items():
        assert abs(t.count - ref.count[k]) < 1e-2  # eps = 1e6 / 3 mechanisms: tiny noise
    # huge eps: truncated geometric keeps every partition with >= 2 privacy
    # ids, those with exactly one only with probability delta / L0.
    many = set(np.flatnonzero(ref.row_count >= 2).tolist())
    assert many <= set(out) <= set(np.flatnonzero(ref.row_count >= 1).tolist())
    kept = set(sel)
    assert many <= kept <= set(np.flatnonzero(ref.row_count >= 1).tolist())


# ---------------------------------------------------------------------------
# Distributional tests (reference recipe: tests/dp_computations_test.py:69-129)
# ---------------------------------------------------------------------------


def _mass_checks(samples, sigma, within1, one_to_two):
    n = len(samples)
    a = np.abs(samples)
    f1 = np.mean(a <= sigma)
    f2 = np.mean((a > sigma) & (a <= 2 * sigma))
    assert abs(f1 - within1) <= 2.4 * math.sqrt(within1 * (1 - within1) / n)
    assert abs(f2 - one_to_two) <= 2.4 * math.sqrt(one_to_two * (1 - one_to_two) / n)


@pytest.mark.parametrize("kind", ["laplace", "gaussian"])
def test_noise_distribution(ex, kind):
    """Noise on a zero count over 2e5 partitions: KS p >= 0.001 against numpy
    and the 1-sigma / 1-2-sigma mass bands of the reference tests."""
    import torch
    from scipy import stats
    from pipelinedp_amd.executor import Accumulators, BoundConfig, ReleaseConfig
    P = 200000
    acc = Accumulators(torch, P, ex.device, 1)
    acc.row_count.zero_()
    acc.count.zero_()
    eps, delta, L0, Linf = 0.8, 1e-6, 3, 2
    rel = ReleaseConfig(1, 0 if kind == "laplace" else 1, 0, [eps, 0, 0, 0, 0, 0], [delta, 0, 0, 0, 0, 0], 1, True,
                        noise_seed=1234)
    keep, out, fields = ex.release(acc, rel, BoundConfig(1, L0, Linf))
    s = out[0].cpu().numpy()
    rng = np.random.default_rng(0)
    if kind == "laplace":
        b = L0 * Linf / eps
        ref = rng.laplace(0, b, P)
        _mass_checks(s, math.sqrt(2) * b, 1 - math.exp(-math.sqrt(2)),
                     math.exp(-math.sqrt(2)) - math.exp(-2 * math.sqrt(2)))
    else:
        sigma = o.gaussian_sigma(eps, delta, math.sqrt(L0) * Linf)
        ref = rng.normal(0, sigma, P)
        _mass_checks(s, sigma, 0.68268949213, 0.27181024396)
    assert stats.ks_2samp(s, ref).pvalue >= 0.001


def test_truncated_geometric_selection_rate(ex):
    """Keep rate of partitions with n privacy ids ~ Binomial(p(n))."""
    import torch
    from pipelinedp_amd.executor import Accumulators, BoundConfig, ReleaseConfig
    P = 100000
    eps, delta, L0 = 1.0, 1e-2, 2
    table = o.truncated_geometric_table(eps, delta, L0)
    acc = Accumulators(torch, P, ex.device, 1)
    nvals = np.arange(P) % 8 + 1
    acc.row_count.copy_(torch.from_numpy(nvals))
    acc.count.zero_()
    rel = ReleaseConfig(1, 0, 1, [1.0, 0, 0, 0, 0, eps], [0, 0, 0, 0, 0, delta], 1, True, noise_seed=77)
    keep, _, _ = ex.release(acc, rel, BoundConfig(1, L0, 1))
    k = keep.cpu().numpy().astype(bool)
    for nv in range(1, 9):
        sel = nvals == nv
        p = table[nv] if nv < len(table) else 1.0
        m = sel.sum()
        assert abs(k[sel].mean() - p) <= 4 * math.sqrt(p * (1 - p) / m) + 1e-12, (nv, k[sel].mean(), p)


# ---------------------------------------------------------------------------
# Multi-GPU ingestion: pdp_shard_rows (device side of the privacy-id shuffle)
# ---------------------------------------------------------------------------


@pytest.mark.parametrize("world", [1, 2, 3, 8, 64])
def test_shard_rows_is_stable_grouping_by_shard(ex, world):
    import torch
    from pipelinedp_amd.distributed import shard_of
    n, U, P = 100003, 5000, 700
    pid, pk, val = o.synth_rows(n, U, P, seed=40 + world, zipf_s=1.1)
    spid, spk, sval, counts = ex.shard_rows(_dev(pid, torch), _dev(pk, torch), _dev(val, torch), world)
    torch.cuda.synchronize()
    dest = shard_of(pid, world)
    order = np.argsort(dest, kind="stable")
    assert counts == np.bincount(dest, minlength=world).tolist()
    np.testing.assert_array_equal(spid.cpu().numpy(), pid[order])
    np.testing.assert_array_equal(spk.cpu().numpy(), pk[order])
    np.testing.assert_array_equal(sval.cpu().numpy(), val[order])
    _, _, none, c2 = ex.shard_rows(_dev(pid, torch), _dev(pk, torch), None, world)
    assert none is None and c2 == counts


# ---------------------------------------------------------------------------
# select_partitions: the reference's probabilistic end-to-end test
# (tests/dp_engine_test.py:444-492) with the MI355X noise
# ---------------------------------------------------------------------------


@pytest.mark.parametrize("seed", range(5))
def test_select_partitions_reference_scenario(seed):
    import pipelinedp_amd as pdp
    col = [(u, "pk-many-contribs") for u in range(25)]
    col += [(100 + u // 10, "pk-many-contribs-few-users") for u in range(30)]
    col += [(200 + u, "pk-few-contribs") for u in range(3)]
    for i in range(30):
        col += [(500 + u, f"few-contribs-after-bound{i}") for u in range(25)]
    acct = pdp.NaiveBudgetAccountant(total_epsilon=1, total_delta=1e-5)
    engine = pdp.DPEngine(acct, pdp.HipBackend(sampling_seed=1000 + seed, noise_seed=2000 + seed))
    res = engine.select_partitions(col, pdp.SelectPartitionsParams(max_partitions_contributed=1),
                                   pdp.DataExtractors(privacy_id_extractor=lambda x: x[0],
                                                      partition_extractor=lambda x: x[1]))
    acct.compute_budgets()
    assert list(res) == ["pk-many-contribs"]


def _gpu_select_counts(ex, pid, pk, P, L0, seed):
    import torch
    from pipelinedp_amd.executor import BoundConfig
    U = int(pid.max()) + 1
    acc = ex.accumulate(_dev(pid, torch), _dev(pk, torch), None, U, P, BoundConfig(0, L0, 1, sampling_seed=seed))
    return acc.row_count.cpu().numpy()


def test_select_partitions_counts_match_reference_golden(ex):
    d = load("select_partitions_nonbinding")
    meta = d["meta"]
    rc = _gpu_select_counts(ex, d["pid"], d["pk"], meta["P"], meta["L0"], seed=3)
    assert np.flatnonzero(rc >= meta["threshold"]).tolist() == d["out_keys"].tolist()


def test_select_partitions_binding_matches_reference_distribution_on_gpu(ex):
    d = load("select_partitions_binding")
    meta = d["meta"]
    runs = int(d["runs"])
    freq = np.zeros(meta["P"])
    for s in range(runs):
        rc = _gpu_select_counts(ex, d["pid"], d["pk"], meta["P"], meta["L0"], seed=5000 + s)
        if s < 5:  # the GPU sampler is the oracle's, bit for bit
            np.testing.assert_array_equal(rc, o.bound_and_accumulate(d["pid"], d["pk"], None, meta["P"],
                                                                     o.BoundParams(meta["L0"], 1), "hash",
                                                                     seed=5000 + s).row_count)
        freq += rc >= meta["threshold"]
    freq /= runs
    p = (freq + d["freq"]) / 2
    sd = np.sqrt(2 * p * (1 - p) / runs) + 1e-9
    assert np.all(np.abs(freq - d["freq"]) <= 4.5 * sd), (freq, d["freq"])


def test_heavy_single_group_generic_path(ex):
    """one privacy id with 2e6 rows in ONE partition (plus a
    spread of ordinary rows) goes through the generic path, whose kept groups
    of more than 2048 rows are summed by a whole block (k_stream_big_groups)
    instead of one lane walking every row.  Counts bit-exact against the
    oracle, sums to 1e-9; the accumulate call stays well under the time a
    single-lane walk of 2e6 rows takes."""
    import time

    import torch
    n0, U, P = 200000, 3000, 500
    pid0, pk0, val0 = o.synth_rows(n0, U, P, seed=4242, zipf_s=1.1, value_lo=-5, value_hi=15)
    heavy = 2_000_000
    rng = np.random.default_rng(7)
    pid = np.concatenate([pid0, np.full(heavy, U, np.int64), np.full(300, U, np.int64)])
    pk = np.concatenate([pk0, np.full(heavy, 17, np.int64), rng.integers(0, P, 300)])
    val = np.concatenate([val0, rng.uniform(-5, 15, heavy), rng.uniform(-5, 15, 300)])
    perm = rng.permutation(len(pid))
    pid, pk, val = pid[perm], pk[perm], val[perm]
    for L0, Linf in ((3, 2), (2, 5000)):
        bp = o.BoundParams(L0, Linf, 0.0, 10.0)
        mask = 1 | 2 | 4 | 8 | 16
        run_gpu(ex, pid, pk, val, U + 1, P, bp, mask, seed=5)  # warm-up
        t0 = time.perf_counter()
        _, _, rc, cnt, x, y = run_gpu(ex, pid, pk, val, U + 1, P, bp, mask, seed=5)
        dt = time.perf_counter() - t0
        assert ex.stats().fallback_rows >= heavy
        ref = o.bound_and_accumulate(pid, pk, val, P, bp, "hash", seed=5)
        check_acc(ref, rc, cnt, x, y, mask, val, bp)
        assert dt < 0.5, dt


@pytest.mark.parametrize("cfgi", [0, 2, 9, 11, 19, 21])
def test_k4_pair_record_forms_bitwise_equal(ex, cfgi):
    """K4's pair passes move 12-byte records {pk << cb | count - 1, x} when the
    partition id and count fit 31 bits, 16-byte {pk, count, x} otherwise
    (debug flag K4_P16 forces them); K2 can write the 12-byte form as split slots
    (keys, then values: the first pass reads 4 bytes of an empty slot; flag
    K4_SOA): the fixed-point sums are integers, so all three forms give
    identical accumulators, sums included.  So do the K2 forms under the L0
    pre-filter (forced on at these sizes): k_thin (default) and the LDS-staged
    k_thin2 (THIN2), each writing a slot per row (default) or compacted pair
    records (K4_COMPACT); and with or without K2's hot-partition tables
    (NO_HOT_CACHE: every kept pair a record)."""
    n, U, P, z, L0, Linf, vb, pb, mask = CONFIGS[cfgi]
    pid, pk, val = o.synth_rows(n, U, P, seed=700 + cfgi, zipf_s=z, value_lo=-5, value_hi=15)
    bp = o.BoundParams(L0, Linf, *(vb or (None, None)), *(pb or (None, None)))
    need_val = bool(mask & (2 | 4 | 8))
    runs = []
    ff, compact, thin2, nohot = 268435456, 1024, 67108864, 524288  # FORCE_FILTER, K4_COMPACT, THIN2, NO_HOT_CACHE
    for form in (K4_SOA, 0, K4_P16 | K4_SOA, compact, nohot, ff, ff | compact, ff | thin2, ff | thin2 | compact,
                 ff | nohot):
        _, _, rc, cnt, x, y = run_gpu(ex, pid, pk, val if need_val else None, U, P, bp, mask, seed=5 + cfgi,
                                      debug_flags=form)
        runs.append((rc, cnt, x, y))
    for other in runs[1:]:
        for a, b in zip(runs[0], other):
            if a is None:
                assert b is None
            else:
                np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("mask", [1 | 2 | 4 | 16, 1 | 2])
def test_hot_tables_dropped_on_whole_input_redo(ex, mask):
    """Round-5 advisor finding: k_lean's K4 hot-partition tables flush their
    kept groups (counts into the accumulators, sums into K4's fixed-point
    scratch) before the host learns that the overflow list is full
    (kCtrFull), which reruns EVERY row on the generic path.  Those groups must
    be dropped then, or they count twice.  Debug flag OVERFLOW_FULL1 sets the
    full flag from the second overflow range on (three privacy ids of 3000 rows
    overflow here), while the hot tables hold Zipf-head pairs (L0 = 32).
    Bit for bit against the oracle, with and without the flag."""
    from pipelinedp_amd import native
    n, U, P, z, L0, Linf, vb, _, _ = CONFIGS[11]
    pid0, pk0, val0 = o.synth_rows(n, U, P, seed=811, zipf_s=z, value_lo=-5, value_hi=15)
    rng = np.random.default_rng(811)
    heavy = 3000
    pid = np.concatenate([pid0] + [np.full(heavy, U + i, np.int64) for i in range(3)])
    pk = np.concatenate([pk0] + [rng.integers(0, P, heavy) for _ in range(3)])
    val = np.concatenate([val0, rng.uniform(-5, 15, 3 * heavy)])
    perm = rng.permutation(len(pid))
    pid, pk, val = pid[perm], pk[perm], val[perm]
    bp = o.BoundParams(L0, Linf, *vb)
    ref = o.bound_and_accumulate(pid, pk, val, P, bp, "hash", seed=19)
    # the hot tables are in play here: they absorb pairs that would otherwise reach K4 as records
    run_gpu(ex, pid, pk, val, U + 3, P, bp, mask, seed=19, debug_flags=native.DEBUG_NO_HOT_CACHE)
    records_without_tables = ex.stats().k4_pairs
    run_gpu(ex, pid, pk, val, U + 3, P, bp, mask, seed=19)
    assert ex.stats().k4_pairs < records_without_tables
    for flags2 in (0, native.DEBUG2_OVERFLOW_FULL1):
        _, _, rc, cnt, x, y = run_gpu(ex, pid, pk, val, U + 3, P, bp, mask, seed=19, debug_flags2=flags2)
        check_acc(ref, rc, cnt, x, y, mask, val, bp)
        st = ex.stats()
        if flags2:
            assert st.fallback_rows == len(pid)  # the whole input went through the generic path
        else:
            assert 3 * heavy <= st.fallback_rows < len(pid)


@pytest.mark.parametrize("p12", [True, False])
@pytest.mark.parametrize("cfgi", [0, 5, 9, 11, 17, 19, 21])
def test_row_counts_only_match_oracle(ex, cfgi, p12):
    """Selection only (no COUNT / SUM: select_partitions' accumulate): K2 does
    not sample rows then, so a pair slot's count is the group's row count, not
    bounded by L_inf; the 12-byte K4 key must not carry count bits (a round-4
    build OR-ed them into the partition id).  Row counts bit-exact vs the
    oracle in both record forms."""
    n, U, P, z, L0, Linf, vb, pb, _ = CONFIGS[cfgi]
    pid, pk, _ = o.synth_rows(n, U, P, seed=900 + cfgi, zipf_s=z, value_lo=0, value_hi=1)
    bp = o.BoundParams(L0, Linf)
    _, _, rc, cnt, x, y = run_gpu(ex, pid, pk, None, U, P, bp, 0, seed=11 + cfgi, debug_flags=0 if p12 else K4_P16)
    ref = o.bound_and_accumulate(pid, pk, None, P, bp, "hash", seed=11 + cfgi)
    np.testing.assert_array_equal(rc, ref.row_count)
