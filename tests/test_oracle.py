"""Pins the CPU oracle (oracle/pdp_oracle.py) against the reference:
golden vectors produced by the reference LocalBackend (oracle/gen_golden.py)
and the known-answer numbers of the reference's own tests."""
import json
import math
import os

import numpy as np
import pytest
from scipy.stats import binom

import pdp_oracle as o
from golden_util import GOLDEN, aggregate_cases, encode_case, known_answers, load, sum_tolerance


def oracle_run(d, sampler="hash", seed=0, noise=False):
    cfg = d["meta"]["cfg"]
    pid, pk, keys = encode_case(d)
    value = d["value"] if len(d["value"]) else None
    bp = o.BoundParams(cfg["L0"], cfg["Linf"], cfg.get("min_value"), cfg.get("max_value"),
                       cfg.get("min_sum_per_partition"), cfg.get("max_sum_per_partition"),
                       cfg.get("already_enforced", False))
    acc = o.bound_and_accumulate(pid, pk, value, len(keys), bp, sampler=sampler, seed=seed)
    metrics = tuple(cfg["metrics"])
    budgets = {m: (0.5, 1e-7) for m in ("count", "sum", "mean", "variance", "privacy_id_count")}
    public = bool(d["has_public"])
    spec = o.ReleaseSpec(metrics, cfg.get("noise_kind", "laplace"), budgets,
                         None if public else "truncated_geometric", (0.5, 1e-7),
                         cfg["Linf"] if cfg.get("already_enforced") else 1)
    keep, out = o.release(acc, bp, spec, seed=seed, noise=noise)
    return keys, keep, out, acc


@pytest.mark.parametrize("name", aggregate_cases())
def test_oracle_matches_reference_golden(name):
    d = load(name)
    keys, keep, out, acc = oracle_run(d)
    fields = d["meta"]["fields"]
    assert fields == o.metric_field_order(d["meta"]["cfg"]["metrics"])
    np.testing.assert_array_equal(keys[keep], d["out_keys"])
    vals = d["out_vals"]
    # scale for float tolerance: sum of |values| bounded by count * max|v|
    vmax = float(np.abs(d["value"]).max()) if len(d["value"]) else 1.0
    for j, f in enumerate(fields):
        got = out[f][keep]
        exp = vals[:, j]
        if f in ("count", "privacy_id_count"):
            np.testing.assert_array_equal(got, exp)
        else:
            scale = (acc.count[keep] + 1) * max(vmax, 1.0)**2
            assert np.all(np.abs(got - exp) <= sum_tolerance(exp, scale)), f


def test_gaussian_sigma_known_answers():
    for c in known_answers()["gaussian_sigma"]:
        l2 = c["l2"] if "l2" in c else math.sqrt(c["l0"]) * c["linf"]
        assert o.gaussian_sigma(c["eps"], c["delta"], l2) == pytest.approx(c["sigma"], abs=1e-12), c


def test_truncated_geometric_known_answers():
    for c in known_answers()["truncated_geometric"]:
        n, p = c["n_binomial"]
        ks = np.arange(n + 1)
        pm = binom.pmf(ks, n, p)
        got = float((pm * o.truncated_geometric_keep_prob(ks, c["eps"], c["delta"], c["k"])).sum())
        assert got == pytest.approx(c["p_keep"], abs=1e-10), c


def test_laplace_std_known_answers():
    for c in known_answers()["laplace_std"]:
        if "std" in c:
            linf = max(abs(c["min_sum"]), abs(c["max_sum"]))
            assert o.noise_scale("laplace", c["eps"], 0, c["l0"], linf) * math.sqrt(2) == pytest.approx(c["std"], abs=1e-10)
        else:
            assert o.noise_scale("laplace", c["eps"], 0, c["l0"], c["linf"]) * math.sqrt(2) == pytest.approx(
                c["l0"] * c["linf"] / c["eps"] * math.sqrt(2), abs=1e-10)


def test_equally_split_budget_known_answer():
    c = known_answers()["equally_split_budget"]
    exp = [(0.5 / 5, 1e-10 / 5) for _ in range(4)] + [(0.5 - 4 * (0.5 / 5), 1e-10 - 4 * (1e-10 / 5))]
    assert o.equally_split_budget(c["eps"], c["delta"], c["n"]) == exp
    with pytest.raises(ValueError):
        o.equally_split_budget(0.5, 1e-10, 0)


def test_bounder_known_answer():
    # contribution_bounders_test.py:60-69: (2, 7, 25) / (2, 3, 5) -> with an
    # accumulator of (len, sum, sum of squares) on values 1..4.
    pid = np.array([0, 0, 0, 0])
    pk = np.array([0, 0, 1, 1])
    v = np.array([1.0, 2.0, 3.0, 4.0])
    acc = o.bound_and_accumulate(pid, pk, v, 2, o.BoundParams(2, 2, -100.0, 100.0))
    mid = 0.0
    np.testing.assert_array_equal(acc.count, [2, 2])
    np.testing.assert_allclose(acc.sum, [3, 7])
    np.testing.assert_allclose(acc.nsumsq, [5, 25])
    assert mid == o.compute_middle(-100.0, 100.0)


def test_accumulator_known_answers():
    # combiners_test.py:337-341 mean acc [1,3] with [0,4] -> (2, 0)
    acc = o.bound_and_accumulate(np.zeros(2), np.zeros(2), np.array([1.0, 3.0]), 1,
                                 o.BoundParams(1, 5, 0.0, 4.0))
    assert (acc.count[0], acc.nsum[0]) == (2, 0.0)
    # combiners_test.py:391-395 variance acc [1,2] -> (2, -1, 1)
    acc = o.bound_and_accumulate(np.zeros(2), np.zeros(2), np.array([1.0, 2.0]), 1,
                                 o.BoundParams(1, 5, 0.0, 4.0))
    assert (acc.count[0], acc.nsum[0], acc.nsumsq[0]) == (2, -1.0, 1.0)
    # combiners_test.py:275-282 per-partition sum clipping [0, 3]
    for vals, exp in ([2, 0.5], 2.5), ([4, 1], 3), ([-10, 5, 3], 0):
        acc = o.bound_and_accumulate(np.zeros(len(vals)), np.zeros(len(vals)), np.array(vals, float), 1,
                                     o.BoundParams(1, 10, None, None, 0.0, 3.0))
        assert acc.sum[0] == exp
    # combiners_test.py:405-412 variance no-noise (4, 0, 2) with [0, 4]
    a = o.Accumulators(np.array([1]), np.array([4]), np.array([8.0]), np.array([0.0]), np.array([2.0]))
    keep, out = o.release(a, o.BoundParams(1, 1, 0.0, 4.0),
                          o.ReleaseSpec(("variance", "mean", "count", "sum"), "laplace",
                                        {"variance": (1.0, 0.0)}), noise=False)
    assert (out["count"][0], out["sum"][0], out["mean"][0], out["variance"][0]) == (4, 8, 2, 0.5)


def test_feistel_is_bijection():
    for bits in (1, 2, 5, 8, 13, 20):
        x = np.arange(1 << bits, dtype=np.uint64)
        y = o.perm_bits(x, bits, np.uint64(12345))
        assert len(np.unique(y)) == len(x) and y.max() < (1 << bits)
    for n in (2, 3, 7, 100, 1000):
        y = o.cycle_walk(np.arange(n), np.full(n, n), np.full(n, 99, dtype=np.uint64))
        assert sorted(y.tolist()) == list(range(n))


def test_hash_sampler_is_uniform():
    """Inclusion frequency of each row of an n-row group under L_inf sampling
    is L_inf / n, and of each partition under L0 sampling is L0 / R."""
    trials = 20000
    for n, linf in ((2, 1), (3, 1), (5, 2), (7, 3), (12, 5)):
        seeds = np.arange(trials)
        pid = np.zeros(trials * n, np.int64)
        gprio = o.group_priority(np.repeat(seeds, n), pid, 2)
        j = np.tile(np.arange(n), trials)
        pr = o.row_priority(gprio, j).reshape(trials, n)
        rank = np.argsort(np.argsort(pr, axis=1, kind="stable"), axis=1, kind="stable")
        freq = (rank < linf).mean(0)
        p = linf / n
        assert np.all(np.abs(freq - p) < 4.5 * math.sqrt(p * (1 - p) / trials)), (n, freq)
    for R, l0 in ((3, 1), (5, 2), (9, 4)):
        seeds = np.repeat(np.arange(trials), R)
        pks = np.tile(np.arange(R), trials)
        pr = o.group_priority(seeds, np.full(len(pks), 7), pks).reshape(trials, R)
        rank = np.argsort(np.argsort(pr, axis=1, kind="stable"), axis=1, kind="stable")
        freq = (rank < l0).mean(0)
        p = l0 / R
        assert np.all(np.abs(freq - p) < 4.5 * math.sqrt(p * (1 - p) / trials)), (R, freq)


def test_partition_ranking_is_uniform_across_privacy_ids():
    """For ONE seed, over many privacy ids (the case the hot path sees): each
    partition is kept with probability L0 / R, each pair with
    L0 (L0 - 1) / (R (R - 1))."""
    pids = np.arange(40000)
    for R, l0 in ((5, 2), (9, 4), (40, 8)):
        pks = np.tile(np.arange(R) * 7919 + 3, len(pids))
        pr = o.group_priority(12345, np.repeat(pids, R), pks).reshape(len(pids), R)
        kept = np.argsort(np.argsort(pr, axis=1, kind="stable"), axis=1, kind="stable") < l0
        p = l0 / R
        freq = kept.mean(0)
        assert np.all(np.abs(freq - p) < 4.5 * math.sqrt(p * (1 - p) / len(pids))), (R, freq)
        p2 = l0 * (l0 - 1) / (R * (R - 1))
        f2 = (kept[:, 0] & kept[:, 1]).mean()
        assert abs(f2 - p2) < 4.5 * math.sqrt(p2 * (1 - p2) / len(pids)), (R, f2, p2)


def test_binding_bounds_match_reference_distribution():
    """oracle feistel sampler vs mean of 400 reference LocalBackend runs."""
    d = load("binding_count_sum_pidcount")
    cfg = d["meta"]["cfg"]
    P = d["mean"].shape[0]
    bp = o.BoundParams(cfg["L0"], cfg["Linf"], cfg["min_value"], cfg["max_value"])
    runs = 400
    res = np.zeros((runs, P, 3))
    for s in range(runs):
        acc = o.bound_and_accumulate(d["pid"], d["pk"], d["value"], P, bp, "hash", seed=1000 + s)
        res[s] = np.stack([acc.count, acc.sum, acc.row_count], 1)
    ref_mean, ref_std = d["mean"], d["std"]
    se = np.sqrt(ref_std**2 / int(d["runs"]) + res.std(0)**2 / runs) + 1e-9
    z = np.abs(res.mean(0) - ref_mean) / se
    assert z.max() < 5.0, z.max()


@pytest.mark.parametrize("kind,scale", [("laplace", 3.7), ("laplace", 1024.0), ("gaussian", 2.5)])
def test_snapped_noise_is_on_grid_and_distributed_right(kind, scale):
    # granularity snapping (pdp_rng.h:add_snapped_noise): outputs are
    # multiples of g = 2^(ceil(log2 scale) - 40); the distribution is the
    # reference's (KS p >= 0.001, tests/dp_computations_test.py:69-83)
    from scipy import stats
    g = o.noise_grid(scale)
    assert g == 2.0**(math.ceil(math.log2(scale)) - 40)
    n = 200000
    x = o.add_snapped_noise(kind, np.full(n, 10.0 + g / 3), seed=77, idx=np.arange(n), stream=3, scale=scale) - 10.0
    assert np.all(np.rint(x / g) * g == x)
    ref = stats.laplace(scale=scale) if kind == "laplace" else stats.norm(scale=scale)
    assert stats.kstest(x, ref.cdf).pvalue >= 0.001
    # tails beyond the 36.7-scale cap of a 53-bit inverse CDF are reachable
    u = o._uniform64(np.uint64(0), np.uint64(1))
    assert -math.log(float(u)) > 43


def _select_counts(pid, pk, P, L0, seed):
    # select_partitions (dp_engine.py:229-281): per pid <= L0 distinct pks,
    # then privacy ids per pk -- the row_count of a COUNT-less bound
    return o.bound_and_accumulate(pid, pk, None, P, o.BoundParams(L0, 1), "hash", seed=seed).row_count


def test_select_partitions_matches_reference_golden():
    d = np.load(os.path.join(GOLDEN, "select_partitions_nonbinding.npz"))
    meta = json.loads(str(d["meta"]))
    rc = _select_counts(d["pid"], d["pk"], meta["P"], meta["L0"], seed=3)
    assert np.flatnonzero(rc >= meta["threshold"]).tolist() == d["out_keys"].tolist()


def test_select_partitions_binding_matches_reference_distribution():
    d = np.load(os.path.join(GOLDEN, "select_partitions_binding.npz"))
    meta = json.loads(str(d["meta"]))
    runs = int(d["runs"])
    freq = np.zeros(meta["P"])
    for s in range(runs):
        freq += _select_counts(d["pid"], d["pk"], meta["P"], meta["L0"], seed=1000 + s) >= meta["threshold"]
    freq /= runs
    p = (freq + d["freq"]) / 2
    sd = np.sqrt(2 * p * (1 - p) / runs) + 1e-9
    assert np.all(np.abs(freq - d["freq"]) <= 4.5 * sd), (freq, d["freq"])


@pytest.mark.parametrize("bits", [32, 16])
@pytest.mark.parametrize("n,U,P,z,L0,Linf", [(200000, 2000, 5000, 1.1, 4, 2), (150000, 1500, 800, 0.0, 8, 4),
                                            (100000, 1000, 20000, 1.3, 1, 1), (50000, 10000, 300, 1.1, 2, 3)])
def test_prefilter_drops_only_rows_the_bounding_drops(n, U, P, z, L0, Linf, bits):
    """The L0 pre-filter restated (pdp_oracle.prefilter_survivors): bounding
    the survivors gives exactly the accumulators of bounding every row, and
    for enough rows per privacy id most rows are dropped."""
    pid, pk, val = o.synth_rows(n, U, P, seed=77, zipf_s=z)
    pk = np.where((pid % 11) == 0, -1, pk)  # some non-public rows
    bp = o.BoundParams(L0, Linf, 0.0, 10.0)
    surv = o.prefilter_survivors(pid, pk, 5, L0, bits)
    full = o.bound_and_accumulate(pid, pk, val, P, bp, "hash", seed=5)
    part = o.bound_and_accumulate(pid[surv], pk[surv], val[surv], P, bp, "hash", seed=5)
    np.testing.assert_array_equal(full.row_count, part.row_count)
    np.testing.assert_array_equal(full.count, part.count)
    np.testing.assert_allclose(full.nsum, part.nsum, rtol=1e-12, atol=1e-9)
    assert not surv[pk < 0].any()
    if n // U >= 16 * L0:
        assert surv.mean() < 0.5


def test_prefilter_level_is_monotone_and_covers_32_levels():
    h = np.array([0, 1, (1 << 24) - 1, 1 << 24, 0x01306FE1, 1 << 25, 1 << 31, 0x9837F051 << 0, 0xD744FCCB,
                  0xFFFFFFFF], dtype=np.uint64)
    lv = o.prefilter_level(np.sort(h))
    assert np.all(np.diff(lv) >= 0) and lv[0] == 0 and lv[-1] == 31
    x = np.sort(np.random.default_rng(1).integers(0, 1 << 32, 100000, dtype=np.uint64))
    lx = o.prefilter_level(x)
    assert np.all(np.diff(lx) >= 0) and set(np.unique(lx)) <= set(range(32))


def test_prefilter_sketch_width_rule():
    assert o.prefilter_sketch_bits(10_000_000) == 32  # c3: 39,063 pids per bucket
    assert o.prefilter_sketch_bits(15_000_000) == 16
    assert o.prefilter_sketch_bits(30_000_000) == 0
