"""Host-side API parity with the reference (no GPU needed: aggregate() is lazy,
so validation, budget requests and the explain report are all host work)."""
import numpy as np
import pytest

import pipelinedp_amd as pdp
from golden_util import aggregate_cases, load

M = pdp.Metrics


def test_budget_split_known_answer():
    # tests/budget_accounting_test.py:56-70
    acct = pdp.NaiveBudgetAccountant(total_epsilon=1, total_delta=1e-6)
    b1 = acct.request_budget(mechanism_type=pdp.MechanismType.LAPLACE)
    b2 = acct.request_budget(mechanism_type=pdp.MechanismType.GAUSSIAN, weight=3)
    with pytest.raises(AssertionError):
        _ = b1.eps
    acct.compute_budgets()
    assert (b1.eps, b1.delta, b2.eps, b2.delta) == (0.25, 0, 0.75, 1e-6)


def test_budget_scopes_known_answer():
    # tests/budget_accounting_test.py:72-110
    acct = pdp.NaiveBudgetAccountant(total_epsilon=1, total_delta=1e-6)
    with acct.scope(weight=0.4):
        b1 = acct.request_budget(mechanism_type=pdp.MechanismType.LAPLACE)
        b2 = acct.request_budget(mechanism_type=pdp.MechanismType.LAPLACE, weight=3)
    with acct.scope(weight=0.6):
        b3 = acct.request_budget(mechanism_type=pdp.MechanismType.LAPLACE)
        b4 = acct.request_budget(mechanism_type=pdp.MechanismType.LAPLACE, weight=4)
    acct.compute_budgets()
    assert b1.eps == 0.4 * (1 / 4) and b2.eps == 0.4 * (3 / 4)
    assert b3.eps == 0.6 * (1 / 5) and b4.eps == 0.6 * (4 / 5)
    acct2 = pdp.NaiveBudgetAccountant(total_epsilon=1, total_delta=1e-6)
    c1 = acct2.request_budget(mechanism_type=pdp.MechanismType.LAPLACE)
    with acct2.scope(weight=0.5):
        c2 = acct2.request_budget(mechanism_type=pdp.MechanismType.LAPLACE)
    acct2.compute_budgets()
    assert c1.eps == 1.0 / 1.5 and c2.eps == 0.5 / 1.5


def test_budget_accountant_errors():
    with pytest.raises(ValueError):
        pdp.NaiveBudgetAccountant(total_epsilon=0, total_delta=1e-6)
    with pytest.raises(ValueError):
        pdp.NaiveBudgetAccountant(total_epsilon=1, total_delta=1)
    acct = pdp.NaiveBudgetAccountant(total_epsilon=1, total_delta=0)
    with pytest.raises(ValueError):
        acct.request_budget(pdp.MechanismType.GAUSSIAN)
    acct = pdp.NaiveBudgetAccountant(total_epsilon=1, total_delta=1e-6, num_aggregations=2)
    acct._compute_budget_for_aggregation(1)
    with pytest.raises(ValueError):
        acct.compute_budgets()


@pytest.mark.parametrize("kwargs,err", [
    (dict(metrics=[M.SUM], max_partitions_contributed=1, max_contributions_per_partition=1), ValueError),
    (dict(metrics=[M.COUNT], max_partitions_contributed=1), ValueError),
    (dict(metrics=[M.COUNT], max_partitions_contributed=0, max_contributions_per_partition=1), ValueError),
    (dict(metrics=[M.COUNT], max_partitions_contributed=1, max_contributions_per_partition=1, min_value=1),
     ValueError),
    (dict(metrics=[M.MEAN], max_partitions_contributed=1, max_contributions_per_partition=1, min_value=2,
          max_value=1), ValueError),
    (dict(metrics=[M.MEAN], max_partitions_contributed=1, max_contributions_per_partition=1,
          min_sum_per_partition=0, max_sum_per_partition=1), ValueError),
    (dict(metrics=[M.COUNT], max_partitions_contributed=1, max_contributions_per_partition=1, low=1), ValueError),
    (dict(metrics=[M.PRIVACY_ID_COUNT], max_partitions_contributed=1, max_contributions_per_partition=1,
          contribution_bounds_already_enforced=True), ValueError),
    (dict(metrics=[M.SUM], max_partitions_contributed=1, max_contributions_per_partition=1, min_value=0,
          max_value=float("inf")), ValueError),
])
def test_aggregate_params_validation(kwargs, err):
    with pytest.raises(err):
        pdp.AggregateParams(**kwargs)


def test_engine_validation_errors():
    acct = pdp.NaiveBudgetAccountant(1, 1e-6)
    engine = pdp.DPEngine(acct, pdp.HipBackend())
    params = pdp.AggregateParams(metrics=[M.COUNT], max_partitions_contributed=1, max_contributions_per_partition=1)
    ex = pdp.DataExtractors(lambda r: r, lambda r: r, lambda r: r)
    with pytest.raises(ValueError, match="col must be non-empty"):
        engine.aggregate([], params, ex)
    with pytest.raises(TypeError):
        engine.aggregate([1], object(), ex)
    with pytest.raises(ValueError, match="data_extractors"):
        engine.aggregate([1], params, None)
    p2 = pdp.AggregateParams(metrics=[M.COUNT], max_contributions=3)
    with pytest.raises(NotImplementedError):
        engine.aggregate([1], p2, ex)
    p3 = pdp.AggregateParams(metrics=[M.PERCENTILE(50)], max_partitions_contributed=1,
                             max_contributions_per_partition=1, min_value=0, max_value=1)
    with pytest.raises(NotImplementedError):
        engine.aggregate([1], p3, ex)
    p4 = pdp.AggregateParams(metrics=[M.COUNT], max_partitions_contributed=1, max_contributions_per_partition=1,
                             contribution_bounds_already_enforced=True)
    with pytest.raises(ValueError, match="privacy_id_extractor"):
        engine.aggregate([1], p4, ex)


def test_result_is_lazy_and_needs_budgets():
    acct = pdp.NaiveBudgetAccountant(1, 1e-6)
    engine = pdp.DPEngine(acct, pdp.HipBackend())
    params = pdp.AggregateParams(metrics=[M.COUNT], max_partitions_contributed=1, max_contributions_per_partition=1)

    def exploding():
        raise AssertionError("input must not be read at graph construction")
        yield  # pragma: no cover

    res = engine.aggregate(exploding(), params, pdp.DataExtractors(lambda r: r, lambda r: r, lambda r: r))
    assert isinstance(res, pdp.DPResult)
    with pytest.raises(AssertionError, match="not calculated yet"):
        res._release_config(1)


def _params_from_cfg(cfg):
    metric = {"count": M.COUNT, "sum": M.SUM, "mean": M.MEAN, "variance": M.VARIANCE,
              "privacy_id_count": M.PRIVACY_ID_COUNT}
    kw = dict(metrics=[metric[m] for m in cfg["metrics"]], noise_kind=pdp.NoiseKind(cfg.get("noise_kind", "laplace")),
              max_partitions_contributed=cfg["L0"], max_contributions_per_partition=cfg["Linf"],
              contribution_bounds_already_enforced=cfg.get("already_enforced", False))
    for k in ("min_value", "max_value", "min_sum_per_partition", "max_sum_per_partition"):
        if cfg.get(k) is not None:
            kw[k] = cfg[k]
    return pdp.AggregateParams(**kw)


@pytest.mark.parametrize("name", aggregate_cases())
def test_explain_report_matches_reference(name):
    """The explain-computation report (stages, budgets, parameter block) is
    byte-identical to the one the reference produced for the golden case."""
    d = load(name)
    cfg = d["meta"]["cfg"]
    acct = pdp.NaiveBudgetAccountant(total_epsilon=cfg.get("eps", 1.0), total_delta=cfg.get("delta", 1e-6))
    engine = pdp.DPEngine(acct, pdp.HipBackend())
    enforced = cfg.get("already_enforced", False)
    ex = pdp.DataExtractors(privacy_id_extractor=None if enforced else (lambda r: r[0]),
                            partition_extractor=lambda r: r[1], value_extractor=lambda r: r[2])
    public = d["public"].tolist() if bool(d["has_public"]) else None
    report = pdp.ExplainComputationReport()
    engine.aggregate([(0, 0, 0.0)], _params_from_cfg(cfg), ex, public, out_explain_computaton_report=report)
    acct.compute_budgets()
    assert report.text() == d["meta"]["report"]


def test_params_readable_string():
    p = pdp.AggregateParams(metrics=[M.SUM], max_partitions_contributed=2, max_contributions_per_partition=10,
                            min_value=1, max_value=5)
    assert str(p) == ("AggregateParams:\n metrics=['SUM']\n noise_kind=laplace\n budget_weight=1\n"
                      " Contribution bounding:\n  max_partitions_contributed=2\n"
                      "  max_contributions_per_partition=10\n  min_value=1\n  max_value=5")


def test_host_encoding():
    from pipelinedp_amd.columnar import encode_rows
    rows = [("u1", "a", 1.0), ("u2", "b", 2.0), ("u1", "c", 3.0), ("u3", "a", 4.0)]
    ex = pdp.DataExtractors(lambda r: r[0], lambda r: r[1], lambda r: r[2])
    e = encode_rows(rows, ex)
    assert e.partition_keys == ["a", "b", "c"] and e.pk.tolist() == [0, 1, 2, 0]
    # privacy ids numbered by the ascending order of their 128-bit key hash (columnar.dense_ids_from_hashes)
    from pipelinedp_amd.columnar import key_hashes
    h = key_hashes(["u1", "u2", "u3"])
    order = sorted(range(3), key=lambda i: (int(h[i, 0]), int(h[i, 1])))
    rank = {["u1", "u2", "u3"][i]: r for r, i in enumerate(order)}
    assert e.pid.tolist() == [rank["u1"], rank["u2"], rank["u1"], rank["u3"]] and e.num_privacy_ids == 3
    # the hash is process-independent (blake2b of canonical bytes; numpy scalars / integral floats as ints)
    hk = lambda k: tuple(key_hashes([k])[0].tolist())  # noqa: E731
    assert hk(5) == hk(np.int64(5)) == hk(5.0) == hk(5 + 0j)
    assert hk(True) == hk(1) == hk(1.0) and hk(False) == hk(0) and hk((True, 2)) == hk((1, 2.0))
    assert len({tuple(r) for r in key_hashes(["5", 5, (5,), b"5", None, 5.5]).tolist()}) == 6
    e = encode_rows(rows, ex, public_partitions=["c", "zz", "a", "c"])
    assert e.partition_keys == ["c", "zz", "a"] and e.pk.tolist() == [2, -1, 0, 2]
    np.testing.assert_array_equal(e.value, [1, 2, 3, 4])


def _dict_groups(keys):
    """The reference's privacy-id grouping: by dict key (pipeline_backend.py:476-485)."""
    first = {}
    return [first.setdefault(k, len(first)) for k in keys]


def _same_partition(a, b):
    """Two labelings of the same items induce the same grouping."""
    a, b = list(a), list(b)
    return all((a[i] == a[j]) == (b[i] == b[j]) for i in range(len(a)) for j in range(len(a)))


MIXED_KEYS = [True, 1, 1.0, np.int64(1), "1", b"1", 2, 2.0, np.float32(2.0), False, 0, 0.0, -0.0, None, (1, 2),
              (True, 2.0), (1, "2"), 3.5, np.float64(3.5), "u", "u", 1 + 0j, 7, "7"]


def test_privacy_ids_grouped_by_dict_equality():
    """True == 1 == 1.0 (and False == 0, numpy scalars, tuples of them) are ONE
    dict key, so ONE privacy id in the reference; the encoding follows it
    (round-5 advisor: bool and int canonicalised differently)."""
    from pipelinedp_amd.columnar import encode_rows
    rows = [(k, "p", 1.0) for k in MIXED_KEYS]
    e = encode_rows(rows, pdp.DataExtractors(lambda r: r[0], lambda r: r[1], lambda r: r[2]))
    assert _same_partition(e.pid, _dict_groups(MIXED_KEYS))
    assert e.num_privacy_ids == len(set(_dict_groups(MIXED_KEYS)))
    assert sorted(set(e.pid.tolist())) == list(range(e.num_privacy_ids))


def test_privacy_ids_exact_under_forced_hash_collisions(monkeypatch):
    """Every key hashed to the SAME 128-bit value (monkeypatched): distinct
    keys must still be distinct privacy ids (told apart by their canonical
    bytes, deterministic order), equal keys one id.  Then a non-binding
    aggregate through DPEngine equals the reference's per-dict-key counts."""
    from pipelinedp_amd import columnar
    real = columnar.key_hashes
    monkeypatch.setattr(columnar, "key_hashes", lambda keys: np.zeros((len(keys), 2), np.int64))
    rows = [(k, "p", 1.0) for k in MIXED_KEYS]
    ex = pdp.DataExtractors(lambda r: r[0], lambda r: r[1], lambda r: r[2])
    e = columnar.encode_rows(rows, ex)
    assert _same_partition(e.pid, _dict_groups(MIXED_KEYS))
    # deterministic: the same ids in another input order
    perm = list(reversed(range(len(rows))))
    e2 = columnar.encode_rows([rows[i] for i in perm], ex)
    assert [int(e2.pid[j]) for j in range(len(perm))] == [int(e.pid[i]) for i in perm]
    # a partial collision (word 0 only) under the real hash: still exact, same grouping
    monkeypatch.setattr(columnar, "key_hashes", lambda keys: real(keys) * np.array([[0, 1]], np.int64))
    e3 = columnar.encode_rows(rows, ex)
    assert _same_partition(e3.pid, _dict_groups(MIXED_KEYS))
    # through the engine (tests/cpu_executor.py stands in for the GPU): non-binding bounds, so the
    # privacy-id count of each partition is the number of distinct dict keys contributing to it
    from cpu_executor import CpuExecutor
    keys = MIXED_KEYS * 3
    rows = [(k, f"part{i % 4}", 1.0) for i, k in enumerate(keys)]
    backend = pdp.HipBackend(sampling_seed=5, noise_seed=9)
    backend._executor = CpuExecutor()
    acct = pdp.NaiveBudgetAccountant(total_epsilon=1e6, total_delta=1e-3)
    engine = pdp.DPEngine(acct, backend)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=4, max_contributions_per_partition=100)
    res = engine.aggregate(rows, params, ex, public_partitions=[f"part{j}" for j in range(4)])
    acct.compute_budgets()
    got = {k: v for k, v in res}
    for j in range(4):
        members = [r[0] for r in rows if r[1] == f"part{j}"]
        assert round(got[f"part{j}"].privacy_id_count) == len(set(_dict_groups(members)))
        assert round(got[f"part{j}"].count) == len(members)


def test_hip_backend_host_ops_follow_local_backend():
    # LocalBackend.sample_fixed_per_key / combine_accumulators_per_key
    # (pipeline_backend.py:504-538), element-wise on the host
    b = pdp.HipBackend(sampling_seed=3)
    col = [("a", i) for i in range(10)] + [("b", 1), ("b", 2)]
    out = dict(b.sample_fixed_per_key(col, 3))
    assert set(out) == {"a", "b"} and len(out["a"]) == 3 and len(set(out["a"])) == 3
    assert set(out["a"]) <= set(range(10)) and sorted(out["b"]) == [1, 2]

    class SumCombiner:

        def merge_accumulators(self, a, b):
            return a + b

    merged = dict(b.combine_accumulators_per_key([("x", 1), ("y", 5), ("x", 2), ("x", 3)], SumCombiner()))
    assert merged == {"x": 6, "y": 5}
    assert sorted(b.sum_per_key([("x", 1), ("x", 2), ("y", 3)])) == [("x", 3), ("y", 3)]


def _engine_with_cpu_executor():
    from cpu_executor import CpuExecutor
    backend = pdp.HipBackend(sampling_seed=1, noise_seed=2)
    backend._executor = CpuExecutor()
    acct = pdp.NaiveBudgetAccountant(total_epsilon=1, total_delta=1e-6)
    return pdp.DPEngine(acct, backend), acct


def test_empty_public_partitions_give_empty_result():
    # reference: public_partitions=[] drops every row and adds no partition
    engine, acct = _engine_with_cpu_executor()
    params = pdp.AggregateParams(metrics=[M.COUNT], max_partitions_contributed=1, max_contributions_per_partition=1)
    ex = pdp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                            value_extractor=lambda r: 0)
    res = engine.aggregate([(1, "a"), (2, "b")], params, ex, public_partitions=[])
    acct.compute_budgets()
    assert list(res) == []


def test_columnar_partition_out_of_range_raises():
    engine, acct = _engine_with_cpu_executor()
    params = pdp.AggregateParams(metrics=[M.COUNT], max_partitions_contributed=1, max_contributions_per_partition=1)
    col = pdp.ColumnarData(partition=np.array([0, 1, 5]), privacy_id=np.array([0, 1, 2]), num_partitions=3)
    res = engine.aggregate(col, params, None, public_partitions=[0, 1])
    acct.compute_budgets()
    with pytest.raises(ValueError, match="num_partitions"):
        list(res)


def test_pipeline_dp_alias_runs_reference_caller_code():
    # a reference caller (run_without_frameworks.py shape) with only the backend changed
    import pipeline_dp
    from cpu_executor import CpuExecutor
    backend = pipeline_dp.HipBackend(sampling_seed=1, noise_seed=2)
    backend._executor = CpuExecutor()
    acct = pipeline_dp.NaiveBudgetAccountant(total_epsilon=100, total_delta=1e-6)
    engine = pipeline_dp.DPEngine(acct, backend)
    params = pipeline_dp.AggregateParams(noise_kind=pipeline_dp.NoiseKind.LAPLACE,
                                         metrics=[pipeline_dp.Metrics.COUNT, pipeline_dp.Metrics.SUM],
                                         max_partitions_contributed=3, max_contributions_per_partition=2,
                                         min_value=1, max_value=5)
    rows = [(u, f"movie{u % 4}", 1 + u % 5) for u in range(400)]
    ext = pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                                     value_extractor=lambda r: r[2])
    res = engine.aggregate(rows, params, ext)
    acct.compute_budgets()
    out = dict(res)
    assert sorted(out) == [f"movie{i}" for i in range(4)]
    assert all(abs(t.count - 100) < 10 for t in out.values())
    import pipeline_dp.aggregate_params as ap
    assert ap.AggregateParams is pipeline_dp.AggregateParams
    with pytest.raises(AttributeError, match="HipBackend"):
        pipeline_dp.LocalBackend  # noqa: B018
