"""Utility analysis (BASELINE configs[4]) on the CPU: the oracle restatement
and the host engine (pipelinedp_amd.analysis, executor replaced by the CPU
stand-in) against golden vectors from the reference UtilityAnalysisEngine,
and the reference tests' own known answers
(analysis/tests/utility_analysis_engine_test.py:157-220, 222-302)."""
import numpy as np
import pytest

import pipelinedp_amd as pdp
from analysis_util import CASES, check_case, run_case
from pipelinedp_amd import analysis as A


def _backend():
    from cpu_executor import CpuExecutor
    b = pdp.HipBackend()
    b._executor = CpuExecutor()
    return b


@pytest.mark.parametrize("name", CASES)
def test_engine_matches_reference_golden_on_cpu_executor(name):
    d, got = run_case(name, _backend())
    check_case(d, got)


def test_reference_per_partition_known_answers():
    # analysis/tests/utility_analysis_engine_test.py:203-220
    _, got = run_case("reference_per_partition_errors", _backend())
    assert len(got) == 10
    for _, v in got.items():
        assert v[1].per_partition_error_max == -10
        assert v[1].expected_cross_partition_error == pytest.approx(-18.0, abs=1e-5)
        assert v[1].std_cross_partition_error == pytest.approx(1.89736, abs=1e-5)
        assert v[1].std_noise == pytest.approx(11.95312, abs=1e-5)


def test_reference_multi_parameters_known_answers():
    # analysis/tests/utility_analysis_engine_test.py:264-302 (public partitions, 2 configurations)
    _, got = run_case("reference_multi_parameters", _backend())
    G = pdp.NoiseKind.GAUSSIAN
    assert got[0] == (A.SumMetrics(1.0, 0.0, 0.0, -0.5, 0.5, 5.87109375, G),
                      A.SumMetrics(1.0, 0.0, 0.0, 0, 0.0, pytest.approx(16.60596081442783), G))
    assert got[1] == (A.SumMetrics(2.0, 0.0, -1.0, -0.5, 0.5, 5.87109375, G),
                      A.SumMetrics(2.0, 0.0, 0.0, 0, 0.0, pytest.approx(16.60596081442783), G))


def test_analysis_validation_errors():
    params = pdp.AggregateParams(metrics=[pdp.Metrics.MEAN], max_partitions_contributed=1,
                                 max_contributions_per_partition=1, min_value=0, max_value=1)
    eng = A.UtilityAnalysisEngine(pdp.NaiveBudgetAccountant(1, 1e-6), _backend())
    ex = pdp.DataExtractors(privacy_id_extractor=lambda r: r, partition_extractor=lambda r: r,
                            value_extractor=lambda r: r)
    with pytest.raises(NotImplementedError, match="unsupported metric"):
        eng.analyze([1], A.UtilityAnalysisOptions(1, 1e-6, params), ex)
    count = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT], max_partitions_contributed=1,
                                max_contributions_per_partition=1)
    with pytest.raises(ValueError, match="PreAggregateExtractors"):
        eng.analyze([1], A.UtilityAnalysisOptions(1, 1e-6, count, pre_aggregated_data=True), ex)
    with pytest.raises(ValueError, match="can't be called"):
        eng.aggregate([1], count, ex)
    with pytest.raises(ValueError):
        A.UtilityAnalysisOptions(1, 1e-6, count, partitions_sampling_prob=0)
    with pytest.raises(ValueError):
        A.MultiParameterConfiguration(max_partitions_contributed=[1, 2], max_contributions_per_partition=[1])


def test_value_sampler_matches_reference_counts():
    # tests/sampling_utils_test.py:54-79 pins ValueSampler on range(1000)
    from golden_util import known_answers
    for c in known_answers()["value_sampler"]:
        s = A.ValueSampler(c["rate"])
        vals = [str(v) for v in range(c["n"])] if c["str"] else range(c["n"])
        assert sum(s.keep(v) for v in vals) == c["kept"]


@pytest.mark.parametrize("name", ["private_gaussian", "public_gaussian", "private_laplace"])
def test_oracle_aggregate_matches_reference_golden(name):
    """pdp_analysis_oracle's perform_utility_analysis restatement against the
    reference (tests/golden/aggregate_*.npz, oracle/gen_golden.py).  Gaussian
    quantiles are closed form (exact); Laplace quantiles are the reference's
    Monte-Carlo estimates, compared by distribution (analysis_util)."""
    from analysis_util import check_aggregate, oracle_aggregate
    from golden_util import load
    d = load("aggregate_" + name)
    check_aggregate(d, oracle_aggregate(d), rtol=1e-8, atol=1e-9, quantile_sigmas=4.0)


def _agg_as_dicts(result):
    """perform_utility_analysis output -> check_aggregate's per-configuration dicts."""
    import dataclasses as dc
    out = []
    lst = list(result)
    assert len(lst) == 1
    for am in lst[0]:
        d = {"selection": None if am.partition_selection_metrics is None else dc.asdict(am.partition_selection_metrics)}
        for m in ("count", "privacy_id_count", "sum"):
            em = getattr(am, m + "_metrics")
            if em is not None:
                d[m] = {k: v for k, v in dc.asdict(em).items() if k != "metric_type"}
        out.append(d)
    return out


def run_perform(name, backend):
    """pipelinedp_amd.analysis.perform_utility_analysis on an aggregate_* golden."""
    from golden_util import load
    d = load("aggregate_" + name)
    meta = d["meta"]
    cfg = meta["cfg"]
    kw = dict(metrics=[{"count": pdp.Metrics.COUNT, "sum": pdp.Metrics.SUM,
                        "privacy_id_count": pdp.Metrics.PRIVACY_ID_COUNT}[m] for m in cfg["metrics"]],
              noise_kind=pdp.NoiseKind(cfg["noise_kind"]), max_partitions_contributed=cfg["L0"],
              max_contributions_per_partition=cfg["Linf"])
    for k in ("min_sum_per_partition", "max_sum_per_partition"):
        if cfg.get(k) is not None:
            kw[k] = cfg[k]
    multi = A.MultiParameterConfiguration(**meta["multi"]) if meta["multi"] else None
    options = A.UtilityAnalysisOptions(epsilon=cfg["eps"], delta=cfg["delta"], aggregate_params=pdp.AggregateParams(**kw),
                                       multi_param_configuration=multi, partitions_sampling_prob=meta["sampling"])
    rows = list(zip(d["pid"].tolist(), d["pk"].tolist(), d["value"].tolist()))
    ex = pdp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                            value_extractor=lambda r: r[2])
    public = d["public"].tolist() if bool(d["has_public"]) else None
    return d, A.perform_utility_analysis(rows, backend, options, ex, public_partitions=public)


@pytest.mark.parametrize("name", ["private_gaussian", "public_gaussian", "private_laplace"])
def test_perform_utility_analysis_host_on_cpu_executor(name):
    """The host side of perform_utility_analysis (budget split, std_noise, the
    compute_metrics divisions, AggregateMetrics packing) with the CPU
    stand-in executor, against the reference goldens."""
    from analysis_util import check_aggregate
    d, res = run_perform(name, _backend())
    check_aggregate(d, _agg_as_dicts(res), rtol=1e-8, atol=1e-9, quantile_sigmas=4.0)
