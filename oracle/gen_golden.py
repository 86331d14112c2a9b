"""Generate golden vectors from the REFERENCE PipelineDP LocalBackend.

CONTAINER-ONLY TEST INFRASTRUCTURE.  Run in the build container (where
/root/reference exists) as

    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden.py

It puts oracle/pydp_stub (identity noise, keep-all selection; PyDP is not
installed) and /root/reference on sys.path, runs the reference
``DPEngine(..., LocalBackend()).aggregate`` on seeded inputs and writes the
inputs plus the reference outputs to tests/golden/*.npz.  The fixtures are
data only; no reference source travels with them.

Cases use non-binding bounds (or deterministic clipping) so that the
LocalBackend result is deterministic, except ``binding_*`` which records the
mean of the reference output over many numpy seeds (a distributional target
for uniform sampling without replacement).
"""
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "pydp_stub"))
sys.path.insert(0, REF)

import numpy as np  # noqa: E402

import pipeline_dp  # noqa: E402  (the reference, via the stub)

# The repo root holds a `pipeline_dp` alias of pipelinedp_amd: make sure the goldens come from the
# reference and not from the implementation under test.
assert os.path.realpath(pipeline_dp.__file__).startswith(os.path.realpath(REF) + os.sep), pipeline_dp.__file__

OUT = os.path.join(REPO, "tests", "golden")

METRIC = {
    "count": pipeline_dp.Metrics.COUNT,
    "sum": pipeline_dp.Metrics.SUM,
    "mean": pipeline_dp.Metrics.MEAN,
    "variance": pipeline_dp.Metrics.VARIANCE,
    "privacy_id_count": pipeline_dp.Metrics.PRIVACY_ID_COUNT,
}


def run_reference(pid, pk, value, cfg, public=None, seed=None):
    if seed is not None:
        np.random.seed(seed)
    acct = pipeline_dp.NaiveBudgetAccountant(total_epsilon=cfg.get("eps", 1.0),
                                             total_delta=cfg.get("delta", 1e-6))
    engine = pipeline_dp.DPEngine(acct, pipeline_dp.LocalBackend())
    kw = dict(metrics=[METRIC[m] for m in cfg["metrics"]],
              noise_kind=pipeline_dp.NoiseKind(cfg.get("noise_kind", "laplace")),
              max_partitions_contributed=cfg["L0"],
              max_contributions_per_partition=cfg["Linf"])
    for k in ("min_value", "max_value", "min_sum_per_partition", "max_sum_per_partition"):
        if cfg.get(k) is not None:
            kw[k] = cfg[k]
    enforced = cfg.get("already_enforced", False)
    kw["contribution_bounds_already_enforced"] = enforced
    params = pipeline_dp.AggregateParams(**kw)
    has_value = value is not None
    rows = [(int(pid[i]) if pid is not None else None, int(pk[i]),
             float(value[i]) if has_value else None) for i in range(len(pk))]
    ex = pipeline_dp.DataExtractors(
        privacy_id_extractor=None if enforced else (lambda r: r[0]),
        partition_extractor=lambda r: r[1],
        value_extractor=lambda r: r[2])
    report = pipeline_dp.ExplainComputationReport()
    res = engine.aggregate(rows, params, ex, public_partitions=public,
                           out_explain_computaton_report=report)
    acct.compute_budgets()
    res = list(res)
    text = report.text()
    if not res:
        return np.zeros(0, np.int64), np.zeros((0, 0)), [], text
    fields = list(res[0][1]._fields)
    keys = np.array([k for k, _ in res], dtype=np.int64)
    vals = np.array([[float(getattr(t, f)) for f in fields] for _, t in res])
    o = np.argsort(keys, kind="stable")
    return keys[o], vals[o], fields, text


def save(name, pid, pk, value, cfg, public=None, **extra):
    keys, vals, fields, text = run_reference(pid, pk, value, cfg, public)
    np.savez_compressed(
        os.path.join(OUT, name + ".npz"),
        pid=np.asarray(pid if pid is not None else [], dtype=np.int64),
        pk=np.asarray(pk, dtype=np.int64),
        value=np.asarray(value if value is not None else [], dtype=np.float64),
        public=np.asarray(public if public is not None else [], dtype=np.int64),
        has_public=np.asarray(public is not None),
        out_keys=keys, out_vals=vals,
        meta=np.asarray(json.dumps(dict(cfg=cfg, fields=fields, report=text, **extra))))
    print(f"{name}: {len(pk)} rows -> {len(keys)} partitions, fields={fields}")


def nonbinding(pid, pk):
    pairs = {}
    per_pid = {}
    for a, b in zip(pid.tolist(), pk.tolist()):
        pairs[(a, b)] = pairs.get((a, b), 0) + 1
        per_pid.setdefault(a, set()).add(b)
    return max(len(s) for s in per_pid.values()), max(pairs.values())


def netflix():
    """contributing/sample_combined_data_1.txt in Netflix format, parsed like
    examples/movie_view_ratings/common_utils.py:51-59 (movie_id line ends
    with ':', then 'user_id,rating,date')."""
    movie, users, movies, ratings = None, [], [], []
    with open(os.path.join(REF, "contributing", "sample_combined_data_1.txt")) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            if line[-1] == ":":
                movie = int(line[:-1])
            else:
                u, r, _ = line.split(",")
                users.append(int(u))
                movies.append(movie)
                ratings.append(float(r))
    return np.array(users), np.array(movies), np.array(ratings)


def main():
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(20250204)

    # A. Netflix sample, configs[0] shape: COUNT+SUM+MEAN(+PID count).
    u, m, r = netflix()
    L0, Linf = nonbinding(u, m)
    save("netflix_count_sum_mean", u, m, r,
         dict(metrics=["count", "sum", "mean", "privacy_id_count"], L0=L0, Linf=Linf,
              min_value=1.0, max_value=5.0))

    # Synthetic data with clipping active (values outside [a, b]).
    n, U, P = 20000, 400, 250
    pid = rng.integers(0, U, n)
    pk = np.minimum(rng.zipf(1.3, n) - 1, P - 1)
    val = rng.normal(5.0, 3.0, n)
    L0, Linf = nonbinding(pid, pk)
    save("synth_count_sum_mean", pid, pk, val,
         dict(metrics=["count", "sum", "mean"], L0=L0, Linf=Linf, min_value=0.0, max_value=10.0))
    save("synth_variance", pid, pk, val,
         dict(metrics=["variance", "mean", "count", "sum"], L0=L0, Linf=Linf,
              min_value=-2.0, max_value=7.0, noise_kind="gaussian"))
    save("synth_count_sum_pidcount", pid, pk, val,
         dict(metrics=["count", "sum", "privacy_id_count"], L0=L0, Linf=Linf,
              min_value=1.0, max_value=8.0))
    save("synth_per_partition_sum", pid, pk, val,
         dict(metrics=["count", "sum"], L0=L0, Linf=Linf,
              min_sum_per_partition=-5.0, max_sum_per_partition=40.0))
    save("synth_mean_min_eq_max", pid, pk, val,
         dict(metrics=["mean", "count"], L0=L0, Linf=Linf, min_value=3.0, max_value=3.0))
    save("synth_count_only", pid, pk, None,
         dict(metrics=["count", "privacy_id_count"], L0=L0, Linf=Linf))

    # Public partitions: a subset of observed keys plus absent ones.
    public = sorted(set(range(0, P, 3)) | {P + 5, P + 17})
    save("synth_public_partitions", pid, pk, val,
         dict(metrics=["count", "sum", "privacy_id_count"], L0=L0, Linf=Linf,
              min_value=0.0, max_value=10.0, noise_kind="gaussian"), public=public)
    save("synth_public_mean_empty", pid, pk, val,
         dict(metrics=["mean", "count", "sum"], L0=L0, Linf=Linf,
              min_value=-1.0, max_value=4.0), public=public)

    # contribution_bounds_already_enforced (no privacy ids).
    save("synth_already_enforced_public", None, pk, val,
         dict(metrics=["count", "sum"], L0=3, Linf=2, min_value=0.0, max_value=10.0,
              already_enforced=True), public=public)
    save("synth_already_enforced_private", None, pk, val,
         dict(metrics=["sum"], L0=3, Linf=2, min_value=0.0, max_value=10.0,
              already_enforced=True))

    # Binding bounds: mean over reference runs (distributional target).
    nb, Ub, Pb = 600, 30, 12
    pidb = rng.integers(0, Ub, nb)
    pkb = rng.integers(0, Pb, nb)
    valb = rng.uniform(0, 10, nb)
    cfg = dict(metrics=["count", "sum", "privacy_id_count"], L0=3, Linf=2,
               min_value=0.0, max_value=10.0)
    runs = 400
    acc = []
    for s in range(runs):
        keys, vals, fields, _ = run_reference(pidb, pkb, valb, cfg, seed=s)
        full = np.zeros((Pb, len(fields)))
        full[keys] = vals
        acc.append(full)
    acc = np.array(acc)
    np.savez_compressed(os.path.join(OUT, "binding_count_sum_pidcount.npz"),
                        pid=pidb, pk=pkb, value=valb, runs=runs,
                        mean=acc.mean(0), std=acc.std(0),
                        meta=np.asarray(json.dumps(dict(cfg=cfg, fields=fields))))
    print(f"binding: {runs} runs, fields={fields}")


def run_select_partitions(pid, pk, L0, threshold, seed=None):
    """Reference DPEngine.select_partitions (dp_engine.py:204-281) with the
    stub's deterministic strategy keep(n) = n >= threshold."""
    if seed is not None:
        np.random.seed(seed)
    os.environ["PDP_STUB_SELECT_THRESHOLD"] = str(threshold)
    try:
        acct = pipeline_dp.NaiveBudgetAccountant(total_epsilon=1.0, total_delta=1e-6)
        engine = pipeline_dp.DPEngine(acct, pipeline_dp.LocalBackend())
        ex = pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1])
        res = engine.select_partitions([(int(a), int(b)) for a, b in zip(pid, pk)],
                                       pipeline_dp.SelectPartitionsParams(max_partitions_contributed=L0), ex)
        acct.compute_budgets()
        return sorted(int(k) for k in res)
    finally:
        del os.environ["PDP_STUB_SELECT_THRESHOLD"]


def select_partitions_cases():
    """select_partitions goldens: non-binding L0 (exact kept set) and binding
    L0 (per-partition inclusion frequency over 400 numpy seeds)."""
    rng = np.random.default_rng(20250205)
    n, U, P = 8000, 600, 300
    pid = rng.integers(0, U, n)
    pk = np.minimum(rng.zipf(1.4, n) - 1, P - 1)
    L0, _ = nonbinding(pid, pk)
    T = 3
    kept = run_select_partitions(pid, pk, L0, T)
    np.savez_compressed(os.path.join(OUT, "select_partitions_nonbinding.npz"), pid=pid, pk=pk,
                        out_keys=np.asarray(kept, np.int64),
                        meta=np.asarray(json.dumps(dict(L0=L0, threshold=T, P=P))))
    print(f"select_partitions_nonbinding: {n} rows, L0={L0}, {len(kept)} kept")
    nb, Ub, Pb, L0b, Tb, runs = 900, 60, 15, 1, 5, 400
    pidb = rng.integers(0, Ub, nb)
    pkb = rng.integers(0, Pb, nb)
    freq = np.zeros(Pb)
    for s in range(runs):
        for k in run_select_partitions(pidb, pkb, L0b, Tb, seed=s):
            freq[k] += 1
    np.savez_compressed(os.path.join(OUT, "select_partitions_binding.npz"), pid=pidb, pk=pkb, freq=freq / runs,
                        runs=runs, meta=np.asarray(json.dumps(dict(L0=L0b, threshold=Tb, P=Pb))))
    print(f"select_partitions_binding: {runs} runs, inclusion frequencies {np.round(freq / runs, 3)}")


def run_analysis(rows, extractors, cfg, multi=None, public=None, pre_aggregated=False, sampling=1.0):
    """Reference UtilityAnalysisEngine.analyze (analysis/utility_analysis_engine.py:53-86)
    -> keys and per-partition arrays: prob [C, P] (private only) and, per
    metric of (SUM, COUNT, PRIVACY_ID_COUNT) present, [C, 6, P] of
    (sum, err_min, err_max, expected_cross, std_cross, std_noise)."""
    import analysis
    from analysis import utility_analysis_engine
    acct = pipeline_dp.NaiveBudgetAccountant(total_epsilon=cfg["eps"], total_delta=cfg["delta"])
    engine = utility_analysis_engine.UtilityAnalysisEngine(acct, pipeline_dp.LocalBackend())
    kw = dict(metrics=[METRIC[m] for m in cfg["metrics"]],
              noise_kind=pipeline_dp.NoiseKind(cfg.get("noise_kind", "laplace")),
              max_partitions_contributed=cfg["L0"], max_contributions_per_partition=cfg["Linf"])
    for k in ("min_sum_per_partition", "max_sum_per_partition"):
        if cfg.get(k) is not None:
            kw[k] = cfg[k]
    if cfg.get("selection"):
        kw["partition_selection_strategy"] = pipeline_dp.PartitionSelectionStrategy[cfg["selection"].upper()]
    params = pipeline_dp.AggregateParams(**kw)
    mp = None
    if multi:
        mk = dict(multi)
        if "partition_selection_strategy" in mk:
            mk["partition_selection_strategy"] = [pipeline_dp.PartitionSelectionStrategy[v.upper()]
                                                  for v in mk["partition_selection_strategy"]]
        if "noise_kind" in mk:
            mk["noise_kind"] = [pipeline_dp.NoiseKind(v) for v in mk["noise_kind"]]
        mp = analysis.MultiParameterConfiguration(**mk)
    options = analysis.UtilityAnalysisOptions(epsilon=cfg["eps"], delta=cfg["delta"], aggregate_params=params,
                                              multi_param_configuration=mp, partitions_sampling_prob=sampling,
                                              pre_aggregated_data=pre_aggregated)
    out = engine.analyze(rows, options, extractors, public_partitions=public)
    acct.compute_budgets()
    out = sorted(list(out), key=lambda kv: kv[0])
    C = options.n_configurations
    present = [m for m in ("sum", "count", "privacy_id_count") if m in cfg["metrics"]]
    per = (0 if public is not None else 1) + len(present)
    P = len(out)
    keys = np.array([k for k, _ in out], dtype=np.int64)
    prob = np.zeros((C, P))
    arr = {m: np.zeros((C, 6, P)) for m in present}
    for p, (_, vals) in enumerate(out):
        vals = list(vals)
        assert len(vals) == C * per, (len(vals), C, per)
        for c in range(C):
            chunk = vals[c * per:(c + 1) * per]
            if public is None:
                prob[c, p] = float(chunk[0])
                chunk = chunk[1:]
            for m, sm in zip(present, chunk):
                arr[m][c, :, p] = (sm.sum, sm.per_partition_error_min, sm.per_partition_error_max,
                                   sm.expected_cross_partition_error, sm.std_cross_partition_error, sm.std_noise)
    return keys, prob, arr


def save_analysis(name, pid, pk, value, cfg, multi=None, public=None, sampling=1.0, pre=None):
    if pre is not None:  # pre-aggregated rows (pk, (count, sum, n_partitions))
        rows = [(int(a), (int(b), float(c), int(d))) for a, b, c, d in zip(*pre)]
        ex = analysis_pre_extractors()
        keys, prob, arr = run_analysis(rows, ex, cfg, multi, public, pre_aggregated=True, sampling=sampling)
    else:
        rows = [(int(a), int(b), float(v)) for a, b, v in zip(pid, pk, value)]
        ex = pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                                        value_extractor=lambda r: r[2])
        keys, prob, arr = run_analysis(rows, ex, cfg, multi, public, sampling=sampling)
    z = np.zeros(0)
    np.savez_compressed(
        os.path.join(OUT, "analysis_" + name + ".npz"),
        pid=np.asarray(pid if pid is not None else z, np.int64), pk=np.asarray(pk if pk is not None else z, np.int64),
        value=np.asarray(value if value is not None else z, np.float64),
        pre=np.asarray(pre if pre is not None else np.zeros((4, 0)), np.float64),
        public=np.asarray(public if public is not None else [], np.int64), has_public=np.asarray(public is not None),
        out_keys=keys, prob=prob, **{"m_" + m: a for m, a in arr.items()},
        meta=np.asarray(json.dumps(dict(cfg=cfg, multi=multi, sampling=sampling, metrics=list(arr)))))
    print(f"analysis_{name}: {len(keys)} partitions, metrics={list(arr)}")


def analysis_pre_extractors():
    import analysis
    return analysis.PreAggregateExtractors(partition_extractor=lambda r: r[0], preaggregate_extractor=lambda r: r[1])


def analysis_cases():
    """Utility-analysis goldens (configs[4]); see pdp_analysis_oracle.py."""
    # A. analysis/tests/utility_analysis_engine_test.py:157-220 (known answers)
    rows = [(i, j) for i in range(10) for j in range(10)] * 3
    save_analysis("reference_per_partition_errors", [r[0] for r in rows], [r[1] for r in rows],
                  [0.0] * len(rows),
                  dict(metrics=["count"], L0=1, Linf=2, eps=2.0, delta=1e-10, noise_kind="gaussian"))
    # B. :222-302 (multi parameters, public partitions)
    save_analysis("reference_multi_parameters", [0, 0, 0], [0, 1, 1], [0.0] * 3,
                  dict(metrics=["count"], L0=1, Linf=1, eps=1.0, delta=1e-10, noise_kind="gaussian"),
                  multi=dict(max_partitions_contributed=[1, 2], max_contributions_per_partition=[1, 2]),
                  public=[0, 1])
    rng = np.random.default_rng(20250206)
    # C. private selection, 6 configs incl. the thresholding strategies, partitions with > 100 privacy ids
    n, U, P = 12000, 800, 60
    pid = rng.integers(0, U, n)
    pk = np.minimum(rng.zipf(1.5, n) - 1, P - 1)
    val = rng.normal(2.0, 3.0, n)
    save_analysis("private_multi", pid, pk, val,
                  dict(metrics=["count", "sum", "privacy_id_count"], L0=2, Linf=2, eps=3.0, delta=1e-5,
                       noise_kind="gaussian", min_sum_per_partition=-3.0, max_sum_per_partition=5.0),
                  multi=dict(max_partitions_contributed=[1, 2, 3, 5, 2, 4],
                             max_contributions_per_partition=[1, 2, 3, 1, 2, 4],
                             min_sum_per_partition=[-3.0, 0.0, -1.0, 1.0, -2.0, 0.5],
                             max_sum_per_partition=[5.0, 2.0, 4.0, 3.0, 8.0, 0.75],
                             partition_selection_strategy=["truncated_geometric", "truncated_geometric",
                                                           "laplace_thresholding", "gaussian_thresholding",
                                                           "truncated_geometric", "laplace_thresholding"]))
    # D. public partitions (absent ones too) with SUM bounds excluding 0 (the empty accumulator matters)
    save_analysis("public_sum", pid, pk, val,
                  dict(metrics=["sum", "count"], L0=3, Linf=2, eps=1.0, delta=1e-6, noise_kind="laplace",
                       min_sum_per_partition=0.5, max_sum_per_partition=6.0),
                  public=list(range(0, P, 2)) + [P + 3, P + 9])
    # E. pre-aggregated input (NoOpContributionBounder)
    gp, gc, gs, gn = [], [], [], []
    for i in range(300):
        npart = int(rng.integers(1, 6))
        for k in rng.choice(40, npart, replace=False):
            gp.append(int(k))
            gc.append(int(rng.integers(1, 5)))
            gs.append(float(rng.normal(1.0, 2.0)))
            gn.append(npart)
    save_analysis("pre_aggregated", None, None, None,
                  dict(metrics=["count", "privacy_id_count", "sum"], L0=2, Linf=2, eps=1.0, delta=1e-6,
                       noise_kind="laplace", min_sum_per_partition=-1.0, max_sum_per_partition=2.0),
                  pre=np.array([gp, gc, gs, gn], dtype=np.float64))
    # F. partition sampling (ValueSampler, sampling_utils.py:38-51)
    save_analysis("partition_sampling", pid, pk, val,
                  dict(metrics=["count"], L0=2, Linf=3, eps=1.0, delta=1e-6, noise_kind="laplace"),
                  sampling=0.5)
    # G. partition sampling with public partitions: unsampled public partitions lose their rows and
    # get the empty accumulator (contribution_bounders.py:57-66 + dp_engine.py:_add_empty_public_partitions)
    save_analysis("public_sampling", pid, pk, val,
                  dict(metrics=["sum", "count", "privacy_id_count"], L0=2, Linf=2, eps=1.0, delta=1e-6,
                       noise_kind="laplace", min_sum_per_partition=-1.0, max_sum_per_partition=4.0),
                  public=list(range(0, P, 3)) + [P + 1, P + 4], sampling=0.6)


def _aggregate_metrics_to_dict(am):
    """AggregateMetrics -> {"selection": {...} | None, metric: {field: value}} (floats only)."""
    out = {"selection": None}
    if am.partition_selection_metrics is not None:
        out["selection"] = {k: float(v) for k, v in vars(am.partition_selection_metrics).items()}
    for m in ("count", "privacy_id_count", "sum"):
        em = getattr(am, m + "_metrics", None)
        if em is None:
            continue
        out[m] = {k: ([float(x) for x in v] if isinstance(v, (list, tuple, np.ndarray)) else float(v))
                  for k, v in vars(em).items() if k != "metric_type"}
    return out


def run_perform_utility_analysis(rows, extractors, cfg, multi=None, public=None, pre_aggregated=False, sampling=1.0):
    """Reference analysis.perform_utility_analysis (analysis/utility_analysis.py:27-161)
    -> list (one per configuration) of _aggregate_metrics_to_dict."""
    import analysis
    kw = dict(metrics=[METRIC[m] for m in cfg["metrics"]],
              noise_kind=pipeline_dp.NoiseKind(cfg.get("noise_kind", "laplace")),
              max_partitions_contributed=cfg["L0"], max_contributions_per_partition=cfg["Linf"])
    for k in ("min_sum_per_partition", "max_sum_per_partition"):
        if cfg.get(k) is not None:
            kw[k] = cfg[k]
    params = pipeline_dp.AggregateParams(**kw)
    mp = None
    if multi:
        mk = dict(multi)
        if "partition_selection_strategy" in mk:
            mk["partition_selection_strategy"] = [pipeline_dp.PartitionSelectionStrategy[v.upper()]
                                                  for v in mk["partition_selection_strategy"]]
        if "noise_kind" in mk:
            mk["noise_kind"] = [pipeline_dp.NoiseKind(v) for v in mk["noise_kind"]]
        mp = analysis.MultiParameterConfiguration(**mk)
    options = analysis.UtilityAnalysisOptions(epsilon=cfg["eps"], delta=cfg["delta"], aggregate_params=params,
                                              multi_param_configuration=mp, partitions_sampling_prob=sampling,
                                              pre_aggregated_data=pre_aggregated)
    out = list(analysis.perform_utility_analysis(rows, pipeline_dp.LocalBackend(), options, extractors,
                                                 public_partitions=public))
    assert len(out) == 1
    return [_aggregate_metrics_to_dict(am) for am in out[0]]


def save_aggregate(name, pid, pk, value, cfg, multi=None, public=None, sampling=1.0, runs=1):
    """Golden of perform_utility_analysis.  With runs > 1 (Laplace noise: the
    reference's error quantiles are 10^3-sample Monte-Carlo estimates,
    analysis/probability_computations.py:20-36) the mean and the standard
    deviation over `runs` numpy seeds are stored."""
    rows = [(int(a), int(b), float(v)) for a, b, v in zip(pid, pk, value)]
    ex = pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                                    value_extractor=lambda r: r[2])
    res = []
    for r in range(runs):
        np.random.seed(1000 + r)
        res.append(run_perform_utility_analysis(rows, ex, cfg, multi, public, sampling=sampling))

    def stat(fn):
        def walk(items):
            first = items[0]
            if first is None:
                return None
            if isinstance(first, dict):
                return {k: walk([i[k] for i in items]) for k in first}
            if isinstance(first, list):
                return [walk([i[j] for i in items]) for j in range(len(first))]
            return fn(np.asarray(items, np.float64))
        return walk(res)

    expected = stat(lambda a: float(a.mean()))
    spread = stat(lambda a: float(a.std(ddof=1)) if len(a) > 1 else 0.0)
    np.savez_compressed(
        os.path.join(OUT, "aggregate_" + name + ".npz"),
        pid=np.asarray(pid, np.int64), pk=np.asarray(pk, np.int64), value=np.asarray(value, np.float64),
        public=np.asarray(public if public is not None else [], np.int64), has_public=np.asarray(public is not None),
        meta=np.asarray(json.dumps(dict(cfg=cfg, multi=multi, sampling=sampling, runs=runs, expected=expected,
                                        spread=spread))))
    print(f"aggregate_{name}: {len(expected)} configurations, runs={runs}")


def aggregate_cases():
    """perform_utility_analysis goldens (cross-partition aggregate error metrics)."""
    rng = np.random.default_rng(20251017)
    n, U, P = 6000, 500, 50
    pid = rng.integers(0, U, n)
    pk = np.minimum(rng.zipf(1.5, n) - 1, P - 1)
    val = rng.normal(2.0, 3.0, n)
    # private selection, Gaussian noise (deterministic: norm.ppf quantiles), 4 configurations
    save_aggregate("private_gaussian", pid, pk, val,
                   dict(metrics=["count", "sum", "privacy_id_count"], L0=2, Linf=2, eps=3.0, delta=1e-5,
                        noise_kind="gaussian", min_sum_per_partition=-3.0, max_sum_per_partition=5.0),
                   multi=dict(max_partitions_contributed=[1, 2, 3, 5], max_contributions_per_partition=[1, 2, 3, 1],
                              min_sum_per_partition=[-3.0, 0.0, -1.0, 1.0],
                              max_sum_per_partition=[5.0, 2.0, 4.0, 3.0]))
    # public partitions (absent ones too), Gaussian
    save_aggregate("public_gaussian", pid, pk, val,
                   dict(metrics=["sum", "count"], L0=3, Linf=2, eps=1.0, delta=1e-6, noise_kind="gaussian",
                        min_sum_per_partition=0.5, max_sum_per_partition=6.0),
                   public=list(range(0, P, 2)) + [P + 3, P + 9])
    # Laplace noise: Monte-Carlo quantiles in the reference -> mean / std over 16 seeds
    save_aggregate("private_laplace", pid, pk, val,
                   dict(metrics=["count", "privacy_id_count"], L0=2, Linf=2, eps=2.0, delta=1e-5,
                        noise_kind="laplace"),
                   multi=dict(max_partitions_contributed=[1, 3], max_contributions_per_partition=[2, 1]), runs=16)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "select":
        select_partitions_cases()
    elif len(sys.argv) > 1 and sys.argv[1] == "analysis":
        analysis_cases()
    elif len(sys.argv) > 1 and sys.argv[1] == "aggregate":
        aggregate_cases()
    else:
        main()
        select_partitions_cases()
        analysis_cases()
        aggregate_cases()
