"""CPU oracle for the utility-analysis path -- TEST INFRASTRUCTURE ONLY.

A numpy restatement of the reference's per-partition utility analysis
(configs[4] of BASELINE.json), imported only by ``tests/`` and the
``cpu_baseline`` leg of ``bench.py``, never by the product:

  * ``preaggregate``   <- SamplingL0LinfContributionBounder.bound_contributions
                          (analysis/contribution_bounders.py:38-75) and
                          analysis/pre_aggregation.py:preaggregate: per
                          (privacy id, partition) the row count, the value sum
                          and the number of distinct partitions of the privacy
                          id (counted before partition sampling).
  * ``per_partition``  <- UtilityAnalysisEngine._create_compound_combiner
                          (analysis/utility_analysis_engine.py:97-142) with
                          SumCombiner / CountCombiner / PrivacyIdCountCombiner
                          (analysis/combiners.py:228-310) and
                          PartitionSelectionCombiner (:99-225) over the exact
                          Poisson-binomial pmf (analysis/poisson_binomial.py:39-50)
                          for <= 100 privacy ids, the refined normal
                          approximation (:62-83) otherwise.

Pinned by golden vectors generated from the reference's
UtilityAnalysisEngine (oracle/gen_golden.py ``analysis`` cases) and by the
reference's own known answers (analysis/tests/utility_analysis_engine_test.py:
157-220, 222-302).  The keep probability of a selection strategy
(PyDP ``probability_of_keep``) is the restatement of pdp_oracle.py; parity
unpinned for max_partitions_contributed > 1 and the thresholding strategies.
"""
import dataclasses
import math
from typing import Optional

import numpy as np

import pdp_oracle as o

MAX_PROBABILITIES_IN_ACCUMULATOR = 100  # analysis/combiners.py:32
METRICS = ("sum", "count", "privacy_id_count")  # combiner order, utility_analysis_engine.py:124-139
FIELDS = ("sum", "per_partition_error_min", "per_partition_error_max", "expected_cross_partition_error",
          "var_cross_partition_error")


@dataclasses.dataclass
class AnalysisConfig:
    """One bounding configuration (MultiParameterConfiguration entry,
    analysis/data_structures.py:46-118) with its selection budget."""
    max_partitions_contributed: int
    max_contributions_per_partition: int
    min_sum_per_partition: Optional[float] = None
    max_sum_per_partition: Optional[float] = None
    selection: Optional[str] = None  # None (public) | truncated_geometric | laplace | gaussian
    selection_eps: float = 0.0
    selection_delta: float = 0.0


def preaggregate(pid, pk, value=None, num_sampled=None):
    """-> (pair_pk, count, sum, n_partitions) in (pid, pk) order.  Rows with
    pk < 0 are dropped first (non-public partitions, dropped before bounding
    in DPEngine._aggregate).  Partitions with id >= num_sampled count toward
    n_partitions but emit no pair (partition sampling: the reference counts
    len(partition_values) before sampler.keep, contribution_bounders.py:63-66)."""
    pid = np.asarray(pid, np.int64)
    pk = np.asarray(pk, np.int64)
    keep = pk >= 0
    pid, pk = pid[keep], pk[keep]
    value = np.zeros(len(pk)) if value is None else np.asarray(value, np.float64)[keep]
    order = np.lexsort((pk, pid))
    spid, spk, sval = pid[order], pk[order], value[order]
    n = len(spid)
    if n == 0:
        z = np.zeros(0, np.int64)
        return z, z, np.zeros(0), z
    start = np.ones(n, bool)
    start[1:] = (spid[1:] != spid[:-1]) | (spk[1:] != spk[:-1])
    gid = np.cumsum(start) - 1
    first = np.flatnonzero(start)
    g_pid, g_pk = spid[first], spk[first]
    cnt = np.bincount(gid).astype(np.int64)
    sm = np.bincount(gid, weights=sval)
    pstart = np.ones(len(g_pid), bool)
    pstart[1:] = g_pid[1:] != g_pid[:-1]
    pidx = np.cumsum(pstart) - 1
    npart = np.bincount(pidx)[pidx].astype(np.int64)
    emit = np.ones(len(g_pk), bool) if num_sampled is None else g_pk < num_sampled
    return g_pk[emit], cnt[emit], sm[emit], npart[emit]


def keep_probability(strategy, eps, delta, k, n):
    """PyDP probability_of_keep(n) restated (pdp_oracle.py; oracle/pydp_stub)."""
    n = np.asarray(n, np.int64)
    if strategy == "truncated_geometric":
        return o.truncated_geometric_keep_prob(n, eps, delta, k) * (n > 0)
    if strategy == "laplace":
        thr, b = o.laplace_threshold(eps, delta, k)
        x = thr - n
        p = np.where(x >= 0, 0.5 * np.exp(-np.abs(x) / b), 1.0 - 0.5 * np.exp(-np.abs(x) / b))
        return p * (n > 0)
    if strategy == "gaussian":
        from scipy.special import erfc
        thr, sigma = o.gaussian_threshold(eps, delta, k)
        return 0.5 * erfc((thr - n) / (sigma * math.sqrt(2.0))) * (n > 0)
    raise ValueError(strategy)


def exact_pmf(probs):
    """poisson_binomial.compute_pmf (analysis/poisson_binomial.py:39-50)."""
    pmf = np.array([1.0])
    for p in probs:
        nxt = np.zeros(len(pmf) + 1)
        nxt[:-1] = pmf * (1 - p)
        nxt[1:] += pmf * p
        pmf = nxt
    return 0, pmf


def approx_pmf(mean, sigma, skewness, n):
    """poisson_binomial.compute_pmf_approximation (:62-83), refined normal."""
    from scipy.stats import norm
    if sigma == 0:
        return int(round(mean)), np.array([1.0])
    start = max(0, int(np.floor(mean - 8 * sigma)))
    end = min(n, int(np.round(mean + 8 * sigma)))
    xs = np.arange(start - 1, end + 1)
    x = (xs + 0.5 - mean) / sigma
    cdf = np.clip(norm.cdf(x) + skewness * (1 - x * x) * norm.pdf(x) / 6, 0, 1)
    return start, np.diff(cdf)


def probability_to_keep(q, cfg: AnalysisConfig):
    """PartitionSelectionCalculator.compute_probability_to_keep (:124-152)."""
    if len(q) <= MAX_PROBABILITIES_IN_ACCUMULATOR:
        start, pmf = exact_pmf(q)
    else:
        mean = float(np.sum(q))
        var = float(np.sum(q * (1 - q)))
        third = float(np.sum(q * (1 - q) * (1 - 2 * q)))
        std = math.sqrt(var)
        skew = 0 if std == 0 else third / std**3
        start, pmf = approx_pmf(mean, std, skew, len(q))
    ks = np.arange(start, start + len(pmf))
    return float(np.sum(pmf * keep_probability(cfg.selection, cfg.selection_eps, cfg.selection_delta,
                                               cfg.max_partitions_contributed, ks)))


def _sum_terms(x, lo, hi, q):
    """SumCombiner.create_accumulator terms per (pid, pk) (combiners.py:237-263)."""
    cc = np.clip(x, lo, hi)
    err = cc - x
    return (x, np.where(x < lo, err, 0.0), np.where(x > hi, err, 0.0), -cc * (1 - q), cc**2 * q * (1 - q))


def per_partition(pair_pk, count, sums, npart, P, configs, metrics, public=False):
    """-> {"sum"|"count"|"privacy_id_count": array [C, 5, P] of FIELDS,
           "prob_keep": array [C, P] (private selection only)}.

    public=True adds, per partition, the empty accumulator of
    _add_empty_public_partitions: one pseudo-contribution (0, 0, 0)
    (analysis/combiners.py:337-342)."""
    pair_pk = np.asarray(pair_pk, np.int64)
    count = np.asarray(count, np.float64)
    sums = np.asarray(sums, np.float64)
    npart = np.asarray(npart, np.float64)
    if public:
        allp = np.arange(P)
        pair_pk = np.concatenate([pair_pk, allp])
        count = np.concatenate([count, np.zeros(P)])
        sums = np.concatenate([sums, np.zeros(P)])
        npart = np.concatenate([npart, np.zeros(P)])
    C = len(configs)
    out = {m: np.zeros((C, 5, P)) for m in metrics}
    if not public:
        out["prob_keep"] = np.zeros((C, P))
        order = np.argsort(pair_pk, kind="stable")
        spk = pair_pk[order]
        bounds = np.searchsorted(spk, np.arange(P + 1))
    for c, cfg in enumerate(configs):
        L0 = cfg.max_partitions_contributed
        q = np.where(npart > 0, np.minimum(1.0, L0 / np.maximum(npart, 1)), 0.0)
        for m in metrics:
            if m == "sum":
                x, lo, hi = sums, cfg.min_sum_per_partition, cfg.max_sum_per_partition
            elif m == "count":
                x, lo, hi = count, 0.0, float(cfg.max_contributions_per_partition)
            else:
                x, lo, hi = np.where(count > 0, 1.0, 0.0), 0.0, 1.0
            for f, t in enumerate(_sum_terms(x, lo, hi, q)):
                out[m][c, f] = np.bincount(pair_pk, weights=t, minlength=P)
        if not public:
            qs = q[order]
            for p in range(P):
                a, b = bounds[p], bounds[p + 1]
                if b > a:
                    out["prob_keep"][c, p] = probability_to_keep(qs[a:b], cfg)
    return out


def noise_std(kind, eps, delta, l0, linf):
    """compute_dp_count_noise_std (dp_computations.py:462-481): the std every
    SumCombiner / CountCombiner / PrivacyIdCountCombiner reports
    (analysis/combiners.py:265-277), linf = max_contributions_per_partition."""
    if kind == "laplace":
        return l0 * linf / eps * math.sqrt(2)
    return o.gaussian_sigma(eps, delta, math.sqrt(l0) * linf)


# ---------------------------------------------------------------------------
# Cross-partition aggregation: perform_utility_analysis
# (analysis/utility_analysis.py:27-161) -- the AggregateErrorMetricsCompoundCombiner
# over every partition's per-partition metrics (analysis/combiners.py:385-723).
# ---------------------------------------------------------------------------

ERROR_QUANTILES = (0.1, 0.5, 0.9, 0.99)  # utility_analysis.py:68
# AggregateErrorMetricsAccumulator fields summed over partitions (combiners.py:385-416), quantile
# lists excluded (they follow as 2 x Q entries: error_quantiles, rel_error_quantiles)
ACC_FIELDS = ("num_partitions", "kept_partitions_expected", "total_aggregate", "data_dropped_l0",
              "data_dropped_linf", "data_dropped_partition_selection", "error_l0_expected", "error_linf_expected",
              "error_linf_min_expected", "error_linf_max_expected", "error_l0_variance", "error_variance",
              "rel_error_l0_expected", "rel_error_linf_expected", "rel_error_linf_min_expected",
              "rel_error_linf_max_expected", "rel_error_l0_variance", "rel_error_variance",
              "error_expected_w_dropped_partitions", "rel_error_expected_w_dropped_partitions")


def _ndtr(z):
    from scipy.special import ndtr
    return ndtr(z)


def laplace_gaussian_cdf(x, b, sigma):
    """CDF of Laplace(0, b) + N(0, sigma^2) at x: E[F_L(x - G)] in closed form,
    the two exponential terms taken as erfcx products so nothing overflows."""
    from scipy.special import erfcx
    x = np.asarray(x, np.float64)
    if sigma == 0:
        return np.where(x < 0, 0.5 * np.exp(np.minimum(x, 0) / b), 1 - 0.5 * np.exp(-np.maximum(x, 0) / b))
    if b == 0:
        return _ndtr(x / sigma)
    r = sigma / b
    u = x / sigma
    g = np.exp(-0.5 * u * u)
    with np.errstate(over="ignore", invalid="ignore"):  # np.where evaluates both branches
        return _lg_cdf(x, b, r, u, g)


def _lg_cdf(x, b, r, u, g):
    from scipy.special import erfcx
    # 1/2 e^{r^2/2 - x/b} Phi(u - r)  and  1/2 e^{r^2/2 + x/b} Phi(-u - r)
    t2 = np.where(u - r < 0, 0.25 * erfcx((r - u) / math.sqrt(2)) * g,
                  0.5 * np.exp(0.5 * r * r - x / b) * _ndtr(u - r))
    t3 = np.where(u + r > 0, 0.25 * erfcx((u + r) / math.sqrt(2)) * g,
                  0.5 * np.exp(0.5 * r * r + x / b) * _ndtr(-u - r))
    return _ndtr(u) - t2 + t3


def laplace_gaussian_quantile(q, b, sigma):
    """The exact q-quantile of Laplace(0, b) + N(0, sigma^2), by bisection on
    laplace_gaussian_cdf.  The reference estimates it from 10^3 Monte-Carlo
    samples (analysis/probability_computations.py:20-36); this is the value
    that estimate converges to."""
    if sigma == 0:
        return b * math.log(2 * q) if q < 0.5 else -b * math.log(2 * (1 - q))
    if b == 0:
        from scipy.special import ndtri
        return sigma * float(ndtri(q))
    lo, hi = -(40 * b + 40 * sigma), 40 * b + 40 * sigma
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        if laplace_gaussian_cdf(mid, b, sigma) < q:
            lo = mid
        else:
            hi = mid
        if hi - lo <= 1e-15 * max(1.0, abs(mid)):
            break
    return 0.5 * (lo + hi)


def error_quantile_values(kind, expected_cross, std_cross, std_noise, quantiles):
    """SumAggregateErrorMetricsCombiner._compute_error_quantiles' distribution
    quantiles (combiners.py:655-674) before the per-partition error is added:
    Gaussian: norm.ppf(q, E, sqrt(std_cross^2 + std_noise^2)); Laplace: the
    Laplace(std_noise / sqrt 2) + N(0, std_cross^2) quantile (exact here, see
    laplace_gaussian_quantile; the reference's Laplace values ignore E)."""
    if kind == "gaussian":
        from scipy.special import ndtri
        s = math.sqrt(std_cross**2 + std_noise**2)
        return [expected_cross + s * float(ndtri(q)) for q in quantiles]
    return [laplace_gaussian_quantile(q, std_noise / math.sqrt(2), std_cross) for q in quantiles]


def aggregate_accumulator(metric, per_part, prob_keep, std_noise, kind, quantiles=ERROR_QUANTILES):
    """Sum over partitions of SumAggregateErrorMetricsCombiner.create_accumulator
    (combiners.py:497-585) for one configuration and metric.  per_part: [5, P]
    (FIELDS), prob_keep: [P] or None (public partitions: 1).  -> dict of
    ACC_FIELDS plus "error_quantiles" / "rel_error_quantiles" lists."""
    inv = [1 - q for q in quantiles]  # _invert_error_quantiles
    P = per_part.shape[1]
    acc = {f: 0.0 for f in ACC_FIELDS}
    acc["error_quantiles"] = [0.0] * len(inv)
    acc["rel_error_quantiles"] = [0.0] * len(inv)
    for p in range(P):
        s, emin, emax, ecross, var_cross = (float(v) for v in per_part[:, p])
        std_cross = math.sqrt(max(var_cross, 0.0))
        pk = 1.0 if prob_keep is None else float(prob_keep[p])
        t = {"num_partitions": 1.0, "kept_partitions_expected": pk, "total_aggregate": s}
        if metric != "sum":
            t["data_dropped_l0"] = -ecross
            t["data_dropped_linf"] = -emax
            t["data_dropped_partition_selection"] = (1 - pk) * (s + ecross + emax)
        t["error_l0_expected"] = pk * ecross
        t["error_linf_min_expected"] = pk * emin
        t["error_linf_max_expected"] = pk * emax
        t["error_linf_expected"] = t["error_linf_min_expected"] + t["error_linf_max_expected"]
        t["error_l0_variance"] = pk * std_cross**2
        t["error_variance"] = pk * (std_cross**2 + std_noise**2)
        eq = [pk * (v + emin + emax) for v in error_quantile_values(kind, ecross, std_cross, std_noise, inv)]
        t["error_expected_w_dropped_partitions"] = pk * (ecross + emin + emax) + (1 - pk) * -s
        if s != 0:
            a = abs(s)
            for f in ("l0_expected", "linf_min_expected", "linf_max_expected"):
                t["rel_error_" + f] = t["error_" + f] / a
            t["rel_error_linf_expected"] = t["rel_error_linf_min_expected"] + t["rel_error_linf_max_expected"]
            t["rel_error_l0_variance"] = t["error_l0_variance"] / s**2
            t["rel_error_variance"] = t["error_variance"] / s**2
            t["rel_error_expected_w_dropped_partitions"] = t["error_expected_w_dropped_partitions"] / a
            req = [e / a for e in eq]
        else:
            req = [0.0] * len(eq)
        for f, v in t.items():
            acc[f] += v
        acc["error_quantiles"] = [x + y for x, y in zip(acc["error_quantiles"], eq)]
        acc["rel_error_quantiles"] = [x + y for x, y in zip(acc["rel_error_quantiles"], req)]
    return acc


def aggregate_error_metrics(acc, std_noise):
    """SumAggregateErrorMetricsCombiner.compute_metrics (combiners.py:590-640)
    -> dict of AggregateErrorMetrics fields (metric_type excluded)."""
    k = acc["kept_partitions_expected"]
    total = max(1.0, acc["total_aggregate"])
    out = {"ratio_data_dropped_l0": acc["data_dropped_l0"] / total,
           "ratio_data_dropped_linf": acc["data_dropped_linf"] / total,
           "ratio_data_dropped_partition_selection": acc["data_dropped_partition_selection"] / total}
    for pre in ("", "rel_"):
        l0 = acc[pre + "error_l0_expected"] / k
        lmin = acc[pre + "error_linf_min_expected"] / k
        lmax = acc[pre + "error_linf_max_expected"] / k
        out[pre + "error_l0_expected"] = l0
        out[pre + "error_linf_expected"] = lmin + lmax
        out[pre + "error_linf_min_expected"] = lmin
        out[pre + "error_linf_max_expected"] = lmax
        out[pre + "error_expected"] = l0 + lmin + lmax
        out[pre + "error_l0_variance"] = acc[pre + "error_l0_variance"] / k
        out[pre + "error_variance"] = acc[pre + "error_variance"] / k
        out[pre + "error_quantiles"] = [v / k for v in acc[pre + "error_quantiles"]]
        out[pre + "error_expected_w_dropped_partitions"] = (acc[pre + "error_expected_w_dropped_partitions"] /
                                                            acc["num_partitions"])
    out["noise_std"] = std_noise
    return out


def partition_selection_metrics(prob_keep):
    """PrivatePartitionSelectionAggregateErrorMetricsCombiner.compute_metrics
    (combiners.py:700-715) over the moments of the keep indicators (:87-96)."""
    p = np.asarray(prob_keep, np.float64)
    return {"num_partitions": len(p), "dropped_partitions_expected": len(p) - float(np.sum(p)),
            "dropped_partitions_variance": float(np.sum(p * (1 - p)))}
