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
