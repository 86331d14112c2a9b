"""Utility analysis on the MI355X (BASELINE.json configs[4]).

Host mirror of the reference's ``analysis`` package for the per-partition
analysis: ``UtilityAnalysisEngine.analyze`` (analysis/utility_analysis_engine.py:
29-210) with ``UtilityAnalysisOptions`` / ``MultiParameterConfiguration`` /
``PreAggregateExtractors`` (analysis/data_structures.py) and ``SumMetrics``
(analysis/metrics.py:23-48), plus ``preaggregate``
(analysis/pre_aggregation.py).  Same validation errors, the same budget
requests in the same order, the same lazy result of
(partition_key, tuple of per-configuration metrics).

The computation -- per (privacy id, partition) pre-aggregation, then for every
configuration at once the Sum / Count / PrivacyIdCount combiner terms and the
Poisson-binomial keep probability of private partition selection -- runs in
libpdp_hip.so (``pdp_utility_analysis``, include/pdp_hip.h).  The noise
standard deviation is host arithmetic (dp_computations.py:462-481).

``perform_utility_analysis`` (analysis/utility_analysis.py:27-161) adds the
cross-partition aggregation on the device (``pdp_utility_aggregate``): the
sums of AggregateErrorMetricsCompoundCombiner's accumulators over every
partition, divided here as compute_metrics does (analysis/combiners.py:
590-640, 700-715).  Laplace error quantiles are exact (closed-form CDF of
Laplace + Gaussian, inverted on the GPU) where the reference uses 10^3
Monte-Carlo samples.  Parameter tuning is out of scope.
"""
import copy
import enum
import dataclasses
import hashlib
import math
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import aggregate_params as agg
from . import native
from .columnar import ColumnarData, _factorize, _index_of, _unique_in_order
from .input_validators import validate_epsilon_delta

_SELECTION = {agg.PartitionSelectionStrategy.TRUNCATED_GEOMETRIC: native.SELECTION_TRUNCATED_GEOMETRIC,
              agg.PartitionSelectionStrategy.LAPLACE_THRESHOLDING: native.SELECTION_LAPLACE,
              agg.PartitionSelectionStrategy.GAUSSIAN_THRESHOLDING: native.SELECTION_GAUSSIAN}


@dataclasses.dataclass
class PreAggregateExtractors:
    """Extractors of pre-aggregated rows: partition key and
    (count, sum, n_partitions) per (privacy id, partition) (data_structures.py:24-43)."""
    partition_extractor: Callable
    preaggregate_extractor: Callable


@dataclasses.dataclass
class MultiParameterConfiguration:
    """Per-configuration parameters (data_structures.py:46-118)."""
    max_partitions_contributed: Sequence[int] = None
    max_contributions_per_partition: Sequence[int] = None
    min_sum_per_partition: Sequence[float] = None
    max_sum_per_partition: Sequence[float] = None
    noise_kind: Sequence[agg.NoiseKind] = None
    partition_selection_strategy: Sequence[agg.PartitionSelectionStrategy] = None

    def __post_init__(self):
        attributes = dataclasses.asdict(self)
        sizes = [len(value) for value in attributes.values() if value]
        if not sizes:
            raise ValueError("MultiParameterConfiguration must have at least 1"
                             " non-empty attribute.")
        if min(sizes) != max(sizes):
            raise ValueError("All set attributes in MultiParameterConfiguration must have "
                             "the same length.")
        if (self.min_sum_per_partition is None) != (self.max_sum_per_partition is None):
            raise ValueError("MultiParameterConfiguration: min_sum_per_partition and "
                             "max_sum_per_partition must be both set or both None.")
        self._size = sizes[0]

    @property
    def size(self):
        return self._size

    def get_aggregate_params(self, params: agg.AggregateParams, index: int) -> agg.AggregateParams:
        """AggregateParams with the index-th parameters."""
        params = copy.copy(params)
        for f in dataclasses.fields(self):
            seq = getattr(self, f.name)
            if seq:
                setattr(params, f.name, seq[index])
        return params


@dataclasses.dataclass
class UtilityAnalysisOptions:
    """Options of the utility analysis (data_structures.py:121-143)."""
    epsilon: float
    delta: float
    aggregate_params: agg.AggregateParams
    multi_param_configuration: Optional[MultiParameterConfiguration] = None
    partitions_sampling_prob: float = 1
    pre_aggregated_data: bool = False

    def __post_init__(self):
        validate_epsilon_delta(self.epsilon, self.delta, "UtilityAnalysisOptions")
        if self.partitions_sampling_prob <= 0 or self.partitions_sampling_prob > 1:
            raise ValueError(f"partitions_sampling_prob must be in the interval"
                             f" (0, 1], but {self.partitions_sampling_prob} given.")

    @property
    def n_configurations(self):
        if self.multi_param_configuration is None:
            return 1
        return self.multi_param_configuration.size


def get_aggregate_params(options: UtilityAnalysisOptions) -> List[agg.AggregateParams]:
    """The AggregateParams of every configuration (data_structures.py:146-156)."""
    m = options.multi_param_configuration
    if m is None:
        return [options.aggregate_params]
    return [m.get_aggregate_params(options.aggregate_params, i) for i in range(m.size)]


@dataclasses.dataclass
class SumMetrics:
    """Per-partition SUM / COUNT / PRIVACY_ID_COUNT utility metrics
    (analysis/metrics.py:23-48)."""
    sum: float
    per_partition_error_min: float
    per_partition_error_max: float
    expected_cross_partition_error: float
    std_cross_partition_error: float
    std_noise: float
    noise_kind: agg.NoiseKind


class ValueSampler:
    """Deterministic partition sampler: keep(v) iff the first 64 bits of
    SHA-1(repr(v)) < round(2^64 * rate) (pipeline_dp/sampling_utils.py:32-51)."""

    def __init__(self, sampling_rate: float):
        self._sample_bound = int(round(2**64 * sampling_rate))

    def keep(self, value) -> bool:
        m = hashlib.sha1()
        m.update(repr(value).encode())
        return int(m.hexdigest()[:16], 16) < self._sample_bound


def noise_std(params: agg.AggregateParams, eps: float, delta: float) -> float:
    """compute_dp_count_noise_std (dp_computations.py:462-481): the std every
    utility-analysis Sum/Count/PrivacyIdCount combiner reports
    (analysis/combiners.py:265-277), linf = max_contributions_per_partition."""
    l0 = params.max_partitions_contributed
    linf = params.max_contributions_per_partition
    if params.noise_kind == agg.NoiseKind.LAPLACE:
        return l0 * linf / eps * math.sqrt(2)
    return native.gaussian_sigma(eps, delta, math.sqrt(l0) * linf)


_ANALYSIS_METRICS = (agg.Metrics.SUM, agg.Metrics.COUNT, agg.Metrics.PRIVACY_ID_COUNT)  # combiner order


class AnalysisResult:
    """Lazy collection of (partition_key, tuple of per-configuration
    metrics): per configuration [keep probability if private] + SumMetrics
    for SUM, COUNT, PRIVACY_ID_COUNT (those requested), in the order of
    UtilityAnalysisEngine._create_compound_combiner
    (utility_analysis_engine.py:114-139)."""

    def __init__(self, engine, col, options, extractors, public_partitions, selection_spec, metric_specs):
        self._engine = engine
        self._col = col
        self._options = options
        self._extractors = extractors
        self._public = public_partitions
        self._selection_spec = selection_spec
        self._metric_specs = metric_specs
        self._out = None

    def __iter__(self):
        if self._out is None:
            self._out = self._compute()
        return iter(self._out)

    def to_arrays(self):
        """(partition keys, metrics [C, nb, 5, P] device tensor, prob_keep [C, P]
        or None, privacy ids with data [P]): the raw GPU result behind the
        per-partition tuples."""
        return self._encode_and_run()[:4]

    def _configs(self):
        cfgs = []
        sel = self._selection_spec
        for p in get_aggregate_params(self._options):
            c = native.AnalysisConfig()
            c.max_partitions_contributed = p.max_partitions_contributed
            c.max_contributions_per_partition = p.max_contributions_per_partition
            c.min_sum_per_partition = float(p.min_sum_per_partition) if p.min_sum_per_partition is not None else 0.0
            c.max_sum_per_partition = float(p.max_sum_per_partition) if p.max_sum_per_partition is not None else 0.0
            if sel is not None:
                c.selection = _SELECTION[p.partition_selection_strategy]
                c.selection_eps, c.selection_delta = sel.eps, sel.delta
            cfgs.append(c)
        return cfgs

    def _encode_and_run(self):
        """The device run behind the result, once (per-partition tuples and the
        cross-partition aggregation share it)."""
        if getattr(self, "_raw", None) is None:
            self._raw = self._encode_and_run_once()
        return self._raw

    def _encode_and_run_once(self):
        backend = self._engine._backend
        ex = backend.executor
        torch = ex.torch
        opts = self._options
        col = self._col
        rows = col if isinstance(col, (list, ColumnarData)) else list(col)
        sampler = ValueSampler(opts.partitions_sampling_prob) if opts.partitions_sampling_prob < 1 else None
        ext = self._extractors
        pre = opts.pre_aggregated_data
        mask = sum(bit for m, bit in ((agg.Metrics.SUM, native.METRIC_SUM), (agg.Metrics.COUNT, native.METRIC_COUNT),
                                      (agg.Metrics.PRIVACY_ID_COUNT, native.METRIC_PRIVACY_ID_COUNT))
                   if m in opts.aggregate_params.metrics)
        need_sum = bool(mask & native.METRIC_SUM)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(ex.device)  # noqa: E731
        if isinstance(rows, ColumnarData):
            if pre:
                raise ValueError("pre_aggregated_data needs rows with PreAggregateExtractors")
            pk = np.asarray(torch.as_tensor(rows.partition).cpu().numpy(), np.int64)
            P0 = rows.num_partitions if rows.num_partitions is not None else (int(pk.max()) + 1 if len(pk) else 0)
            raw_keys = list(rows.partition_keys) if rows.partition_keys is not None else list(range(P0))
            pk_raw = None
            pid = np.asarray(torch.as_tensor(rows.privacy_id).cpu().numpy(), np.int64)
            U = rows.num_privacy_ids if rows.num_privacy_ids is not None else (int(pid.max()) + 1 if len(pid) else 1)
            value = np.asarray(torch.as_tensor(rows.value).cpu().numpy(), np.float64) if need_sum else None
        else:
            pk_raw = [ext.partition_extractor(r) for r in rows]
            raw_keys = None
        # partition dictionary: public partitions in the given order, else
        # first appearance; sampled partitions get the low ids
        if self._public is not None:
            keys = _unique_in_order(self._public)
        elif pk_raw is not None:
            keys = _unique_in_order(pk_raw)
        else:
            keys = raw_keys
        if sampler is not None:
            # public partitions too (analysis/contribution_bounders.py:57-66 drops the rows of unsampled
            # partitions whether or not they are public; _add_empty_public_partitions then gives the
            # unsampled public ones the empty accumulator, while n_partitions still counts them)
            s = [k for k in keys if sampler.keep(k)]
            ns = [k for k in keys if not sampler.keep(k)]
            keys, num_sampled = s + ns, len(s)
        else:
            num_sampled = len(keys)
        if pk_raw is not None:
            pk = _index_of(keys, pk_raw)
        elif keys is not raw_keys:
            lut = _index_of(keys, raw_keys)
            pk = np.where(pk >= 0, lut[np.clip(pk, 0, max(len(raw_keys) - 1, 0))], -1)
        P = len(keys)
        if P == 0:
            return keys, None, None, None, num_sampled
        cfgs = self._configs()
        if pre:
            agg_rows = [ext.preaggregate_extractor(r) for r in rows]
            cnt = np.asarray([a[0] for a in agg_rows], np.int64)
            sm = np.asarray([a[1] for a in agg_rows], np.float64)
            npart = np.asarray([a[2] for a in agg_rows], np.int64)
            metrics, prob, pids = ex.analyze(None, t(pk), t(sm), 0, P, mask, cfgs, pre_count=t(cnt),
                                             pre_n_partitions=t(npart))
        else:
            if pk_raw is not None:
                pid_raw = [ext.privacy_id_extractor(r) for r in rows]
                pid, uniq = _factorize(pid_raw) if rows else (np.zeros(0, np.int64), [])
                U = max(len(uniq), 1)
                value = np.asarray([ext.value_extractor(r) for r in rows], np.float64) if need_sum else None
            metrics, prob, pids = ex.analyze(t(pid), t(pk), None if value is None else t(value), U, P, mask, cfgs,
                                             num_sampled_partitions=num_sampled)
        return keys, metrics, prob, pids, num_sampled

    def _compute(self):
        keys, metrics, prob, pids, num_sampled = self._encode_and_run()
        if metrics is None:
            return []
        opts = self._options
        params_list = get_aggregate_params(opts)
        present = [m for m in _ANALYSIS_METRICS if m in opts.aggregate_params.metrics]
        met = metrics.cpu().numpy()
        pr = prob.cpu().numpy() if prob is not None else None
        C = len(params_list)
        stds = [[noise_std(p, self._metric_specs[m].eps, self._metric_specs[m].delta) for m in present]
                for p in params_list]
        public = self._public is not None
        if public:
            parts = range(len(keys))
        else:  # partitions present in the (sampled) data
            parts = np.flatnonzero(pids.cpu().numpy() > 0).tolist()
        out = []
        for p in parts:
            vals = []
            for c in range(C):
                if not public:
                    vals.append(float(pr[c, p]))
                for b, m in enumerate(present):
                    f = met[c, b, :, p]
                    vals.append(SumMetrics(float(f[0]), float(f[1]), float(f[2]), float(f[3]),
                                           math.sqrt(max(float(f[4]), 0.0)), stds[c][b],
                                           params_list[c].noise_kind))
            out.append((keys[p], tuple(vals)))
        return out


class UtilityAnalysisEngine:
    """Utility analysis of DP aggregations per partition
    (analysis/utility_analysis_engine.py:29-173), computed by the HIP
    library for all configurations at once."""

    def __init__(self, budget_accountant, backend):
        self._budget_accountant = budget_accountant
        self._backend = backend

    def aggregate(self, col, params, data_extractors, public_partitions=None):
        raise ValueError("UtilityAnalysisEngine.aggregate can't be called.\n"
                         "If you like to perform utility analysis use "
                         "UtilityAnalysisEngine.aggregate.\n"
                         "If you like to perform DP computations use "
                         "DPEngine.aggregate.")

    def analyze(self, col, options: UtilityAnalysisOptions, data_extractors, public_partitions=None):
        """-> lazy collection of (partition_key, per-partition metrics tuple)."""
        from .dp_engine import DPEngine
        _check_utility_analysis_params(options, data_extractors)
        params = options.aggregate_params
        DPEngine(self._budget_accountant, self._backend)._check_aggregate_params(col, params, None,
                                                                                  check_data_extractors=False)
        if not getattr(self._backend, "supports_columnar_aggregate", False):
            raise NotImplementedError("UtilityAnalysisEngine runs on HipBackend (the MI355X analysis path).")
        if agg.Metrics.SUM in params.metrics:
            for p in get_aggregate_params(options):
                if p.min_sum_per_partition is None:
                    raise ValueError("utility analysis of SUM needs min_sum_per_partition and max_sum_per_partition")
        with self._budget_accountant.scope(weight=params.budget_weight):
            # budget requests of _create_compound_combiner (:100-111): selection first, then one per metric
            selection = None
            if public_partitions is None:
                selection = self._budget_accountant.request_budget(agg.MechanismType.GENERIC,
                                                                   weight=params.budget_weight)
            mech = params.noise_kind.convert_to_mechanism_type()
            specs = {m: self._budget_accountant.request_budget(mech, weight=params.budget_weight)
                     for m in params.metrics}
            result = AnalysisResult(self, col, options, data_extractors, public_partitions, selection, specs)
            self._budget_accountant._compute_budget_for_aggregation(params.budget_weight)
            return result


def _check_utility_analysis_params(options, data_extractors):
    """utility_analysis_engine.py:176-209 (same errors)."""
    from .dp_engine import DataExtractors
    if options.pre_aggregated_data:
        if not isinstance(data_extractors, PreAggregateExtractors):
            raise ValueError("options.pre_aggregated_data is set to true but "
                             "PreAggregateExtractors aren't provided. PreAggregateExtractors"
                             " should be specified for pre-aggregated data.")
    elif not isinstance(data_extractors, DataExtractors) and data_extractors is not None:
        raise ValueError("pipeline_dp.DataExtractors should be specified for raw data.")
    params = options.aggregate_params
    if params.custom_combiners is not None:
        raise NotImplementedError("custom combiners are not supported")
    allowed = {agg.Metrics.COUNT, agg.Metrics.SUM, agg.Metrics.PRIVACY_ID_COUNT}
    if not set(params.metrics).issubset(allowed):
        not_supported_metrics = list(set(params.metrics).difference(allowed))
        raise NotImplementedError(f"unsupported metric in metrics={not_supported_metrics}")
    if params.contribution_bounds_already_enforced:
        raise NotImplementedError("utility analysis when contribution bounds are already enforced is "
                                  "not supported")


def preaggregate(col, data_extractors, partitions_sampling_prob: float = 1, device=None):
    """analysis/pre_aggregation.py:preaggregate on the GPU: a list of
    (partition_key, (count, sum, n_partitions)), one per (privacy id,
    partition) present in the data (partitions sampled with
    partitions_sampling_prob; n_partitions counts all of the privacy id's
    partitions)."""
    from .executor import HipExecutor
    rows = list(col)
    pk_raw = [data_extractors.partition_extractor(r) for r in rows]
    keys = _unique_in_order(pk_raw)
    if partitions_sampling_prob < 1:
        sampler = ValueSampler(partitions_sampling_prob)
        s = [k for k in keys if sampler.keep(k)]
        keys, num_sampled = s + [k for k in keys if not sampler.keep(k)], len(s)
    else:
        num_sampled = len(keys)
    pk = _index_of(keys, pk_raw)
    pid, uniq = _factorize([data_extractors.privacy_id_extractor(r) for r in rows])
    value = np.asarray([data_extractors.value_extractor(r) for r in rows], np.float64)
    ex = HipExecutor(device)
    pairs = ex.preaggregate(*(ex.torch.from_numpy(a).to(ex.device) for a in (pid, pk, value)), len(uniq), len(keys),
                            num_sampled)
    ppk, cnt, sm, npart = (a.cpu().numpy() for a in pairs)
    return [(keys[k], (int(c), float(s), int(n))) for k, c, s, n in zip(ppk, cnt, sm, npart)]


# ---------------------------------------------------------------------------
# Cross-partition aggregation (perform_utility_analysis)
# ---------------------------------------------------------------------------


class AggregateMetricType(enum.Enum):
    """analysis/metrics.py:51-54."""
    PRIVACY_ID_COUNT = 'privacy_id_count'
    COUNT = 'count'
    SUM = 'sum'


@dataclasses.dataclass
class AggregateErrorMetrics:
    """Cross-partition error metrics of one aggregation (analysis/metrics.py:57-120):
    averages over partitions weighted by the keep probability, except the
    ratio_* fields (ratios of the totals) and the *_w_dropped_partitions ones
    (averages over all partitions)."""
    metric_type: AggregateMetricType
    ratio_data_dropped_l0: float
    ratio_data_dropped_linf: float
    ratio_data_dropped_partition_selection: float
    error_l0_expected: float
    error_linf_expected: float
    error_linf_min_expected: float
    error_linf_max_expected: float
    error_expected: float
    error_l0_variance: float
    error_variance: float
    error_quantiles: List[float]
    rel_error_l0_expected: float
    rel_error_linf_expected: float
    rel_error_linf_min_expected: float
    rel_error_linf_max_expected: float
    rel_error_expected: float
    rel_error_l0_variance: float
    rel_error_variance: float
    rel_error_quantiles: List[float]
    error_expected_w_dropped_partitions: float
    rel_error_expected_w_dropped_partitions: float
    noise_std: float

    def absolute_rmse(self) -> float:
        return math.sqrt(self.error_expected**2 + self.error_variance)

    def relative_rmse(self) -> float:
        return math.sqrt(self.rel_error_expected**2 + self.rel_error_variance)


@dataclasses.dataclass
class PartitionSelectionMetrics:
    """analysis/metrics.py:123-129."""
    num_partitions: float
    dropped_partitions_expected: float
    dropped_partitions_variance: float


@dataclasses.dataclass
class AggregateMetrics:
    """Utility analysis result for one configuration (analysis/metrics.py:132-150)."""
    input_aggregate_params: agg.AggregateParams
    count_metrics: Optional[AggregateErrorMetrics] = None
    privacy_id_count_metrics: Optional[AggregateErrorMetrics] = None
    partition_selection_metrics: Optional[PartitionSelectionMetrics] = None
    sum_metrics: Optional[AggregateErrorMetrics] = None


ERROR_QUANTILES = (0.1, 0.5, 0.9, 0.99)  # utility_analysis.py:68
_METRIC_TYPE = {agg.Metrics.SUM: AggregateMetricType.SUM, agg.Metrics.COUNT: AggregateMetricType.COUNT,
                agg.Metrics.PRIVACY_ID_COUNT: AggregateMetricType.PRIVACY_ID_COUNT}


def _error_metrics(metric_type, acc, Q, std_noise) -> AggregateErrorMetrics:
    """SumAggregateErrorMetricsCombiner.compute_metrics (combiners.py:590-640)
    on one row of pdp_utility_aggregate's sums."""
    f = dict(zip(native.AGG_FIELDS, (float(v) for v in acc[:native.AGG_NUM_FIELDS])))
    eq = [float(v) for v in acc[native.AGG_NUM_FIELDS:native.AGG_NUM_FIELDS + Q]]
    req = [float(v) for v in acc[native.AGG_NUM_FIELDS + Q:native.AGG_NUM_FIELDS + 2 * Q]]
    k = f["kept_partitions_expected"]
    total = max(1.0, f["total_aggregate"])
    l0, lmin, lmax = f["error_l0_expected"] / k, f["error_linf_min_expected"] / k, f["error_linf_max_expected"] / k
    rl0 = f["rel_error_l0_expected"] / k
    rlmin, rlmax = f["rel_error_linf_min_expected"] / k, f["rel_error_linf_max_expected"] / k
    n = f["num_partitions"]
    return AggregateErrorMetrics(
        metric_type=metric_type,
        ratio_data_dropped_l0=f["data_dropped_l0"] / total,
        ratio_data_dropped_linf=f["data_dropped_linf"] / total,
        ratio_data_dropped_partition_selection=f["data_dropped_partition_selection"] / total,
        error_l0_expected=l0, error_linf_expected=lmin + lmax, error_linf_min_expected=lmin,
        error_linf_max_expected=lmax, error_expected=l0 + lmin + lmax,
        error_l0_variance=f["error_l0_variance"] / k, error_variance=f["error_variance"] / k,
        error_quantiles=[v / k for v in eq],
        rel_error_l0_expected=rl0, rel_error_linf_expected=rlmin + rlmax, rel_error_linf_min_expected=rlmin,
        rel_error_linf_max_expected=rlmax, rel_error_expected=rl0 + rlmin + rlmax,
        rel_error_l0_variance=f["rel_error_l0_variance"] / k, rel_error_variance=f["rel_error_variance"] / k,
        rel_error_quantiles=[v / k for v in req],
        error_expected_w_dropped_partitions=f["error_expected_w_dropped_partitions"] / n,
        rel_error_expected_w_dropped_partitions=f["rel_error_expected_w_dropped_partitions"] / n,
        noise_std=std_noise)


class AggregateResult:
    """Lazy one-element collection holding the list of AggregateMetrics (one
    per configuration), as perform_utility_analysis returns it."""

    def __init__(self, per_partition: "AnalysisResult", quantiles):
        self._pp = per_partition
        self._quantiles = list(quantiles)
        self._out = None

    def __iter__(self):
        if self._out is None:
            self._out = [self._pp._aggregate(self._quantiles)]
        return iter(self._out)


def _aggregate(self, quantiles):
    """AnalysisResult -> [AggregateMetrics per configuration] via
    pdp_utility_aggregate on the device arrays of the per-partition result."""
    keys, metrics, prob, pids, _ = self._encode_and_run()
    opts = self._options
    params_list = get_aggregate_params(opts)
    present = [m for m in _ANALYSIS_METRICS if m in opts.aggregate_params.metrics]
    private = self._public is None
    C, Q = len(params_list), len(quantiles)
    stds = [[noise_std(p, self._metric_specs[m].eps, self._metric_specs[m].delta) for m in present]
            for p in params_list]
    if metrics is None or len(keys) == 0:
        raise ValueError("utility analysis over an empty partition set")
    kinds = [native.NOISE_GAUSSIAN if p.noise_kind == agg.NoiseKind.GAUSSIAN else native.NOISE_LAPLACE
             for p in params_list]
    mask = sum(bit for m, bit in ((agg.Metrics.SUM, native.METRIC_SUM), (agg.Metrics.COUNT, native.METRIC_COUNT),
                                  (agg.Metrics.PRIVACY_ID_COUNT, native.METRIC_PRIVACY_ID_COUNT))
               if m in opts.aggregate_params.metrics)
    errors, sel = self._engine._backend.executor.aggregate_errors(metrics, prob, pids, mask, stds, kinds, quantiles,
                                                                  private)
    errors = errors.cpu().numpy()
    sel = sel.cpu().numpy() if sel is not None else None
    out = []
    for c, p in enumerate(params_list):
        am = AggregateMetrics(input_aggregate_params=p)
        if private:
            n, e, v = (float(x) for x in sel[c])
            am.partition_selection_metrics = PartitionSelectionMetrics(num_partitions=n,
                                                                       dropped_partitions_expected=n - e,
                                                                       dropped_partitions_variance=v)
        for b, m in enumerate(present):
            em = _error_metrics(_METRIC_TYPE[m], errors[c, b], Q, stds[c][b])
            setattr(am, {agg.Metrics.SUM: "sum_metrics", agg.Metrics.COUNT: "count_metrics",
                         agg.Metrics.PRIVACY_ID_COUNT: "privacy_id_count_metrics"}[m], em)
        out.append(am)
    return out


AnalysisResult._aggregate = _aggregate


def perform_utility_analysis(col, backend, options: UtilityAnalysisOptions, data_extractors, public_partitions=None,
                             return_per_partition: bool = False):
    """Utility analysis of DP aggregations (analysis/utility_analysis.py:27-119):
    the per-partition analysis of UtilityAnalysisEngine, then its
    cross-partition aggregation.  Returns a one-element collection holding
    the list of AggregateMetrics (one per configuration); with
    return_per_partition, (that collection, the per-partition result)."""
    from .budget_accounting import NaiveBudgetAccountant
    accountant = NaiveBudgetAccountant(total_epsilon=options.epsilon, total_delta=options.delta)
    engine = UtilityAnalysisEngine(budget_accountant=accountant, backend=backend)
    per_partition = engine.analyze(col, options=options, data_extractors=data_extractors,
                                   public_partitions=public_partitions)
    accountant.compute_budgets()
    result = AggregateResult(per_partition, ERROR_QUANTILES)
    if return_per_partition:
        return result, per_partition
    return result
