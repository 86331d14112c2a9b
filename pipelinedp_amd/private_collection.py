"""``make_private(...)`` — the high-level caller shape of the reference's
private APIs (``pipeline_dp/private_spark.py:21-382``), over a local
collection and the HipBackend instead of a Spark RDD.

Each method builds AggregateParams exactly like the reference (e.g.
``PrivateRDD.mean`` :122-176) and calls DPEngine.aggregate; results are lazy
``(partition_key, value)`` iterables.
"""
from typing import Callable, Optional

from . import aggregate_params as agg
from .dp_engine import DataExtractors, DPEngine
from .pipeline_backend import HipBackend


class PrivateCollection:
    """Collection of (privacy_id, element) pairs that can only be released
    through DP aggregations."""

    def __init__(self, col, budget_accountant, privacy_id_extractor: Optional[Callable] = None, backend=None):
        if privacy_id_extractor:
            self._col = [(privacy_id_extractor(x), x) for x in col]
        else:
            self._col = col if isinstance(col, list) else list(col)
        self._budget_accountant = budget_accountant
        self._backend = backend or HipBackend()

    def map(self, fn: Callable) -> "PrivateCollection":
        return PrivateCollection([(k, fn(v)) for k, v in self._col], self._budget_accountant, None, self._backend)

    def flat_map(self, fn: Callable) -> "PrivateCollection":
        return PrivateCollection([(k, y) for k, v in self._col for y in fn(v)], self._budget_accountant, None,
                                 self._backend)

    def _pid_extractor(self, already_enforced: bool):
        return None if already_enforced else (lambda x: x[0])

    def _run(self, params, pe, ve, public_partitions, report, field):
        engine = DPEngine(self._budget_accountant, self._backend)
        ex = DataExtractors(privacy_id_extractor=self._pid_extractor(params.contribution_bounds_already_enforced),
                            partition_extractor=lambda x: pe(x[1]),
                            value_extractor=(lambda x: ve(x[1])) if ve else (lambda x: None))
        res = engine.aggregate(self._col, params, ex, public_partitions, out_explain_computaton_report=report)
        return _LazyMap(res, lambda v: getattr(v, field))

    def variance(self, variance_params: agg.VarianceParams, public_partitions=None,
                 out_explain_computaton_report=None):
        p = variance_params
        params = agg.AggregateParams(noise_kind=p.noise_kind, metrics=[agg.Metrics.VARIANCE],
                                     max_partitions_contributed=p.max_partitions_contributed,
                                     max_contributions_per_partition=p.max_contributions_per_partition,
                                     min_value=p.min_value, max_value=p.max_value, budget_weight=p.budget_weight,
                                     contribution_bounds_already_enforced=p.contribution_bounds_already_enforced)
        return self._run(params, p.partition_extractor, p.value_extractor, public_partitions,
                         out_explain_computaton_report, "variance")

    def mean(self, mean_params: agg.MeanParams, public_partitions=None, out_explain_computaton_report=None):
        p = mean_params
        params = agg.AggregateParams(noise_kind=p.noise_kind, metrics=[agg.Metrics.MEAN],
                                     max_partitions_contributed=p.max_partitions_contributed,
                                     max_contributions_per_partition=p.max_contributions_per_partition,
                                     min_value=p.min_value, max_value=p.max_value, budget_weight=p.budget_weight,
                                     contribution_bounds_already_enforced=p.contribution_bounds_already_enforced)
        return self._run(params, p.partition_extractor, p.value_extractor, public_partitions,
                         out_explain_computaton_report, "mean")

    def sum(self, sum_params: agg.SumParams, public_partitions=None, out_explain_computaton_report=None):
        p = sum_params
        params = agg.AggregateParams(noise_kind=p.noise_kind, metrics=[agg.Metrics.SUM],
                                     max_partitions_contributed=p.max_partitions_contributed,
                                     max_contributions_per_partition=p.max_contributions_per_partition,
                                     min_value=p.min_value, max_value=p.max_value, budget_weight=p.budget_weight,
                                     contribution_bounds_already_enforced=p.contribution_bounds_already_enforced)
        return self._run(params, p.partition_extractor, p.value_extractor, public_partitions,
                         out_explain_computaton_report, "sum")

    def count(self, count_params: agg.CountParams, public_partitions=None, out_explain_computaton_report=None):
        p = count_params
        params = agg.AggregateParams(noise_kind=p.noise_kind, metrics=[agg.Metrics.COUNT],
                                     max_partitions_contributed=p.max_partitions_contributed,
                                     max_contributions_per_partition=p.max_contributions_per_partition,
                                     budget_weight=p.budget_weight,
                                     contribution_bounds_already_enforced=p.contribution_bounds_already_enforced)
        return self._run(params, p.partition_extractor, None, public_partitions, out_explain_computaton_report,
                         "count")

    def privacy_id_count(self, privacy_id_count_params: agg.PrivacyIdCountParams, public_partitions=None,
                         out_explain_computaton_report=None):
        p = privacy_id_count_params
        params = agg.AggregateParams(noise_kind=p.noise_kind, metrics=[agg.Metrics.PRIVACY_ID_COUNT],
                                     max_partitions_contributed=p.max_partitions_contributed,
                                     max_contributions_per_partition=1,
                                     contribution_bounds_already_enforced=p.contribution_bounds_already_enforced)
        return self._run(params, p.partition_extractor, None, public_partitions, out_explain_computaton_report,
                         "privacy_id_count")

    def select_partitions(self, select_partitions_params: agg.SelectPartitionsParams,
                          partition_extractor: Callable):
        engine = DPEngine(self._budget_accountant, self._backend)
        ex = DataExtractors(privacy_id_extractor=lambda x: x[0], partition_extractor=lambda x: partition_extractor(x[1]))
        params = agg.SelectPartitionsParams(
            max_partitions_contributed=select_partitions_params.max_partitions_contributed)
        return engine.select_partitions(self._col, params, ex)


class _LazyMap:
    """Lazy, re-iterable map_values over a DPResult."""

    def __init__(self, src, fn):
        self._src, self._fn = src, fn

    def __iter__(self):
        return ((k, self._fn(v)) for k, v in self._src)


def make_private(col, budget_accountant, privacy_id_extractor=None, backend=None) -> PrivateCollection:
    """reference private_spark.make_private (:377-382)."""
    return PrivateCollection(col, budget_accountant, privacy_id_extractor, backend)
