"""User-facing parameter types of the aggregate path.

Mirrors the reference API (``pipeline_dp/aggregate_params.py``) so callers of
``DPEngine.aggregate`` and ``make_private(...).sum/count/mean/...`` are
unchanged: same class and field names, same defaults, same validation errors
(``AggregateParams.__post_init__``, reference :175-270).
"""
import dataclasses
import enum
import logging
import math
from typing import Any, Callable, Iterable, List, Optional, Sequence


@dataclasses.dataclass
class Metric:
    """A DP metric; ``parameter`` is used by PERCENTILE (reference :23-51)."""
    name: str
    parameter: Optional[float] = None

    def __eq__(self, other) -> bool:
        return isinstance(other, Metric) and (self.name, self.parameter) == (other.name, other.parameter)

    def __hash__(self):
        return hash(str(self))

    def __str__(self):
        return self.name if self.parameter is None else f"{self.name}({self.parameter})"

    __repr__ = __str__

    @property
    def is_percentile(self) -> bool:
        return self.name == "PERCENTILE"


class Metrics:
    """All metrics of the reference (:54-65).  PERCENTILE and VECTOR_SUM are
    accepted by the parameter classes but are outside the GPU path."""
    COUNT = Metric("COUNT")
    PRIVACY_ID_COUNT = Metric("PRIVACY_ID_COUNT")
    SUM = Metric("SUM")
    MEAN = Metric("MEAN")
    VARIANCE = Metric("VARIANCE")
    VECTOR_SUM = Metric("VECTOR_SUM")

    @classmethod
    def PERCENTILE(cls, percentile_to_compute: float) -> Metric:
        return Metric("PERCENTILE", percentile_to_compute)


class MechanismType(enum.Enum):
    LAPLACE = "Laplace"
    GAUSSIAN = "Gaussian"
    GENERIC = "Generic"


class NoiseKind(enum.Enum):
    LAPLACE = "laplace"
    GAUSSIAN = "gaussian"

    def convert_to_mechanism_type(self) -> MechanismType:
        return {NoiseKind.LAPLACE.value: MechanismType.LAPLACE,
                NoiseKind.GAUSSIAN.value: MechanismType.GAUSSIAN}[self.value]


class NormKind(enum.Enum):
    Linf = "linf"
    L0 = "l0"
    L1 = "l1"
    L2 = "l2"


class PartitionSelectionStrategy(enum.Enum):
    TRUNCATED_GEOMETRIC = "Truncated Geometric"
    LAPLACE_THRESHOLDING = "Laplace Thresholding"
    GAUSSIAN_THRESHOLDING = "Gaussian Thresholding"


def _is_bad_number(x: Any) -> bool:
    return math.isnan(x) or math.isinf(x)


def _require_positive_int(value: Any, name: str) -> None:
    if not (isinstance(value, int) and value > 0):
        raise ValueError(f"{name} has to be positive integer, but {value} given.")


@dataclasses.dataclass
class AggregateParams:
    """Parameters of ``DPEngine.aggregate`` (reference :98-296)."""
    metrics: List[Metric]
    noise_kind: NoiseKind = NoiseKind.LAPLACE
    max_partitions_contributed: Optional[int] = None
    max_contributions_per_partition: Optional[int] = None
    max_contributions: Optional[int] = None
    budget_weight: float = 1
    low: float = None  # deprecated
    high: float = None  # deprecated
    min_value: float = None
    max_value: float = None
    min_sum_per_partition: float = None
    max_sum_per_partition: float = None
    public_partitions: Any = None  # deprecated
    custom_combiners: Sequence[Any] = None
    vector_norm_kind: Optional[NormKind] = None
    vector_max_norm: Optional[float] = None
    vector_size: Optional[int] = None
    contribution_bounds_already_enforced: bool = False
    public_partitions_already_filtered: bool = False
    partition_selection_strategy: PartitionSelectionStrategy = PartitionSelectionStrategy.TRUNCATED_GEOMETRIC

    @property
    def metrics_str(self) -> str:
        if self.custom_combiners:
            return f"custom combiners={[c.metrics_names() for c in self.custom_combiners]}"
        return f"metrics={[str(m) for m in self.metrics]}"

    @property
    def bounds_per_contribution_are_set(self) -> bool:
        return self.min_value is not None and self.max_value is not None

    @property
    def bounds_per_partition_are_set(self) -> bool:
        return self.min_sum_per_partition is not None and self.max_sum_per_partition is not None

    def _pair_consistent(self, lo: str, hi: str) -> None:
        if (getattr(self, lo) is None) != (getattr(self, hi) is None):
            raise ValueError(f"AggregateParams: {lo} and {hi} should be both set or both None.")

    def _range_ok(self, lo: str, hi: str) -> None:
        for name in (lo, hi):
            if _is_bad_number(getattr(self, name)):
                raise ValueError(f"AggregateParams: {name} must be a finite number")
        if getattr(self, lo) > getattr(self, hi):
            raise ValueError(f"AggregateParams: {hi} must be equal to or greater than {lo}")

    def _check_metric_compatibility(self, value_bound: bool, partition_bound: bool) -> None:
        metrics = set(self.metrics)
        if Metrics.VECTOR_SUM in metrics:
            if metrics & {Metrics.SUM, Metrics.MEAN, Metrics.VARIANCE}:
                raise ValueError("AggregateParams: vector sum can not be computed together"
                                 " with scalar metrics such as sum, mean etc")
            return
        if partition_bound:
            extra = metrics - {Metrics.SUM, Metrics.PRIVACY_ID_COUNT, Metrics.COUNT}
            if extra:
                raise ValueError(f"AggregateParams: min_sum_per_partition is not "
                                 f"compatible with metrics {extra}. Please"
                                 f"use min_value/max_value.")
        elif not value_bound:
            extra = metrics - {Metrics.PRIVACY_ID_COUNT, Metrics.COUNT}
            if extra:
                raise ValueError(f"AggregateParams: for metrics {extra} "
                                 f"bounds per partition are required (e.g. min_value,"
                                 f"max_value).")

    def _check_contribution_bounds(self) -> None:
        if self.max_contributions is not None:
            _require_positive_int(self.max_contributions, "max_contributions")
            if self.max_partitions_contributed is not None or self.max_contributions_per_partition is not None:
                raise ValueError("AggregateParams: only one in max_contributions or "
                                 "both max_partitions_contributed and "
                                 "max_contributions_per_partition must be set")
            return
        n_set = sum(x is not None for x in (self.max_partitions_contributed,
                                            self.max_contributions_per_partition))
        if n_set == 0:
            raise ValueError("AggregateParams: either max_contributions must be set or "
                             "both max_partitions_contributed and "
                             "max_contributions_per_partition must be set.")
        if n_set == 1:
            raise ValueError("AggregateParams: either none or both from "
                             "max_partitions_contributed and "
                             " max_contributions_per_partition must be set.")
        _require_positive_int(self.max_partitions_contributed, "max_partitions_contributed")
        _require_positive_int(self.max_contributions_per_partition, "max_contributions_per_partition")

    def __post_init__(self):
        if self.low is not None:
            raise ValueError("AggregateParams: please use min_value instead of low")
        if self.high is not None:
            raise ValueError("AggregateParams: please use max_value instead of high")
        self._pair_consistent("min_value", "max_value")
        self._pair_consistent("min_sum_per_partition", "max_sum_per_partition")
        value_bound = self.min_value is not None
        partition_bound = self.min_sum_per_partition is not None
        if value_bound and partition_bound:
            raise ValueError("min_value and min_sum_per_partition can not be both set.")
        if value_bound:
            self._range_ok("min_value", "max_value")
        if partition_bound:
            self._range_ok("min_sum_per_partition", "max_sum_per_partition")
        if self.metrics:
            self._check_metric_compatibility(value_bound, partition_bound)
            if self.contribution_bounds_already_enforced and Metrics.PRIVACY_ID_COUNT in self.metrics:
                raise ValueError("AggregateParams: Cannot calculate PRIVACY_ID_COUNT when "
                                 "contribution_bounds_already_enforced is set to True.")
        if self.custom_combiners:
            logging.warning("Warning: custom combiners are used. This is an "
                            "experimental feature. It might not work properly "
                            "and it might be changed or removed without any "
                            "notifications.")
            if self.metrics:
                raise ValueError("Custom combiners can not be used with standard metrics")
        if self.public_partitions:
            raise ValueError("AggregateParams.public_partitions is deprecated. Please use public_partitions "
                             "argument in DPEngine.aggregate insead.")
        self._check_contribution_bounds()

    def __str__(self):
        return parameters_to_readable_string(self)


@dataclasses.dataclass
class SelectPartitionsParams:
    """Parameters of ``DPEngine.select_partitions`` (reference :299-321)."""
    max_partitions_contributed: int
    budget_weight: float = 1
    partition_selection_strategy: PartitionSelectionStrategy = PartitionSelectionStrategy.TRUNCATED_GEOMETRIC

    def __str__(self):
        return "Private Partitions"


def _reject_deprecated_public(obj, name: str, message: str) -> None:
    if getattr(obj, "public_partitions", None):
        raise ValueError(message)


@dataclasses.dataclass
class SumParams:
    """make_private(...).sum parameters (reference :324-377)."""
    max_partitions_contributed: int
    max_contributions_per_partition: int
    min_value: float
    max_value: float
    partition_extractor: Callable
    value_extractor: Callable
    low: float = None  # deprecated
    high: float = None  # deprecated
    budget_weight: float = 1
    noise_kind: NoiseKind = NoiseKind.LAPLACE
    contribution_bounds_already_enforced: bool = False
    public_partitions: Any = None  # deprecated

    def __post_init__(self):
        if self.low is not None:
            raise ValueError("SumParams: please use min_value instead of low")
        if self.high is not None:
            raise ValueError("SumParams: please use max_value instead of high")
        _reject_deprecated_public(self, "SumParams",
                                  "SumParams.public_partitions is deprecated. Please read API documentation "
                                  "for anonymous Sum transform.")


@dataclasses.dataclass
class VarianceParams:
    """make_private(...).variance parameters (reference :380-421)."""
    max_partitions_contributed: int
    max_contributions_per_partition: int
    min_value: float
    max_value: float
    partition_extractor: Callable
    value_extractor: Callable
    budget_weight: float = 1
    noise_kind: NoiseKind = NoiseKind.LAPLACE
    contribution_bounds_already_enforced: bool = False
    public_partitions: Any = None  # deprecated

    def __post_init__(self):
        _reject_deprecated_public(self, "VarianceParams",
                                  "VarianceParams.public_partitions is deprecated. Please read API "
                                  "documentation for anonymous Variance transform.")


@dataclasses.dataclass
class MeanParams:
    """make_private(...).mean parameters (reference :424-467)."""
    max_partitions_contributed: int
    max_contributions_per_partition: int
    min_value: float
    max_value: float
    partition_extractor: Callable
    value_extractor: Callable
    budget_weight: float = 1
    noise_kind: NoiseKind = NoiseKind.LAPLACE
    contribution_bounds_already_enforced: bool = False
    public_partitions: Any = None  # deprecated

    def __post_init__(self):
        _reject_deprecated_public(self, "MeanParams",
                                  "MeanParams.public_partitions is deprecated. Please read API documentation "
                                  "for anonymous Mean transform.")


@dataclasses.dataclass
class CountParams:
    """make_private(...).count parameters (reference :470-502)."""
    noise_kind: NoiseKind
    max_partitions_contributed: int
    max_contributions_per_partition: int
    partition_extractor: Callable
    budget_weight: float = 1
    contribution_bounds_already_enforced: bool = False
    public_partitions: Any = None  # deprecated

    def __post_init__(self):
        _reject_deprecated_public(self, "CountParams",
                                  "CountParams.public_partitions is deprecated. Please read API documentation "
                                  "for anonymous Count transform.")


@dataclasses.dataclass
class PrivacyIdCountParams:
    """make_private(...).privacy_id_count parameters (reference :505-535)."""
    noise_kind: NoiseKind
    max_partitions_contributed: int
    partition_extractor: Callable
    budget_weight: float = 1
    contribution_bounds_already_enforced: bool = False
    public_partitions: Any = None  # deprecated

    def __post_init__(self):
        _reject_deprecated_public(self, "PrivacyIdCountParams",
                                  "PrivacyIdCountParams.public_partitions is deprecated. Please "
                                  "read API documentation for anonymous PrivacyIdCountParams "
                                  "transform.")


_BOUND_FIELDS = ("max_partitions_contributed", "max_contributions_per_partition", "max_contributions",
                 "min_value", "max_value", "min_sum_per_partition", "max_sum_per_partition")
_VECTOR_FIELDS = ("vector_max_norm", "vector_size", "vector_norm_kind")


def parameters_to_readable_string(params, is_public_partition: Optional[bool] = None) -> str:
    """Human readable parameter block of the explain report (reference
    :565-594); the text is byte-identical to the reference's."""
    lines = [f"{type(params).__name__}:"]
    if hasattr(params, "metrics_str"):
        lines.append(f" {params.metrics_str}")
    if hasattr(params, "noise_kind"):
        lines.append(f" noise_kind={params.noise_kind.value}")
    if hasattr(params, "budget_weight"):
        lines.append(f" budget_weight={params.budget_weight}")
    lines.append(" Contribution bounding:")

    def add(name):
        value = getattr(params, name, None)
        if value is not None:
            lines.append(f"  {name}={value}")

    for name in _BOUND_FIELDS:
        add(name)
    if getattr(params, "contribution_bounds_already_enforced", False):
        lines.append("  contribution_bounds_already_enforced=True")
    for name in _VECTOR_FIELDS:
        add(name)
    if is_public_partition is not None:
        kind = "public" if is_public_partition else "private"
        lines.append(f" Partition selection: {kind} partitions")
    return "\n".join(lines)
