"""Bounding sweep: the data-parallel core of the reference's utility analysis.

The reference's `UtilityAnalysisEngine` (analysis/utility_analysis_engine.py:
88-173) re-runs contribution bounding and the combiners once per bounding
configuration of a `MultiParameterConfiguration`
(analysis/data_structures.py:41-118).  Here the rows are encoded once, sorted
by privacy id once on the GPU, and bounded + accumulated per configuration by
`pdp_bound_accumulate_sweep` (include/pdp_hip.h).  The result of each
configuration is what `DPEngine.aggregate` computes before noise and
selection: per partition, the privacy-id count, the bounded row count and the
clipped sum.

Out of scope: the analysis metrics built on top of these
accumulators (error expectations, Poisson-binomial keep probabilities).
"""
import dataclasses
from typing import Dict, List, Optional, Sequence

from .aggregate_params import AggregateParams
from .columnar import encode_rows


@dataclasses.dataclass
class MultiParameterConfiguration:
    """Per-configuration bounding parameters; every set field has one entry per
    configuration (validation as analysis/data_structures.py:78-91)."""
    max_partitions_contributed: Optional[Sequence[int]] = None
    max_contributions_per_partition: Optional[Sequence[int]] = None
    min_sum_per_partition: Optional[Sequence[float]] = None
    max_sum_per_partition: Optional[Sequence[float]] = None

    def __post_init__(self):
        lengths = [len(v) for v in dataclasses.asdict(self).values() if v]
        if not lengths:
            raise ValueError("MultiParameterConfiguration must have at least 1 non-empty attribute.")
        if len(set(lengths)) != 1:
            raise ValueError("All set attributes in MultiParameterConfiguration must have the same length.")
        if (self.min_sum_per_partition is None) != (self.max_sum_per_partition is None):
            raise ValueError("MultiParameterConfiguration: min_sum_per_partition and max_sum_per_partition "
                             "must be both set or both None.")
        self._size = lengths[0]

    @property
    def size(self) -> int:
        return self._size

    def get_aggregate_params(self, params: AggregateParams, index: int) -> AggregateParams:
        """`params` with the index-th configuration's bounds substituted."""
        changes = {}
        for f in dataclasses.fields(self):
            seq = getattr(self, f.name)
            if seq:
                changes[f.name] = seq[index]
        return dataclasses.replace(params, **changes)


@dataclasses.dataclass
class PartitionAccumulators:
    """Per-partition accumulators of one configuration (before noise)."""
    privacy_id_count: int
    count: int
    sum: float


def bounded_accumulators_sweep(col, params: AggregateParams, data_extractors,
                               multi: MultiParameterConfiguration, public_partitions=None, device: int = 0,
                               sampling_seed: Optional[int] = None) -> List[Dict[object, PartitionAccumulators]]:
    """For each configuration of `multi`: {partition_key: PartitionAccumulators}.

    Bounding per configuration follows SamplingCrossAndPerPartitionContributionBounder
    (contribution_bounders.py:66-105): at most max_contributions_per_partition
    rows per (privacy id, partition), then at most max_partitions_contributed
    partitions per privacy id; values clipped to [min_value, max_value], or
    per-partition sums clipped to [min_sum_per_partition, max_sum_per_partition].
    Partitions that keep no row are absent unless they are public.
    """
    import torch

    from . import native
    from .executor import BoundConfig, HipExecutor

    cfgs = [multi.get_aggregate_params(params, i) for i in range(multi.size)]
    need_value = any(c.min_value is not None or c.min_sum_per_partition is not None for c in cfgs)
    enc = encode_rows(col, data_extractors, public_partitions, need_pid=True, need_value=need_value)
    ex = HipExecutor(device)
    t = lambda a: None if a is None else torch.from_numpy(a).to(ex.device)  # noqa: E731
    P = max(len(enc.partition_keys), 1)
    bounds = []
    for i, c in enumerate(cfgs):
        mask = native.METRIC_COUNT | native.METRIC_PRIVACY_ID_COUNT
        if need_value:
            mask |= native.METRIC_SUM
        bounds.append(BoundConfig(mask, c.max_partitions_contributed, c.max_contributions_per_partition,
                                  c.min_value, c.max_value, c.min_sum_per_partition, c.max_sum_per_partition,
                                  sampling_seed=None if sampling_seed is None else sampling_seed + i))
    accs = ex.accumulate_sweep(t(enc.pid), t(enc.pk), t(enc.value), enc.num_privacy_ids, P, bounds)
    out = []
    public = public_partitions is not None
    for acc in accs:
        rc = acc.row_count.cpu().numpy()
        cnt = acc.count.cpu().numpy()
        sm = acc.x.cpu().numpy() if need_value else None
        res = {}
        for i, key in enumerate(enc.partition_keys):
            if rc[i] or public:
                res[key] = PartitionAccumulators(int(rc[i]), int(cnt[i]), float(sm[i]) if sm is not None else 0.0)
        out.append(res)
    return out
