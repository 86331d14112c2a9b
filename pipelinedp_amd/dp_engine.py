"""DPEngine: the user-facing aggregate / select_partitions API.

Same call shape and semantics as the reference ``pipeline_dp/dp_engine.py``
(DPEngine.aggregate :66-109, _aggregate :111-181, select_partitions
:204-281): eager parameter validation with the same errors, budget requests
in the same order and weights, the same explain-computation stages, and a
LAZY result that computes only when iterated after
``budget_accountant.compute_budgets()``.  The computation itself is the
fused HIP pipeline of ``HipBackend`` (libpdp_hip.so); there is no
element-wise CPU execution of the hot path.
"""
import collections
import dataclasses
from typing import Callable, List, Optional

import numpy as np

from . import aggregate_params as agg
from . import native
from .columnar import ColumnarData, encode_rows, remap_public
from .executor import BoundConfig, ReleaseConfig
from .report_generator import ExplainComputationReport, ReportGenerator


@dataclasses.dataclass
class DataExtractors:
    """privacy id / partition key / value extractors (reference :27-37)."""
    privacy_id_extractor: Callable = None
    partition_extractor: Callable = None
    value_extractor: Callable = None


_MECH_SLOT = {"count": native.MECH_COUNT, "sum": native.MECH_SUM, "mean": native.MECH_MEAN,
              "variance": native.MECH_VARIANCE, "privacy_id_count": native.MECH_PRIVACY_ID_COUNT}
_EXPLAIN_NAME = {"count": "count", "sum": "sum", "mean": "mean", "variance": "variance",
                 "privacy_id_count": "privacy id count"}
_SELECTION = {agg.PartitionSelectionStrategy.TRUNCATED_GEOMETRIC: native.SELECTION_TRUNCATED_GEOMETRIC,
              agg.PartitionSelectionStrategy.LAPLACE_THRESHOLDING: native.SELECTION_LAPLACE,
              agg.PartitionSelectionStrategy.GAUSSIAN_THRESHOLDING: native.SELECTION_GAUSSIAN}

_tuple_types = {}


def metrics_tuple_type(fields):
    key = tuple(fields)
    t = _tuple_types.get(key)
    if t is None:
        t = collections.namedtuple("MetricsTuple", key)
        _tuple_types[key] = t
    return t


def metrics_mask(metrics) -> int:
    m = set(metrics)
    mask = 0
    for metric, bit in ((agg.Metrics.COUNT, native.METRIC_COUNT), (agg.Metrics.SUM, native.METRIC_SUM),
                        (agg.Metrics.MEAN, native.METRIC_MEAN), (agg.Metrics.VARIANCE, native.METRIC_VARIANCE),
                        (agg.Metrics.PRIVACY_ID_COUNT, native.METRIC_PRIVACY_ID_COUNT)):
        if metric in m:
            mask |= bit
    return mask


@dataclasses.dataclass
class _Plan:
    """What _aggregate decided at graph-construction time."""
    slots: list  # [(combiner name, MechanismSpec)]
    selection_spec: object = None
    max_rows_per_privacy_id: int = 1


class DPResult:
    """Lazy collection of (partition_key, MetricsTuple).  Iterating it runs
    the GPU pipeline once (after compute_budgets()) and caches the result."""

    def __init__(self, engine, col, params, extractors, public_partitions, plan, select_only=False):
        self._engine = engine
        self._backend = engine._backend
        self._col = col
        self._params = params
        self._extractors = extractors
        self._public = public_partitions
        self._plan = plan
        self._select_only = select_only
        self._arrays = None

    # -- public API ----------------------------------------------------------
    def __iter__(self):
        keys, keep, fields, values = self.to_arrays()
        idx = np.flatnonzero(keep)
        if self._select_only:
            return iter([keys[i] for i in idx])
        T = metrics_tuple_type(fields)
        cols = values[:, idx].T.tolist() if len(fields) else [[] for _ in idx]
        return iter([(keys[i], T(*row)) for i, row in zip(idx.tolist(), cols)])

    def to_arrays(self):
        """(partition keys, keep mask [P] bool, field names, values [F, P])."""
        if self._arrays is None:
            self._arrays = self._compute()
        return self._arrays

    # -- execution -------------------------------------------------------------
    def _release_config(self, mask):
        eps = [0.0] * native.NUM_MECH
        delta = [0.0] * native.NUM_MECH
        for name, spec in self._plan.slots:
            eps[_MECH_SLOT[name]] = spec.eps
            delta[_MECH_SLOT[name]] = spec.delta
        selection = native.SELECTION_NONE
        if self._plan.selection_spec is not None:
            selection = _SELECTION[self._params.partition_selection_strategy]
            eps[native.MECH_SELECTION] = self._plan.selection_spec.eps
            delta[native.MECH_SELECTION] = self._plan.selection_spec.delta
        noise_kind = native.NOISE_GAUSSIAN if getattr(self._params, "noise_kind",
                                                      agg.NoiseKind.LAPLACE) == agg.NoiseKind.GAUSSIAN \
            else native.NOISE_LAPLACE
        return ReleaseConfig(mask, noise_kind, selection, eps, delta, self._plan.max_rows_per_privacy_id,
                             add_noise=not self._backend._disable_noise, noise_seed=self._backend.noise_seed)

    def _inputs(self, torch, device, need_pid, need_value, world=None):
        """-> pid, pk, value device tensors, U, P, partition keys, and whether
        the rows are already sharded by privacy id over the world's ranks."""
        col = self._col
        public = self._public
        multi = world is not None and world.size > 1

        def global_max(t, local):
            # multi-rank: the id ranges are the union over ranks
            if not multi:
                return local
            import torch.distributed as dist
            m = torch.tensor([local], dtype=torch.int64, device=device)
            dist.all_reduce(m, op=dist.ReduceOp.MAX, group=world.group)
            return int(m.item())

        if isinstance(col, ColumnarData):
            pk = torch.as_tensor(col.partition).to(device=device, dtype=torch.int64).contiguous()
            P = col.num_partitions
            if P is None:
                P = global_max(pk, int(pk.max().item()) + 1 if pk.numel() else 0)
            elif pk.numel() and int(pk.max().item()) >= P:
                raise ValueError(f"partition id {int(pk.max().item())} >= num_partitions={P}")
            keys = list(col.partition_keys) if col.partition_keys is not None else list(range(P))
            if public is not None:
                lut, keys = remap_public(pk, col.partition_keys, P, public)
                lut_t = torch.as_tensor(lut, device=device)
                pk = torch.where(pk >= 0, lut_t[pk.clamp(min=0, max=max(P - 1, 0))], pk.new_full((), -1))
                P = len(keys)
            pid = None
            U = 0
            if need_pid:
                pid = torch.as_tensor(col.privacy_id).to(device=device, dtype=torch.int64).contiguous()
                U = col.num_privacy_ids
                if U is None:
                    U = global_max(pid, int(pid.max().item()) + 1 if pid.numel() else 1)
            value = None
            if need_value:
                value = torch.as_tensor(col.value).to(device=device, dtype=torch.float64).contiguous()
            return pid, pk, value, U, P, keys, bool(col.privacy_id_sharded), 0
        enc = encode_rows(col, self._extractors, public, need_pid=need_pid, need_value=need_value, world=world)
        t = lambda a: torch.from_numpy(a).to(device)  # noqa: E731
        pid, pk, value = (t(enc.pid) if enc.pid is not None else None, t(enc.pk),
                          t(enc.value) if enc.value is not None else None)
        U, sharded, base = enc.num_privacy_ids, False, 0
        if enc.pid_hash is not None:  # multi-rank host rows: to the owner of their privacy-id key hash
            # rank-local ids [0, U) with the global numbering's offset `base` (hashed as base + id)
            pid, pk, value, U, base = world.exchange_by_key_hash(t(enc.pid_hash), pk, value)
            sharded = True
        return pid, pk, value, U, len(enc.partition_keys), enc.partition_keys, sharded, base

    def _compute(self):
        backend = self._backend
        ex = backend.executor
        torch = ex.torch
        p = self._params
        if self._select_only:
            mask = 0
            enforced = False
            bounds = BoundConfig(0, p.max_partitions_contributed, 1, sampling_seed=backend.sampling_seed)
        else:
            mask = metrics_mask(p.metrics)
            enforced = p.contribution_bounds_already_enforced
            bounds = BoundConfig(mask, p.max_partitions_contributed, p.max_contributions_per_partition,
                                 p.min_value, p.max_value, p.min_sum_per_partition, p.max_sum_per_partition,
                                 enforced, backend.sampling_seed, backend._debug_force_fallback)
        rel = self._release_config(mask)  # raises before any work if budgets are not computed
        need_value = bool(mask & (native.METRIC_SUM | native.METRIC_MEAN | native.METRIC_VARIANCE))
        # A World (also of size 1: the RCCL identity, tests/test_gpu_rccl.py) runs the collective path.
        world = backend.world
        pid, pk, value, U, P, keys, presharded, pid_base = self._inputs(torch, ex.device, not enforced, need_value,
                                                                        world)
        if pid_base:
            bounds = dataclasses.replace(bounds, pid_base=pid_base)
        fields = native.metric_fields(mask)
        if world is not None and world.size > 1:
            # every rank must take the same branch below (a rank with P == 0 alone would leave the others
            # blocked in the collectives): agree on P first, raising on disagreement
            world.check_same(P, "num_partitions", pk.device)
        if P == 0:  # e.g. public_partitions=[]: nothing to release (reference: empty collection)
            return keys, np.zeros(0, dtype=bool), fields, np.zeros((len(fields), 0))
        if world is not None:
            keep, out, fields = world.aggregate(ex, pid, pk, value, U, P, bounds, rel,
                                                shuffle=not presharded and pid is not None)
        else:
            acc = ex.accumulate(pid, pk, value, U, P, bounds)
            keep, out, fields = ex.release(acc, rel, bounds)
        keep = keep.cpu().numpy().astype(bool)
        out = out.cpu().numpy()
        return keys, keep, fields, out[:len(fields)]


class DPEngine:
    """Performs DP aggregations on the MI355X backend."""

    def __init__(self, budget_accountant, backend):
        self._budget_accountant = budget_accountant
        self._backend = backend
        self._report_generators = []

    @property
    def _current_report_generator(self):
        return self._report_generators[-1]

    def _add_report_stage(self, stage_description):
        self._current_report_generator.add_stage(stage_description)

    def _add_report_stages(self, stages):
        for s in stages:
            self._add_report_stage(s)

    def explain_computations_report(self):
        return [g.report() for g in self._report_generators]

    # -- aggregate --------------------------------------------------------------
    def aggregate(self, col, params: agg.AggregateParams, data_extractors: Optional[DataExtractors],
                  public_partitions=None, out_explain_computaton_report: Optional[ExplainComputationReport] = None):
        """Computes DP metrics per partition; returns a lazy DPResult of
        (partition_key, MetricsTuple) (reference dp_engine.py:66-109)."""
        self._check_aggregate_params(col, params, data_extractors,
                                     check_data_extractors=not isinstance(col, ColumnarData))
        self._check_backend_supports(params)
        with self._budget_accountant.scope(weight=params.budget_weight):
            self._report_generators.append(ReportGenerator(params, "aggregate", public_partitions is not None))
            if out_explain_computaton_report is not None:
                out_explain_computaton_report._set_report_generator(self._current_report_generator)
            plan = self._plan_aggregate(params, public_partitions)
            result = DPResult(self, col, params, data_extractors, public_partitions, plan)
            budget = self._budget_accountant._compute_budget_for_aggregation(params.budget_weight)
            return self._backend.annotate(result, "annotation", params=params, budget=budget)

    def _check_backend_supports(self, params):
        if not getattr(self._backend, "supports_columnar_aggregate", False):
            raise NotImplementedError("pipelinedp_amd.DPEngine runs on HipBackend (the MI355X aggregate path).")
        if params.custom_combiners:
            raise NotImplementedError("custom combiners are not part of the MI355X aggregate path")
        for m in params.metrics:
            if m.is_percentile or m == agg.Metrics.VECTOR_SUM:
                raise NotImplementedError(f"metric {m} is not part of the MI355X aggregate path")

    def _request_combiner_budgets(self, params) -> List:
        """Budget requests of create_compound_combiner (combiners.py:652-720)."""
        mech = params.noise_kind.convert_to_mechanism_type()
        metrics = set(params.metrics)
        req = lambda: self._budget_accountant.request_budget(mech, weight=params.budget_weight)  # noqa: E731
        slots = []
        if agg.Metrics.VARIANCE in metrics:
            slots.append(("variance", req()))
        elif agg.Metrics.MEAN in metrics:
            slots.append(("mean", req()))
        else:
            if agg.Metrics.COUNT in metrics:
                slots.append(("count", req()))
            if agg.Metrics.SUM in metrics:
                slots.append(("sum", req()))
        if agg.Metrics.PRIVACY_ID_COUNT in metrics:
            slots.append(("privacy_id_count", req()))
        return slots

    def _plan_aggregate(self, params, public_partitions) -> _Plan:
        """Budget requests and explain stages in the order of the reference's
        _aggregate (dp_engine.py:111-181)."""
        plan = _Plan(self._request_combiner_budgets(params))
        if public_partitions is not None and not params.public_partitions_already_filtered:
            self._add_report_stage("Public partition selection: dropped non public partitions")
        if not params.contribution_bounds_already_enforced:
            self._add_bounding_stages(params.max_partitions_contributed, params.max_contributions_per_partition)
        if public_partitions:
            self._add_report_stage("Adding empty partitions for public partitions that are missing in data")
        if public_partitions is None:
            max_rows = 1
            if params.contribution_bounds_already_enforced:
                max_rows = params.max_contributions or params.max_contributions_per_partition
            plan.max_rows_per_privacy_id = max_rows
            plan.selection_spec = self._request_selection_budget(params.partition_selection_strategy)
        for name, spec in plan.slots:
            self._add_report_stage(self._explain_combiner(name, spec))
        return plan

    def _add_bounding_stages(self, l0, linf):
        # contribution_bounders.py:77-80, 94-97 (text kept byte-identical)
        self._add_report_stage(f"Per-partition contribution bounding: for each privacy_id and each"
                               f"partition, randomly select max(actual_contributions_per_partition"
                               f", {linf}) contributions.")
        self._add_report_stage(f"Cross-partition contribution bounding: for each privacy_id "
                               f"randomly select max(actual_partition_contributed, "
                               f"{l0}) partitions")

    def _request_selection_budget(self, strategy):
        spec = self._budget_accountant.request_budget(mechanism_type=agg.MechanismType.GENERIC)
        self._add_report_stage(lambda: f"Private Partition selection: using {strategy.value} "
                               f"method with (eps={spec.eps}, delta={spec.delta})")
        return spec

    @staticmethod
    def _explain_combiner(name, spec):
        label = _EXPLAIN_NAME[name]
        return lambda: f"Computed {label} with (eps={spec.eps} delta={spec.delta})"

    # -- select_partitions -------------------------------------------------------
    def select_partitions(self, col, params: agg.SelectPartitionsParams, data_extractors: DataExtractors):
        """DP partition selection (reference dp_engine.py:204-281): per privacy
        id keep <= max_partitions_contributed distinct partitions, count
        privacy ids per partition, keep partitions by the selection strategy."""
        self._check_select_private_partitions(col, params, data_extractors)
        if not getattr(self._backend, "supports_columnar_aggregate", False):
            raise NotImplementedError("pipelinedp_amd.DPEngine runs on HipBackend.")
        with self._budget_accountant.scope(weight=params.budget_weight):
            self._report_generators.append(ReportGenerator(params, "select_partitions"))
            plan = _Plan([], self._request_selection_budget(params.partition_selection_strategy), 1)
            result = DPResult(self, col, params, data_extractors, None, plan, select_only=True)
            budget = self._budget_accountant._compute_budget_for_aggregation(params.budget_weight)
            return self._backend.annotate(result, "annotation", params=params, budget=budget)

    # -- validation (same errors as the reference) -------------------------------
    def _check_select_private_partitions(self, col, params, data_extractors):
        if col is None or not col:
            raise ValueError("col must be non-empty")
        if params is None:
            raise ValueError("params must be set to a valid SelectPrivatePartitionsParams")
        if not isinstance(params, agg.SelectPartitionsParams):
            raise TypeError("params must be set to a valid SelectPrivatePartitionsParams")
        if not isinstance(params.max_partitions_contributed, int) or params.max_partitions_contributed <= 0:
            raise ValueError("params.max_partitions_contributed must be set (to a positive integer)")
        if isinstance(col, ColumnarData):
            return
        if data_extractors is None:
            raise ValueError("data_extractors must be set to a DataExtractors")
        if not isinstance(data_extractors, DataExtractors):
            raise TypeError("data_extractors must be set to a DataExtractors")

    def _check_aggregate_params(self, col, params, data_extractors, check_data_extractors: bool = True):
        if params is not None and getattr(params, "max_contributions", None) is not None:
            raise NotImplementedError("max_contributions is not supported yet.")
        if col is None or not col:
            raise ValueError("col must be non-empty")
        if params is None:
            raise ValueError("params must be set to a valid AggregateParams")
        if not isinstance(params, agg.AggregateParams):
            raise TypeError("params must be set to a valid AggregateParams")
        if check_data_extractors:
            if data_extractors is None:
                raise ValueError("data_extractors must be set to a DataExtractors")
            if not isinstance(data_extractors, DataExtractors):
                raise TypeError("data_extractors must be set to a DataExtractors")
        if params.contribution_bounds_already_enforced:
            if data_extractors is not None and data_extractors.privacy_id_extractor:
                raise ValueError("privacy_id_extractor should be set iff "
                                 "contribution_bounds_already_enforced is False")
            if agg.Metrics.PRIVACY_ID_COUNT in params.metrics:
                raise ValueError("PRIVACY_ID_COUNT cannot be computed when "
                                 "contribution_bounds_already_enforced is True.")
