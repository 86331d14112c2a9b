"""Device-side execution of the aggregate path through libpdp_hip.so.

``HipExecutor`` owns one pdp_ctx, a cached device workspace and the stream
it launches on (torch's current stream of the device).  Torch is used for
device memory and streams only; all compute is in the HIP library.
"""
import ctypes
import dataclasses
import secrets
from typing import List, Optional, Sequence

from . import native


@dataclasses.dataclass
class BoundConfig:
    """Bounding parameters (AggregateParams subset)."""
    metrics_mask: int
    max_partitions_contributed: int
    max_contributions_per_partition: int
    min_value: Optional[float] = None
    max_value: Optional[float] = None
    min_sum_per_partition: Optional[float] = None
    max_sum_per_partition: Optional[float] = None
    bounds_already_enforced: bool = False
    sampling_seed: Optional[int] = None
    debug_force_fallback: bool = False
    debug_flags: int = 0
    debug_flags2: int = 0  # pdp_bound_params.reserved2 (testing: DEBUG2_* in native.py)
    # the pid columns hold (privacy id - pid_base); the sampling hashes pid_base + pid (ABI 3): a rank passes
    # its contiguous range of global ids rebased to [0, U_local) and gets the global ids' result
    pid_base: int = 0


@dataclasses.dataclass
class ReleaseConfig:
    """Noise / selection parameters after compute_budgets()."""
    metrics_mask: int
    noise_kind: int
    selection: int
    eps: Sequence[float]
    delta: Sequence[float]
    max_rows_per_privacy_id: int = 1
    add_noise: bool = True
    noise_seed: Optional[int] = None


c_void = ctypes.c_void_p


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class Accumulators:
    """Dense per-partition accumulators on the device."""

    def __init__(self, torch, num_partitions: int, device, metrics_mask: int, counts=None):
        """counts: (row_count, count) tensors to use instead of allocating them (finalize_partials
        reuses the summed partials' rows)."""
        m = metrics_mask
        i64, f64 = torch.int64, torch.float64
        P = max(int(num_partitions), 1)
        self.num_partitions = int(num_partitions)
        need_count = bool(m & (native.METRIC_COUNT | native.METRIC_MEAN | native.METRIC_VARIANCE))
        need_x = bool(m & (native.METRIC_SUM | native.METRIC_MEAN | native.METRIC_VARIANCE))
        if counts is not None:
            self.row_count, self.count = counts[0], counts[1] if need_count else None
        else:
            self.row_count = torch.empty(P, dtype=i64, device=device)
            self.count = torch.empty(P, dtype=i64, device=device) if need_count else None
        self.x = torch.empty(P, dtype=f64, device=device) if need_x else None
        self.y = torch.empty(P, dtype=f64, device=device) if m & native.METRIC_VARIANCE else None

    def tensors(self):
        return [t for t in (self.row_count, self.count, self.x, self.y) if t is not None]

    def as_struct(self, offset: int = 0) -> native.Accumulators:

        def p(t):
            return ctypes.c_void_p(t.data_ptr() + 8 * offset) if t is not None else None

        return native.Accumulators(p(self.row_count), p(self.count), p(self.x), p(self.y))


class Partials:
    """Per-partition partials in K4's exported 64-bit fixed point
    (pdp_bound_accumulate_partials): one int64 tensor ``data`` [K, P] whose
    rows are ``fields`` (row_count, count, x_hi, x_lo, y_hi, y_lo, nan as the
    metrics need them).  Partials of several ranks add up exactly (an int64
    SUM), and finalize() converts the sum once."""

    def __init__(self, data, fields, num_partitions: int):
        self.data = data
        self.fields = list(fields)
        self.num_partitions = int(num_partitions)

    @staticmethod
    def fields_for(metrics_mask: int):
        m = metrics_mask
        f = ["row_count"]
        if m & (native.METRIC_COUNT | native.METRIC_MEAN | native.METRIC_VARIANCE):
            f.append("count")
        if m & (native.METRIC_SUM | native.METRIC_MEAN | native.METRIC_VARIANCE):
            f += ["x_hi", "x_lo", "nan"]
        if m & native.METRIC_VARIANCE:
            f += ["y_hi", "y_lo"]
        return f

    def row(self, name):
        return self.data[self.fields.index(name)] if name in self.fields else None

    def as_struct(self) -> native.Partials:

        def p(name):
            t = self.row(name)
            return ctypes.c_void_p(t.data_ptr()) if t is not None else None

        return native.Partials(p("row_count"), p("count"), p("x_hi"), p("x_lo"), p("y_hi"), p("y_lo"), p("nan"))


class HipExecutor:

    def __init__(self, device=None):
        import torch
        if not torch.cuda.is_available():
            raise native.NativeError("HipBackend needs a ROCm GPU (torch.cuda.is_available() is False); "
                                     "the aggregate path has no CPU fallback.")
        self.torch = torch
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.lib = native.lib()
        self.ctx = self.lib.pdp_ctx_create(self.device.index)
        self._ws = None

    def __del__(self):
        try:
            if getattr(self, "ctx", None):
                self.lib.pdp_ctx_destroy(self.ctx)
        except Exception:
            pass

    @property
    def stream_handle(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def _workspace(self, nbytes: int):
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = None
            self._ws = self.torch.empty(max(nbytes, 256), dtype=self.torch.uint8, device=self.device)
        return self._ws

    def _columns(self, pid, pk, value, num_privacy_ids, num_partitions):
        torch = self.torch
        n = int(pk.numel())
        for t, dt in ((pid, torch.int64), (pk, torch.int64), (value, torch.float64)):
            if t is not None:
                assert t.device == self.device and t.dtype == dt and t.is_contiguous(), (t.device, t.dtype)
                assert t.numel() == n
        return native.Columns(_ptr(pid), _ptr(pk), _ptr(value), n, int(max(num_privacy_ids, 1)),
                              int(num_partitions))

    @staticmethod
    def _bound_params(cfg: BoundConfig, flags: int = 0):
        seed = cfg.sampling_seed if cfg.sampling_seed is not None else secrets.randbits(64)
        return native.BoundParams(
            cfg.metrics_mask, int(cfg.bounds_already_enforced), cfg.max_partitions_contributed,
            cfg.max_contributions_per_partition, int(cfg.min_value is not None),
            int(cfg.min_sum_per_partition is not None),
            float(cfg.min_value or 0.0), float(cfg.max_value or 0.0),
            float(cfg.min_sum_per_partition or 0.0), float(cfg.max_sum_per_partition or 0.0),
            seed, int(cfg.debug_force_fallback), int(cfg.debug_flags), int(flags), int(cfg.debug_flags2),
            int(cfg.pid_base))

    def accumulate(self, pid, pk, value, num_privacy_ids: int, num_partitions: int, cfg: BoundConfig,
                   acc: Optional[Accumulators] = None, sync: bool = True) -> Accumulators:
        """pdp_bound_accumulate on int64 pid/pk and float64 value device tensors.
        sync=False (PDP_BOUND_ASYNC): only enqueues work on the current stream
        (hipGraph-capturable); check status() once the stream has drained."""
        cols = self._columns(pid, pk, value, num_privacy_ids, num_partitions)
        bp = self._bound_params(cfg, 0 if sync else native.BOUND_ASYNC)
        if acc is None:
            acc = Accumulators(self.torch, num_partitions, self.device, cfg.metrics_mask)
        nbytes = ctypes.c_size_t(0)
        native.check(self.lib.pdp_workspace_size(ctypes.byref(cols), ctypes.byref(bp), ctypes.byref(nbytes)),
                     "pdp_workspace_size")
        ws = self._workspace(nbytes.value)
        accs = acc.as_struct()
        native.check(self.lib.pdp_bound_accumulate(self.ctx, ctypes.byref(cols), ctypes.byref(bp), ctypes.byref(accs),
                                                   ctypes.c_void_p(ws.data_ptr()), ws.numel(), self.stream_handle),
                     "pdp_bound_accumulate")
        return acc

    def accumulate_partials(self, pid, pk, value, num_privacy_ids: int, num_partitions: int,
                            cfg: BoundConfig, sync: bool = True, padded: Optional[int] = None) -> Partials:
        """pdp_bound_accumulate_partials: the rank-local accumulate of the
        multi-GPU path, sums in exported fixed point (see Partials).
        ``padded``: allocate that many columns (>= num_partitions, the tail
        zero) so a reduce-scatter over equal rank blocks needs no copy."""
        cols = self._columns(pid, pk, value, num_privacy_ids, num_partitions)
        bp = self._bound_params(cfg, 0 if sync else native.BOUND_ASYNC)
        fields = Partials.fields_for(cfg.metrics_mask)
        P = max(int(num_partitions), 1)
        W = max(P, int(padded or 0))
        data = self.torch.empty((len(fields), W), dtype=self.torch.int64, device=self.device)
        if W > P:
            data[:, P:].zero_()
        parts = Partials(data, fields, num_partitions)
        nbytes = ctypes.c_size_t(0)
        native.check(self.lib.pdp_workspace_size(ctypes.byref(cols), ctypes.byref(bp), ctypes.byref(nbytes)),
                     "pdp_workspace_size")
        ws = self._workspace(nbytes.value)
        ps = parts.as_struct()
        native.check(self.lib.pdp_bound_accumulate_partials(self.ctx, ctypes.byref(cols), ctypes.byref(bp),
                                                            ctypes.byref(ps), ctypes.c_void_p(ws.data_ptr()),
                                                            ws.numel(), self.stream_handle),
                     "pdp_bound_accumulate_partials")
        return parts

    def finalize_partials(self, parts: Partials, cfg: BoundConfig) -> Accumulators:
        """pdp_finalize_partials: (summed) partials -> Accumulators for release."""
        P = parts.num_partitions
        acc = Accumulators(self.torch, P, self.device, cfg.metrics_mask,
                           counts=(parts.row("row_count"), parts.row("count")))
        bp = self._bound_params(cfg)
        ps, accs = parts.as_struct(), acc.as_struct()
        native.check(self.lib.pdp_finalize_partials(self.ctx, ctypes.byref(ps), P, ctypes.byref(bp),
                                                    ctypes.byref(accs), self.stream_handle), "pdp_finalize_partials")
        return acc

    def accumulate_sweep(self, pid, pk, value, num_privacy_ids: int, num_partitions: int,
                         cfgs: Sequence[BoundConfig]) -> List[Accumulators]:
        """pdp_bound_accumulate_sweep: one sort by privacy id, then bounding +
        accumulation per configuration (utility-analysis sweep over bounding
        parameters, analysis/utility_analysis_engine.py:88-173).  Result c
        equals accumulate(..., cfgs[c])."""
        cols = self._columns(pid, pk, value, num_privacy_ids, num_partitions)
        k = len(cfgs)
        if k == 0:
            return []
        bps = (native.BoundParams * k)(*[self._bound_params(c) for c in cfgs])
        out = [Accumulators(self.torch, num_partitions, self.device, c.metrics_mask) for c in cfgs]
        accs = (native.Accumulators * k)(*[a.as_struct() for a in out])
        nbytes = ctypes.c_size_t(0)
        native.check(self.lib.pdp_sweep_workspace_size(ctypes.byref(cols), ctypes.byref(nbytes)),
                     "pdp_sweep_workspace_size")
        ws = self._workspace(nbytes.value)
        native.check(self.lib.pdp_bound_accumulate_sweep(self.ctx, ctypes.byref(cols), bps, k, accs,
                                                         ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                                                         self.stream_handle),
                     "pdp_bound_accumulate_sweep")
        return out

    @staticmethod
    def _release_params(cfg: ReleaseConfig, bounds: BoundConfig):
        eps = (ctypes.c_double * native.NUM_MECH)(*cfg.eps)
        delta = (ctypes.c_double * native.NUM_MECH)(*cfg.delta)
        seed = cfg.noise_seed if cfg.noise_seed is not None else secrets.randbits(64)
        return native.ReleaseParams(
            cfg.metrics_mask, cfg.noise_kind, cfg.selection, int(cfg.add_noise), bounds.max_partitions_contributed,
            bounds.max_contributions_per_partition, int(bounds.min_value is not None),
            int(bounds.min_sum_per_partition is not None), float(bounds.min_value or 0.0),
            float(bounds.max_value or 0.0), float(bounds.min_sum_per_partition or 0.0),
            float(bounds.max_sum_per_partition or 0.0), eps, delta, int(cfg.max_rows_per_privacy_id), seed)

    def prepare_release(self, cfg: ReleaseConfig, bounds: BoundConfig):
        """pdp_prepare_release: build release's device-side table (truncated
        geometric selection) now, outside any stream capture, so that a
        release() captured in a CUDA/HIP graph enqueues kernels only."""
        rp = self._release_params(cfg, bounds)
        native.check(self.lib.pdp_prepare_release(self.ctx, ctypes.byref(rp)), "pdp_prepare_release")

    def release(self, acc: Accumulators, cfg: ReleaseConfig, bounds: BoundConfig, pk_offset: int = 0,
                num_partitions: Optional[int] = None, offset_in_acc: int = 0):
        """pdp_release -> (keep uint8 [P], metrics float64 [F, P], field names).
        Under stream capture call prepare_release() first (else NEEDS_SYNC)."""
        torch = self.torch
        P = acc.num_partitions if num_partitions is None else int(num_partitions)
        fields = native.metric_fields(cfg.metrics_mask)
        keep = torch.empty(max(P, 1), dtype=torch.uint8, device=self.device)
        out = torch.empty((max(len(fields), 1), max(P, 1)), dtype=torch.float64, device=self.device)
        rp = self._release_params(cfg, bounds)
        outs = native.Outputs(ctypes.c_void_p(keep.data_ptr()), ctypes.c_void_p(out.data_ptr()))
        accs = acc.as_struct(offset_in_acc)
        native.check(self.lib.pdp_release(self.ctx, ctypes.byref(accs), P, int(pk_offset), ctypes.byref(rp),
                                          ctypes.byref(outs), self.stream_handle), "pdp_release")
        return keep[:P], out[:, :P], fields

    def _analysis_outputs(self, cfgs, num_partitions, metrics_mask, private):
        torch = self.torch
        nb = bin(metrics_mask & (native.METRIC_SUM | native.METRIC_COUNT | native.METRIC_PRIVACY_ID_COUNT)).count("1")
        P = int(num_partitions)
        metrics = torch.empty((len(cfgs), nb, 5, P), dtype=torch.float64, device=self.device)
        prob = torch.empty((len(cfgs), P), dtype=torch.float64, device=self.device) if private else None
        pids = torch.empty(P, dtype=torch.int64, device=self.device)
        return metrics, prob, pids, native.AnalysisOutputs(_ptr(metrics), _ptr(prob), _ptr(pids))

    def analyze(self, pid, pk, value, num_privacy_ids: int, num_partitions: int, metrics_mask: int,
                cfgs: Sequence["native.AnalysisConfig"], num_sampled_partitions: Optional[int] = None,
                pre_count=None, pre_n_partitions=None):
        """pdp_utility_analysis (raw rows) or, with pre_count / pre_n_partitions,
        pdp_utility_analysis_preaggregated (pk = pair partitions, value = pair
        sums) -> (metrics [C, nb, 5, P], prob_keep [C, P] or None, privacy ids
        with data per partition [P])."""
        k = len(cfgs)
        carr = (native.AnalysisConfig * k)(*cfgs)
        private = cfgs[0].selection != native.SELECTION_NONE
        n = int(pk.numel())
        P = int(num_partitions)
        pre = pre_count is not None
        U = n if pre else int(max(num_privacy_ids, 1))
        nbytes = ctypes.c_size_t(0)
        native.check(self.lib.pdp_analysis_workspace_size(n, U, P, carr, k, ctypes.byref(nbytes)),
                     "pdp_analysis_workspace_size")
        ws = self._workspace(nbytes.value)
        metrics, prob, pids, outs = self._analysis_outputs(cfgs, P, metrics_mask, private)
        if pre:
            native.check(self.lib.pdp_utility_analysis_preaggregated(
                self.ctx, _ptr(pk), _ptr(pre_count), _ptr(value), _ptr(pre_n_partitions), n, P, metrics_mask, carr, k,
                ctypes.byref(outs), ctypes.c_void_p(ws.data_ptr()), ws.numel(), self.stream_handle),
                "pdp_utility_analysis_preaggregated")
        else:
            cols = self._columns(pid, pk, value, U, P)
            ns = P if num_sampled_partitions is None else int(num_sampled_partitions)
            native.check(self.lib.pdp_utility_analysis(self.ctx, ctypes.byref(cols), ns, metrics_mask, carr, k,
                                                       ctypes.byref(outs), ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                                                       self.stream_handle), "pdp_utility_analysis")
        return metrics, prob, pids

    def aggregate_errors(self, metrics, prob_keep, privacy_ids, metrics_mask: int, std_noise, noise_kinds,
                         quantiles, private: bool):
        """pdp_utility_aggregate: cross-partition sums of the per-partition
        utility metrics (analyze's outputs) -> (errors [C, nb, 20 + 2Q],
        selection [C, 3] or None) device tensors; field order native.AGG_FIELDS,
        then error_quantiles[Q], rel_error_quantiles[Q]."""
        torch = self.torch
        C, nb, _, P = (int(v) for v in metrics.shape)
        Q = len(quantiles)
        errors = torch.empty((C, nb, native.AGG_NUM_FIELDS + 2 * Q), dtype=torch.float64, device=self.device)
        sel = torch.empty((C, 3), dtype=torch.float64, device=self.device) if private else None
        qs = (ctypes.c_double * max(Q, 1))(*quantiles)
        sn = (ctypes.c_double * (C * nb))(*[float(v) for row in std_noise for v in row])
        nk = (ctypes.c_int32 * C)(*noise_kinds)
        ap = native.AggregateParams(C, metrics_mask, Q, 0, ctypes.cast(qs, c_void), ctypes.cast(sn, c_void),
                                    ctypes.cast(nk, c_void))
        native.check(self.lib.pdp_utility_aggregate(self.ctx, _ptr(metrics.contiguous()),
                                                    _ptr(prob_keep) if private else None,
                                                    _ptr(privacy_ids) if private else None, P, ctypes.byref(ap),
                                                    _ptr(errors), _ptr(sel), self.stream_handle),
                     "pdp_utility_aggregate")
        return errors, sel

    def preaggregate(self, pid, pk, value, num_privacy_ids: int, num_partitions: int,
                     num_sampled_partitions: Optional[int] = None):
        """pdp_preaggregate -> (pk, count, sum, n_partitions) device tensors, one
        per (privacy id, sampled partition) pair."""
        torch = self.torch
        n = int(pk.numel())
        P = int(num_partitions)
        cols = self._columns(pid, pk, value, num_privacy_ids, P)
        cfg = native.AnalysisConfig(1, 1, 0.0, 0.0, 0, 0, 0.0, 0.0)
        nbytes = ctypes.c_size_t(0)
        native.check(self.lib.pdp_analysis_workspace_size(n, int(max(num_privacy_ids, 1)), P, ctypes.byref(cfg), 1,
                                                          ctypes.byref(nbytes)), "pdp_analysis_workspace_size")
        ws = self._workspace(nbytes.value)
        m = max(n, 1)
        opk = torch.empty(m, dtype=torch.int64, device=self.device)
        ocnt = torch.empty(m, dtype=torch.int64, device=self.device)
        osum = torch.empty(m, dtype=torch.float64, device=self.device)
        onp = torch.empty(m, dtype=torch.int64, device=self.device)
        cnt = ctypes.c_int64(0)
        ns = P if num_sampled_partitions is None else int(num_sampled_partitions)
        native.check(self.lib.pdp_preaggregate(self.ctx, ctypes.byref(cols), ns, _ptr(opk), _ptr(ocnt), _ptr(osum),
                                               _ptr(onp), ctypes.byref(cnt), ctypes.c_void_p(ws.data_ptr()),
                                               ws.numel(), self.stream_handle), "pdp_preaggregate")
        k = cnt.value
        return opk[:k], ocnt[:k], osum[:k], onp[:k]

    def shard_rows(self, pid, pk, value, world_size: int):
        """pdp_shard_rows: rows grouped by destination rank shard_of(pid)
        (stable) -> (pid, pk, value, rows_per_rank list)."""
        torch = self.torch
        n = int(pk.numel())
        cols = self._columns(pid, pk, value, 1, 1)
        opid = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)[:n]
        opk = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)[:n]
        oval = torch.empty(max(n, 1), dtype=torch.float64, device=self.device)[:n] if value is not None else None
        nbytes = ctypes.c_size_t(0)
        native.check(self.lib.pdp_shard_workspace_size(n, int(world_size), ctypes.byref(nbytes)),
                     "pdp_shard_workspace_size")
        ws = torch.empty(max(nbytes.value, 256), dtype=torch.uint8, device=self.device)
        counts = (ctypes.c_int64 * int(world_size))()
        native.check(self.lib.pdp_shard_rows(self.ctx, ctypes.byref(cols), int(world_size), _ptr(opid), _ptr(opk),
                                             _ptr(oval), counts, ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                                             self.stream_handle), "pdp_shard_rows")
        return opid, opk, oval, list(counts)

    def set_debug(self, flags: int = 0):
        """pdp_ctx_set_debug (testing): alternative-form flags for every later
        call on this executor (DEBUG_* in native.py); 0 = the shipped path."""
        native.check(self.lib.pdp_ctx_set_debug(self.ctx, int(flags)), "pdp_ctx_set_debug")

    def profile(self, enable: bool = True):
        native.check(self.lib.pdp_profile_enable(self.ctx, int(enable)), "pdp_profile_enable")

    def profile_read(self, reset: bool = True):
        """-> {stage: (total ms, launches)} of the recorded kernels."""
        n = len(native.STAGES)
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_int64 * n)()
        native.check(self.lib.pdp_profile_read(self.ctx, ms, cnt, int(reset)), "pdp_profile_read")
        return {s: (ms[i], cnt[i]) for i, s in enumerate(native.STAGES)}

    def status(self) -> int:
        """pdp_get_status: 0, or the PDP_ERR_* code of the last accumulate(sync=False)
        (native.ERR_NEEDS_SYNC: redo it with sync=True).  Call after the stream drained."""
        st = ctypes.c_int32(0)
        native.check(self.lib.pdp_get_status(self.ctx, ctypes.byref(st)), "pdp_get_status")
        return int(st.value)

    def stats(self) -> native.Stats:
        s = native.Stats()
        native.check(self.lib.pdp_get_stats(self.ctx, ctypes.byref(s)), "pdp_get_stats")
        return s

    def generate(self, n: int, num_privacy_ids: int, num_partitions: int, seed: int, zipf_s: float = 0.0,
                 value_kind: int = 0, lo: float = 0.0, hi: float = 10.0, row_offset: int = 0, with_value=True):
        torch = self.torch
        pid = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)[:n]
        pk = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)[:n]
        val = torch.empty(max(n, 1), dtype=torch.float64, device=self.device)[:n] if with_value else None
        native.check(self.lib.pdp_generate_synthetic(_ptr(pid), _ptr(pk), _ptr(val), n, row_offset, num_privacy_ids,
                                                     num_partitions, zipf_s, value_kind, lo, hi, seed,
                                                     self.stream_handle), "pdp_generate_synthetic")
        return pid, pk, val
