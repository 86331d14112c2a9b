"""CPU stand-in for ``pipelinedp_amd.executor.HipExecutor`` -- TEST
INFRASTRUCTURE ONLY.

Implements the executor interface (accumulate / release / shard_rows) on CPU
torch tensors with the numpy oracle, so that the host logic around the HIP
library -- DPEngine's lazy result, the multi-rank dictionary agreement, the
privacy-id shuffle, reduce-scatter and owner-side release of
``pipelinedp_amd/distributed.py`` -- can run under gloo in the CPU suite.
The product never imports this: HipBackend builds a HipExecutor, which
fails loudly without a GPU; tests inject this object instead.
"""
import numpy as np

import pdp_oracle as o
from pipelinedp_amd import native

_NAMES = ((native.METRIC_VARIANCE, "variance"), (native.METRIC_MEAN, "mean"), (native.METRIC_COUNT, "count"),
          (native.METRIC_SUM, "sum"), (native.METRIC_PRIVACY_ID_COUNT, "privacy_id_count"))
_SLOTS = {"count": native.MECH_COUNT, "sum": native.MECH_SUM, "mean": native.MECH_MEAN,
          "variance": native.MECH_VARIANCE, "privacy_id_count": native.MECH_PRIVACY_ID_COUNT}
_SEL = {native.SELECTION_TRUNCATED_GEOMETRIC: "truncated_geometric", native.SELECTION_LAPLACE: "laplace",
        native.SELECTION_GAUSSIAN: "gaussian"}


def _bound_params(b):
    return o.BoundParams(b.max_partitions_contributed, b.max_contributions_per_partition, b.min_value, b.max_value,
                         b.min_sum_per_partition, b.max_sum_per_partition, b.bounds_already_enforced)


class _Acc:

    def __init__(self, torch, acc, mask, P):
        self.num_partitions = P
        mean_like = mask & (native.METRIC_MEAN | native.METRIC_VARIANCE)
        self.row_count = torch.from_numpy(acc.row_count.astype(np.int64))
        self.count = torch.from_numpy(acc.count.astype(np.int64))
        self.x = torch.from_numpy(np.asarray(acc.nsum if mean_like else acc.sum, np.float64))
        self.y = torch.from_numpy(np.asarray(acc.nsumsq, np.float64))


class CpuExecutor:

    def __init__(self):
        import torch
        self.torch = torch
        self.device = torch.device("cpu")
        self.calls = []

    def accumulate(self, pid, pk, value, num_privacy_ids, num_partitions, cfg, acc=None, sync=True):
        self.calls.append(("accumulate", int(pk.numel())))
        acc = o.bound_and_accumulate(None if pid is None else pid.numpy() + int(getattr(cfg, 'pid_base', 0)), pk.numpy(),
                                     None if value is None else value.numpy(), num_partitions, _bound_params(cfg),
                                     "hash", seed=cfg.sampling_seed or 0)
        # the per-partition merge in K4's fixed point, as the GPU sums (pdp_reduce.inc)
        bp, m = _bound_params(cfg), cfg.metrics_mask
        x, y = o.k4_finalize(o.k4_partials(acc, num_partitions, bp, m), bp, m)
        if x is not None:
            if m & (native.METRIC_MEAN | native.METRIC_VARIANCE):
                acc.nsum = x
            else:
                acc.sum = x
        if y is not None:
            acc.nsumsq = y
        return _Acc(self.torch, acc, cfg.metrics_mask, num_partitions)

    def accumulate_partials(self, pid, pk, value, num_privacy_ids, num_partitions, cfg, sync=True, padded=None):
        """pdp_bound_accumulate_partials restated: the oracle's kept pairs in
        K4's exported fixed point (pdp_oracle.k4_partials)."""
        from pipelinedp_amd.executor import Partials
        self.calls.append(("accumulate", int(pk.numel())))
        acc = o.bound_and_accumulate(None if pid is None else pid.numpy() + int(getattr(cfg, 'pid_base', 0)), pk.numpy(),
                                     None if value is None else value.numpy(), num_partitions, _bound_params(cfg),
                                     "hash", seed=cfg.sampling_seed or 0)
        parts = o.k4_partials(acc, num_partitions, _bound_params(cfg), cfg.metrics_mask)
        fields = Partials.fields_for(cfg.metrics_mask)
        return Partials(self.torch.from_numpy(np.stack([parts[f] for f in fields])), fields, num_partitions)

    def finalize_partials(self, parts, cfg):
        """pdp_finalize_partials restated (pdp_oracle.k4_finalize)."""
        torch = self.torch
        d = {f: parts.row(f).numpy() for f in parts.fields}
        x, y = o.k4_finalize(d, _bound_params(cfg), cfg.metrics_mask)

        class A:
            pass

        a = A()
        a.num_partitions = parts.num_partitions
        a.row_count = parts.row("row_count")
        a.count = parts.row("count")
        a.x = None if x is None else torch.from_numpy(x)
        a.y = None if y is None else torch.from_numpy(y)
        return a

    def release(self, acc, cfg, bounds, pk_offset=0, num_partitions=None):
        torch = self.torch
        P = acc.num_partitions if num_partitions is None else int(num_partitions)
        mask = cfg.metrics_mask
        names = tuple(n for bit, n in _NAMES if mask & bit)
        budgets = {n: (cfg.eps[s], cfg.delta[s]) for n, s in _SLOTS.items() if n in names}
        sel = _SEL.get(cfg.selection)
        spec = o.ReleaseSpec(names, "gaussian" if cfg.noise_kind == native.NOISE_GAUSSIAN else "laplace", budgets, sel,
                             (cfg.eps[native.MECH_SELECTION], cfg.delta[native.MECH_SELECTION]),
                             cfg.max_rows_per_privacy_id)
        mean_like = mask & (native.METRIC_MEAN | native.METRIC_VARIANCE)
        x = acc.x.numpy()[:P] if acc.x is not None else np.zeros(P)
        y = acc.y.numpy()[:P] if acc.y is not None else np.zeros(P)
        z = np.zeros(P)
        oacc = o.Accumulators(acc.row_count.numpy()[:P], acc.count.numpy()[:P] if acc.count is not None else z,
                              z if mean_like else x, x if mean_like else z, y)
        keep, out = o.release(oacc, _bound_params(bounds), spec, seed=cfg.noise_seed or 0, noise=cfg.add_noise,
                              pk_idx=np.arange(pk_offset, pk_offset + P))
        fields = o.metric_field_order(names)
        metrics = np.stack([out[f] for f in fields]) if fields else np.zeros((1, P))
        return torch.from_numpy(keep.astype(np.uint8)), torch.from_numpy(metrics), fields

    def shard_rows(self, pid, pk, value, world_size):
        """pdp_shard_rows restated: stable grouping by shard_of(pid)."""
        from pipelinedp_amd.distributed import shard_of
        torch = self.torch
        dest = shard_of(pid.numpy(), world_size)
        order = np.argsort(dest, kind="stable")
        counts = np.bincount(dest, minlength=world_size).tolist()
        take = lambda t: None if t is None else torch.from_numpy(np.ascontiguousarray(t.numpy()[order]))  # noqa
        return take(pid), take(pk), take(value), counts

    # -- utility analysis (pdp_utility_analysis restated) -------------------
    def analyze(self, pid, pk, value, num_privacy_ids, num_partitions, metrics_mask, cfgs,
                num_sampled_partitions=None, pre_count=None, pre_n_partitions=None):
        import pdp_analysis_oracle as ao
        torch = self.torch
        P = int(num_partitions)
        sel = {native.SELECTION_NONE: None, **_SEL}
        ocfgs = [ao.AnalysisConfig(c.max_partitions_contributed, c.max_contributions_per_partition,
                                   c.min_sum_per_partition, c.max_sum_per_partition, sel[c.selection],
                                   c.selection_eps, c.selection_delta) for c in cfgs]
        public = ocfgs[0].selection is None
        if pre_count is not None:
            ppk = pk.numpy()
            keep = (ppk >= 0) & (ppk < P)
            pairs = (ppk[keep], pre_count.numpy()[keep], value.numpy()[keep], pre_n_partitions.numpy()[keep])
        else:
            pairs = ao.preaggregate(pid.numpy(), pk.numpy(), None if value is None else value.numpy(),
                                    num_sampled=num_sampled_partitions)
        names = [m for m, bit in (("sum", native.METRIC_SUM), ("count", native.METRIC_COUNT),
                                  ("privacy_id_count", native.METRIC_PRIVACY_ID_COUNT)) if metrics_mask & bit]
        out = ao.per_partition(*pairs, P, ocfgs, names, public=public)
        metrics = np.stack([np.stack([out[m][c] for m in names]) for c in range(len(ocfgs))])
        prob = None if public else torch.from_numpy(out["prob_keep"])
        pids = np.bincount(pairs[0], minlength=P).astype(np.int64)
        return torch.from_numpy(metrics), prob, torch.from_numpy(pids)

    def aggregate_errors(self, metrics, prob_keep, privacy_ids, metrics_mask, std_noise, noise_kinds, quantiles,
                         private):
        """pdp_utility_aggregate restated with pdp_analysis_oracle.aggregate_accumulator."""
        import pdp_analysis_oracle as ao
        torch = self.torch
        m = metrics.numpy()
        C, nb, _, P = m.shape
        names = [n for n, bit in (("sum", native.METRIC_SUM), ("count", native.METRIC_COUNT),
                                  ("privacy_id_count", native.METRIC_PRIVACY_ID_COUNT)) if metrics_mask & bit]
        present = np.flatnonzero(privacy_ids.numpy() > 0) if private else np.arange(P)
        prob = prob_keep.numpy() if private else None
        Q = len(quantiles)
        errors = np.zeros((C, nb, native.AGG_NUM_FIELDS + 2 * Q))
        for c in range(C):
            kind = "gaussian" if noise_kinds[c] == native.NOISE_GAUSSIAN else "laplace"
            for b, name in enumerate(names):
                acc = ao.aggregate_accumulator(name, m[c, b][:, present], None if prob is None else prob[0, present],
                                               std_noise[c][b], kind, tuple(quantiles))
                errors[c, b] = [acc[f] for f in ao.ACC_FIELDS] + acc["error_quantiles"] + acc["rel_error_quantiles"]
        sel = None
        if private:
            sel = np.array([[len(present), prob[c, present].sum(), (prob[c, present] * (1 - prob[c, present])).sum()]
                            for c in range(C)])
            sel = torch.from_numpy(sel)
        return torch.from_numpy(errors), sel
