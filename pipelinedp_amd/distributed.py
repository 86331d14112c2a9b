"""Multi-GPU execution: one process per GPU, rows sharded by privacy id.

Bounding is per privacy id, so once every row of a privacy id lives on one
rank (rank = shard_of(pid)), contribution bounding is rank-local
(contribution_bounders.py:87-92 groups by pid).  Each rank reduces its rows
to dense per-partition partials over all P partitions, with the sums in K4's
exported 64-bit fixed point (pdp_bound_accumulate_partials); ONE int64 SUM
reduce-scatter of all partial arrays leaves rank r with the exact integer
sums of partition block [r*B, (r+1)*B), which are converted to fp64 once
there (pdp_finalize_partials).  Counts AND sums are therefore identical bit
for bit to a one-GPU run, whatever the world size or the collective's
reduction order (the fixed-order merge of combine_accumulators_per_key,
pipeline_backend.py:528-538).  Selection and noise run once on the owner;
Philox counters use the global partition id, so released values do not
depend on the rank count either.

The collective backend is whatever ``torch.distributed`` was initialised
with: ``nccl`` (= RCCL over xGMI on MI355X) for GPUs, ``gloo`` in CPU tests.

Restriction: the exported partials need K4's fixed point, which runs for
every input except a rank-local share of >= 2^32 rows with L_inf >= 131072
(and the testing-only debug flag NO_K4).  World.aggregate checks this before
any collective and raises ValueError, on every rank alike (the condition
depends only on the bounds and the agreed row counts); there is no fp64
fallback, whose sums would depend on the reduction order.
"""
import dataclasses
from typing import Optional

PID_SHARD_SALT = 0x9E3779B97F4A7C15
K4_MAX_LINF_BEYOND_2_32 = 131072  # pdp_kernels.hip k4_enabled: (2^32) / kK4Chunk


def shard_of(pid, world_size: int):
    """Rank owning a (dense) privacy id: splitmix64(pid ^ salt) % world_size
    (numpy / torch int64 arrays or ints)."""
    import numpy as np
    x = np.asarray(pid, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x ^ np.uint64(PID_SHARD_SALT)
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z % np.uint64(world_size)).astype(np.int64)


@dataclasses.dataclass
class World:
    """Process group view: ``rank``/``size`` and the torch.distributed group."""
    rank: int
    size: int
    group: Optional[object] = None

    @classmethod
    def from_env(cls, backend: Optional[str] = None):
        import os
        import torch.distributed as dist
        if not dist.is_initialized():
            dist.init_process_group(backend=backend or ("nccl" if _has_gpu() else "gloo"))
        return cls(dist.get_rank(), dist.get_world_size(), None)

    def block(self, num_partitions: int):
        """Partition block owned by this rank: (offset, length, padded P)."""
        b = (num_partitions + self.size - 1) // self.size
        off = min(self.rank * b, num_partitions)
        return off, max(0, min(b, num_partitions - off)), b * self.size

    def check_same(self, value: int, what: str, device=None):
        """All ranks must agree on `value` (e.g. the number of partitions of
        the dense key space they reduce-scatter); raises otherwise."""
        import torch
        import torch.distributed as dist
        t = torch.tensor([int(value), -int(value)], dtype=torch.int64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        if int(t[0]) != -int(t[1]):
            raise ValueError(f"ranks disagree on {what}: {int(value)} here, range [{-int(t[1])}, {int(t[0])}]")

    def shuffle_by_privacy_id(self, ex, pid, pk, value):
        """Moves every row to rank shard_of(pid): pdp_shard_rows groups the
        local rows by destination (stable), then one all-to-all per column
        (RCCL over xGMI on GPUs).  Rank r receives rank 0's rows for it first,
        then rank 1's, ...: the input order of the concatenated ranks is kept
        within every privacy id, so the bounding result equals one process
        over the concatenated input (the reference's group-by-pid shuffle,
        pipeline_backend.py:261,401,476-485)."""
        import torch
        import torch.distributed as dist
        spid, spk, sval, counts = ex.shard_rows(pid, pk, value, self.size)
        send = torch.tensor(counts, dtype=torch.int64, device=pk.device)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        out_splits = [int(x) for x in recv.tolist()]
        total = sum(out_splits)

        def move(t):
            if t is None:
                return None
            out = t.new_empty(total)
            dist.all_to_all_single(out, t.contiguous(), out_splits, counts, group=self.group)
            return out

        return move(spid), move(spk), move(sval)

    @staticmethod
    def key_owner(h, size: int):
        """Rank owning a privacy-id key hash (int64 tensor of hash word 0):
        ranks own contiguous ranges of the signed hash order, rank 0 the
        lowest."""
        hi = ((h >> 32) & 0xFFFFFFFF) ^ 0x80000000
        return (hi * size) >> 32

    def exchange_by_key_hash(self, h, pk, value):
        """Rows of host-encoded input (columnar.encode_rows with a world) ->
        the rank owning their privacy-id key hash, then dense privacy ids there.
        ``h`` is the rows' [N, 2] int64 hash pairs (columnar.key_hashes); word 0
        picks the owner, and the owner numbers its distinct PAIRS in ascending
        (word 0, word 1) order, offset by the distinct counts of the lower ranks
        (one all-gather of one integer): two keys that share word 0 but not
        word 1 stay two privacy ids.  No key crosses a rank.  The numbering
        equals one process's (columnar.dense_ids_from_hashes /
        dense_ids_exact), and rank r receives rank 0's rows for it first, then
        rank 1's, ...: within a privacy id the concatenated input order is
        kept, so bounding equals one process over the concatenated input
        (pipeline_backend.py:476-485).
        -> (pid, pk, value, num_privacy_ids, pid_base): the rank's ids are
        returned rebased to [0, num_privacy_ids) = its own distinct count, with
        pid_base = the lower ranks' count, so the library hashes pid_base + pid
        (BoundConfig.pid_base, ABI 3) -- the global numbering's result -- while
        sizing the L0 pre-filter by the rank's own ids."""
        import torch
        import torch.distributed as dist
        h = h.reshape(-1, 2)
        dest = self.key_owner(h[:, 0], self.size)
        order = torch.argsort(dest, stable=True)
        counts = torch.bincount(dest, minlength=self.size).to(torch.int64)
        recv = torch.empty_like(counts)
        dist.all_to_all_single(recv, counts, group=self.group)
        in_splits, out_splits = [int(x) for x in counts.tolist()], [int(x) for x in recv.tolist()]
        total = sum(out_splits)

        def move(t):
            if t is None:
                return None
            out = t.new_empty(total)
            dist.all_to_all_single(out, t[order].contiguous(), out_splits, in_splits, group=self.group)
            return out

        h0, h1, pkr, vr = move(h[:, 0]), move(h[:, 1]), move(pk), move(value)
        # ids = rank of (h0, h1) among the distinct received pairs: lexicographic order by two stable sorts
        o = torch.argsort(h1, stable=True)
        o = o[torch.argsort(h0[o], stable=True)]
        new = torch.ones(total, dtype=torch.bool, device=h.device)
        if total > 1:
            new[1:] = (h0[o][1:] != h0[o][:-1]) | (h1[o][1:] != h1[o][:-1])
        ids = torch.empty(total, dtype=torch.int64, device=h.device)
        ids[o] = torch.cumsum(new.to(torch.int64), 0) - 1
        mine = torch.tensor([int(new.sum().item()) if total else 0], dtype=torch.int64, device=h.device)
        every = [torch.empty_like(mine) for _ in range(self.size)]
        dist.all_gather(every, mine, group=self.group)
        n_each = [int(x.item()) for x in every]
        return ids, pkr, vr, n_each[self.rank], sum(n_each[:self.rank])

    def reduce_scatter_partials(self, parts, num_partitions: int):
        """Sums the ranks' fixed-point partials (int64, exact) and returns the
        owned block's as an executor.Partials of B = padded / size partitions.
        Each field's row is already rank-major (rank r owns columns
        [r*B, (r+1)*B)), so one reduce_scatter_tensor per field (K <= 7) runs
        on the row in place: no re-layout copy.  Partials allocated with
        ``padded`` columns (aggregate does) need no padding copy either."""
        import torch
        import torch.distributed as dist

        from .executor import Partials
        _, _, padded = self.block(num_partitions)
        b = padded // self.size
        data = parts.data
        k = data.shape[0]
        if data.shape[1] < padded:
            data = torch.cat([data[:, :num_partitions], data.new_zeros((k, padded - num_partitions))], dim=1)
        elif data.shape[1] > num_partitions:
            data[:, num_partitions:padded].zero_()  # padding columns sum to zero
        dst = data.new_empty((k, b))
        for i in range(k):
            dist.reduce_scatter_tensor(dst[i], data[i, :padded], op=dist.ReduceOp.SUM, group=self.group)
        return Partials(dst, parts.fields, b)

    def aggregate(self, ex, pid, pk, value, num_privacy_ids, num_partitions, bounds, rel, gather=True,
                  shuffle=False):
        """Rank-local bound+accumulate, reduce-scatter, owner-side release.

        ``shuffle``: first move every row to rank shard_of(pid)
        (``shuffle_by_privacy_id``); without it the rows must already be
        sharded by privacy id.  Returns (keep [P], metrics [F, P], fields) of
        ALL partitions on every rank when ``gather`` (all-gather of the owned
        blocks), else of the owned block only.  The rank-local accumulate is
        synchronous: its partials are complete before they are reduce-scattered
        and released (an input that needs the generic path is finished)."""
        return self._aggregate(ex, pid, pk, value, num_privacy_ids, num_partitions, bounds, rel, gather, shuffle,
                               True)

    def aggregate_async(self, ex, pid, pk, value, num_privacy_ids, num_partitions, bounds, rel, gather=False):
        """Benchmark / graph-capture form of ``aggregate`` (rows already sharded
        by privacy id): the rank-local accumulate does not wait for its stream,
        so the reduce-scatter and release are enqueued before any rank knows
        whether its input needed the generic path.  The outputs are valid only
        after ``check_async_status(ex)`` returned on every rank once the
        streams drained; it raises (on every rank) when one rank reported
        ERR_NEEDS_SYNC or an error -- then run ``aggregate`` instead.  Not part
        of the DPEngine path."""
        return self._aggregate(ex, pid, pk, value, num_privacy_ids, num_partitions, bounds, rel, gather, False,
                               False)

    def check_async_status(self, ex, device=None):
        """All ranks' ``ex.status()`` after ``aggregate_async`` (streams drained):
        raises native.NativeError everywhere if any rank's is not 0."""
        import torch
        import torch.distributed as dist

        from . import native
        st = int(ex.status())
        t = torch.tensor([-st], dtype=torch.int64, device=device)  # codes are <= 0: MAX of the negation
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        worst = -int(t.item())
        if worst != 0:
            raise native.NativeError(f"aggregate_async: a rank's accumulate returned {worst} "
                                     "(ERR_NEEDS_SYNC: its input needs the generic path; use aggregate())")

    def _aggregate(self, ex, pid, pk, value, num_privacy_ids, num_partitions, bounds, rel, gather, shuffle, sync):
        import torch
        import torch.distributed as dist
        if shuffle and pid is not None:
            pid, pk, value = self.shuffle_by_privacy_id(ex, pid, pk, value)
        linf = int(getattr(bounds, "max_contributions_per_partition", 1) or 1)
        if linf >= K4_MAX_LINF_BEYOND_2_32:
            n_local = torch.tensor([int(pk.numel()) if pk is not None else 0], dtype=torch.int64)
            if dist.get_backend(self.group) == "nccl":
                n_local = n_local.cuda()
            dist.all_reduce(n_local, op=dist.ReduceOp.MAX, group=self.group)
            if int(n_local.item()) >= 1 << 32:
                raise ValueError(f"multi-GPU partials need K4's fixed point: a rank-local share of >= 2^32 rows "
                                 f"needs max_contributions_per_partition < {K4_MAX_LINF_BEYOND_2_32} (got {linf})")
        off, length, padded = self.block(num_partitions)
        parts = ex.accumulate_partials(pid, pk, value, num_privacy_ids, num_partitions, bounds, sync=sync,
                                       padded=padded)
        owned = self.reduce_scatter_partials(parts, num_partitions)
        block_acc = ex.finalize_partials(owned, bounds)
        keep, out, fields = ex.release(block_acc, rel, bounds, pk_offset=off, num_partitions=padded // self.size)
        if not gather:
            return keep[:length], out[:, :length], fields
        b = padded // self.size
        keep_all = keep.new_empty(padded)
        dist.all_gather_into_tensor(keep_all, keep.contiguous()[:b], group=self.group)
        f = out.shape[0]
        # concatenated along dim 0 ((size*F, B): the layout every backend accepts)
        out_all = out.new_empty((self.size * f, b))
        dist.all_gather_into_tensor(out_all, out[:, :b].contiguous(), group=self.group)
        out_all = out_all.reshape(self.size, f, b).permute(1, 0, 2).reshape(f, padded)
        return keep_all[:num_partitions], out_all[:, :num_partitions], fields


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
