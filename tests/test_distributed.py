"""Multi-process path (pipelinedp_amd/distributed.py) on CPU: world_size 2 over
gloo on 127.0.0.1, the same World.aggregate code the RCCL bench runs.

Each rank bounds/accumulates only the rows of its privacy ids (rank =
shard_of(pid)), the dense partials are reduce-scattered, the owned partition
block is released with global partition ids, and the blocks are
all-gathered.  The per-rank compute is the CPU oracle (test-only stand-in
for HipExecutor, same accumulate/release interface): what is under test is
the sharding, the collectives and the block bookkeeping.  Expected result:
one single-process oracle run over all rows.  Counts, privacy-id counts and
keep decisions bit-exact; fp64 sums to 1e-9 relative (summation order);
noisy outputs with identical Philox draws to 1e-9.
"""
import os
import socket

import numpy as np
import pytest

import pdp_oracle as o

N, U, P = 30000, 900, 257  # P not divisible by the world size: padded last block
BP = o.BoundParams(3, 2, 0.0, 10.0)
SPEC = o.ReleaseSpec(("mean", "count", "sum", "privacy_id_count"), "laplace",
                     {"mean": (0.5, 0.0), "privacy_id_count": (0.25, 0.0)}, "truncated_geometric", (2.0, 1e-3))
FIELDS = ["mean", "count", "sum", "privacy_id_count"]  # create_compound_combiner order for this mask


def _rows():
    return o.synth_rows(N, U, P, seed=17, zipf_s=1.1)


class OracleExecutor:
    """accumulate / release with HipExecutor's signatures, computed by the
    CPU oracle on torch CPU tensors (test infrastructure only)."""

    def accumulate(self, pid, pk, value, num_privacy_ids, num_partitions, bounds):
        import torch
        acc = o.bound_and_accumulate(pid.numpy(), pk.numpy(), value.numpy(), num_partitions, BP, "hash", seed=5)

        class A:
            pass

        a = A()
        a.num_partitions = num_partitions
        a.row_count = torch.from_numpy(acc.row_count.astype(np.int64))
        a.count = torch.from_numpy(acc.count.astype(np.int64))
        a.x = torch.from_numpy(acc.nsum.astype(np.float64))
        a.y = None
        return a

    def release(self, acc, rel, bounds, pk_offset=0, num_partitions=None):
        import torch
        Pb = int(num_partitions)
        z = np.zeros(Pb)
        oacc = o.Accumulators(acc.row_count.numpy()[:Pb], acc.count.numpy()[:Pb], z, acc.x.numpy()[:Pb], z)
        keep, out = o.release(oacc, BP, SPEC, seed=9, pk_idx=np.arange(pk_offset, pk_offset + Pb))
        metrics = np.stack([out[f] for f in FIELDS])
        return torch.from_numpy(keep.astype(np.uint8)), torch.from_numpy(metrics), FIELDS


def _worker(rank, world_size, port, outdir):
    import torch
    import torch.distributed as dist

    from pipelinedp_amd.distributed import World, shard_of
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world_size)
    try:
        pid, pk, val = _rows()
        mine = shard_of(pid, world_size) == rank
        w = World(rank, world_size)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a[mine]))  # noqa: E731
        keep, out, fields = w.aggregate(OracleExecutor(), t(pid), t(pk), t(val), U, P, None, None, gather=True)
        acc = OracleExecutor().accumulate(t(pid), t(pk), t(val), U, P, None)
        owned = w.reduce_scatter_accumulators(acc, P)
        off, length, _ = w.block(P)
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), keep=keep.numpy(), out=out.numpy(),
                 rows=np.int64(mine.sum()), off=off, length=length, row_count=owned[0].numpy()[:length])
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module")
def two_rank_run(tmp_path_factory):
    import torch.multiprocessing as mp
    outdir = str(tmp_path_factory.mktemp("dist"))
    mp.spawn(_worker, args=(2, _free_port(), outdir), nprocs=2, join=True)
    return [dict(np.load(os.path.join(outdir, f"rank{r}.npz"))) for r in range(2)]


def test_shard_of_is_deterministic_and_balanced():
    from pipelinedp_amd.distributed import shard_of
    pid = np.arange(100000)
    s = shard_of(pid, 8)
    assert np.array_equal(s, shard_of(pid, 8))
    assert s.min() == 0 and s.max() == 7
    counts = np.bincount(s, minlength=8)
    assert np.all(np.abs(counts - 12500) < 5 * np.sqrt(12500))


def test_world_block_covers_partitions():
    from pipelinedp_amd.distributed import World
    for size in (1, 2, 3, 8):
        for P_ in (1, 7, 257, 1000):
            blocks = [World(r, size).block(P_) for r in range(size)]
            covered = np.concatenate([np.arange(off, off + ln) for off, ln, _ in blocks])
            assert np.array_equal(covered, np.arange(P_))
            assert all(pad == blocks[0][2] and pad >= P_ for _, _, pad in blocks)


def test_two_ranks_shard_all_rows(two_rank_run):
    assert sum(int(r["rows"]) for r in two_rank_run) == N
    assert min(int(r["rows"]) for r in two_rank_run) > N // 4


def test_two_ranks_match_single_process(two_rank_run):
    pid, pk, val = _rows()
    acc = o.bound_and_accumulate(pid, pk, val, P, BP, "hash", seed=5)
    keep, out = o.release(acc, BP, SPEC, seed=9)
    for r in two_rank_run:  # every rank holds the gathered result
        assert np.array_equal(r["keep"].astype(bool), keep)
        for i, f in enumerate(FIELDS):
            np.testing.assert_allclose(r["out"][i], out[f], rtol=1e-9, atol=1e-9, err_msg=f)
    # the reduce-scattered privacy-id counts are exact on each owned block
    for r in two_rank_run:
        off, ln = int(r["off"]), int(r["length"])
        assert np.array_equal(r["row_count"], acc.row_count[off:off + ln])
