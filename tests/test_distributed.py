"""Multi-process path (pipelinedp_amd/distributed.py) on CPU: world_size 2 over
gloo on 127.0.0.1, the same World.aggregate code the RCCL bench runs.

Each rank bounds/accumulates only the rows of its privacy ids (rank =
shard_of(pid)), the dense fixed-point partials are reduce-scattered as int64,
converted once on the owner, the owned partition block is released with
global partition ids, and the blocks are all-gathered.  The per-rank compute
is the CPU oracle (test-only stand-in for HipExecutor, same
accumulate_partials / finalize_partials / release interface, K4's fixed
point restated in pdp_oracle.k4_partials): what is under test is the
sharding, the collectives and the block bookkeeping.  Expected result: one
single-process run over all rows with the same fixed-point merge --
everything bit for bit, sums and noisy outputs included, because integer
partial sums do not depend on how the pairs are split over ranks.
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


MASK = 1 | 2 | 4 | 16


def _single_process_fixed(pid, pk, val):
    """One process over all rows, sums merged in K4's fixed point."""
    acc = o.bound_and_accumulate(pid, pk, val, P, BP, "hash", seed=5)
    x, _ = o.k4_finalize(o.k4_partials(acc, P, BP, MASK), BP, MASK)
    acc.nsum = x
    return acc


class OracleExecutor:
    """accumulate_partials / finalize_partials / release with HipExecutor's
    signatures, computed by the CPU oracle on torch CPU tensors (test
    infrastructure only)."""

    def accumulate_partials(self, pid, pk, value, num_privacy_ids, num_partitions, bounds, sync=True, padded=None):
        import torch

        from pipelinedp_amd.executor import Partials
        base = int(getattr(bounds, "pid_base", 0) or 0)  # World.aggregate's rebased ids
        acc = o.bound_and_accumulate(pid.numpy() + base, pk.numpy(), value.numpy(), num_partitions, BP, "hash", seed=5)
        parts = o.k4_partials(acc, num_partitions, BP, MASK)
        fields = Partials.fields_for(MASK)
        data = np.stack([parts[f] for f in fields])
        if padded and padded > num_partitions:  # HipExecutor's padded columns (reduce-scatter without a copy)
            data = np.concatenate([data, np.full((len(fields), padded - num_partitions), -1, np.int64)], axis=1)
        return Partials(torch.from_numpy(data), fields, num_partitions)

    def finalize_partials(self, parts, bounds):
        import torch
        x, _ = o.k4_finalize({f: parts.row(f).numpy() for f in parts.fields}, BP, MASK)

        class A:
            pass

        a = A()
        a.num_partitions = parts.num_partitions
        a.row_count, a.count = parts.row("row_count"), parts.row("count")
        a.x, a.y = torch.from_numpy(x), None
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
        parts = OracleExecutor().accumulate_partials(t(pid), t(pk), t(val), U, P, None)
        owned = w.reduce_scatter_partials(parts, P)
        x = OracleExecutor().finalize_partials(owned, None).x
        off, length, _ = w.block(P)
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), keep=keep.numpy(), out=out.numpy(),
                 rows=np.int64(mine.sum()), off=off, length=length, row_count=owned.row("row_count").numpy()[:length],
                 x=x.numpy()[:length])
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
    acc = _single_process_fixed(pid, pk, val)
    keep, out = o.release(acc, BP, SPEC, seed=9)
    for r in two_rank_run:  # every rank holds the gathered result
        assert np.array_equal(r["keep"].astype(bool), keep)
        for i, f in enumerate(FIELDS):
            np.testing.assert_array_equal(r["out"][i], out[f], err_msg=f)
    # the reduce-scattered privacy-id counts and the converted sums are exact on each owned block
    for r in two_rank_run:
        off, ln = int(r["off"]), int(r["length"])
        assert np.array_equal(r["row_count"], acc.row_count[off:off + ln])
        np.testing.assert_array_equal(r["x"], acc.nsum[off:off + ln])
    # and the fixed-point sums are the fp64 sums to 1e-12 (per-pair rounding 2^-63 max|x|)
    ref = o.bound_and_accumulate(pid, pk, val, P, BP, "hash", seed=5)
    np.testing.assert_allclose(acc.nsum, ref.nsum, rtol=1e-12, atol=1e-9)


# --- DPEngine.aggregate with a 2-rank world (gloo) ---------------------------
# Rows are dealt round-robin (NOT sharded by privacy id) and carry string keys,
# so the run exercises the cross-rank partition dictionary (columnar._global_keys),
# the num_partitions agreement, the privacy-id exchange by key hash
# (World.exchange_by_key_hash over all_to_all_single; dense ids numbered by the
# owner), reduce-scatter and owner-side release.  The HIP executor is replaced
# by tests/cpu_executor.py (oracle on CPU tensors).  Expected: one process over
# the concatenation [rank 0 rows, rank 1 rows] -- the same dense ids, the same
# privacy-id row order, hence identical sampling and Philox draws: bit for bit.


def _engine_rows():
    pid, pk, val = o.synth_rows(6000, 300, 40, seed=23, zipf_s=1.1)
    return [(f"user{a}", f"movie{b}", float(v)) for a, b, v in zip(pid, pk, val)]


def _run_engine(rows, world):
    import pipelinedp_amd as pdp
    from cpu_executor import CpuExecutor
    backend = pdp.HipBackend(world=world, sampling_seed=5, noise_seed=9)
    backend._executor = CpuExecutor()
    acct = pdp.NaiveBudgetAccountant(total_epsilon=10, total_delta=1e-3)
    engine = pdp.DPEngine(acct, backend)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.MEAN,
                                          pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=3, max_contributions_per_partition=2,
                                 min_value=0.0, max_value=10.0)
    ex = pdp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                            value_extractor=lambda r: r[2])
    res = engine.aggregate(rows, params, ex)
    acct.compute_budgets()
    return sorted((k, tuple(t)) for k, t in res), list(backend._executor.calls)


def _engine_worker(rank, world_size, port, outdir):
    import json

    import torch.distributed as dist

    from pipelinedp_amd.distributed import World
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world_size)
    try:
        rows = _engine_rows()[rank::world_size]
        out, calls = _run_engine(rows, World(rank, world_size))
        with open(os.path.join(outdir, f"engine{rank}.json"), "w") as f:
            json.dump({"out": out, "calls": calls, "rows_in": len(rows)}, f)
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def engine_two_ranks(tmp_path_factory):
    import json

    import torch.multiprocessing as mp
    outdir = str(tmp_path_factory.mktemp("engine"))
    mp.spawn(_engine_worker, args=(2, _free_port(), outdir), nprocs=2, join=True)
    return [json.load(open(os.path.join(outdir, f"engine{r}.json"))) for r in range(2)]


def test_dp_engine_two_ranks_matches_one_process(engine_two_ranks):
    rows = _engine_rows()
    concat = rows[0::2] + rows[1::2]
    want, _ = _run_engine(concat, None)
    assert len(want) > 5
    for r in engine_two_ranks:
        got = [(k, tuple(v)) for k, v in r["out"]]
        assert [k for k, _ in got] == [k for k, _ in want]
        for (_, g), (_, w) in zip(got, want):
            np.testing.assert_array_equal(g, w)


def test_dp_engine_two_ranks_shuffle_moves_rows_by_privacy_id(engine_two_ranks):
    # after the shuffle each rank bounds only its own privacy ids: the rows
    # each rank accumulates add up to all rows, and differ from what it was given
    acc_rows = [c[1] for r in engine_two_ranks for c in r["calls"] if c[0] == "accumulate"]
    assert sum(acc_rows) == len(_engine_rows())
    assert acc_rows != [r["rows_in"] for r in engine_two_ranks]


def test_world_check_same_raises_on_disagreement(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_disagree_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert sorted(os.listdir(tmp_path)) == ["raised0", "raised1"]


def _disagree_worker(rank, world_size, port, outdir):
    import torch.distributed as dist

    from pipelinedp_amd.distributed import World
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world_size)
    try:
        World(rank, world_size).check_same(10, "num_partitions")
        try:
            World(rank, world_size).check_same(10 + rank, "num_partitions")
        except ValueError:
            open(os.path.join(outdir, f"raised{rank}"), "w").close()
    finally:
        dist.destroy_process_group()


# --- scalable host encoding: 1e5 distinct privacy ids over 2 ranks -----------
# No privacy-id key crosses a rank: the rows carry their key hashes and
# World.exchange_by_key_hash moves them to the hash owner, which numbers them;
# only the partition dictionary is all-gathered.  Bitwise equal to one process.


def _many_user_rows():
    pid, pk, val = o.synth_rows(200_000, 100_000, 50, seed=29, zipf_s=1.1)
    return [(f"user{a}", f"movie{b}", float(v)) for a, b, v in zip(pid, pk, val)]


def _many_users_worker(rank, world_size, port, outdir):
    import json

    import torch.distributed as dist

    from pipelinedp_amd.distributed import World
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world_size)
    gathered = []
    real = dist.all_gather_object

    def spy(out, obj, group=None):
        gathered.append(len(obj) if hasattr(obj, "__len__") else 1)
        return real(out, obj, group=group)

    dist.all_gather_object = spy
    try:
        rows = _many_user_rows()[rank::world_size]
        out, calls = _run_engine(rows, World(rank, world_size))
        with open(os.path.join(outdir, f"many{rank}.json"), "w") as f:
            json.dump({"out": out, "calls": calls, "gathered": gathered}, f)
    finally:
        dist.all_gather_object = real
        dist.destroy_process_group()


def test_many_privacy_ids_two_ranks_no_key_exchange_bitwise(tmp_path):
    import json

    import torch.multiprocessing as mp
    mp.spawn(_many_users_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    runs = [json.load(open(os.path.join(tmp_path, f"many{r}.json"))) for r in range(2)]
    rows = _many_user_rows()
    want, _ = _run_engine(rows[0::2] + rows[1::2], None)
    assert len(want) > 20
    for r in runs:
        # one all_gather_object per rank: the partition keys (<= 50), never the 1e5 privacy-id keys
        assert len(r["gathered"]) == 1 and r["gathered"][0] <= 50, r["gathered"]
        got = [(k, tuple(v)) for k, v in r["out"]]
        assert [k for k, _ in got] == [k for k, _ in want]
        for (_, g), (_, w) in zip(got, want):
            np.testing.assert_array_equal(g, w)
    acc_rows = [c[1] for r in runs for c in r["calls"] if c[0] == "accumulate"]
    assert sum(acc_rows) == len(rows)


# --- privacy-id hash collisions across ranks -----------------------------------
# Word 0 of every key hash (the owning rank) keeps only its top 2 bits, so most
# privacy ids share word 0 with others on their rank; the owner must still tell
# them apart by word 1 (World.exchange_by_key_hash numbers distinct PAIRS).
# Bitwise equal to one process under the same patch.


def _collide_hashes(keys):
    from pipelinedp_amd import columnar
    h = columnar._real_key_hashes(keys)
    h[:, 0] = (h[:, 0] >> 62) << 62
    return h


def _patch_hashes():
    from pipelinedp_amd import columnar
    if not hasattr(columnar, "_real_key_hashes"):
        columnar._real_key_hashes = columnar.key_hashes
    columnar.key_hashes = _collide_hashes


def _unpatch_hashes():
    from pipelinedp_amd import columnar
    if hasattr(columnar, "_real_key_hashes"):
        columnar.key_hashes = columnar._real_key_hashes


def _collide_worker(rank, world_size, port, outdir):
    import json

    import torch.distributed as dist

    from pipelinedp_amd.distributed import World
    _patch_hashes()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world_size)
    try:
        rows = _engine_rows()[rank::world_size]
        out, _ = _run_engine(rows, World(rank, world_size))
        with open(os.path.join(outdir, f"collide{rank}.json"), "w") as f:
            json.dump({"out": out}, f)
    finally:
        dist.destroy_process_group()


def test_two_ranks_word0_hash_collisions_bitwise(tmp_path):
    import json

    import torch.multiprocessing as mp
    mp.spawn(_collide_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    runs = [json.load(open(os.path.join(tmp_path, f"collide{r}.json"))) for r in range(2)]
    rows = _engine_rows()
    _patch_hashes()
    try:
        from pipelinedp_amd import columnar
        enc = columnar.encode_rows(rows, __import__("pipelinedp_amd").DataExtractors(
            lambda r: r[0], lambda r: r[1], lambda r: r[2]))
        assert enc.num_privacy_ids == len({r[0] for r in rows})  # 4 word-0 values, still every user distinct
        want, _ = _run_engine(rows[0::2] + rows[1::2], None)
    finally:
        _unpatch_hashes()
    assert len(want) > 5
    for r in runs:
        got = [(k, tuple(v)) for k, v in r["out"]]
        assert [k for k, _ in got] == [k for k, _ in want]
        for (_, g), (_, w) in zip(got, want):
            np.testing.assert_array_equal(g, w)


def test_aggregate_refuses_partials_k4_cannot_make(tmp_path):
    """A rank-local share of >= 2^32 rows with L_inf >= 131072 has no fixed-point
    partials (pdp_kernels.hip k4_enabled): World.aggregate raises before any
    accumulate or data collective (world size 1, gloo; the row count is a stub)."""
    import torch
    import torch.distributed as dist

    from pipelinedp_amd.distributed import World
    from pipelinedp_amd.executor import BoundConfig

    class Huge:  # numel() only: the check must not touch the rows
        def numel(self):
            return 1 << 32

    class NoAccumulate:
        def accumulate_partials(self, *a, **k):
            raise AssertionError("must not accumulate")

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        w = World(0, 1)
        with pytest.raises(ValueError, match="2\\^32"):
            w.aggregate(NoAccumulate(), None, Huge(), None, 10, 10, BoundConfig(1, 1, 131072), None)
    finally:
        dist.destroy_process_group()
