"""Columnar input and host-side dictionary encoding.

The GPU path consumes dictionary-encoded int64 privacy-id / partition
columns and float64 values.  Rows of arbitrary Python objects are encoded
once on the host (the DataExtractors of ``dp_engine.py:27-37`` applied in
one pass, then pandas.factorize); device-resident columnar data is passed
straight through.
"""
import dataclasses
from typing import Any, Optional, Sequence

import numpy as np


@dataclasses.dataclass
class ColumnarData:
    """Already-encoded columns.

    partition:   dense partition ids in [0, num_partitions) (torch tensor on
                 the GPU or anything numpy can read); negative = drop.
    privacy_id:  dense privacy ids in [0, num_privacy_ids) (None when
                 contribution bounds are already enforced).
    value:       float64 values (None for COUNT / PRIVACY_ID_COUNT).
    partition_keys: optional original key of each dense partition id; when
                 given, public_partitions are expressed in this key space.
    privacy_id_sharded: multi-GPU only -- every privacy id's rows are on one
                 rank already (rank = distributed.shard_of(pid)), so no
                 all-to-all shuffle is needed.  Ids must be GLOBAL (the same
                 dense id means the same key on every rank).
    """
    partition: Any
    privacy_id: Any = None
    value: Any = None
    num_partitions: Optional[int] = None
    num_privacy_ids: Optional[int] = None
    partition_keys: Optional[Sequence] = None
    privacy_id_sharded: bool = False

    def __len__(self):
        return int(self.partition.shape[0]) if hasattr(self.partition, "shape") else len(self.partition)

    def __bool__(self):
        return True


@dataclasses.dataclass
class EncodedColumns:
    pid: Optional[np.ndarray]
    pk: np.ndarray
    value: Optional[np.ndarray]
    num_privacy_ids: int
    partition_keys: list
    # multi-rank: the rows' privacy-id key hashes, not yet dense ids -- World.exchange_by_key_hash
    # moves every row to the rank owning its hash and numbers the privacy ids there
    pid_hash: Optional[np.ndarray] = None


def _canon(k) -> bytes:
    """Canonical bytes of a privacy-id key, identical in every process (Python's
    hash() is salted per process).  Keys equal as dict keys encode equally:
    numpy scalars as their Python value, integral floats as ints."""
    if isinstance(k, np.generic):
        k = k.item()
    if isinstance(k, bool):
        return b"b1" if k else b"b0"
    if isinstance(k, float) and k.is_integer():
        k = int(k)
    if isinstance(k, int):
        return b"i" + str(k).encode()
    if isinstance(k, str):
        return b"s" + k.encode("utf-8", "surrogatepass")
    if isinstance(k, float):
        return b"f" + float.hex(k).encode()
    if isinstance(k, bytes):
        return b"y" + k
    if isinstance(k, tuple):
        return b"t(" + b",".join(_canon(x) for x in k) + b")"
    if k is None:
        return b"n"
    return b"r" + repr(k).encode()


def key_hashes(keys) -> np.ndarray:
    """64-bit hash (int64) of each key: blake2b of its canonical bytes."""
    import hashlib
    out = np.empty(len(keys), dtype=np.int64)
    for i, k in enumerate(keys):
        out[i] = int.from_bytes(hashlib.blake2b(_canon(k), digest_size=8).digest(), "little", signed=True)
    return out


def dense_ids_from_hashes(h):
    """Privacy ids numbered by the ascending (signed) order of their key hash:
    the numbering World.exchange_by_key_hash reproduces across ranks without
    exchanging keys (ranks own contiguous hash ranges).  Distinct keys with
    equal 64-bit hashes (probability ~U^2 / 2^65) share one privacy id: their
    contributions are bounded together -- stricter bounding, never weaker
    privacy."""
    uniq, inv = np.unique(np.asarray(h, dtype=np.int64), return_inverse=True)
    return inv.astype(np.int64).reshape(-1), len(uniq)


def _factorize(values):
    import pandas as pd
    codes, uniques = pd.factorize(pd.Series(values, dtype=object) if not isinstance(values, np.ndarray) else values,
                                  use_na_sentinel=False)
    return codes.astype(np.int64), list(uniques)


def _unique_in_order(keys):
    seen = {}
    for k in keys:
        if k not in seen:
            seen[k] = len(seen)
    return list(seen)


def _index_of(keys, raw):
    """Dense ids of `raw` in the key list `keys` (-1 = absent)."""
    import pandas as pd
    if not len(raw):
        return np.zeros(0, np.int64)
    idx = pd.Index(keys, dtype=object) if len(keys) else pd.Index([], dtype=object)
    return idx.get_indexer(pd.Index(raw, dtype=object)).astype(np.int64)


def _global_keys(local_keys, world):
    """One key dictionary for all ranks: every rank's keys (first-appearance
    order) concatenated in rank order, deduplicated.  Ranks that
    reduce-scatter dense per-partition accumulators must number partitions
    identically."""
    import torch.distributed as dist
    gathered = [None] * world.size
    dist.all_gather_object(gathered, list(local_keys), group=world.group)
    return _unique_in_order(k for ks in gathered for k in ks)


def encode_rows(rows, extractors, public_partitions=None, need_pid=True, need_value=True,
                world=None) -> EncodedColumns:
    """Apply the extractors once per row and dictionary-encode.

    Partition ids: public partitions (deduplicated, in the given order) get
    ids [0, len(public)); rows of other partitions get -1 (dropped, like
    ``_drop_not_public_partitions`` dp_engine.py:283-293).  Without public
    partitions ids follow first appearance.  With a multi-rank ``world``
    (``distributed.World``) the partition dictionary is agreed across ranks
    (``_global_keys``: dense partition ids mean the same key on every rank,
    which the reduce-scatter of [P] partials needs).

    Privacy ids are numbered by their key hash (``dense_ids_from_hashes``),
    in one process and across ranks alike, so the sampling (keyed by the
    dense id) is the same whatever the world size.  With a multi-rank world
    no privacy-id key leaves its rank: the rows carry their key hashes
    (``pid_hash``), and ``World.exchange_by_key_hash`` moves them to the rank
    owning the hash (the reference's group-by-privacy-id shuffle,
    pipeline_backend.py:476-485) and numbers them there.
    """
    rows = rows if isinstance(rows, list) else list(rows)
    multi = world is not None and world.size > 1
    pk_raw = [extractors.partition_extractor(r) for r in rows]
    if public_partitions is not None:
        keys = _unique_in_order(public_partitions)
        pk = _index_of(keys, pk_raw)
    elif multi:
        keys = _global_keys(_unique_in_order(pk_raw), world)
        pk = _index_of(keys, pk_raw)
    else:
        pk, keys = _factorize(pk_raw) if rows else (np.zeros(0, np.int64), [])
    pid, U, pid_hash = None, 0, None
    if need_pid:
        pid_raw = [extractors.privacy_id_extractor(r) for r in rows]
        if rows:
            codes, uniq = _factorize(pid_raw)  # hash each distinct key once
            h = key_hashes(uniq)[codes]
        else:
            h = np.zeros(0, np.int64)
        if multi:
            pid_hash = h
        else:
            pid, U = dense_ids_from_hashes(h)
    value = None
    if need_value:
        value = np.asarray([extractors.value_extractor(r) for r in rows], dtype=np.float64)
    return EncodedColumns(pid, pk, value, U, keys, pid_hash)


def remap_public(pk, partition_keys, num_partitions, public_partitions):
    """Columnar input + public partitions: returns (lut, new_keys) mapping
    old dense ids to ids in public order (-1 = not public)."""
    keys = partition_keys if partition_keys is not None else list(range(num_partitions))
    pos = {k: i for i, k in enumerate(keys)}
    public = _unique_in_order(public_partitions)
    lut = np.full(max(len(keys), 1), -1, dtype=np.int64)
    for j, k in enumerate(public):
        i = pos.get(k)
        if i is not None:
            lut[i] = j
    return lut, public
