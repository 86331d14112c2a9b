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
    (``distributed.World``) the partition and privacy-id dictionaries are
    agreed across ranks (``_global_keys``), so dense ids mean the same key
    on every rank.
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
    pid, U = None, 0
    if need_pid:
        pid_raw = [extractors.privacy_id_extractor(r) for r in rows]
        if multi:
            pid_keys = _global_keys(_unique_in_order(pid_raw), world)
            pid = _index_of(pid_keys, pid_raw)
            U = len(pid_keys)
        elif rows:
            pid, uniq = _factorize(pid_raw)
            U = len(uniq)
        else:
            pid = np.zeros(0, np.int64)
    value = None
    if need_value:
        value = np.asarray([extractors.value_extractor(r) for r in rows], dtype=np.float64)
    return EncodedColumns(pid, pk, value, U, keys)


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
