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
    """
    partition: Any
    privacy_id: Any = None
    value: Any = None
    num_partitions: Optional[int] = None
    num_privacy_ids: Optional[int] = None
    partition_keys: Optional[Sequence] = None

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


def encode_rows(rows, extractors, public_partitions=None, need_pid=True, need_value=True) -> EncodedColumns:
    """Apply the extractors once per row and dictionary-encode.

    Partition ids: public partitions (deduplicated, in the given order) get
    ids [0, len(public)); rows of other partitions get -1 (dropped, like
    ``_drop_not_public_partitions`` dp_engine.py:283-293).  Without public
    partitions ids follow first appearance.
    """
    rows = rows if isinstance(rows, list) else list(rows)
    pk_raw = [extractors.partition_extractor(r) for r in rows]
    if public_partitions is not None:
        import pandas as pd
        keys = _unique_in_order(public_partitions)
        idx = pd.Index(keys, dtype=object) if keys else pd.Index([], dtype=object)
        pk = idx.get_indexer(pd.Index(pk_raw, dtype=object)).astype(np.int64) if rows else np.zeros(0, np.int64)
    else:
        pk, keys = _factorize(pk_raw) if rows else (np.zeros(0, np.int64), [])
    pid, U = None, 0
    if need_pid:
        pid_raw = [extractors.privacy_id_extractor(r) for r in rows]
        if rows:
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
