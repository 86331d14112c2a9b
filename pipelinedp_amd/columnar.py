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
    # multi-rank: the rows' privacy-id key hash pairs [N, 2], not yet dense ids -- World.exchange_by_key_hash
    # moves every row to the rank owning its hash and numbers the privacy ids there
    pid_hash: Optional[np.ndarray] = None


def _canon(k) -> bytes:
    """Canonical bytes of a privacy-id key, identical in every process (Python's
    hash() is salted per process).  Keys that are equal as dict keys -- the
    reference groups privacy ids by dict key (pipeline_backend.py:476-485) --
    encode equally: numpy scalars as their Python value, bools and integral
    floats as ints (True == 1 == 1.0, False == 0), complex numbers with a zero
    imaginary part as their real part, tuples element-wise."""
    if isinstance(k, np.generic):
        k = k.item()
    if isinstance(k, complex) and k.imag == 0:
        k = k.real
    if isinstance(k, bool):
        k = int(k)
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


def _digest_words(canon: bytes):
    import hashlib
    d = hashlib.blake2b(canon, digest_size=16).digest()
    return int.from_bytes(d[:8], "little", signed=True), int.from_bytes(d[8:], "little", signed=True)


def key_hashes(keys) -> np.ndarray:
    """128-bit hash of each key as two int64 words [len(keys), 2]: the
    blake2b-128 digest of its canonical bytes (``_canon``).  Word 0 picks the
    owning rank (distributed.World.key_owner); the pair orders the dense ids."""
    out = np.empty((len(keys), 2), dtype=np.int64)
    for i, k in enumerate(keys):
        out[i] = _digest_words(_canon(k))
    return out


def _pair_order(h):
    """Row order of an [M, 2] int64 array sorted by (word 0, word 1), signed."""
    h = np.asarray(h, dtype=np.int64).reshape(-1, 2)
    return np.lexsort((h[:, 1], h[:, 0]))


def dense_ids_from_hashes(h):
    """Dense privacy ids numbered by the ascending (signed) order of the
    128-bit key hash pairs [N, 2]: the numbering World.exchange_by_key_hash
    reproduces across ranks without exchanging keys (ranks own contiguous
    ranges of word 0).  -> (ids [N], number of distinct pairs)."""
    h = np.asarray(h, dtype=np.int64).reshape(-1, 2)
    if not len(h):
        return np.zeros(0, np.int64), 0
    o = _pair_order(h)
    hs = h[o]
    new = np.ones(len(h), dtype=bool)
    new[1:] = (hs[1:, 0] != hs[:-1, 0]) | (hs[1:, 1] != hs[:-1, 1])
    ids = np.empty(len(h), np.int64)
    ids[o] = np.cumsum(new) - 1
    return ids, int(new.sum())


def dense_ids_exact(uniq_keys, hashes):
    """Dense ids of distinct keys (``uniq_keys``: one per dict-equality class,
    as pandas.factorize yields them) in the order of their hash pairs, with
    EXACT handling of collisions: keys whose 128-bit hashes are equal are told
    apart by their canonical bytes (then by first appearance), so distinct
    keys always get distinct ids and equal keys one id -- the reference's
    dict grouping (pipeline_backend.py:476-485).  Without a collision the
    numbering is dense_ids_from_hashes'.  -> ids [M]."""
    M = len(uniq_keys)
    h = np.asarray(hashes, dtype=np.int64).reshape(-1, 2)
    o = _pair_order(h)
    hs = h[o]
    same = np.zeros(M, dtype=bool)
    if M > 1:
        same[1:] = (hs[1:, 0] == hs[:-1, 0]) & (hs[1:, 1] == hs[:-1, 1])
    if same.any():  # runs of equal hash pairs: order each run by (canonical bytes, first appearance)
        o = o.copy()
        i = 0
        while i < M:
            j = i + 1
            while j < M and same[j]:
                j += 1
            if j - i > 1:
                run = o[i:j]
                o[i:j] = sorted(run, key=lambda r: (_canon(uniq_keys[r]), r))
            i = j
    ids = np.empty(M, np.int64)
    ids[o] = np.arange(M, dtype=np.int64)
    return ids


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

    Privacy ids are grouped by dict equality, as the reference groups them
    (pipeline_backend.py:476-485: ``True``, ``1`` and ``1.0`` are one id), and
    numbered by their 128-bit key hash, in one process and across ranks
    alike, so the sampling (keyed by the dense id) is the same whatever the
    world size.  In one process the numbering is exact (``dense_ids_exact``:
    colliding hashes are told apart by the keys).  With a multi-rank world no
    privacy-id key leaves its rank: the rows carry their key hash pairs
    (``pid_hash`` [N, 2]), and ``World.exchange_by_key_hash`` moves them to the
    rank owning the hash (the reference's group-by-privacy-id shuffle) and
    numbers the distinct pairs there; only a full 128-bit collision of two
    distinct keys (probability ~U^2 / 2^129) would merge them.
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
            codes, uniq = _factorize(pid_raw)  # dict-equal keys share a code; hash each distinct key once
            hu = key_hashes(uniq)
        else:
            codes, uniq, hu = np.zeros(0, np.int64), [], np.zeros((0, 2), np.int64)
        if multi:
            pid_hash = hu[codes]
        else:
            pid, U = dense_ids_exact(uniq, hu)[codes], len(uniq)
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
