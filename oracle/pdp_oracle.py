"""CPU oracle for the DPEngine.aggregate hot path — TEST INFRASTRUCTURE ONLY.

This module is a vectorised numpy restatement of the reference algorithm
(/root/reference, PipelineDP snapshot 2025-02-04).  It is imported only by
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py``, always as the checker / baseline, never as the product path.
The product (``pipelinedp_amd``) must never import it.

Parity pinning: the restatement is checked against
  * golden vectors generated from the reference LocalBackend itself
    (``oracle/gen_golden.py`` -> ``tests/golden/*.npz``), and
  * the known-answer numbers the reference's own tests hold
    (``tests/golden/reference_known_answers.json``), e.g. the PyDP Gaussian
    sigma values and truncated-geometric keep probabilities.
LAPLACE_THRESHOLDING / GAUSSIAN_THRESHOLDING thresholds and the k>1
per-partition (eps / k, 1 - (1 - delta)^(1/k)) adjustment shared by all three
selection strategies are "parity unpinned" (PyDP is absent and the reference
tests only mock it).

Each function cites the reference file:line it restates.

Randomness specification (shared bit-for-bit with the HIP kernels, see
DESIGN.md "Randomness"):
  * sampling (contribution bounding) ranks 64-bit splitmix priorities: the
    kept L_inf rows of a (pid, pk) group are the L_inf rows with the smallest
    (row_priority(j), j), j = input-order rank in the group; the kept L0
    partitions of a pid are the L0 with the smallest (group_priority, pk).
    This is exactly uniform sampling without replacement (given the hash).
    ``sampler='hash'`` reproduces the GPU exactly;
    ``sampler='numpy'`` draws uniform subsets with numpy like LocalBackend
    (``pipeline_backend.py:504-520``).
  * noise / selection draws use Philox4x32-10 keyed by the 64-bit noise seed
    with counter (pk_lo, pk_hi, stream, 0); Laplace noise is a two-sided
    geometric on the grid 2^(ceil(log2 b) - 40), Gaussian noise is rounded to
    that grid, and the released value is snapped to it (granularity
    snapping as in PyDP's secure mechanisms; not PyDP's implementation).
"""
import functools
import math
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)

# ----------------------------------------------------------------------------
# Randomness primitives (spec shared with pipelinedp_amd/csrc/pdp_rng.h)
# ----------------------------------------------------------------------------

STREAM_SELECT = 1
STREAM_PID_COUNT = 2
STREAM_COUNT = 3
STREAM_SUM = 4
STREAM_MEAN_COUNT = 5
STREAM_MEAN_NSUM = 6
STREAM_VAR_NSQ = 7


def _u64(x):
    return np.asarray(x, dtype=np.uint64)


def splitmix64(x):
    """splitmix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = _u64(x) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _mask(bits):
    return np.uint64((1 << int(bits)) - 1) if bits > 0 else np.uint64(0)


_M32 = np.uint64(0xFFFFFFFF)


def fmix32(h):
    """murmur3 32-bit finaliser on uint64 arrays holding 32-bit values."""
    h = _u64(h) & _M32
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & _M32
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & _M32
    h ^= h >> np.uint64(16)
    return h


def _mask32(bits):
    return np.uint64((1 << int(bits)) - 1) if bits > 0 else np.uint64(0)


def perm_bits(x, bits, key):
    """Keyed 4-round Feistel bijection on [0, 2**bits) (bits <= 32) with
    round function F_r(R) = fmix32(R * 0x9E3779B1 + k_r), round keys
    (lo32(key), hi32(key), lo32 ^ 0x85EBCA6B, hi32 ^ 0xC2B2AE35)."""
    x = _u64(x)
    key = _u64(key)
    k0, k1 = key & _M32, key >> np.uint64(32)
    rk = [k0, k1, k0 ^ np.uint64(0x85EBCA6B), k1 ^ np.uint64(0xC2B2AE35)]
    h1 = (bits + 1) >> 1
    h2 = bits >> 1
    wl, wr = h1, h2
    left = x >> np.uint64(h2)
    right = x & _mask32(h2)
    with np.errstate(over="ignore"):
        for r in range(4):
            f = fmix32((right * np.uint64(0x9E3779B1) + rk[r]) & _M32)
            left, right = right, left ^ (f & _mask32(wl))
            wl, wr = wr, wl
    return (left << np.uint64(h2)) | right


def ceil_log2(n):
    n = int(n)
    return 0 if n <= 1 else (n - 1).bit_length()


def cycle_walk(j, n, key):
    """Pseudo-random permutation of [0, n) evaluated at j (numpy arrays of
    equal shape; n varies per element).  Elements with n <= 1 map to j."""
    j = _u64(j).copy()
    n = np.asarray(n, dtype=np.int64)
    key = _u64(key)
    out = j.copy()
    bits = np.zeros(n.shape, dtype=np.int64)
    nz = n > 1
    bits[nz] = np.ceil(np.log2(n[nz].astype(np.float64))).astype(np.int64)
    # guard float rounding of log2 on exact powers / near powers
    for b_fix in range(2):
        too_small = nz & ((np.int64(1) << bits) < n)
        bits[too_small] += 1
        too_big = nz & (bits > 0) & ((np.int64(1) << (bits - 1)) >= n)
        bits[too_big] -= 1
    for b in np.unique(bits[nz]):
        sel = nz & (bits == b)
        y = j[sel]
        k = key[sel]
        nn = n[sel].astype(np.uint64)
        y = perm_bits(y, int(b), k)
        todo = y >= nn
        while todo.any():
            y[todo] = perm_bits(y[todo], int(b), k[todo])
            todo = y >= nn
        out[sel] = y
    return out


def pid_key(seed, pid):
    """Per privacy-id key: splitmix64(seed ^ splitmix64(pid + 1))."""
    with np.errstate(over="ignore"):
        return splitmix64(_u64(seed) ^ splitmix64(_u64(pid) + np.uint64(1)))


def group_priority(seed, pid, pk):
    """L0 priority of partition pk for privacy id pid."""
    with np.errstate(over="ignore"):
        return splitmix64(pid_key(seed, pid) + (_u64(pk) + np.uint64(1)) * np.uint64(0xD1B54A32D192ED03))


def row_priority(gprio, j):
    """L_inf priority of the j-th (input order) row of a (pid, pk) group."""
    with np.errstate(over="ignore"):
        gkey = splitmix64(_u64(gprio) ^ np.uint64(0xA0761D6478BD642F))
        return splitmix64(gkey + (_u64(j) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15))


_PHILOX_M0 = np.uint64(0xD2511F53)
_PHILOX_M1 = np.uint64(0xCD9E8D57)
_PHILOX_W0 = np.uint64(0x9E3779B9)
_PHILOX_W1 = np.uint64(0xBB67AE85)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (Random123) on uint64 arrays holding 32-bit values."""
    c0, c1, c2, c3 = (_u64(c) & _M32 for c in (c0, c1, c2, c3))
    k0 = _u64(k0) & _M32
    k1 = _u64(k1) & _M32
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _PHILOX_M0 * c0
            p1 = _PHILOX_M1 * c2
            hi0, lo0 = p0 >> np.uint64(32), p0 & _M32
            hi1, lo1 = p1 >> np.uint64(32), p1 & _M32
            c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & _M32, lo1, (hi0 ^ c3 ^ k1) & _M32, lo0
            k0 = (k0 + _PHILOX_W0) & _M32
            k1 = (k1 + _PHILOX_W1) & _M32
    return c0, c1, c2, c3


def _uniform53(a, b):
    """Two 32-bit words -> uniform double strictly inside (0, 1)."""
    return ((a >> np.uint64(5)).astype(np.float64) * 67108864.0 +
            (b >> np.uint64(6)).astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)


def philox_uniforms(seed, idx, stream):
    """Two independent uniforms in (0,1) per index for (seed, stream)."""
    idx = _u64(idx)
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    x0, x1, x2, x3 = philox4x32_10(idx & _M32, idx >> np.uint64(32),
                                   np.uint64(stream), np.uint64(0),
                                   np.uint64(seed & 0xFFFFFFFF),
                                   np.uint64(seed >> 32))
    return _uniform53(x0, x1), _uniform53(x2, x3)


def _uniform64(hi, lo):
    """Uniform in (0,1) from a 64-bit word, exact near 0 (pdp_rng.h:uniform64)."""
    w = (hi << np.uint64(32)) | lo
    big = w >= np.uint64(1 << 53)
    top = ((w >> np.uint64(11)).astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)
    low = (np.where(big, np.uint64(0), w).astype(np.float64) + 0.5) * 5.421010862427522e-20
    return np.where(big, top, low)


def noise_grid(scale):
    """Noise grid 2^(ceil(log2 scale) - 40) (pdp_rng.h:noise_grid)."""
    m, e = math.frexp(scale)
    return math.ldexp(1.0, (e - 1 if m == 0.5 else e) - 40)


def laplace_on_grid(seed, idx, stream, b, g):
    """Laplace(0, b) as a two-sided geometric on the grid g: g (G1 - G2),
    G_i = floor(E_i b / g), E_i = -log(u_i) from the two 64-bit Philox words."""
    idx = _u64(idx)
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    x0, x1, x2, x3 = philox4x32_10(idx & _M32, idx >> np.uint64(32), np.uint64(stream), np.uint64(0),
                                   np.uint64(seed & 0xFFFFFFFF), np.uint64(seed >> 32))
    e1 = -np.log(_uniform64(x0, x1))
    e2 = -np.log(_uniform64(x2, x3))
    return g * (np.floor(e1 * (b / g)) - np.floor(e2 * (b / g)))


def gaussian_on_grid(seed, idx, stream, sigma, g):
    """N(0, sigma^2) by Box-Muller, rounded to the grid g."""
    idx = _u64(idx)
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    x0, x1, x2, x3 = philox4x32_10(idx & _M32, idx >> np.uint64(32), np.uint64(stream), np.uint64(0),
                                   np.uint64(seed & 0xFFFFFFFF), np.uint64(seed >> 32))
    z = np.sqrt(-2.0 * np.log(_uniform64(x0, x1))) * np.cos(2.0 * math.pi * _uniform53(x2, x3))
    return g * np.rint(sigma * z / g)


def add_snapped_noise(kind, value, seed, idx, stream, scale):
    """value + noise, both on the grid of `scale` (pdp_rng.h:add_snapped_noise)."""
    g = noise_grid(scale)
    z = laplace_on_grid(seed, idx, stream, scale, g) if kind == "laplace" else \
        gaussian_on_grid(seed, idx, stream, scale, g)
    return g * np.rint(np.asarray(value, dtype=np.float64) / g) + z


# ----------------------------------------------------------------------------
# DP arithmetic (dp_computations.py restatement + PyDP calibration)
# ----------------------------------------------------------------------------


def compute_middle(min_value, max_value):
    """dp_computations.py:65-69."""
    return min_value + (max_value - min_value) / 2


def compute_squares_interval(min_value, max_value):
    """dp_computations.py:58-62."""
    if min_value < 0 < max_value:
        return 0, max(min_value**2, max_value**2)
    return min_value**2, max_value**2


def equally_split_budget(eps, delta, no_mechanisms):
    """dp_computations.py:224-252."""
    if no_mechanisms <= 0:
        raise ValueError("The number of mechanisms must be a positive integer.")
    eps_used = delta_used = 0
    budgets = []
    for _ in range(no_mechanisms - 1):
        budget = (eps / no_mechanisms, delta / no_mechanisms)
        eps_used += budget[0]
        delta_used += budget[1]
        budgets.append(budget)
    budgets.append((eps - eps_used, delta - delta_used))
    return budgets


def _std_normal_cdf(x):
    return 0.5 * math.erfc(-x / math.sqrt(2.0))


def _gaussian_delta(sigma, eps, l2):
    """Analytic-Gaussian delta(sigma) (Balle & Wang 2018), as used by PyDP's
    GaussianMechanism."""
    a = l2 / (2.0 * sigma)
    b = eps * sigma / l2
    return _std_normal_cdf(a - b) - math.exp(eps) * _std_normal_cdf(-a - b)


def gaussian_sigma(eps, delta, l2_sensitivity):
    """PyDP GaussianMechanism(eps, delta, l2).std restated
    (dp_computations.py:98-108 calls it).  Unit-sensitivity search: double
    the upper bound while delta(hi) > delta, then bisect until
    hi - lo <= 1e-3 * lo; return hi * l2.  Pinned by
    tests/dp_computations_test.py:62-67,557-587,623-657 (5 values)."""
    if delta <= 0:
        raise ValueError("Gaussian mechanism requires delta > 0")
    lo, hi = 0.0, 1.0
    while _gaussian_delta(hi, eps, 1.0) > delta:
        lo = hi
        hi *= 2.0
    while hi - lo > 1e-3 * lo:
        mid = lo + (hi - lo) / 2.0
        if _gaussian_delta(mid, eps, 1.0) > delta:
            lo = mid
        else:
            hi = mid
    return hi * l2_sensitivity


def adjusted_delta(delta, k):
    """Per-partition delta over k = max_partitions_contributed partitions:
    1 - (1 - delta)^(1/k) (k independent decisions compose to delta); the
    one adjustment of all three selection strategies here.  Parity unpinned
    for k > 1 (PyDP is absent; the reference pins only k = 1, where this is
    delta).  Differs from delta / k by less than delta^2 / 2."""
    if k <= 1:
        return delta
    return -math.expm1(math.log1p(-delta) / k)


@functools.lru_cache(maxsize=256)
def truncated_geometric_table(eps, delta, max_partitions, max_len=1 << 22):
    """Keep probability p(n) of PyDP's truncated-geometric partition
    selection, n = 0..len-1; p(n) = 1 for n beyond the table.
    Recurrence (pinned for k=1 by analysis/tests/combiners_test.py:197-224):
      p(0) = 0; p(n) = min(e^eps p(n-1) + delta,
                           1 - e^-eps (1 - p(n-1) - delta), 1)
    with eps / k and adjusted_delta(delta, k), k = max_partitions (k > 1:
    parity unpinned).
    """
    e = eps / max_partitions
    d = adjusted_delta(delta, max_partitions)
    ee = math.exp(e)
    eme = math.exp(-e)
    p = [0.0]
    while p[-1] < 1.0:
        prev = p[-1]
        nxt = min(ee * prev + d, 1.0 - eme * (1.0 - prev - d), 1.0)
        p.append(nxt)
        if len(p) >= max_len:
            raise ValueError("truncated geometric table too long (eps too small)")
        if nxt <= prev:  # delta == 0 and eps tiny: never reaches 1
            raise ValueError("truncated geometric selection cannot keep partitions")
    t = np.asarray(p, dtype=np.float64)
    t.flags.writeable = False  # cached: shared by every caller
    return t


def truncated_geometric_keep_prob(n, eps, delta, max_partitions):
    t = truncated_geometric_table(eps, delta, max_partitions)
    n = np.asarray(n, dtype=np.int64)
    return np.where(n < len(t), t[np.clip(n, 0, len(t) - 1)], 1.0)


def laplace_threshold(eps, delta, max_partitions):
    """LAPLACE_THRESHOLDING (PyDP LaplacePartitionSelection) — parity
    unpinned restatement.  Returns (threshold, diversity)."""
    adj_delta = adjusted_delta(delta, max_partitions)
    b = max_partitions / eps
    if adj_delta > 0.5:
        thr = 1.0 + b * math.log(2.0 * (1.0 - adj_delta))
    else:
        thr = 1.0 - b * math.log(2.0 * adj_delta)
    return thr, b


def _norm_ppf(p):
    from scipy.stats import norm
    return float(norm.ppf(p))


def gaussian_threshold(eps, delta, max_partitions):
    """GAUSSIAN_THRESHOLDING (PyDP GaussianPartitionSelection) — parity
    unpinned restatement.  Returns (threshold, sigma)."""
    thr_delta = delta / 2.0
    noise_delta = delta - thr_delta
    sigma = gaussian_sigma(eps, noise_delta, math.sqrt(max_partitions))
    adj = adjusted_delta(thr_delta, max_partitions)
    return 1.0 + sigma * _norm_ppf(1.0 - adj), sigma


def noise_scale(kind, eps, delta, l0, linf):
    """_add_random_noise (dp_computations.py:146-175): Laplace b = l0*linf/eps
    (l1 sensitivity, :72-82, :111-124); Gaussian sigma(eps, delta,
    sqrt(l0)*linf) (:85-108, :127-143)."""
    if kind == "laplace":
        return l0 * linf / eps
    if kind == "gaussian":
        return gaussian_sigma(eps, delta, math.sqrt(l0) * linf)
    raise ValueError("Noise kind must be either Laplace or Gaussian.")


# ----------------------------------------------------------------------------
# Contribution bounding + per-partition accumulation
# ----------------------------------------------------------------------------


@dataclass
class BoundParams:
    max_partitions_contributed: int
    max_contributions_per_partition: int
    min_value: Optional[float] = None
    max_value: Optional[float] = None
    min_sum_per_partition: Optional[float] = None
    max_sum_per_partition: Optional[float] = None
    contribution_bounds_already_enforced: bool = False


@dataclass
class Accumulators:
    """Dense per-partition accumulators (CompoundCombiner state,
    combiners.py:507-603): row_count = #(pid,pk) pairs (== privacy id count),
    count = #kept rows, sum = sum of clipped values (SumCombiner),
    nsum / nsumsq = normalised sums (Mean/VarianceCombiner)."""
    row_count: np.ndarray
    count: np.ndarray
    sum: np.ndarray
    nsum: np.ndarray
    nsumsq: np.ndarray
    kept_rows: int = 0
    kept_pairs: int = 0
    # the kept (pid, pk) accumulators before the per-partition merge:
    # (pk, count, sum, nsum, nsumsq) arrays, one entry per kept pair
    pairs: Optional[tuple] = None


def _group_starts(keys_sorted_list):
    n = len(keys_sorted_list[0])
    start = np.zeros(n, dtype=bool)
    if n:
        start[0] = True
        for k in keys_sorted_list:
            start[1:] |= k[1:] != k[:-1]
    return start


def _bit_length32(h):
    """Bit length of uint64 arrays holding 32-bit values (0 for 0)."""
    h = _u64(h).copy()
    n = np.zeros(h.shape, dtype=np.int64)
    for sh in (16, 8, 4, 2, 1):
        big = h >= (np.uint64(1) << np.uint64(sh))
        n[big] += sh
        h[big] >>= np.uint64(sh)
    return n + (h > 0)


def prefilter_level(h):
    """Level of a 32-bit group priority h on a log scale with 4 levels per
    octave, 0..31 (pdp_filter.inc:filt_level): 4 (7 - e) + #{thresholds
    2^(k/4) 2^31 <= mantissa}, e = leading zeros of h; 0 when e >= 8."""
    h = _u64(h) & _M32
    e = 32 - _bit_length32(h)
    m = (h << np.minimum(e, 31).astype(np.uint64)) & _M32
    f = (m >= np.uint64(0x9837F052)).astype(np.int64) + (m >= np.uint64(0xB504F334)) + (m >= np.uint64(0xD744FCCB))
    return np.where(e >= 8, 0, 4 * (7 - e) + f)


PREFILTER_WORDS = 39936  # LDS sketch words per bucket (pdp_filter.inc kFiltWords)


def prefilter_sketch_bits(num_privacy_ids):
    """Sketch width the GPU uses for U privacy ids (pdp_kernels.hip
    filter_plan): 256 buckets of pids with (pid * mult) >> 32 = b,
    mult = floor(2^40 / U); 32 bits per pid when the widest bucket has <=
    PREFILTER_WORDS pids, 16 bits up to twice that, else no filter (0)."""
    U = int(num_privacy_ids)
    mult = (1 << 40) // U
    lo = [((b << 32) + mult - 1) // mult for b in range(257)]
    width = max(min(lo[b + 1], U) - lo[b] for b in range(256))
    return 32 if width <= PREFILTER_WORDS else (16 if width <= 2 * PREFILTER_WORDS else 0)


def prefilter_survivors(pid, pk, seed, l0, sketch_bits=32):
    """Restatement of the L0 pre-filter (pdp_filter.inc) for
    checking: per privacy id a sketch with bit level(top32(group priority))
    set for each of its rows; K = level of the L0-th set bit (the top level
    when fewer); a row survives iff its level <= K.  With 16-bit sketches
    (buckets wider than PREFILTER_WORDS pids) levels are halved.  Rows with
    pk < 0 never survive.  (The GPU groups privacy ids into buckets first;
    that changes nothing per privacy id.)  Returns the boolean survivor mask."""
    pid = np.asarray(pid, dtype=np.int64)
    pk = np.asarray(pk, dtype=np.int64)
    ok = pk >= 0
    lvl = np.zeros(len(pid), dtype=np.int64)
    lvl[ok] = prefilter_level(group_priority(seed, pid[ok], pk[ok]) >> np.uint64(32))
    if sketch_bits == 16:
        lvl = lvl >> 1
    uniq, inv = np.unique(pid, return_inverse=True)
    sketch = np.zeros(len(uniq), dtype=np.uint64)
    np.bitwise_or.at(sketch, inv[ok], np.left_shift(np.uint64(1), lvl[ok].astype(np.uint64)))
    bits = ((sketch[:, None] >> np.arange(sketch_bits, dtype=np.uint64)) & np.uint64(1)).astype(np.int64)
    cs = np.cumsum(bits, axis=1)
    K = np.where(cs[:, -1] >= l0, np.argmax(cs >= l0, axis=1), sketch_bits - 1)
    return ok & (lvl <= K[inv])


def bound_and_accumulate(pid, pk, value, num_partitions, params: BoundParams,
                         sampler="hash", seed=0, rng=None) -> Accumulators:
    """SamplingCrossAndPerPartitionContributionBounder.bound_contributions
    (contribution_bounders.py:66-105) + CompoundCombiner.create_accumulator /
    merge_accumulators (combiners.py:558-573) + combine_accumulators_per_key
    (pipeline_backend.py:528-538), dense over partitions [0, num_partitions).

    Rows with pk < 0 are dropped (non-public partitions,
    dp_engine.py:283-293).  ``sampler``: 'hash' (GPU-identical),
    'numpy' (uniform subsets from ``rng``, like LocalBackend), or 'none'
    (keep everything; valid when bounds are non-binding).
    """
    P = int(num_partitions)
    pk = np.asarray(pk, dtype=np.int64)
    keep_row = pk >= 0
    value = None if value is None else np.asarray(value, dtype=np.float64)
    L0 = params.max_partitions_contributed
    Linf = params.max_contributions_per_partition
    have_vb = params.min_value is not None
    have_pb = params.min_sum_per_partition is not None
    if have_vb:
        a, b = params.min_value, params.max_value
        mid = compute_middle(a, b)

    if params.contribution_bounds_already_enforced:
        # dp_engine.py:139-150: every row is its own accumulator
        # create_accumulator([value]).
        pkk = pk[keep_row]
        row_count = np.bincount(pkk, minlength=P).astype(np.int64)
        count = row_count.copy()
        s = ns = nsq = np.zeros(P)
        if value is not None:
            v = value[keep_row]
            if have_vb:
                cv = np.clip(v, a, b)
                s = np.bincount(pkk, weights=cv, minlength=P)
                nv = cv - mid
                ns = np.bincount(pkk, weights=nv, minlength=P)
                nsq = np.bincount(pkk, weights=nv * nv, minlength=P)
            elif have_pb:
                s = np.bincount(pkk, weights=np.clip(v, params.min_sum_per_partition,
                                                     params.max_sum_per_partition), minlength=P)
        m = len(pkk)
        ps = pns = pnsq = np.zeros(m)
        if value is not None and have_vb:
            ps, pns, pnsq = cv, nv, nv * nv
        elif value is not None and have_pb:
            ps = np.clip(v, params.min_sum_per_partition, params.max_sum_per_partition)
        return Accumulators(row_count, count, np.asarray(s, np.float64),
                            np.asarray(ns, np.float64), np.asarray(nsq, np.float64),
                            int(keep_row.sum()), int(keep_row.sum()),
                            pairs=(pkk, np.ones(m, np.int64), ps, pns, pnsq))

    pid = np.asarray(pid, dtype=np.int64)[keep_row]
    pk = pk[keep_row]
    if value is not None:
        value = value[keep_row]
    n = len(pid)
    order = np.lexsort((pk, pid))  # stable: input order within (pid, pk)
    spid, spk = pid[order], pk[order]
    gstart = _group_starts([spid, spk])
    gid = np.cumsum(gstart) - 1
    G = int(gstart.sum())
    gsize = np.bincount(gid, minlength=G)
    gfirst = np.flatnonzero(gstart)
    j = np.arange(n) - gfirst[gid]
    gn = gsize[gid]

    if sampler == "hash":
        sampler = "hash"
    g_pid = spid[gfirst]
    g_pk = spk[gfirst]
    # --- per-partition (L_inf) sampling, contribution_bounders.py:74-76
    if sampler == "hash":
        gprio = group_priority(seed, g_pid, g_pk)
        rprio = row_priority(gprio[gid], j)
        o2 = np.lexsort((j, rprio, gid))
        rank = np.empty(n, dtype=np.int64)
        rank[o2] = np.arange(n) - gfirst[gid[o2]]
        keep = rank < Linf
    elif sampler == "numpy":
        rng = rng or np.random.default_rng()
        prio = rng.random(n)
        o2 = np.lexsort((prio, gid))
        rank = np.empty(n, dtype=np.int64)
        rank[o2] = np.arange(n) - gfirst[gid[o2]]
        keep = rank < Linf
    elif sampler == "none":
        keep = np.ones(n, dtype=bool)
    else:
        raise ValueError(sampler)

    # --- per-group accumulators (create_accumulator over kept values)
    kg = gid[keep]
    g_count = np.bincount(kg, minlength=G).astype(np.int64)
    g_sum = np.zeros(G)
    g_nsum = np.zeros(G)
    g_nsq = np.zeros(G)
    if value is not None:
        sv = value[order][keep]
        if have_vb:
            cv = np.clip(sv, a, b)
            g_sum = np.bincount(kg, weights=cv, minlength=G)
            nv = cv - mid
            g_nsum = np.bincount(kg, weights=nv, minlength=G)
            g_nsq = np.bincount(kg, weights=nv * nv, minlength=G)
        elif have_pb:
            # SumCombiner per-partition bounding, combiners.py:256-259
            g_sum = np.clip(np.bincount(kg, weights=sv, minlength=G),
                            params.min_sum_per_partition,
                            params.max_sum_per_partition)

    # --- cross-partition (L0) sampling, contribution_bounders.py:87-92
    if sampler == "hash":
        o3 = np.lexsort((g_pk, gprio, g_pid))
    elif sampler == "numpy":
        o3 = np.lexsort((rng.random(G), g_pid))
    else:
        o3 = np.arange(G)
    pstart = _group_starts([g_pid[o3]])
    pfirst = np.flatnonzero(pstart)
    pidx = np.cumsum(pstart) - 1
    grank = np.empty(G, dtype=np.int64)
    grank[o3] = np.arange(G) - pfirst[pidx]
    gkeep = grank < L0 if sampler != "none" else np.ones(G, dtype=bool)

    kp = g_pk[gkeep]
    acc = Accumulators(
        row_count=np.bincount(kp, minlength=P).astype(np.int64),
        count=np.bincount(kp, weights=g_count[gkeep], minlength=P).astype(np.int64),
        sum=np.bincount(kp, weights=g_sum[gkeep], minlength=P),
        nsum=np.bincount(kp, weights=g_nsum[gkeep], minlength=P),
        nsumsq=np.bincount(kp, weights=g_nsq[gkeep], minlength=P),
        kept_rows=int(g_count[gkeep].sum()),
        kept_pairs=int(gkeep.sum()),
        pairs=(kp, g_count[gkeep], g_sum[gkeep], g_nsum[gkeep], g_nsq[gkeep]))
    return acc


# ----------------------------------------------------------------------------
# K4 fixed point (pipelinedp_amd/csrc/pdp_reduce.inc): the per-partition merge
# of the pair accumulators (combine_accumulators_per_key,
# pipeline_backend.py:528-538) in 64-bit fixed point, and its multi-GPU
# export (pdp_bound_accumulate_partials / pdp_finalize_partials)
# ----------------------------------------------------------------------------

METRIC_BITS = {"count": 1, "sum": 2, "mean": 4, "variance": 8, "privacy_id_count": 16}


def k4_exponent(M):
    """F = 62 - ceil(log2 M) (k4_exponent: frexp's e, M < 2^e), clamped."""
    if not (M > 0.0) or not math.isfinite(M):
        return 0
    _, e = math.frexp(M)
    return max(-1000, min(1000, 62 - e))


def k4_exponents(params: BoundParams, metrics_mask):
    """(F_x, F_y, x kind) as k4_plan / make_seg pick them: the largest |x| of
    one pair is L_inf (b - a) / 2 for normalised sums (MEAN / VARIANCE),
    L_inf max(|a|, |b|) for clipped SUM, max(|min_sum|, |max_sum|) for SUM
    with per-partition sum bounds; y: L_inf ((b - a) / 2)^2."""
    linf = 1.0 if params.contribution_bounds_already_enforced else float(params.max_contributions_per_partition)
    a = params.min_value if params.min_value is not None else 0.0
    b = params.max_value if params.max_value is not None else 0.0
    half = abs(b - a) / 2.0
    m = metrics_mask
    if m & (METRIC_BITS["mean"] | METRIC_BITS["variance"]):
        kind, mx = "nsum", linf * half
    elif m & METRIC_BITS["sum"]:
        if params.min_value is not None:
            kind, mx = "sum", linf * max(abs(a), abs(b))
        else:
            kind, mx = "sum", max(abs(params.min_sum_per_partition or 0.0), abs(params.max_sum_per_partition or 0.0))
    else:
        kind, mx = None, 0.0
    return k4_exponent(mx), k4_exponent(linf * half * half), kind


def k4_fixed_sums(pair_pk, pair_x, num_partitions, F):
    """Exported fixed-point sums (hi, lo, nan count) [P] of the pair values:
    q = rint(x 2^F) per pair, hi = sum(q >> 32) + (sum(q mod 2^32) >> 32),
    lo = sum(q mod 2^32) mod 2^32 (pdp_hip.h pdp_partials)."""
    P = int(num_partitions)
    x = np.asarray(pair_x, np.float64)
    pk = np.asarray(pair_pk, np.int64)
    isnan = np.isnan(x)
    q = np.rint(np.where(isnan, 0.0, x) * math.ldexp(1.0, F)).astype(np.int64)
    hi = np.zeros(P, np.int64)
    lo = np.zeros(P, np.int64)
    np.add.at(hi, pk, q >> 32)
    np.add.at(lo, pk, q & 0xFFFFFFFF)
    hi += lo >> 32
    lo &= 0xFFFFFFFF
    return hi, lo, np.bincount(pk[isnan], minlength=P).astype(np.int64)


def k4_to_double(hi, lo, nan, F):
    """(summed) fixed-point partials -> fp64 (k4_value): h = hi + (lo >> 32),
    l = lo mod 2^32, h 2^(32-F) + l 2^-F; NaN where a NaN term was added."""
    hi = np.asarray(hi, np.int64)
    lo = np.asarray(lo, np.int64)
    h = hi + (lo >> 32)
    v = h.astype(np.float64) * math.ldexp(1.0, 32 - F) + (lo & 0xFFFFFFFF).astype(np.float64) * math.ldexp(1.0, -F)
    return np.where(np.asarray(nan) != 0, np.nan, v)


PARTIAL_FIELDS = ("row_count", "count", "x_hi", "x_lo", "nan", "y_hi", "y_lo")


def k4_partials(acc: Accumulators, num_partitions, params: BoundParams, metrics_mask):
    """The rank-local partials of pdp_bound_accumulate_partials from an
    oracle result: {field: int64 [P]} (nan: + 1 per x NaN, + 2^32 per y NaN)."""
    fx, fy, kind = k4_exponents(params, metrics_mask)
    pk, _, s, ns, nsq = acc.pairs
    out = {"row_count": acc.row_count.astype(np.int64), "count": acc.count.astype(np.int64)}
    if kind is not None:
        out["x_hi"], out["x_lo"], nx = k4_fixed_sums(pk, ns if kind == "nsum" else s, num_partitions, fx)
        out["nan"] = nx
    if metrics_mask & METRIC_BITS["variance"]:
        out["y_hi"], out["y_lo"], ny = k4_fixed_sums(pk, nsq, num_partitions, fy)
        out["nan"] = out["nan"] + (ny << 32)
    return out


def k4_finalize(parts, params: BoundParams, metrics_mask):
    """pdp_finalize_partials restated: -> (x, y) fp64 arrays (None if absent)."""
    fx, fy, kind = k4_exponents(params, metrics_mask)
    x = y = None
    if kind is not None:
        x = k4_to_double(parts["x_hi"], parts["x_lo"], parts["nan"] & 0xFFFFFFFF, fx)
    if metrics_mask & METRIC_BITS["variance"]:
        y = k4_to_double(parts["y_hi"], parts["y_lo"], parts["nan"] >> 32, fy)
    return x, y


# ----------------------------------------------------------------------------
# Release: partition selection + noisy metrics
# ----------------------------------------------------------------------------


@dataclass
class ReleaseSpec:
    """Which combiners run and their (eps, delta) after compute_budgets
    (combiners.py:652-720; budget_accounting.py:368-396)."""
    metrics: tuple  # subset of names: count, sum, mean, variance, privacy_id_count
    noise_kind: str  # 'laplace' | 'gaussian'
    budgets: Dict[str, tuple] = field(default_factory=dict)  # combiner -> (eps, delta)
    selection: Optional[str] = None  # None (public) | 'truncated_geometric' | 'laplace' | 'gaussian'
    selection_budget: tuple = (0.0, 0.0)
    max_rows_per_privacy_id: int = 1


def _noisy(value, seed, pk_idx, stream, kind, scale, enabled):
    """value + snapped noise of `scale` (k_release: noisy); value if off."""
    value = np.asarray(value, dtype=np.float64)
    if not enabled or scale == 0:
        return value
    return add_snapped_noise(kind, value, seed, pk_idx, stream, scale)


def release(acc: Accumulators, bp: BoundParams, spec: ReleaseSpec, seed=0,
            noise=True, pk_idx=None):
    """Partition selection (dp_engine.py:312-362) + compute_metrics of the
    compound combiner (combiners.py:575-597 -> dp_computations.py:255-459).
    Returns (keep mask, dict metric -> array) over all partitions."""
    P = len(acc.row_count)
    idx = np.arange(P, dtype=np.uint64) if pk_idx is None else _u64(pk_idx)
    L0 = bp.max_partitions_contributed
    Linf = bp.max_contributions_per_partition
    kind = spec.noise_kind
    m = set(spec.metrics)
    out = {}

    if spec.selection is None:
        keep = np.ones(P, dtype=bool)
    else:
        eps, delta = spec.selection_budget
        r = spec.max_rows_per_privacy_id
        nn = (acc.row_count + r - 1) // r
        if spec.selection == "truncated_geometric":
            p = truncated_geometric_keep_prob(nn, eps, delta, L0)
            u, _ = philox_uniforms(seed, idx, STREAM_SELECT)
            keep = (nn > 0) & (u < p) if noise else (nn > 0) & (p > 0)
        else:
            if spec.selection == "laplace":
                thr, scale = laplace_threshold(eps, delta, L0)
            else:
                thr, scale = gaussian_threshold(eps, delta, L0)
            v = _noisy(nn, seed, idx, STREAM_SELECT, spec.selection, scale, noise)
            keep = (nn > 0) & (v > thr)

    def lin_sum_linf():
        if bp.min_value is not None:
            return Linf * max(abs(bp.min_value), abs(bp.max_value))
        return max(abs(bp.min_sum_per_partition), abs(bp.max_sum_per_partition))

    if "variance" in m:
        eps, delta = spec.budgets["variance"]
        (ce, cd), (se, sd), (qe, qd) = equally_split_budget(eps, delta, 3)
        a, b = bp.min_value, bp.max_value
        dp_count = _noisy(acc.count, seed, idx, STREAM_MEAN_COUNT, kind, noise_scale(kind, ce, cd, L0, Linf), noise)
        denom = np.maximum(1.0, dp_count)
        if a == b:
            dp_mean = np.full(P, float(a))
        else:
            mid = compute_middle(a, b)
            dp_mean = (_noisy(acc.nsum, seed, idx, STREAM_MEAN_NSUM, kind,
                                         noise_scale(kind, se, sd, L0, Linf * abs(mid - a)), noise)) / denom
        sa, sb = compute_squares_interval(a, b)
        if sa == sb:
            dp_msq = np.full(P, float(sa))
        else:
            msq = compute_middle(sa, sb)
            dp_msq = (_noisy(acc.nsumsq, seed, idx, STREAM_VAR_NSQ, kind,
                                          noise_scale(kind, qe, qd, L0, Linf * abs(msq - sa)), noise)) / denom
        var = dp_msq - dp_mean**2
        if a != b:
            dp_mean = dp_mean + compute_middle(a, b)
        out["variance"] = var
        if "mean" in m:
            out["mean"] = dp_mean
        if "count" in m:
            out["count"] = dp_count
        if "sum" in m:
            out["sum"] = dp_mean * dp_count
    elif "mean" in m:
        eps, delta = spec.budgets["mean"]
        (ce, cd), (se, sd) = equally_split_budget(eps, delta, 2)
        a, b = bp.min_value, bp.max_value
        dp_count = _noisy(acc.count, seed, idx, STREAM_MEAN_COUNT, kind, noise_scale(kind, ce, cd, L0, Linf), noise)
        if a == b:
            dp_mean = np.full(P, float(a))
        else:
            mid = compute_middle(a, b)
            dp_mean = (_noisy(acc.nsum, seed, idx, STREAM_MEAN_NSUM, kind,
                                         noise_scale(kind, se, sd, L0, Linf * abs(mid - a)), noise)) / np.maximum(1.0, dp_count)
            dp_mean = dp_mean + mid
        out["mean"] = dp_mean
        if "count" in m:
            out["count"] = dp_count
        if "sum" in m:
            out["sum"] = dp_mean * dp_count
    else:
        if "count" in m:
            eps, delta = spec.budgets["count"]
            out["count"] = _noisy(acc.count, seed, idx, STREAM_COUNT, kind, noise_scale(kind, eps, delta, L0, Linf), noise)
        if "sum" in m:
            eps, delta = spec.budgets["sum"]
            linf = lin_sum_linf()
            if linf == 0:
                out["sum"] = np.zeros(P)
            else:
                out["sum"] = _noisy(acc.sum, seed, idx, STREAM_SUM, kind, noise_scale(kind, eps, delta, L0, linf), noise)
    if "privacy_id_count" in m:
        eps, delta = spec.budgets["privacy_id_count"]
        out["privacy_id_count"] = _noisy(acc.row_count, seed, idx, STREAM_PID_COUNT, kind,
                                                         noise_scale(kind, eps, delta, L0, Linf), noise)
    # a partition that private selection drops is not in the reference's result
    # (dp_engine.py:312-362): its metrics are NaN (k_release computes no noise for it)
    if spec.selection is not None:
        out = {k: np.where(keep, v, np.nan) for k, v in out.items()}
    return keep, out


def metric_field_order(metrics):
    """MetricsTuple field order produced by create_compound_combiner
    (combiners.py:652-720)."""
    m = set(metrics)
    names = []
    if "variance" in m:
        # VarianceCombiner.compute_metrics dict order (combiners.py:386-392)
        names.append("variance")
        for x in ("count", "sum", "mean"):
            if x in m:
                names.append(x)
    elif "mean" in m:
        names.append("mean")
        for x in ("count", "sum"):
            if x in m:
                names.append(x)
    else:
        for x in ("count", "sum"):
            if x in m:
                names.append(x)
    if "privacy_id_count" in m:
        names.append("privacy_id_count")
    return names


# ----------------------------------------------------------------------------
# Synthetic workload generator (same spec as the on-device generator)
# ----------------------------------------------------------------------------


def synth_rows(n, num_pids, num_partitions, seed, zipf_s=0.0, value_kind="uniform",
               value_lo=0.0, value_hi=10.0, row_offset=0):
    """Rows i = row_offset .. row_offset+n-1 of the synthetic workload
    (bench.py / pdp_generate in the HIP library):
      pid   = floor(u0 * num_pids)
      pk    = floor(u1 * P) (uniform) or Zipf(s) rank by inverse CDF of the
              continuous approximation, then scrambled by perm_bits
      value = lo + u2 * (hi - lo)  or integer ratings 1..5 ('rating').
    u* from Philox(seed, counter=(i_lo, i_hi, 0x53594E54, 0))."""
    i = np.arange(row_offset, row_offset + n, dtype=np.uint64)
    x0, x1, x2, x3 = philox4x32_10(i & _M32, i >> np.uint64(32), np.uint64(0x53594E54),
                                   np.uint64(0), np.uint64(seed & 0xFFFFFFFF),
                                   np.uint64((seed >> 32) & 0xFFFFFFFF))
    inv = 1.0 / 4294967296.0
    u0 = (x0.astype(np.float64) + 0.5) * inv
    u1 = (x1.astype(np.float64) + 0.5) * inv
    u2 = (x2.astype(np.float64) + 0.5) * inv
    pid = np.minimum((u0 * num_pids).astype(np.int64), num_pids - 1)
    P = num_partitions
    if zipf_s and zipf_s > 0:
        rank = zipf_rank(u1, P, zipf_s)
        pkb = max(1, ceil_log2(P))
        y = perm_bits(_u64(rank), pkb, np.uint64(0x5A495046))
        while True:
            bad = y >= np.uint64(P)
            if not bad.any():
                break
            y[bad] = perm_bits(y[bad], pkb, np.uint64(0x5A495046))
        pk = y.astype(np.int64)
    else:
        pk = np.minimum((u1 * P).astype(np.int64), P - 1)
    if value_kind == "rating":
        value = 1.0 + np.minimum((u2 * 5).astype(np.int64), 4).astype(np.float64)
    else:
        value = value_lo + u2 * (value_hi - value_lo)
    return pid, pk, value


def zipf_rank(u, P, s):
    """Truncated Zipf(s) rank in [0, P) by inverting the continuous
    approximation F(x) = (x^(1-s) - 1) / (P^(1-s) - 1) on x in [1, P+1)."""
    t = 1.0 - s
    hi = (P + 1.0)**t
    x = (1.0 + u * (hi - 1.0))**(1.0 / t)
    return np.minimum(np.floor(x).astype(np.int64) - 1, P - 1).clip(0)
