// Counter-based randomness for the DP aggregate path (host + device).
//
// Bit-for-bit the same specification as oracle/pdp_oracle.py (the CPU
// checker):
//   * splitmix64 priorities ranked per group -> uniform sampling without
//     replacement (replaces np.random.choice in
//     LocalBackend.sample_fixed_per_key,
//     /root/reference/pipeline_dp/pipeline_backend.py:504-520);
//   * a keyed Feistel bijection (only used to scramble Zipf ranks in the
//     synthetic generator);
//   * Philox4x32-10 (Random123) -> uniform doubles in (0,1) -> Laplace by
//     inverse CDF, Gaussian by Box-Muller.
// The noise is Philox-based and is NOT PyDP's secure (granularity-rounded)
// noise; see DESIGN.md.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define PDP_HD __host__ __device__ __forceinline__
#else
#define PDP_HD inline
#endif

namespace pdp {

enum : uint32_t {
  kStreamSelect = 1,
  kStreamPidCount = 2,
  kStreamCount = 3,
  kStreamSum = 4,
  kStreamMeanCount = 5,
  kStreamMeanNsum = 6,
  kStreamVarNsq = 7,
  kStreamSynth = 0x53594E54u,
};

PDP_HD uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

PDP_HD uint64_t bitmask(int bits) { return bits >= 64 ? ~0ull : ((1ull << bits) - 1ull); }

PDP_HD uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

PDP_HD uint32_t mask32(int bits) { return bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u); }

// Keyed 4-round Feistel bijection on [0, 2^bits), bits in [0, 32]; 32-bit
// round function F_r(R) = fmix32(R * 0x9E3779B1 + k_r).
PDP_HD uint32_t perm_bits(uint32_t x, int bits, uint64_t key) {
  const uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
  const uint32_t rk[4] = {k0, k1, k0 ^ 0x85EBCA6Bu, k1 ^ 0xC2B2AE35u};
  const int h1 = (bits + 1) >> 1, h2 = bits >> 1;
  int wl = h1, wr = h2;
  uint32_t left = h2 >= 32 ? 0u : (x >> h2), right = x & mask32(h2);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t f = fmix32(right * 0x9E3779B1u + rk[r]);
    const uint32_t nl = right;
    const uint32_t nr = left ^ (f & mask32(wl));
    left = nl;
    right = nr;
    const int t = wl; wl = wr; wr = t;
  }
  return (left << h2) | right;
}

PDP_HD int ceil_log2_u64(uint64_t n) {
  if (n <= 1) return 0;
#if defined(__HIP_DEVICE_COMPILE__)
  return 64 - __clzll((long long)(n - 1));
#else
  return 64 - __builtin_clzll(n - 1);
#endif
}

// Pseudo-random permutation of [0, n) at j (cycle walking), n <= 2^32.
PDP_HD uint32_t cycle_walk(uint32_t j, uint64_t n, uint64_t key) {
  if (n <= 1) return j;
  const int bits = ceil_log2_u64(n);
  uint32_t y = perm_bits(j, bits, key);
  while ((uint64_t)y >= n) y = perm_bits(y, bits, key);
  return y;
}

// Contribution-bounding priorities (uniform sampling without replacement by
// ranking 64-bit hashes; ties broken by pk / input order):
//   L0:    keep the L0 partitions of a pid with the smallest (group_priority, pk)
//   L_inf: keep the L_inf rows of a (pid, pk) group with the smallest
//          (row_priority(gprio, j), j), j = input-order rank within the group.
PDP_HD uint64_t pid_key(uint64_t seed, uint64_t pid) { return splitmix64(seed ^ splitmix64(pid + 1ull)); }

PDP_HD uint64_t group_priority(uint64_t pidkey, uint64_t pk) {
  return splitmix64(pidkey + (pk + 1ull) * 0xD1B54A32D192ED03ull);
}

PDP_HD uint64_t row_priority(uint64_t gprio, uint64_t j) {
  const uint64_t gkey = splitmix64(gprio ^ 0xA0761D6478BD642Full);
  return splitmix64(gkey + (j + 1ull) * 0x9E3779B97F4A7C15ull);
}

struct u32x4 { uint32_t x, y, z, w; };

PDP_HD void mulhilo32(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  const uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

PDP_HD u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo32(0xD2511F53u, c.x, hi0, lo0);
    mulhilo32(0xCD9E8D57u, c.z, hi1, lo1);
    u32x4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

PDP_HD double uniform53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6) + 0.5) * (1.0 / 9007199254740992.0);
}

PDP_HD void philox_uniforms(uint64_t seed, uint64_t idx, uint32_t stream, double& u1, double& u2) {
  u32x4 c{(uint32_t)idx, (uint32_t)(idx >> 32), stream, 0u};
  const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  u1 = uniform53(r.x, r.y);
  u2 = uniform53(r.z, r.w);
}

PDP_HD double unit_laplace(uint64_t seed, uint64_t idx, uint32_t stream) {
  double u, unused;
  philox_uniforms(seed, idx, stream, u, unused);
  const double d = u - 0.5;
  const double m = log1p(-2.0 * fabs(d));
  return d > 0.0 ? -m : (d < 0.0 ? m : 0.0);
}

PDP_HD double unit_gaussian(uint64_t seed, uint64_t idx, uint32_t stream) {
  double u1, u2;
  philox_uniforms(seed, idx, stream, u1, u2);
  return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

}  // namespace pdp
