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
//   * Philox4x32-10 (Random123) -> uniforms in (0,1) -> Laplace as a
//     two-sided geometric on a power-of-two grid, Gaussian by Box-Muller
//     rounded to that grid; released values are snapped to the grid too.
// The noise is Philox-based: granularity-snapped like PyDP's secure
// mechanisms, but not PyDP's implementation; see DESIGN.md.
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

// Uniform in (0, 1) from a 64-bit word (hi:lo), with full relative precision
// near 0: u >= 2^-11 from the top 53 bits, below that exactly (w + 1/2) 2^-64.
// -log(u) then reaches 45 instead of the 36.7 of a 53-bit uniform, so the
// noise tails are not cut at 36.7 scales.
PDP_HD double uniform64(uint32_t hi, uint32_t lo) {
  const uint64_t w = ((uint64_t)hi << 32) | lo;
  if (w >= (1ull << 53)) return ((double)(w >> 11) + 0.5) * (1.0 / 9007199254740992.0);
  return ((double)w + 0.5) * 5.421010862427522e-20;  // 2^-64
}

// Noise grid of a mechanism with scale s (Laplace b or Gaussian sigma):
// g = 2^(ceil(log2 s) - 40).  Released values are multiples of g (the
// granularity snapping of PyDP's secure mechanisms, against the
// floating-point attack on textbook Laplace; the grid is 2^-40 of the scale,
// invisible to every distributional test).
PDP_HD double noise_grid(double s) {
  int e = 0;
  const double m = frexp(s, &e);
  return ldexp(1.0, (m == 0.5 ? e - 1 : e) - 40);
}

// Laplace(0, b) on the grid g: g * (G1 - G2) with G_i = floor(E_i b / g),
// E_i ~ Exp(1) from the two 64-bit Philox words -- the two-sided geometric
// distribution P(k g) ~ exp(-|k| g / b).
PDP_HD double laplace_on_grid(uint64_t seed, uint64_t idx, uint32_t stream, double b, double g) {
  u32x4 c{(uint32_t)idx, (uint32_t)(idx >> 32), stream, 0u};
  const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const double e1 = -log(uniform64(r.x, r.y)), e2 = -log(uniform64(r.z, r.w));
  return g * (floor(e1 * (b / g)) - floor(e2 * (b / g)));
}

// N(0, sigma^2) by Box-Muller, rounded to the grid g.
PDP_HD double gaussian_on_grid(uint64_t seed, uint64_t idx, uint32_t stream, double sigma, double g) {
  u32x4 c{(uint32_t)idx, (uint32_t)(idx >> 32), stream, 0u};
  const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const double z = sqrt(-2.0 * log(uniform64(r.x, r.y))) * cos(6.283185307179586 * uniform53(r.z, r.w));
  return g * rint(sigma * z / g);
}

// value + noise with both on the grid of `scale` (kind 0 Laplace, 1 Gaussian).
PDP_HD double add_snapped_noise(int gaussian, double value, uint64_t seed, uint64_t idx, uint32_t stream,
                                double scale) {
  const double g = noise_grid(scale);
  const double z = gaussian ? gaussian_on_grid(seed, idx, stream, scale, g)
                            : laplace_on_grid(seed, idx, stream, scale, g);
  return g * rint(value / g) + z;
}

}  // namespace pdp
