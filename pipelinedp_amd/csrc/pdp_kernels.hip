// libpdp_hip.so — MI355X (gfx950) kernels for PipelineDP's DPEngine.aggregate
// hot path.  C ABI in include/pdp_hip.h; design in DESIGN.md.
//
// Pipeline of pdp_bound_accumulate (main path):
//   K0 k_histogram  : one read of pid/pk -> digit histograms of every radix
//                     pass (+ count of dropped / invalid rows)
//   K1 k_onesweep   : stable LSD radix passes on the privacy id (decoupled
//                     look-back); pass 0 packs the SoA int64/int64/f64 columns
//                     into 16-byte records and drops non-public rows
//   K2 k_segments   : per privacy-id segment batches, one wave each: register
//                     bitonic sort by (pid, pk, row), L0 / L_inf sampling by
//                     ranked hash priorities, clipping, per-(pid,pk) sums,
//                     fp64/int64 atomics into the dense [P] accumulators
//                     (k_segments_big for 257..1024-row batches)
//   KF generic path : segments > 1024 rows: LSD sorts + device-wide scans
//                     (rare; exactly the same sampling).
// pdp_release: K5/K6 k_release — selection + Laplace/Gaussian noise from
// Philox, one thread per partition.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "pdp_hip.h"
#include "pdp_rng.h"

namespace {

constexpr int kThreads = 256;
#ifndef PDP_OS_ITEMS
#define PDP_OS_ITEMS 16
#endif
#ifndef PDP_OS_OCC
#define PDP_OS_OCC 3
#endif
#ifndef PDP_OS_RANK_ATOMIC
#define PDP_OS_RANK_ATOMIC 0
#endif
#ifndef PDP_OS_STAGE_DIV
#define PDP_OS_STAGE_DIV 2
#endif
constexpr int kItems = PDP_OS_ITEMS;         // rows per thread in a radix tile
constexpr int kTile = kThreads * kItems;     // 4096 rows per radix tile (16 rows per thread)
// k_histogram_tiles' 16-byte column loads take rows in pairs; the variant builds that pass the GPU suite
// (16 rows per thread, and 12 in round 4's r04a) are the ones allowed here.
static_assert(kItems % 2 == 0 && (kItems == 16 || kItems == 12), "tile shape not validated on the GPU");
// Round 3's 12-rows-per-thread build (3072-row tiles) faulted: the per-tile
// count loops stepped over the items in groups of kHistUnroll = 8 rows per
// thread (items 0-7, 8-15) without stopping at kItems = 12, so every tile's
// digit counts also took 1024 rows of the NEXT tile; the tile bases then
// overran the record buffer in the bucket pass's scatter.  The record-pass
// loads had the same overrun (groups of kRecGroup = 16 past r[12]).  Every
// grouped item loop is now bounded by kItems.
constexpr int kMaxPasses = 12;
constexpr int kHist = 257;                   // 256 digits + drop bucket
constexpr int kStatusStride = 256;
constexpr unsigned kOverflowCap = 1u << 16;
constexpr unsigned kNumCounters = 64;

enum Counter {
  kCtrInvalid = 0,
  kCtrNKept = 1,
  kCtrNRanges = 2,
  kCtrFull = 3,
  kCtrErr = 4,
  kCtrNGeneric = 5,
  kCtrNBig = 6,
  kCtrBigNext = 7,
  kCtrSweepCycles = 8,  // 8..11: onesweep load / rank / look-back / scatter cycles (profiling)
  kCtrSweepTiles = 12,
  kCtrAnaPairs = 13,  // utility analysis: pairs of sampled partitions
  kCtrNSurv = 14,     // rows that survive the L0 pre-filter (pdp_filter.inc)
  kCtrNDropped = 15,  // rows of non-public partitions seen by k_filter
  kCtrK4In = 16,      // K4: records in the first pair pass's input (slots + generic-path pairs)
  kCtrK4Pairs = 17,   // K4: (pid, pk) pair records (non-empty slots)
  kCtrK4Chunk = 18,   // K4: pair records per reduce chunk (k4_total: ~1024 chunks, 4096 .. kK4Chunk)
  kCtrK4Slots = 19,   // K4: compacted pair records written by K2 (SegParams.k4ctr)
  kCtrTile0 = 20,  // 20..63 tile claim counters, one per onesweep launch
};

struct __align__(16) Rec {
  uint32_t pid;
  uint32_t pk;
  double val;
};

#ifndef PDP_OS_NT
#define PDP_OS_NT 0
#endif
#ifndef PDP_SCATTER_CHECK
#define PDP_SCATTER_CHECK 0
#endif
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// 16-byte record load / store of the radix passes (streamed once: optionally
// non-temporal so they do not displace the L2's working set).
__device__ __forceinline__ Rec ld_rec(const Rec* p) {
#if PDP_OS_NT & 1
  const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
  Rec r;
  r.pid = v.x;
  r.pk = v.y;
  r.val = __longlong_as_double((long long)(((uint64_t)v.w << 32) | v.z));
  return r;
#else
  return *p;
#endif
}

__device__ __forceinline__ void st_rec(Rec* p, const Rec& r) {
#if PDP_OS_NT & 2
  const uint64_t b = (uint64_t)__double_as_longlong(r.val);
  u32x4 v;
  v.x = r.pid;
  v.y = r.pk;
  v.z = (unsigned int)b;
  v.w = (unsigned int)(b >> 32);
  __builtin_nontemporal_store(v, (u32x4*)p);
#else
  *p = r;
#endif
}

constexpr uint32_t kK4EmptyKey = 0xFFFFFFFFu;  // K4 empty pair slot (pdp_reduce.inc kK4Empty)

// K4 12-byte pair records (pdp_reduce.inc): {key, x lo, x hi} with key = pk << cb | (count - 1) (the y
// records' count is 0 -> key = pk << cb); an empty slot keeps key 0xFFFFFFFF.  In registers and LDS a
// record stays a Rec (pid slot = key, pk slot unused).
__device__ __forceinline__ Rec k4_pack12(Rec r, int cb) {
  if (r.pid != kK4EmptyKey) r.pid = (r.pid << cb) | ((r.pk > 0u ? r.pk - 1u : 0u) & ((1u << cb) - 1u));
  return r;
}
__device__ __forceinline__ Rec k4_ld12(const Rec* base, int64_t i) {
  const uint32_t* p = reinterpret_cast<const uint32_t*>(base) + 3 * i;
  Rec r;
  r.pid = p[0];
  r.pk = 0u;
  r.val = __longlong_as_double((long long)(((uint64_t)p[2] << 32) | p[1]));
  return r;
}
// split slots (SegParams.k4soa): the key array, then the values; the offset keeps the values 16-B aligned
// and inside a buffer of 16 bytes per slot (at most 12 n + 12 bytes)
inline int64_t k4_soa_offset(int64_t nslots) { return (std::max<int64_t>(nslots, 1) * 4 + 15) / 16 * 16; }
__device__ __forceinline__ void k4_st12(Rec* base, int64_t i, const Rec& r) {
  uint32_t* p = reinterpret_cast<uint32_t*>(base) + 3 * i;
  const uint64_t b = (uint64_t)__double_as_longlong(r.val);
  p[0] = r.pid;
  p[1] = (uint32_t)b;
  p[2] = (uint32_t)(b >> 32);
}

struct KeySpec {
  int mode;  // 0: key = pid >> low ; 1: key = (pid << pkb) | pk ; 3: key = (pid, bits(val)) 96-bit ;
             // 4: bucketed pid: passes with shift >= 64 take the bucket digit (pid * mult) >> 32, others pid bits ;
             // 6: K4 pair records {pk, count, x}: key = pk >> low (the partition block), empty slots dropped
  int passes;
  int shift[kMaxPasses];
  int bits[kMaxPasses];
  int low;
  int pkb;
  uint64_t seed;
  uint64_t num_pids;  // up to 2^32 (pid values 0 .. 2^32 - 1)
  uint64_t pid_base;  // the sampling hashes pid_base + pid (pdp_bound_params.pid_base)
  uint32_t num_parts;
  uint64_t mult;  // mode 4: bucket digit multiplier (pdp_filter.inc)
  // the pre-filter's bucket pass (TAG): within a tile's run of a bucket, rows of sketch level <= tau come
  // first (a stable split by one class bit; the order within a (pid, pk) group -- one level -- is kept)
  int tau;
  // ... and in every odd tile they come LAST: the class-0 rows of tiles 2i+1 and 2i+2 then sit side by side
  // in the bucket's region, so k_filter's survivor gather reads about half as many lines
  int flip;
  int prof;  // accumulate per-phase s_memtime cycles of k_onesweep (kDebugSweepStamps)
  int ablate;  // kDebugNoLookback / kDebugLinearWrite (timing ablations, results invalid)
  int xcd_remap;  // reduce-then-scan passes: blocks sharing an XCD take one contiguous run of tiles
  int64_t cap;  // mode 6: records the output holds; a scatter position beyond it is reported, not written
  // mode 6, first pass of k_pair_pass12s: the slots are split (keys u32[], then values f64[] at these byte
  // offsets from rin / rin2), so an empty slot costs its 4-byte key
  int64_t soa_a, soa_b;
};

// How a row's value feeds the accumulators (combiners.py:254-261, 305-311,
// 364-373).
enum XMode { kXNone = 0, kXNsum = 1, kXClipSum = 2, kXRawSum = 3 };

struct SegParams {
  int low;
  int pkb;
  uint64_t seed;
  int64_t l0;
  int64_t linf;
  int xmode;
  int want_y;
  int want_count;
  int has_value;
  double a, b, mid;
  double smin, smax;
  int packed;  // row_count word holds (count << 32) | row_count until k_unpack_counts
  int debug;   // experiment flags (bench ablations), kDebugBatchKernel
  // K4 (deterministic per-partition reduction, pdp_reduce.inc).  k4x != null: K2 writes one pair
  // record {pk, count, x} per kept (pid, pk) group into slot k4x[s + i] of its segment [s, s + n)
  // (empty records in the segment's other slots) instead of adding to the accumulators, and
  // counts the records' partition-block digits in k4hist; VARIANCE writes {pk, 0, y} to k4y.
  // k4cb >= 0: the slots are the 12-byte records {pk << k4cb | count - 1, x} of the pair passes
  // (k4_pack12; an empty slot writes only its all-ones key); -1: 16-byte Rec slots.
  Rec* k4x;
  Rec* k4y;
  int k4cb;
  // k4cb >= 0 and k4soa > 0: split slots instead -- keys u32[slot] at k4x / k4y and the values f64[slot]
  // k4soa bytes further (k4_soa_offset), so the first pair pass reads 4 bytes of an empty slot, not 12
  int64_t k4soa;
  unsigned int* k4hist;  // [kK4Rep][kK4MaxPasses][256]
  // != null: compacted pair records -- K2 writes only its kept groups, at slots claimed from this
  // counter (k4_claim, one atomic per wave), no empty records; null: the slot form above
  unsigned long long* k4ctr;
  int k4sh;              // partition block = pk >> k4sh
  int k4passes;
  int k4shift[3];
  int k4bits[3];
  uint64_t pid_base;  // pdp_bound_params.pid_base: the sampling hashes pid_base + pid
  // K4 hot-partition table (pdp_reduce.inc, K4Hot): k4hot != 0 -- the K2 kernel holds a per-block LDS
  // table whose pairs are added in fixed point (q = rint(x * k4q)) and flushed with integer atomics
  // into the accumulators' counts and K4's fixed-point scratch k4glo / k4ghi / k4gfl.
  int k4hot;
  double k4q;
  unsigned long long* k4glo;
  unsigned long long* k4ghi;
  unsigned int* k4gfl;
};

constexpr int kDebugBatchKernel = 4096;  // use k_segments even when k_lean applies
constexpr int kDebugSweepStamps = 8192;  // per-phase cycle stamps in k_onesweep -> pdp_stats
// Timing ablations of the radix passes (bench experiments only; accumulators
// are left zero): stop after the sort, skip the look-back (prefix 0), write
// each tile back to its own rows instead of scattering digit runs.
constexpr int kDebugSortOnly = 16384;
constexpr int kDebugNoLookback = 32768;
constexpr int kDebugLinearWrite = 65536;
constexpr int kDebugNoScatter = 2048;  // with kDebugSortOnly: the radix passes stage in LDS but store nothing
constexpr int kDebugLookback = 131072;  // radix passes by decoupled look-back instead of reduce-then-scan
constexpr int kDebugNoAtomics = 262144;  // K2 skips its accumulator atomics (timing ablation)
constexpr int kDebugNoHotCache = 524288;  // K2 without its LDS hot-partition table (K4 off: HotCache; on: K4Hot)
constexpr int kDebugLeanMinSearch = 1048576;  // k_lean ranks L0 by minimum searches even when L0 >= kSortMinL0
constexpr int kDebugWalkOnly = 2097152;  // k_lean loads rows and finds segments only (timing floor, results invalid)
constexpr int kDebugNoLinf = 8388608;     // k_lean skips the L_inf ranking (timing ablation, results invalid)
constexpr int kDebugNoSums = 16777216;    // k_lean skips the kept-row sums (timing ablation, results invalid)
constexpr int kDebugForceHotCache = 33554432;  // k_lean uses the LDS partition cache at any L0
constexpr int kDebugThin2 = 67108864;          // K4 on: the LDS-staged k_thin2 instead of k_thin (round 5 experiment)
constexpr int kDebugNoFilter = 134217728;      // never use the L0 pre-filter (pdp_filter.inc)
constexpr int kDebugForceFilter = 268435456;   // use the L0 pre-filter whenever it applies (small inputs too)
constexpr int kDebugNoThin = 536870912;        // bound the pre-filter's survivors with k_lean instead of k_thin
constexpr int kDebugFilterTiming = 1073741824;  // k_filter timing ablation: phase 1 only (results invalid)
constexpr int kDebugLinfSort = 1 << 22;  // lean_segment_sorted: L_inf by a second wave sort (round-2 form)
// Alternative forms with identical results (parity tests A/B them; pdp_bound_params.reserved or
// pdp_ctx_set_debug), replacing round 4's PDP_* environment knobs: the shipped library reads no
// environment and has one semantics ("Determinism").
constexpr int kDebugNoK4 = 1;               // K4 off: the round-2 fp64-atomic accumulation (last bits differ)
constexpr int kDebugK4P16 = 2;              // K4 pair passes on 16-byte records even when 12-byte ones fit
constexpr int kDebugK4Soa = 4;              // K4 12-byte slots written split (keys, then values)
constexpr int kDebugOddGrid = 8;            // K2 grids of 7 (k_thin) / 5 (k_lean) blocks: determinism tests
constexpr int kDebugSortTileScan = 16;      // sort_recs by reduce-then-scan instead of decoupled look-back
constexpr int kDebugAnaNpartAtomics = 32;   // utility analysis: n_partitions by one atomic per pair
constexpr int kDebugAnaPack = 64;           // utility analysis: separate pack kernel before the sort
constexpr int kDebugAnaFlags = 128;         // utility analysis: round-3 per-row flags + scan pair extraction
constexpr int kDebugAnaSelLds = 256;        // utility analysis: round-3 per-regime selection kernels
constexpr int kDebugDevOcc2 = 512;          // device-sized look-back passes at 2 blocks per CU (no spills, slower)
constexpr int kDebugK4Compact = 1024;       // K2 writes compacted K4 pair records (k4_claim) instead of a slot per row
// Second word of testing flags (pdp_bound_params.reserved2; the first word's 31 bits are taken).
constexpr int kDebug2OverflowFull1 = 1;     // a second overflow range already sets kCtrFull (the whole-input redo)
// the pre-filter's bucket pass carries 8-byte {pk, row index} records and k_filter gathers the survivors'
// values by row index (round-6 experiment: bucket pass 9.13 -> 7.6 ms, filter 3.26 -> 5.2 ms: slower, r06c)
constexpr int kDebug2FilterRec8 = 2;
constexpr int kDebug2NoGroup = 4;        // survivor grouping by the round-5 second look-back pass, not k_group
constexpr int kDebug2GroupFallback = 8;  // k_filter hands every grouping to the look-back pass (kGrpBig = 1)
constexpr int kDebug2NoClassSplit = 16;  // bucket pass: no low-level-first order within a tile's bucket run
constexpr int kDebug2ThinChunk2048 = 32;  // k_thin's 2048-row chunks whatever the expected survivor count
// Timing ablations whose results are invalid: accepted only by a -DPDP_DEBUG_BUILD library.
constexpr int kAblationFlags = kDebugSortOnly | kDebugNoLookback | kDebugLinearWrite | kDebugNoScatter |
                               kDebugNoAtomics | kDebugWalkOnly | kDebugNoLinf | kDebugNoSums | kDebugFilterTiming;
#ifdef PDP_DEBUG_BUILD
constexpr bool kDebugBuild = true;
#else
constexpr bool kDebugBuild = false;
#endif

struct AccPtrs {
  unsigned long long* row_count;
  unsigned long long* count;
  double* x;
  double* y;
};

struct OvList {
  unsigned long long* ranges;  // [cap][2] (start, end)
  unsigned long long* counters;
  // testing (debug2 flag OVERFLOW_FULL1): more than this many overflow ranges also set kCtrFull (the ranges
  // stay recorded and valid); 0 = only beyond kOverflowCap
  unsigned long long full_at;
};

// Digit of radix pass `pass` of record r.  Mode 3 sorts by the 96-bit key
// (pid field, bit pattern of val): passes with shift >= 64 read the pid field.
__device__ __forceinline__ uint32_t digit_of(const KeySpec& ks, int pass, const Rec& r) {
  const uint64_t mask = (1ull << ks.bits[pass]) - 1ull;
  const int sh = ks.shift[pass];
  uint64_t key;
  // Mode 6 (K4 pair records) keys like mode 0; its empty slots are dropped by
  // the caller (onesweep_body).  (Round 3's "miscompile" of an early-return
  // branch here was stale look-back status words)
  if (ks.mode == 0 || ks.mode == 6) {
    key = (uint64_t)(r.pid >> ks.low);
  } else if (ks.mode == 4) {
    if (sh >= 64) return (uint32_t)(((uint64_t)r.pid * ks.mult) >> 32);
    key = (uint64_t)r.pid;
  } else if (ks.mode == 1) {
    key = ((uint64_t)r.pid << ks.pkb) | (uint64_t)r.pk;
  } else {
    if (sh >= 64) return (uint32_t)(((uint64_t)r.pid >> (sh - 64)) & mask);
    key = (uint64_t)__double_as_longlong(r.val);
  }
  return (uint32_t)((key >> sh) & mask);
}

__device__ __forceinline__ double clip(double v, double lo, double hi) {
  // NaN-propagating like np.clip.
  return v < lo ? lo : (v > hi ? hi : v);
}

// ---------------------------------------------------------------------------
// Block-level helpers (256 threads = 4 waves of 64)
// ---------------------------------------------------------------------------

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T x = __shfl_up(v, o);
    if (lane >= o) v += x;
  }
  return v;
}

// Exclusive scan across the block; returns exclusive prefix, sets total.
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* s_tmp /*[4]*/, T& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  T inc = wave_incl_scan(v);
  if (lane == 63) s_tmp[wave] = inc;
  __syncthreads();
  T add = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const T s = s_tmp[w];
    if (w < wave) add += s;
    tot += s;
  }
  __syncthreads();
  total = tot;
  return add + inc - v;
}

template <typename T>
__device__ __forceinline__ T block_min(T v, T* s_tmp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T x = __shfl_xor(v, o);
    v = x < v ? x : v;
  }
  if (lane == 0) s_tmp[wave] = v;
  __syncthreads();
  T r = s_tmp[0];
#pragma unroll
  for (int w = 1; w < 4; ++w) r = s_tmp[w] < r ? s_tmp[w] : r;
  __syncthreads();
  return r;
}

template <typename T>
__device__ __forceinline__ T block_max(T v, T* s_tmp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T x = __shfl_xor(v, o);
    v = x > v ? x : v;
  }
  if (lane == 0) s_tmp[wave] = v;
  __syncthreads();
  T r = s_tmp[0];
#pragma unroll
  for (int w = 1; w < 4; ++w) r = s_tmp[w] > r ? s_tmp[w] : r;
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------
// K0: digit histograms of every pass from one read of the keys
// ---------------------------------------------------------------------------

#ifndef PDP_HIST_UNROLL
#define PDP_HIST_UNROLL 8
#endif
#ifndef PDP_HIST_NT
#define PDP_HIST_NT 1  // non-temporal column loads in k_histogram_tiles (c3 K0 1.60 -> 1.49 ms, r04b)
#endif
#ifndef PDP_HIST_V3
#define PDP_HIST_V3 1  // k_histogram_tiles<PID_ONLY>: one LDS atomic per row (the histogram adds the tile counts)
#endif
#ifndef PDP_HIST_V2
#define PDP_HIST_V2 1  // k_histogram_tiles: 16-byte column loads (two rows per lane) for full, aligned tiles
#endif
constexpr int kHistUnroll = PDP_HIST_UNROLL;  // rows per thread with loads in flight together (K0, K1u)

// Utility-analysis record of a row (k_ana_pack restated for the fused first pass):
// {pk, pid, value} for a row in range, the all-ones key (sorts last) otherwise;
// `invalid` counts the out-of-range rows that are errors (pk >= P, or a public
// row's pid out of range).
__device__ __forceinline__ Rec ana_rec(int64_t a, int64_t b, double v, const KeySpec& ks, unsigned int& invalid) {
  const bool ok = b >= 0 && b < (int64_t)ks.num_parts && a >= 0 && a < (int64_t)ks.num_pids;
  invalid += b >= (int64_t)ks.num_parts || (b >= 0 && (a < 0 || a >= (int64_t)ks.num_pids));
  return ok ? Rec{(uint32_t)b, (uint32_t)a, v} : Rec{0xFFFFFFFFu, 0xFFFFFFFFu, 0.0};
}

// MODE 0: records; 1: SoA columns (rows out of range dropped); 2: SoA columns of the utility
// analysis (the records k_ana_pack would write: {pk, pid}, rows out of range as the all-ones
// key that sorts last, pdp_analysis.inc)
// n_dev != null: the row count is *n_dev (device memory; n is then an upper bound).
template <int MODE>
__global__ __launch_bounds__(kThreads) void k_histogram(const int64_t* __restrict__ pid,
                                                        const int64_t* __restrict__ pk,
                                                        const Rec* __restrict__ rin, int64_t n,
                                                        KeySpec ks, unsigned long long* __restrict__ hist,
                                                        unsigned long long* __restrict__ counters,
                                                        const unsigned long long* __restrict__ n_dev) {
  __shared__ unsigned int sh[kMaxPasses * kHist];
  if (n_dev) n = (int64_t)*n_dev;
  for (int i = threadIdx.x; i < kMaxPasses * kHist; i += kThreads) sh[i] = 0;
  __syncthreads();
  unsigned int invalid = 0;
  // kHistUnroll rows per thread per step, loads first (clamped indices), so
  // they are in flight together instead of one HBM round trip per row.
  const int64_t stride = (int64_t)gridDim.x * kThreads * kHistUnroll;
  for (int64_t i0 = (int64_t)blockIdx.x * kThreads * kHistUnroll + threadIdx.x; i0 < n; i0 += stride) {
    Rec r[kHistUnroll];
    int64_t a[kHistUnroll], b[kHistUnroll];
#pragma unroll
    for (int u = 0; u < kHistUnroll; ++u) {
      const int64_t i = i0 + (int64_t)u * kThreads, ic = i < n ? i : n - 1;
      if (MODE != 0) {
        a[u] = pid[ic];
        b[u] = pk[ic];
      } else {
        r[u] = rin[ic];
      }
    }
#pragma unroll
    for (int u = 0; u < kHistUnroll; ++u) {
      if (i0 + (int64_t)u * kThreads >= n) break;
      if (MODE == 2) {
        r[u] = ana_rec(a[u], b[u], 0.0, ks, invalid);
      } else if (MODE == 1) {
        if (b[u] < 0 || b[u] >= (int64_t)ks.num_parts || a[u] < 0 || a[u] >= (int64_t)ks.num_pids) {
          if (b[u] >= 0) ++invalid;
          atomicAdd(&sh[256], 1u);
          continue;
        }
        r[u].pid = (uint32_t)a[u];
        r[u].pk = (uint32_t)b[u];
        r[u].val = 0.0;
      }
      for (int p = 0; p < ks.passes; ++p) atomicAdd(&sh[p * kHist + digit_of(ks, p, r[u])], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ks.passes * kHist; i += kThreads)
    if (sh[i]) atomicAdd(&hist[i], (unsigned long long)sh[i]);
  if (invalid) atomicAdd(&counters[kCtrInvalid], (unsigned long long)invalid);
}

// K0 (tile form): the same histograms, plus the pass-0 digit count of every
// 4096-row input tile (tile_cnt[tile][256], u32) for the reduce-then-scan
// radix pass.  Blocks stride over whole tiles.
// PID_ONLY (the bucket pass of the L0 pre-filter): the partition column is
// not read; a row is dropped only for an out-of-range privacy id, and rows of
// non-public partitions are placed too (k_onesweep<true, true> tags them,
// k_filter drops them).
template <bool PID_ONLY>
__global__ __launch_bounds__(kThreads) void k_histogram_tiles(const int64_t* __restrict__ pid,
                                                              const int64_t* __restrict__ pk, int64_t n,
                                                              KeySpec ks, unsigned long long* __restrict__ hist,
                                                              unsigned int* __restrict__ tile_cnt,
                                                              unsigned long long* __restrict__ counters) {
  // PID_ONLY (the pre-filter's bucket digit): one pass, so the histogram is the sum of the tile counts
  constexpr bool kFromTiles = PID_ONLY && PDP_HIST_V3;
  __shared__ unsigned int sh[(kFromTiles ? 1 : kMaxPasses) * kHist];
  __shared__ unsigned int st[256];
  const int t = threadIdx.x;
  for (int i = t; i < (kFromTiles ? 1 : kMaxPasses) * kHist; i += kThreads) sh[i] = 0;
  st[t] = 0;
  __syncthreads();
  unsigned int invalid = 0;
  const int64_t tiles = (n + kTile - 1) / kTile;
  // 16-byte loads (two rows per lane, PDP_HIST_V2) need 16-byte aligned columns
  const bool v2 = PDP_HIST_V2 && ((reinterpret_cast<uintptr_t>(pid) | (PID_ONLY ? 0 : reinterpret_cast<uintptr_t>(pk))) & 15) == 0;
  auto count_row = [&](int64_t a, int64_t b) {
    if (b < 0 || b >= (int64_t)ks.num_parts || a < 0 || a >= (int64_t)ks.num_pids) {
      if (b >= 0) ++invalid;
      atomicAdd(&sh[256], 1u);
      return;
    }
    Rec r;
    r.pid = (uint32_t)a;
    r.pk = (uint32_t)b;
    r.val = 0.0;
    const uint32_t d0 = digit_of(ks, 0, r);
    atomicAdd(&st[d0], 1u);
    if constexpr (!kFromTiles) {
      atomicAdd(&sh[d0], 1u);
      for (int p = 1; p < ks.passes; ++p) atomicAdd(&sh[p * kHist + digit_of(ks, p, r)], 1u);
    }
  };
  for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int64_t base = tile * kTile + t;
    const bool full = (tile + 1) * kTile <= n;
    if (v2 && full) {  // the tile as kItems / 2 slices of 2 * kThreads rows; lane t reads rows 2t, 2t + 1
      typedef long long ll2 __attribute__((ext_vector_type(2)));
      const ll2* pv = reinterpret_cast<const ll2*>(pid + tile * kTile);
      const ll2* kv = reinterpret_cast<const ll2*>(pk + tile * kTile);
      ll2 a[kItems / 2], b[kItems / 2];
#pragma unroll
      for (int u = 0; u < kItems / 2; ++u) {
        a[u] = __builtin_nontemporal_load(pv + u * kThreads + t);
        if (!PID_ONLY) b[u] = __builtin_nontemporal_load(kv + u * kThreads + t);
      }
#pragma unroll
      for (int u = 0; u < kItems / 2; ++u) {
        count_row(a[u].x, PID_ONLY ? 0 : b[u].x);
        count_row(a[u].y, PID_ONLY ? 0 : b[u].y);
      }
      __syncthreads();
      tile_cnt[tile * 256 + t] = st[t];
      if (kFromTiles) sh[t] += st[t];
      st[t] = 0;
      __syncthreads();
      continue;
    }
#pragma unroll
    for (int g = 0; g < kItems; g += kHistUnroll) {
      int64_t a[kHistUnroll], b[kHistUnroll];
#pragma unroll
      for (int u = 0; u < kHistUnroll && g + u < kItems; ++u) {  // loads first (clamped), then the counting
        const int64_t i = base + (int64_t)(g + u) * kThreads, ic = full || i < n ? i : n - 1;
#if PDP_HIST_NT
        a[u] = __builtin_nontemporal_load(pid + ic);
        b[u] = PID_ONLY ? 0 : __builtin_nontemporal_load(pk + ic);
#else
        a[u] = pid[ic];
        b[u] = PID_ONLY ? 0 : pk[ic];
#endif
      }
#pragma unroll
      for (int u = 0; u < kHistUnroll && g + u < kItems; ++u) {
        if (!full && base + (int64_t)(g + u) * kThreads >= n) break;
        count_row(a[u], b[u]);
      }
    }
    __syncthreads();
    tile_cnt[tile * 256 + t] = st[t];
    if (kFromTiles) sh[t] += st[t];
    st[t] = 0;
    __syncthreads();
  }
  for (int i = t; i < (kFromTiles ? 1 : ks.passes) * kHist; i += kThreads)
    if (sh[i]) atomicAdd(&hist[i], (unsigned long long)sh[i]);
  if (invalid) atomicAdd(&counters[kCtrInvalid], (unsigned long long)invalid);
}

// K1u (upsweep of a records pass): digit count of every tile of `rin`.
// (Tried: pid / pk / value split into three arrays between passes so this
// reads 4 B per row -- it did, 2.1 -> 0.95 ms per launch at c3, but the
// 4- and 8-byte digit-run scatters of the passes cost more: pass 0 11.3 ->
// 17.4 ms.  Records stay 16-B AoS.)
__global__ __launch_bounds__(kThreads) void k_tile_counts(const Rec* __restrict__ rin,
                                                          const unsigned long long* __restrict__ counters_n,
                                                          int n_slot, KeySpec ks, int pass, int64_t tiles,
                                                          unsigned int* __restrict__ tile_cnt) {
  __shared__ unsigned int st[256];
  const int t = threadIdx.x;
  st[t] = 0;
  __syncthreads();
  const int64_t n = (int64_t)counters_n[n_slot];
  for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int64_t base = tile * kTile + t;
#pragma unroll
    for (int g = 0; g < kItems; g += kHistUnroll) {
      Rec r[kHistUnroll];
#pragma unroll
      for (int u = 0; u < kHistUnroll && g + u < kItems; ++u) {
        const int64_t i = base + (int64_t)(g + u) * kThreads;
        if (n > 0) r[u] = rin[i < n ? i : n - 1];  // n == 0 (every row dropped): no load at all
      }
#pragma unroll
      for (int u = 0; u < kHistUnroll && g + u < kItems; ++u)
        if (base + (int64_t)(g + u) * kThreads < n) atomicAdd(&st[digit_of(ks, pass, r[u])], 1u);
    }
    __syncthreads();
    tile_cnt[tile * 256 + t] = st[t];
    st[t] = 0;
    __syncthreads();
  }
}

// The same for the K4 pair passes (reduce-then-scan instead of decoupled
// look-back; round 4): records read as the pass reads them (P12: 12-byte
// records; pass 0 also reads the generic path's pairs after `split`), empty
// slots not counted.
template <int P12>
__global__ __launch_bounds__(kThreads) void k_pair_tile_counts(const Rec* __restrict__ rin,
                                                               const Rec* __restrict__ rin2, int64_t split,
                                                               const unsigned long long* __restrict__ counters_n,
                                                               int n_slot, KeySpec ks, int pass, int64_t tiles,
                                                               unsigned int* __restrict__ tile_cnt) {
  __shared__ unsigned int st[256];
  const int t = threadIdx.x;
  st[t] = 0;
  __syncthreads();
  const int64_t n = (int64_t)counters_n[n_slot];
  for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int64_t base = tile * kTile + t;
#pragma unroll
    for (int g = 0; g < kItems; g += kHistUnroll) {
      Rec r[kHistUnroll];
#pragma unroll
      for (int u = 0; u < kHistUnroll && g + u < kItems; ++u) {
        const int64_t i = base + (int64_t)(g + u) * kThreads;
        const int64_t ic = i < n ? i : n - 1;
        if (n > 0) {
          if constexpr (P12 != 0) {
            r[u] = ic < split ? k4_ld12(rin, ic) : k4_ld12(rin2, ic - split);
          } else {
            r[u] = ld_rec(ic < split ? rin + ic : rin2 + (ic - split));
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kHistUnroll && g + u < kItems; ++u)
        if (base + (int64_t)(g + u) * kThreads < n && r[u].pid != kK4EmptyKey)
          atomicAdd(&st[digit_of(ks, pass, r[u])], 1u);
    }
    __syncthreads();
    tile_cnt[tile * 256 + t] = st[t];
    st[t] = 0;
    __syncthreads();
  }
}

// Tile-offset scan, step 1: per chunk of kScanTiles tiles, the digit sums.
constexpr int kScanTiles = 256;
__global__ __launch_bounds__(kThreads) void k_tile_chunk_sums(const unsigned int* __restrict__ tile_cnt,
                                                              int64_t tiles, unsigned int* __restrict__ chunk) {
  const int t = threadIdx.x;
  const int64_t t0 = (int64_t)blockIdx.x * kScanTiles;
  const int64_t t1 = t0 + kScanTiles < tiles ? t0 + kScanTiles : tiles;
  unsigned int s = 0;
#pragma unroll 8
  for (int64_t i = t0; i < t1; ++i) s += tile_cnt[i * 256 + t];
  chunk[(int64_t)blockIdx.x * 256 + t] = s;
}

// Step 2 (one block per digit): exclusive scan of the chunk sums of digit d,
// plus the global digit start off[d].
__global__ __launch_bounds__(kThreads) void k_tile_chunk_scan(unsigned int* __restrict__ chunk, int64_t nchunks,
                                                              const unsigned long long* __restrict__ off) {
  __shared__ unsigned int s_tmp[4];
  const int t = threadIdx.x, d = blockIdx.x;
  const int64_t per = (nchunks + kThreads - 1) / kThreads;
  const int64_t c0 = (int64_t)t * per;
  unsigned int s = 0;
  for (int64_t c = c0; c < c0 + per && c < nchunks; ++c) s += chunk[c * 256 + d];
  unsigned int total;
  unsigned int run = (unsigned int)off[d] + block_excl_scan(s, s_tmp, total);
  for (int64_t c = c0; c < c0 + per && c < nchunks; ++c) {
    const unsigned int v = chunk[c * 256 + d];
    chunk[c * 256 + d] = run;
    run += v;
  }
}

// Step 3: tile_cnt[tile][d] <- global start of digit d's run of this tile.
__global__ __launch_bounds__(kThreads) void k_tile_bases(unsigned int* __restrict__ tile_cnt, int64_t tiles,
                                                         const unsigned int* __restrict__ chunk) {
  const int t = threadIdx.x;
  const int64_t t0 = (int64_t)blockIdx.x * kScanTiles;
  const int64_t t1 = t0 + kScanTiles < tiles ? t0 + kScanTiles : tiles;
  unsigned int run = chunk[(int64_t)blockIdx.x * 256 + t];
#pragma unroll 8
  for (int64_t i = t0; i < t1; ++i) {
    const unsigned int v = tile_cnt[i * 256 + t];
    tile_cnt[i * 256 + t] = run;
    run += v;
  }
}

// Bucket start offsets (exclusive scan of each pass histogram) and the number
// of rows that survive pass 0.
__global__ __launch_bounds__(kThreads) void k_offsets(const unsigned long long* __restrict__ hist,
                                                      unsigned long long* __restrict__ off, int passes,
                                                      int64_t n, unsigned long long* __restrict__ counters,
                                                      int n_slot, const unsigned long long* __restrict__ n_dev) {
  __shared__ unsigned long long s_tmp[4];
  if (n_dev) n = (int64_t)*n_dev;
  for (int p = 0; p < passes; ++p) {
    const unsigned long long v = hist[p * kHist + threadIdx.x];
    unsigned long long tot;
    const unsigned long long ex = block_excl_scan(v, s_tmp, tot);
    off[p * kHist + threadIdx.x] = ex;
  }
  if (threadIdx.x == 0) counters[n_slot] = (unsigned long long)n - hist[256];
}

#include "pdp_filter.inc"

// ---------------------------------------------------------------------------
// K1: one stable LSD radix pass, single sweep with decoupled look-back.
// ---------------------------------------------------------------------------

constexpr uint64_t kFlagAgg = 1ull << 46;
constexpr uint64_t kFlagPre = 2ull << 46;
constexpr uint64_t kFlagMask = 3ull << 46;
constexpr uint64_t kValMask = (1ull << 46) - 1ull;
#ifndef PDP_LOOKBACK
#define PDP_LOOKBACK 8
#endif
constexpr int kLookback = PDP_LOOKBACK;

// LDS per block ~39 KB (half-tile record staging, digits recomputed from the
// staged record) and <= 128 VGPRs, so 4 blocks (16 waves) share a CU: the
// per-tile latency chain (tile claim, loads, look-back) is hidden by the
// other blocks instead of idling the CU.
constexpr int kHalfTile = kTile / PDP_OS_STAGE_DIV;
// SoA rows loaded per batch (first pass / bucket pass).  All of a thread's rows at once (3 x 16 loads in
// flight per lane, then the digits / tags): bucket pass 11.3 -> 8.9 ms against one row at a time (r04a,
// same box; the no-scatter ablation put the old load phase at 8.2 ms of 11.3).
#ifndef PDP_SOA_GROUP
#define PDP_SOA_GROUP 16
#endif
constexpr int kSoaGroup = PDP_SOA_GROUP < kItems ? PDP_SOA_GROUP : kItems;
// Non-temporal loads of the SoA input columns (read once per pass).
#ifndef PDP_SOA_NT
#define PDP_SOA_NT 0
#endif
template <typename T>
__device__ __forceinline__ T ld_soa(const T* p) {
#if PDP_SOA_NT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}
#ifndef PDP_REC_GROUP
#define PDP_REC_GROUP 16
#endif
constexpr int kRecGroup = PDP_REC_GROUP;  // records loaded per batch (passes on records)
constexpr uint32_t kNoPos = 0xFFFFu;

// TAG (the bucket pass of the L0 pre-filter, pdp_filter.inc): also writes,
// for every placed row, tag = bucket << 22 | (pid - first pid of its bucket)
// << 5 | level of its group priority (kTagDropped set for a non-public row),
// into tag_out at the row's sorted position.  The record carries the tag in
// its pid slot (k_filter rebuilds the pid), so no extra registers or LDS hold
// it between the load and the scatter (a separate tag array spilled 64 B per
// lane to scratch: ~8 GB of extra traffic per 1e9 rows).
// rin2 / split (K4 pair passes): input record i is rin[i] for i < split, else rin2[i - split] (the
// first pair pass reads K2's slots followed by the generic path's pairs).
// Bijective XCD swizzle (cdna_hip_programming.md T1): blocks b with equal
// b % 8 get one contiguous range of ids, in dispatch order.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nwg) {
  const uint32_t q = nwg / 8u, r = nwg % 8u, x = b % 8u;
  return (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + b / 8u;
}

// P12 (K4 pair passes with 12-byte records {key = pk << cb | count - 1, x}, pdp_reduce.inc): 12-B
// records in (K2's slots, then the generic path's pairs after `split`) and out.
// ANA (with SOA): the utility analysis' first pass -- the columns become the {pk, pid, value} records of
// ana_rec (k_ana_pack fused in); no row is dropped (out-of-range rows carry the all-ones key).
// Returns false when the claimed tile lies beyond the row count (the block is done): the look-back
// wrappers loop over tiles claimed in order, so a grid smaller than the tile count (sized from a host
// upper bound while the row count lives in device memory) covers every tile.
// TAG 1: the bucket pass's 16-byte records {tag, pk, value}.  TAG 2 (round-6 experiment, debug2 flag
// FILTER_REC8): the pass does not carry the values -- a row's record is 8 bytes {pk, row index} (rows <
// 2^32: the pre-filter needs the reduce-then-scan passes), and k_filter gathers the value of each SURVIVOR
// from the input column by its row index.  The pass reads 16 instead of 24 B and writes 12 instead of 20
// B per row (c3: 9.13 -> 7.6 ms), but the filter's two extra random gathers per survivor (value, tag)
// cost more (3.26 -> 5.2 ms, r06c): off by default.
template <bool SOA, int TAG = 0, int P12 = 0, bool ANA = false>
__device__ __forceinline__ bool onesweep_body(
    const int64_t* __restrict__ pid, const int64_t* __restrict__ pk, const double* __restrict__ val,
    const Rec* __restrict__ rin, Rec* __restrict__ rout, int64_t n_in,
    const unsigned long long* __restrict__ counters_n, int n_slot, KeySpec ks, int pass,
    const unsigned long long* __restrict__ off, unsigned long long* __restrict__ status, uint32_t epoch,
    unsigned long long* __restrict__ counters, int tile_slot, const unsigned int* __restrict__ tile_base,
    uint32_t* __restrict__ tag_out, const uint32_t* __restrict__ tag_lo, const Rec* __restrict__ rin2,
    int64_t split) {
  // TAG: the in-tile ranking key is the sub-digit 2 d + class (512 sub-digits, 512 dropped, 513 padding)
  constexpr int kSub = TAG ? 2 : 1;
  constexpr int kCntW = TAG ? 2 * 256 + 2 : kHist + 1;
  constexpr int kDrShift = TAG ? 10 : 9;
  constexpr uint32_t kDrMask = (1u << kDrShift) - 1u;
  constexpr uint32_t kValidSub = 256u * kSub;  // sub-digits below this are placed rows
  __shared__ Rec s_rec[kHalfTile];
  __shared__ uint32_t s_lo[TAG ? 256 : 1];
  __shared__ unsigned int s_cnt[4][kCntW];
  __shared__ unsigned int s_dstart[256 * kSub];
  __shared__ long long s_gbase[256];
  __shared__ unsigned int s_tmp[4];
  __shared__ unsigned int s_tile;
  __shared__ unsigned int s_total;

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const long long c0 = ks.prof ? (long long)__builtin_amdgcn_s_memtime() : 0;
  // Reduce-then-scan mode (tile_base != null): tile = block, its digit bases
  // are precomputed; otherwise tiles are claimed in order for the look-back.
  if (t == 0 && !tile_base) s_tile = (unsigned int)atomicAdd(&counters[tile_slot], 1ull);
  for (int i = t; i < 4 * kCntW; i += kThreads) (&s_cnt[0][0])[i] = 0;
  if (TAG) s_lo[t] = tag_lo[t];
  __syncthreads();
  // Reduce-then-scan: any tile order is valid, so blocks that share an XCD
  // (blockIdx % 8, round-robin dispatch) take one contiguous run of tiles:
  // neighbouring tiles' runs of a digit are then written through one L2.
  const int64_t tile = tile_base ? (ks.xcd_remap ? (int64_t)xcd_tile(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x)
                                 : (int64_t)s_tile;
  // prefetch this tile's digit bases (their latency hides behind the loads)
  const unsigned int tb = (tile_base && t < 256) ? tile_base[tile * 256 + t] : 0u;
  const int64_t n_eff = SOA ? n_in : (int64_t)counters_n[n_slot];
  // split = -(len(rin2)) - 1 (K4's first pass): rin holds the first n_eff - len(rin2) records, a count
  // that lives in device memory
  if (split < 0) split += n_eff + 1;
  const int64_t tile_start = tile * kTile;
  if (tile_start >= n_eff) return false;
  const int radix_bits = ks.bits[pass];
  const int radix = 1 << radix_bits;

  Rec r[kItems];
  uint32_t dr[kItems];  // digit (9 bits) | rank in wave << 9; later the sorted position
  const int64_t base = tile_start + (int64_t)wave * (kItems * 64) + lane;
  // Loads first, all of them in flight at once: indices are clamped (a
  // padding item re-reads the tile's last row and is marked 257 below), so
  // no load sits under a divergent branch.  With the loads inside the
  // per-item `idx < n` branch the compiler waited for each item's load before
  // issuing the next one (16 serial HBM round trips per tile).
  const bool full = tile_start + kTile <= n_eff;
  const int64_t last = n_eff - 1;
  uint32_t ninv = 0;
  if constexpr (SOA) {
#pragma unroll
   for (int g = 0; g < kItems; g += kSoaGroup) {
    int64_t a[kItems], b[kItems];
#pragma unroll
    for (int k = g; k < g + kSoaGroup && k < kItems; ++k) {
      const int64_t idx = base + k * 64;
      const int64_t ic = full ? idx : (idx < last ? idx : last);
      a[k] = ld_soa(pid + ic);
      b[k] = ld_soa(pk + ic);
    }
    if constexpr (TAG == 2) {  // the row index rides in the value slot (k_filter gathers the value)
#pragma unroll
      for (int k = g; k < g + kSoaGroup && k < kItems; ++k) r[k].val = __longlong_as_double(base + k * 64);
    } else if (val) {
#pragma unroll
      for (int k = g; k < g + kSoaGroup && k < kItems; ++k) {
        const int64_t idx = base + k * 64;
        r[k].val = ld_soa(val + (full ? idx : (idx < last ? idx : last)));
      }
    } else {
#pragma unroll
      for (int k = g; k < g + kSoaGroup && k < kItems; ++k) r[k].val = 0.0;
    }
#pragma unroll
    for (int k = g; k < g + kSoaGroup && k < kItems; ++k) {
      uint32_t d;
      const bool valid = full || base + k * 64 <= last;
      r[k].pid = (uint32_t)a[k];
      r[k].pk = (uint32_t)b[k];
      if constexpr (ANA) {
        unsigned int inv = 0;  // counted by k_histogram<2>
        r[k] = ana_rec(a[k], b[k], r[k].val, ks, inv);
        d = digit_of(ks, pass, r[k]);
      } else if constexpr (TAG) {
        // placed unless the privacy id is out of range (k_histogram_tiles<true>); a non-public row
        // (pk < 0) is tagged dropped, an out-of-range pk is an error
        if (a[k] < 0 || a[k] >= (int64_t)ks.num_pids) {
          d = 512;  // dropped (sub-digit space)
        } else {
          d = digit_of(ks, pass, r[k]);
          if (b[k] < 0 || b[k] >= (int64_t)ks.num_parts) {
            ninv += valid && b[k] >= 0;
            r[k].pid = kTagDropped | (d << 22);
            d = 2u * d;
          } else {
            const uint32_t lv = filt_level(filt_prio(ks.seed, ks.pid_base + r[k].pid, r[k].pk));
            r[k].pid = (d << 22) | ((r[k].pid - s_lo[d]) << 5) | lv;
            d = 2u * d + ((lv > (uint32_t)ks.tau ? 1u : 0u) ^ ((uint32_t)tile & (uint32_t)ks.flip));
          }
        }
      } else {
        if (b[k] < 0 || b[k] >= (int64_t)ks.num_parts || a[k] < 0 || a[k] >= (int64_t)ks.num_pids)
          d = 256;  // dropped
        else
          d = digit_of(ks, pass, r[k]);
      }
      dr[k] = valid ? d : (TAG ? 513u : 257u);  // 257 (TAG 513): padding, ignored
    }
   }
  } else {
#pragma unroll
   for (int g = 0; g < kItems; g += kRecGroup) {
#pragma unroll
    for (int k = g; k < g + kRecGroup && k < kItems; ++k) {
      const int64_t idx = base + k * 64;
      const int64_t ic = full ? idx : (idx < last ? idx : last);
      if constexpr (P12 == 3) {  // split slots: keys first, all in flight
        r[k].pid = ic < split ? reinterpret_cast<const uint32_t*>(rin)[ic]
                              : reinterpret_cast<const uint32_t*>(rin2)[ic - split];
        r[k].pk = 0u;
      } else if constexpr (P12 != 0) {
        r[k] = ic < split ? k4_ld12(rin, ic) : k4_ld12(rin2, ic - split);
      } else {
        r[k] = ld_rec(ic < split ? rin + ic : rin2 + (ic - split));
      }
    }
    if constexpr (P12 == 3) {  // ... then the values of the non-empty slots
#pragma unroll
      for (int k = g; k < g + kRecGroup && k < kItems; ++k) {
        const int64_t idx = base + k * 64;
        const int64_t ic = full ? idx : (idx < last ? idx : last);
        const double* vp = ic < split ? reinterpret_cast<const double*>(reinterpret_cast<const char*>(rin) + ks.soa_a) + ic
                                      : reinterpret_cast<const double*>(reinterpret_cast<const char*>(rin2) + ks.soa_b) +
                                            (ic - split);
        r[k].val = r[k].pid != kK4EmptyKey ? *vp : 0.0;
      }
    }
#pragma unroll
    for (int k = g; k < g + kRecGroup && k < kItems; ++k) {
      const uint32_t d = (ks.mode == 6 && r[k].pid == kK4EmptyKey) ? 256u : digit_of(ks, pass, r[k]);  // K4: empty slot
      dr[k] = (full || base + k * 64 <= last) ? d : 257u;
    }
   }
  }
  if (TAG && ninv) atomicAdd(&counters[kCtrInvalid], (unsigned long long)ninv);

  long long ca = 0;
  if (ks.prof) {
    uint32_t dsum = 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) dsum += dr[k];
    ca = (long long)__builtin_amdgcn_s_memtime() + (dsum == 0xFFFFFFFFu);  // after every load landed
  }
  // Wave-level multisplit ranking (stable: item order = wave, k, lane).
  // Peers = lanes with the same digit (one ballot per digit bit, plus a
  // validity ballot when the tile can hold dropped / padding rows).  The
  // lowest peer adds the group size to the wave's digit counter with an LDS
  // atomic; LDS ops of one wave complete in issue order, so the returned
  // bases are the sequential ones and the 16 atomics pipeline (no wave
  // barriers).  The base reaches the other peers by a lane shuffle.
  const uint64_t lt = (1ull << lane) - 1ull;
  const bool any_invalid = SOA || ks.mode == 6 || tile_start + kTile > n_eff;
#if PDP_OS_RANK_ATOMIC
  static_assert(TAG == 0, "PDP_OS_RANK_ATOMIC variant builds do not rank the bucket pass's sub-digits");
  constexpr int kRankGroup = kItems < 8 ? kItems : 8;  // atomics in flight before their shuffles
#pragma unroll
  for (int k0 = 0; k0 < kItems; k0 += kRankGroup) {
    uint32_t old[kRankGroup];
#pragma unroll
    for (int k = k0; k < k0 + kRankGroup; ++k) {
      const uint32_t d = dr[k];
      uint64_t peers = ~0ull;
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        if (b < radix_bits) {
          const bool bit = (d >> b) & 1u;
          const uint64_t bb = __ballot(bit);
          peers &= bit ? bb : ~bb;
        }
      }
      if (any_invalid) {
        const bool v = d < 256;
        const uint64_t bb = __ballot(v);
        peers &= v ? bb : ~bb;
      }
      const uint32_t before = __popcll(peers & lt);
      const uint32_t leader = (uint32_t)__ffsll((unsigned long long)peers) - 1u;
      old[k - k0] = 0;
      if (d < 256 && before == 0) old[k - k0] = atomicAdd(&s_cnt[wave][d], (unsigned int)__popcll(peers));
      dr[k] = d | (before << 9) | (leader << 15);
    }
#pragma unroll
    for (int k = k0; k < k0 + kRankGroup; ++k) {
      const uint32_t basec = (uint32_t)__shfl((int)old[k - k0], (int)(dr[k] >> 15));
      dr[k] = (dr[k] & 511u) | ((basec + ((dr[k] >> 9) & 63u)) << 9);
    }
  }
  __syncthreads();
#else
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const uint32_t d = dr[k];
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < (TAG ? 9 : 8); ++b) {
      if (TAG || b < radix_bits) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        peers &= bit ? bb : ~bb;
      }
    }
    if (any_invalid) {  // digits 256 (dropped) / 257 (padding) share a counter (TAG: 512 / 513)
      const bool v = d < kValidSub;
      const uint64_t bb = __ballot(v);
      peers &= v ? bb : ~bb;
    }
    const uint32_t before = __popcll(peers & lt);
    const uint32_t c = __popcll(peers);
    const uint32_t basec = s_cnt[wave][d];
    __builtin_amdgcn_wave_barrier();
    if (before == 0 && d < kValidSub) s_cnt[wave][d] = basec + c;
    __builtin_amdgcn_wave_barrier();
    dr[k] = d | ((basec + before) << kDrShift);
  }
  __syncthreads();
#endif

  // Per-digit tile counts, per-wave exclusive offsets, digit starts.
  unsigned int tcount = 0, tcount0 = 0;
#pragma unroll
  for (int u = 0; u < kSub; ++u) {  // TAG: the digit's two sub-digits (class 0, then class 1)
    const int sd = kSub * t + u;
    const unsigned int c0w = s_cnt[0][sd], c1w = s_cnt[1][sd], c2w = s_cnt[2][sd], c3w = s_cnt[3][sd];
    const unsigned int cs = c0w + c1w + c2w + c3w;
    tcount += cs;
    if (u == 0) tcount0 = cs;
    __syncthreads();
    s_cnt[0][sd] = 0;
    s_cnt[1][sd] = c0w;
    s_cnt[2][sd] = c0w + c1w;
    s_cnt[3][sd] = c0w + c1w + c2w;
  }
  unsigned int total;
  const unsigned int dstart = block_excl_scan(tcount, s_tmp, total);
  s_dstart[kSub * t] = dstart;
  if (TAG) s_dstart[kSub * t + (kSub - 1)] = dstart + tcount0;
  if (t == 0) s_total = total;

  const long long c1 = ks.prof ? (long long)__builtin_amdgcn_s_memtime() : 0;
  // Decoupled look-back per digit.
  if (tile_base) {
    if (t < radix) s_gbase[t] = (long long)tb - (long long)dstart;
  } else if (t < radix && (ks.ablate & kDebugNoLookback)) {
    s_gbase[t] = (long long)off[t] - (long long)dstart;
  } else if (t < radix) {
    unsigned long long* st = status + (size_t)tile * kStatusStride;
    const uint64_t ep = (uint64_t)epoch << 48;
    uint64_t excl = 0;
    if (tile == 0) {
      __hip_atomic_store(&st[t], ep | kFlagPre | (uint64_t)tcount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_store(&st[t], ep | kFlagAgg | (uint64_t)tcount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // Look back kLookback predecessors per round trip (independent loads in
      // flight), consuming them nearest-first up to the first inclusive
      // prefix or the first one not published yet.
      int64_t j = tile - 1;
      unsigned int spins = 0;
      while (true) {
        uint64_t sv[kLookback];
#pragma unroll
        for (int w = 0; w < kLookback; ++w)
          sv[w] = j - w >= 0 ? __hip_atomic_load(&status[(size_t)(j - w) * kStatusStride + t], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : 0ull;
        int used = 0;
        bool done = false;
#pragma unroll
        for (int w = 0; w < kLookback; ++w) {
          const uint64_t s = sv[w];
          const uint64_t f = s & kFlagMask;
          if (!done && used == w && (s >> 48) == (uint64_t)epoch && f != 0) {
            excl += s & kValMask;
            used = w + 1;
            done = f == kFlagPre;
          }
        }
        if (done) break;
        j -= used;
        if (used == 0) {
          if (++spins > (1u << 24)) {
            atomicOr(&counters[kCtrErr], 1ull);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __hip_atomic_store(&st[t], ep | kFlagPre | (excl + tcount), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_gbase[t] = (long long)off[t] + (long long)excl - (long long)dstart;
  }
  __syncthreads();
  const long long c2 = ks.prof ? (long long)__builtin_amdgcn_s_memtime() : 0;

  // Sorted position of every item in the tile.
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const uint32_t d = dr[k] & kDrMask;
    dr[k] = d < kValidSub ? s_dstart[d] + s_cnt[wave][d] + (dr[k] >> kDrShift) : kNoPos;
  }
  // Two halves: stage positions [h, h + kHalfTile) in LDS, write contiguous
  // digit runs (the digit is recomputed from the staged record).
  const unsigned int tot = s_total;
  for (unsigned int h = 0; h < tot; h += kHalfTile) {
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const uint32_t q = dr[k] - h;
      if (q < (uint32_t)kHalfTile) s_rec[q] = r[k];
    }
    __syncthreads();
    const unsigned int e = (ks.ablate & kDebugNoScatter) ? 0u
                           : tot - h < (unsigned int)kHalfTile ? tot - h : (unsigned int)kHalfTile;
    for (unsigned int i = t; i < e; i += kThreads) {
      const Rec rc = s_rec[i];
      if (ks.ablate & kDebugLinearWrite) {
        st_rec(rout + tile_start + (long long)(h + i), rc);
      } else {
        const long long q = s_gbase[TAG ? (rc.pid >> 22) & 255u : digit_of(ks, pass, rc)] + (long long)(h + i);
        if (ks.mode == 6 && (q < 0 || q >= ks.cap)) {  // the pair histogram disagrees with the records
          atomicOr(&counters[kCtrErr], 4ull);
          continue;
        }
#if PDP_SCATTER_CHECK  // variant builds: every scatter position inside the input's row count
        if (q < 0 || q >= n_eff) {
          atomicOr(&counters[kCtrErr], 8ull);
          continue;
        }
#endif
        if constexpr (P12 != 0) k4_st12(rout, q, rc);
        else if constexpr (TAG == 2)
          reinterpret_cast<uint2*>(rout)[q] = make_uint2(rc.pk, (uint32_t)__double_as_longlong(rc.val));
        else st_rec(rout + q, rc);
        if constexpr (TAG) tag_out[q] = rc.pid;
      }
    }
    __syncthreads();
  }
  if (ks.prof && t == 0) {
    const long long c3 = (long long)__builtin_amdgcn_s_memtime();
    atomicAdd(&counters[kCtrSweepCycles], (unsigned long long)(ca - c0));
    atomicAdd(&counters[kCtrSweepCycles + 1], (unsigned long long)(c1 - ca));
    atomicAdd(&counters[kCtrSweepCycles + 2], (unsigned long long)(c2 - c1));
    atomicAdd(&counters[kCtrSweepCycles + 3], (unsigned long long)(c3 - c2));
    atomicAdd(&counters[kCtrSweepTiles], 1ull);
  }
  (void)radix_bits;
  return true;
}

// Distinct symbols per use, so rocprofv3 --stats (which truncates template
// arguments with -T) reports each stage on its own line.
#define PDP_ONESWEEP_ARGS                                                                                  \
  const int64_t *__restrict__ pid, const int64_t *__restrict__ pk, const double *__restrict__ val,         \
      const Rec *__restrict__ rin, Rec *__restrict__ rout, int64_t n_in,                                   \
      const unsigned long long *__restrict__ counters_n, int n_slot, KeySpec ks, int pass,                 \
      const unsigned long long *__restrict__ off, unsigned long long *__restrict__ status, uint32_t epoch, \
      unsigned long long *__restrict__ counters, int tile_slot, const unsigned int *__restrict__ tile_base, \
      uint32_t *__restrict__ tag_out, const uint32_t *__restrict__ tag_lo, const Rec *__restrict__ rin2,  \
      int64_t split
#define PDP_ONESWEEP_PASS                                                                                  \
  pid, pk, val, rin, rout, n_in, counters_n, n_slot, ks, pass, off, status, epoch, counters, tile_slot,    \
      tile_base, tag_out, tag_lo, rin2, split
// Launches whose tile count the host knows run one tile per block.  The passes over a row count that
// lives in device memory (the survivor sort, K4's pair passes) loop over tiles claimed in order, so a
// grid sized from a host bound covers every tile.  The loop costs registers (round 5: 80-108 B of
// scratch at 3 blocks per CU; none at 2), so only those kernels have it.  3 blocks per CU nevertheless
// (r05f: c4 pair passes 9.25 -> 7.62 ms, c3 survivor sort 1.94 -> 1.81 ms against 2; debug flag
// DEV_OCC2: 2, debug library PDP_DEV_OCC=2|3|4).
#define PDP_ONESWEEP_LOOP(B, ...)                        \
  while (B<__VA_ARGS__>(PDP_ONESWEEP_PASS) && !tile_base) \
    __syncthreads();
// records -> records (passes >= 1 of the pid sort, generic path, utility analysis)
__global__ __launch_bounds__(kThreads, PDP_OS_OCC) void k_onesweep(PDP_ONESWEEP_ARGS) {
  onesweep_body<false, 0>(PDP_ONESWEEP_PASS);
}
// ... over a device-side record count (the L0 pre-filter's survivors)
template <int OCC>
__global__ __launch_bounds__(kThreads, OCC) void k_onesweep_dev(PDP_ONESWEEP_ARGS) {
  PDP_ONESWEEP_LOOP(onesweep_body, false, 0, 0, false)
}
// SoA columns -> records (first pass of the pid sort, non-public rows dropped)
__global__ __launch_bounds__(kThreads, PDP_OS_OCC) void k_sort_first(PDP_ONESWEEP_ARGS) {
  onesweep_body<true, 0>(PDP_ONESWEEP_PASS);
}
// the utility analysis' first (pk, pid) pass from the SoA columns (pdp_analysis.inc)
__global__ __launch_bounds__(kThreads, PDP_OS_OCC) void k_ana_sort_first(PDP_ONESWEEP_ARGS) {
  onesweep_body<true, 0, 0, true>(PDP_ONESWEEP_PASS);
}
// the L0 pre-filter's bucket pass (SoA columns -> tagged 16-byte records + tags, pdp_filter.inc)
__global__ __launch_bounds__(kThreads, PDP_OS_OCC) void k_bucket_pass(PDP_ONESWEEP_ARGS) {
  onesweep_body<true, 1>(PDP_ONESWEEP_PASS);
}
// ... debug2 flag FILTER_REC8: 8-byte {pk, row index} records (the values gathered by k_filter)
__global__ __launch_bounds__(kThreads, PDP_OS_OCC) void k_bucket_pass8(PDP_ONESWEEP_ARGS) {
  onesweep_body<true, 2>(PDP_ONESWEEP_PASS);
}
// K4 pair records by partition block (pdp_reduce.inc); device-side record counts
template <int OCC>
__global__ __launch_bounds__(kThreads, OCC) void k_pair_pass(PDP_ONESWEEP_ARGS) {
  PDP_ONESWEEP_LOOP(onesweep_body, false, 0, 0, false)
}
// ... with 12-byte pair records (K2 writes its slots in that form)
template <int OCC>
__global__ __launch_bounds__(kThreads, OCC) void k_pair_pass12(PDP_ONESWEEP_ARGS) {
  PDP_ONESWEEP_LOOP(onesweep_body, false, 0, 2, false)
}
// ... whose first pass reads K2's split slots (keys, then the values of the non-empty ones)
template <int OCC>
__global__ __launch_bounds__(kThreads, OCC) void k_pair_pass12s(PDP_ONESWEEP_ARGS) {
  PDP_ONESWEEP_LOOP(onesweep_body, false, 0, 3, false)
}

// Clears the look-back status words of the tiles of *rows_dev + add rows (a row count that lives in
// device memory: the survivor sort, the K4 pair passes); grid-stride.
__global__ __launch_bounds__(kThreads) void k_status_clear(unsigned long long* __restrict__ status,
                                                           const unsigned long long* __restrict__ rows_dev, int64_t add) {
  const int64_t rows = (int64_t)*rows_dev + add;
  const int64_t words = (rows + kTile - 1) / kTile * kStatusStride;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < words; i += (int64_t)gridDim.x * kThreads)
    status[i] = 0ull;
}

// Zeroes `words` 8-byte words (grid-stride).  The aggregate path clears its buffers with this kernel
// rather than hipMemsetAsync, so a call captured in a hipGraph (PDP_BOUND_ASYNC) holds kernel nodes
// only.
__global__ __launch_bounds__(kThreads) void k_zero64(unsigned long long* __restrict__ p, int64_t words) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < words; i += (int64_t)gridDim.x * kThreads)
    p[i] = 0ull;
}
__global__ __launch_bounds__(kThreads) void k_zero_bytes(unsigned char* __restrict__ p, int64_t bytes) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < bytes; i += (int64_t)gridDim.x * kThreads)
    p[i] = 0u;
}

// End of a pdp_bound_accumulate call: the counters the host needs (errors, the generic-path request,
// statistics) -> the context's device status block (kStat*), read back by ONE copy (or, for an
// asynchronous call, by pdp_get_status after the stream has drained).
enum StatWord {
  kStatErr = 0, kStatInvalid, kStatRanges, kStatFull, kStatKeptRows, kStatSurvivors, kStatK4Slots, kStatK4Pairs,
  kStatSweep0, kStatSweepTiles = kStatSweep0 + 4, kStatBig, kStatWords = 16
};
__global__ void k_latch(const unsigned long long* __restrict__ counters, unsigned long long* __restrict__ st) {
  if (threadIdx.x == 0) {
    st[kStatErr] = counters[kCtrErr];
    st[kStatInvalid] = counters[kCtrInvalid];
    st[kStatRanges] = counters[kCtrNRanges];
    st[kStatFull] = counters[kCtrFull];
    st[kStatKeptRows] = counters[kCtrNKept] - counters[kCtrNDropped];
    st[kStatSurvivors] = counters[kCtrNSurv];
    st[kStatK4Slots] = counters[kCtrK4In];
    st[kStatK4Pairs] = counters[kCtrK4Pairs];
    for (int i = 0; i < 4; ++i) st[kStatSweep0 + i] = counters[kCtrSweepCycles + i];
    st[kStatSweepTiles] = counters[kCtrSweepTiles];
    st[kStatBig] = counters[kCtrNBig];
  }
}

// ---------------------------------------------------------------------------
// K2: privacy-id buckets in LDS: bounding + per-(pid,pk) accumulation
// ---------------------------------------------------------------------------

__device__ __forceinline__ void record_overflow(const OvList& ov, int64_t s, int64_t e) {
  const unsigned long long i = atomicAdd(&ov.counters[kCtrNRanges], 1ull);
  if (i < kOverflowCap) {
    ov.ranges[2 * i] = (unsigned long long)s;
    ov.ranges[2 * i + 1] = (unsigned long long)e;
  }
  if (i >= kOverflowCap || (ov.full_at && i >= ov.full_at)) atomicOr(&ov.counters[kCtrFull], 1ull);
}

__device__ __forceinline__ void row_terms(const SegParams& sp, double v, double& x, double& y) {
  x = 0.0;
  y = 0.0;
  if (sp.xmode == kXNsum) {
    const double c = clip(v, sp.a, sp.b) - sp.mid;
    x = c;
    y = c * c;
  } else if (sp.xmode == kXClipSum) {
    x = clip(v, sp.a, sp.b);
  } else if (sp.xmode == kXRawSum) {
    x = v;
  }
}

__device__ __forceinline__ void emit_group(const SegParams& sp, const AccPtrs& acc, uint32_t pk, uint32_t cnt,
                                           double x, double y) {
  if (sp.debug & kDebugNoAtomics) return;
  if (sp.packed) {
    // one 64-bit atomic for (count, row_count); both stay < 2^32 (rows < 2^32)
    atomicAdd(&acc.row_count[pk], ((unsigned long long)cnt << 32) | 1ull);
  } else {
    atomicAdd(&acc.row_count[pk], 1ull);
    if (sp.want_count) atomicAdd(&acc.count[pk], (unsigned long long)cnt);
  }
  if (sp.xmode != kXNone) {
    if (sp.xmode == kXRawSum) x = clip(x, sp.smin, sp.smax);  // combiners.py:256-259
    atomicAdd(&acc.x[pk], x);
  }
  if (sp.want_y) atomicAdd(&acc.y[pk], y);
}

#include "pdp_group.inc"
#include "pdp_reduce.inc"
#include "pdp_segments.inc"
#include "pdp_thin.inc"
#include "pdp_analysis.inc"
#include "pdp_aggregate.inc"

// ---------------------------------------------------------------------------
// KF: generic sorted-stream path (fallback for buckets that overflow LDS)
// ---------------------------------------------------------------------------

__global__ void k_gather_ranges(const Rec* __restrict__ src, Rec* __restrict__ dst,
                                const long long* __restrict__ rsrc, const long long* __restrict__ rdst,
                                int nranges, int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int lo = 0, hi = nranges - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (rdst[mid] <= i) lo = mid; else hi = mid - 1;
    }
    dst[i] = src[rsrc[lo] + (i - rdst[lo])];
  }
}

__global__ void k_stream_flags(const Rec* __restrict__ r, int64_t m, long long* __restrict__ gs,
                               long long* __restrict__ ps) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const Rec a = r[i];
    bool g = true, p = true;
    if (i > 0) {
      const Rec b = r[i - 1];
      p = a.pid != b.pid;
      g = p || a.pk != b.pk;
    }
    gs[i] = g;
    ps[i] = p;
  }
}

// Inclusive scan of 2048-element chunks; chunk totals to sums.
__global__ __launch_bounds__(kThreads) void k_scan_chunks(long long* __restrict__ a, int64_t n,
                                                          long long* __restrict__ sums) {
  __shared__ long long s_tmp[4];
  const int64_t base = (int64_t)blockIdx.x * 2048 + threadIdx.x * 8;
  long long v[8];
  long long acc = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v[k] = base + k < n ? a[base + k] : 0;
    acc += v[k];
    v[k] = acc;
  }
  long long tot;
  const long long ex = block_excl_scan(acc, s_tmp, tot);
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (base + k < n) a[base + k] = v[k] + ex;
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ void k_scan_add(long long* __restrict__ a, int64_t n, const long long* __restrict__ sums) {
  if (blockIdx.x == 0) return;
  const long long add = sums[blockIdx.x - 1];
  const int64_t base = (int64_t)blockIdx.x * 2048;
  for (int k = threadIdx.x; k < 2048; k += blockDim.x)
    if (base + k < n) a[base + k] += add;
}

__global__ void k_stream_starts(const long long* __restrict__ gs_raw_scan, const long long* __restrict__ ps_scan,
                                const Rec* __restrict__ r, int64_t m, long long* __restrict__ gpos,
                                long long* __restrict__ pfirst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const long long g = gs_raw_scan[i] - 1;
    const long long p = ps_scan[i] - 1;
    const bool gstart = i == 0 || gs_raw_scan[i - 1] != gs_raw_scan[i];
    const bool pstart = i == 0 || ps_scan[i - 1] != ps_scan[i];
    if (gstart) gpos[g] = i;
    if (pstart) pfirst[p] = g;
    if (i == m - 1) gpos[g + 1] = m;
  }
}

// L_inf priorities: R2[i] = {group id, row index, bits(row priority)}.
__global__ void k_stream_row_prio(const Rec* __restrict__ r, int64_t m, const long long* __restrict__ gsc,
                                  const long long* __restrict__ gpos, uint64_t seed, uint64_t base,
                                  Rec* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const long long g = gsc[i] - 1;
    const Rec a = r[i];
    const uint64_t gp = pdp::group_priority(pdp::pid_key(seed, base + a.pid), a.pk);
    const uint64_t rp = pdp::row_priority(gp, (uint64_t)(i - gpos[g]));
    out[i] = Rec{(uint32_t)g, (uint32_t)i, __longlong_as_double((long long)rp)};
  }
}

// L0 priorities: R3[g] = {pid ordinal, group id, bits(group priority)}.
__global__ void k_stream_group_prio(const Rec* __restrict__ r, const long long* __restrict__ psc,
                                    const long long* __restrict__ gpos, int64_t ngroups, uint64_t seed,
                                    uint64_t base, Rec* __restrict__ out) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups;
       g += (int64_t)gridDim.x * blockDim.x) {
    const long long q = gpos[g];
    const Rec a = r[q];
    const uint64_t gp = pdp::group_priority(pdp::pid_key(seed, base + a.pid), a.pk);
    out[g] = Rec{(uint32_t)(psc[q] - 1), (uint32_t)g, __longlong_as_double((long long)gp)};
  }
}

// Sorted (group, priority) records -> rank within the group segment.
__global__ void k_stream_ranks(const Rec* __restrict__ sorted, int64_t m, const long long* __restrict__ seg_first,
                               int64_t limit, uint8_t* __restrict__ keep8, int32_t* __restrict__ rank32) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += (int64_t)gridDim.x * blockDim.x) {
    const Rec a = sorted[q];
    const long long rank = q - seg_first[a.pid];
    if (keep8) keep8[a.pk] = rank < limit;
    if (rank32) rank32[a.pk] = (int32_t)(rank < 0x7FFFFFFF ? rank : 0x7FFFFFFF);
  }
}

// Kept groups: the L_inf-kept rows of each L0-kept group summed in input
// order (deterministic), then one accumulator add (or, K4, one pair record in
// slot g of the generic path's pair array; sp.k4x / k4y point there).  A kept
// group of more than kBigGroupRows rows (a heavy privacy id in one partition)
// is not walked by one lane: it goes to `big` for k_stream_big_groups.
constexpr int64_t kBigGroupRows = 2048;
__global__ void k_stream_groups(const Rec* __restrict__ r, const long long* __restrict__ gpos,
                                const int32_t* __restrict__ grank, const uint8_t* __restrict__ row_keep,
                                int64_t ngroups, SegParams sp, AccPtrs acc, unsigned long long* __restrict__ big) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups;
       g += (int64_t)gridDim.x * blockDim.x) {
    uint32_t c = 0;
    double x = 0.0, y = 0.0;
    if (grank[g] < sp.l0 && gpos[g + 1] - gpos[g] > kBigGroupRows) {
      big[1 + atomicAdd(&big[0], 1ull)] = (unsigned long long)g;  // big[0]: count, then the group ids
      continue;
    }
    if (grank[g] < sp.l0) {
      for (long long q = gpos[g]; q < gpos[g + 1]; ++q) {
        if (!row_keep[q]) continue;
        double xt, yt;
        row_terms(sp, r[q].val, xt, yt);
        ++c;
        x += xt;
        y += yt;
      }
    }
    if (sp.k4x) {
      if (c > 0) k4_put(sp, g, r[gpos[g]].pk, c, x, y, sp.k4hist);
      else k4_empty(sp, g);
    } else if (c > 0) {
      emit_group(sp, acc, r[gpos[g]].pk, c, x, y);
    }
  }
}

// The big kept groups: one block per group.  Each round the block reads 256
// consecutive rows (coalesced keep bytes and values) and stages the kept rows'
// terms in LDS; one thread adds them in row order.  The sum is therefore the
// sequential input-order sum of k_stream_groups (and of the reference's
// per-group accumulator), bit for bit (round 4 used a block tree here).
__global__ __launch_bounds__(kThreads) void k_stream_big_groups(const Rec* __restrict__ r,
                                                                const long long* __restrict__ gpos,
                                                                const uint8_t* __restrict__ row_keep, SegParams sp,
                                                                AccPtrs acc, const unsigned long long* __restrict__ big) {
  __shared__ double s_x[kThreads], s_y[kThreads];
  __shared__ unsigned long long s_m[kThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t nbig = (int64_t)big[0];
  for (int64_t b = blockIdx.x; b < nbig; b += gridDim.x) {
    const int64_t g = (int64_t)big[1 + b];
    const long long q0 = gpos[g], q1 = gpos[g + 1];
    uint32_t c = 0;
    double x = 0.0, y = 0.0;
    for (long long base = q0; base < q1; base += kThreads) {
      const long long q = base + threadIdx.x;
      const bool kept = q < q1 && row_keep[q];
      if (kept) row_terms(sp, r[q].val, s_x[threadIdx.x], s_y[threadIdx.x]);
      const unsigned long long m = __ballot(kept);
      if (lane == 0) s_m[w] = m;
      __syncthreads();
      if (threadIdx.x == 0) {
        for (int i = 0; i < kThreads / 64; ++i) {
          unsigned long long mm = s_m[i];
          c += (uint32_t)__popcll(mm);
          while (mm) {
            const int l = 64 * i + __builtin_ctzll(mm);
            mm &= mm - 1ull;
            x += s_x[l];
            y += s_y[l];
          }
        }
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      if (sp.k4x) {
        if (c > 0) k4_put(sp, g, r[q0].pk, c, x, y, sp.k4hist);
        else k4_empty(sp, g);
      } else if (c > 0) {
        emit_group(sp, acc, r[q0].pk, c, x, y);
      }
    }
  }
}

// contribution_bounds_already_enforced: every row is its own accumulator
// (dp_engine.py:139-150, combiners.py create_accumulator([value])).
// K4: row i -> slot i (empty for a dropped row).
__global__ void k_enforced(const int64_t* __restrict__ pk, const double* __restrict__ val, int64_t n,
                           int64_t num_parts, SegParams sp, AccPtrs acc, unsigned long long* __restrict__ counters) {
  k4_begin(sp);
  unsigned int invalid = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = pk[i];
    if (b < 0 || b >= num_parts) {
      if (b >= num_parts) ++invalid;
      if (sp.k4x) k4_empty(sp, i);
      continue;
    }
    double x = 0.0, y = 0.0;
    if (sp.has_value) {
      row_terms(sp, val[i], x, y);
    }
    if (sp.k4x) k4_put(sp, i, (uint32_t)b, 1u, x, y, k4_lds_hist());
    else emit_group(sp, acc, (uint32_t)b, 1u, x, y);
  }
  if (invalid) atomicAdd(&counters[kCtrInvalid], (unsigned long long)invalid);
  k4_end(sp);
}

// Packed (count << 32 | row_count) words -> the two int64 accumulators.
__global__ void k_unpack_counts(unsigned long long* __restrict__ row_count, unsigned long long* __restrict__ count,
                                int64_t P) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long v = row_count[i];
    row_count[i] = v & 0xFFFFFFFFull;
    count[i] = v >> 32;
  }
}

// ---------------------------------------------------------------------------
// K5/K6: partition selection + noisy metrics, one thread per partition
// ---------------------------------------------------------------------------

struct RelParams {
  int metrics, kind, selection, add_noise;
  int nfields;
  int field[5];
  double s_count, s_sum, s_mean_count, s_mean_nsum, s_var_nsq, s_pid;
  int sum_zero, mean_degenerate, sq_degenerate;
  double a, mid, sq_a, sq_mid;
  double sel_thr, sel_scale;
  const double* table;
  int64_t tlen;
  int64_t max_rows;
  uint64_t seed;
};

// value + Laplace/Gaussian noise of `scale`, both snapped to the noise grid
// (pdp_rng.h: add_snapped_noise); exact value when noise is off.
__device__ __forceinline__ double noisy(const RelParams& rp, double value, uint64_t idx, uint32_t stream,
                                        double scale) {
  if (!rp.add_noise || scale == 0.0) return value;
  return pdp::add_snapped_noise(rp.kind == PDP_NOISE_GAUSSIAN, value, rp.seed, idx, stream, scale);
}

__global__ void k_release(const unsigned long long* __restrict__ row_count,
                          const unsigned long long* __restrict__ count, const double* __restrict__ xs,
                          const double* __restrict__ ys, int64_t P, int64_t pk_offset, RelParams rp,
                          uint8_t* __restrict__ keep, double* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t gidx = (uint64_t)(pk_offset + i);
    const long long rc = (long long)row_count[i];
    uint8_t kp = 1;
    if (rp.selection != PDP_SELECTION_NONE) {
      const long long nn = (rc + rp.max_rows - 1) / rp.max_rows;
      if (nn <= 0) {
        kp = 0;
      } else if (rp.selection == PDP_SELECTION_TRUNCATED_GEOMETRIC) {
        const double p = nn < rp.tlen ? rp.table[nn] : 1.0;
        if (rp.add_noise) {
          double u, u2;
          pdp::philox_uniforms(rp.seed, gidx, pdp::kStreamSelect, u, u2);
          kp = u < p;
        } else {
          kp = p > 0.0;
        }
      } else {
        const int gauss = rp.selection == PDP_SELECTION_GAUSSIAN_THRESHOLDING;
        const double v = rp.add_noise
                             ? pdp::add_snapped_noise(gauss, (double)nn, rp.seed, gidx, pdp::kStreamSelect, rp.sel_scale)
                             : (double)nn;
        kp = v > rp.sel_thr;
      }
    }
    keep[i] = kp;
    if (!kp) {  // dropped by private selection: not in the result (dp_engine.py:312-362), no noise drawn
      for (int k = 0; k < rp.nfields; ++k) out[(int64_t)k * P + i] = __longlong_as_double(0x7FF8000000000000ll);
      continue;
    }
    double f[5] = {0, 0, 0, 0, 0};  // variance, mean, count, sum, pid_count
    const int m = rp.metrics;
    if (m & (PDP_METRIC_VARIANCE | PDP_METRIC_MEAN)) {
      const double dp_count = noisy(rp, (double)(long long)count[i], gidx, pdp::kStreamMeanCount, rp.s_mean_count);
      const double denom = dp_count > 1.0 ? dp_count : 1.0;
      double dp_mean;
      if (rp.mean_degenerate) {
        dp_mean = rp.a;
      } else {
        dp_mean = noisy(rp, xs[i], gidx, pdp::kStreamMeanNsum, rp.s_mean_nsum) / denom;
      }
      if (m & PDP_METRIC_VARIANCE) {
        double msq;
        if (rp.sq_degenerate)
          msq = rp.sq_a;
        else
          msq = noisy(rp, ys[i], gidx, pdp::kStreamVarNsq, rp.s_var_nsq) / denom;
        f[0] = msq - dp_mean * dp_mean;
      }
      if (!rp.mean_degenerate) dp_mean += rp.mid;
      f[1] = dp_mean;
      f[2] = dp_count;
      f[3] = dp_mean * dp_count;
    } else {
      if (m & PDP_METRIC_COUNT) f[2] = noisy(rp, (double)(long long)count[i], gidx, pdp::kStreamCount, rp.s_count);
      if (m & PDP_METRIC_SUM) f[3] = rp.sum_zero ? 0.0 : noisy(rp, xs[i], gidx, pdp::kStreamSum, rp.s_sum);
    }
    if (m & PDP_METRIC_PRIVACY_ID_COUNT) f[4] = noisy(rp, (double)rc, gidx, pdp::kStreamPidCount, rp.s_pid);
    for (int k = 0; k < rp.nfields; ++k) out[(int64_t)k * P + i] = f[rp.field[k]];
  }
}

// ---------------------------------------------------------------------------
// Row shuffle by privacy-id shard (multi-GPU input not sharded by pid): the
// device side of the reference's group-by-pid shuffles
// (pipeline_backend.py:261, 401, 476-485).  Stable counting sort of the rows
// by destination rank shard_of(pid) = splitmix64(pid ^ salt) % world; the
// RCCL all-to-all then moves each destination's contiguous run.
// ---------------------------------------------------------------------------

constexpr int kShardMax = 64;
constexpr int kShardChunk = 8192;  // rows per block, in order
constexpr uint64_t kPidShardSalt = 0x9E3779B97F4A7C15ull;  // distributed.py:PID_SHARD_SALT

__device__ __forceinline__ uint32_t shard_dest(int64_t pid, int world) {
  return (uint32_t)(pdp::splitmix64((uint64_t)pid ^ kPidShardSalt) % (uint64_t)world);
}

__global__ __launch_bounds__(kThreads) void k_shard_count(const int64_t* __restrict__ pid, int64_t n, int world,
                                                          unsigned long long* __restrict__ counts) {
  __shared__ unsigned int c[kShardMax];
  const int t = threadIdx.x;
  if (t < kShardMax) c[t] = 0;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * kShardChunk;
  const int64_t hi = lo + kShardChunk < n ? lo + kShardChunk : n;
  for (int64_t i = lo + t; i < hi; i += kThreads) atomicAdd(&c[shard_dest(pid[i], world)], 1u);
  __syncthreads();
  if (t < world) counts[(size_t)blockIdx.x * world + t] = c[t];
}

// One block: counts[b][d] -> global output offset of block b's rows for d
// (destination-major, then block order); totals[d] = rows for rank d.
__global__ __launch_bounds__(kThreads) void k_shard_scan(unsigned long long* __restrict__ counts, int64_t nblocks,
                                                         int world, unsigned long long* __restrict__ totals) {
  __shared__ unsigned long long s_tmp[4];
  const int t = threadIdx.x;
  const int64_t per = (nblocks + kThreads - 1) / kThreads;
  const int64_t b0 = (int64_t)t * per;
  unsigned long long run0 = 0;
  for (int d = 0; d < world; ++d) {
    unsigned long long s = 0;
    for (int64_t b = b0; b < b0 + per && b < nblocks; ++b) s += counts[(size_t)b * world + d];
    unsigned long long total;
    unsigned long long run = run0 + block_excl_scan(s, s_tmp, total);
    for (int64_t b = b0; b < b0 + per && b < nblocks; ++b) {
      const unsigned long long v = counts[(size_t)b * world + d];
      counts[(size_t)b * world + d] = run;
      run += v;
    }
    if (t == 0) totals[d] = total;
    run0 += total;
  }
}

__global__ __launch_bounds__(kThreads) void k_shard_scatter(const int64_t* __restrict__ pid,
                                                            const int64_t* __restrict__ pk,
                                                            const double* __restrict__ val, int64_t n, int world,
                                                            const unsigned long long* __restrict__ offsets,
                                                            int64_t* __restrict__ opid, int64_t* __restrict__ opk,
                                                            double* __restrict__ oval) {
  __shared__ unsigned long long base[kShardMax];
  __shared__ unsigned int wcnt[4][kShardMax];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t < world) base[t] = offsets[(size_t)blockIdx.x * world + t];
  if (t < kShardMax) wcnt[0][t] = wcnt[1][t] = wcnt[2][t] = wcnt[3][t] = 0;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * kShardChunk;
  const int64_t hi = lo + kShardChunk < n ? lo + kShardChunk : n;
  const int dbits = pdp::ceil_log2_u64((uint64_t)world);
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int64_t b0 = lo; b0 < hi; b0 += kThreads) {
    const int64_t i = b0 + t;
    const bool valid = i < hi;
    int64_t a = 0, k = 0;
    double v = 0.0;
    uint32_t d = 0;
    if (valid) {
      a = pid[i];
      k = pk[i];
      if (val) v = val[i];
      d = shard_dest(a, world);
    }
    // stable rank among the wave's rows with the same destination
    uint64_t peers = __ballot(valid);
    if (!valid) peers = ~peers;
    for (int bit = 0; bit < dbits; ++bit) {
      const bool x = (d >> bit) & 1u;
      const uint64_t bb = __ballot(x);
      peers &= x ? bb : ~bb;
    }
    const uint32_t before = (uint32_t)__popcll(peers & lt);
    if (valid && before == 0) wcnt[wave][d] = (unsigned int)__popcll(peers);
    __syncthreads();
    if (valid) {
      unsigned long long o = base[d] + before;
      for (int w = 0; w < wave; ++w) o += wcnt[w][d];
      opid[o] = a;
      opk[o] = k;
      if (val) oval[o] = v;
    }
    __syncthreads();
    if (t < world) {
      base[t] += (unsigned long long)wcnt[0][t] + wcnt[1][t] + wcnt[2][t] + wcnt[3][t];
      wcnt[0][t] = wcnt[1][t] = wcnt[2][t] = wcnt[3][t] = 0;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Achievable-HBM probe (bench.py roofline.copy_peak_measured): 16 bytes per
// lane, four loads in flight per lane before their stores -- the float4 copy
// shape MI355X_MICROARCH.md measures at 6.29 TB/s.
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_stream_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                     int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

// fp64 FMA chains (pdp_fp64_probe): 8 independent chains per lane, no memory traffic but one store.
__global__ __launch_bounds__(256) void k_fp64_probe(double* __restrict__ out, int iters, double a, double b) {
  double v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = (double)(threadIdx.x + k) * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = fma(v[k], a, b);
  }
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += v[k];
  if (s == 12345.678) out[blockIdx.x] = s;  // keeps the chains alive
}

// Variants: 8 loads in flight per lane; NTL / NTS = non-temporal loads / stores (streaming data that is
// never re-read should not displace L2 / Infinity-Cache lines).  RD: read only (the XOR of the loaded
// words stays in a register; one store per lane if it equals a magic value), WR: write only.
enum CopyKind { kCopyRW = 0, kCopyRead = 1, kCopyWrite = 2 };
template <bool NTL, bool NTS, int KIND>
__global__ __launch_bounds__(256) void k_stream_copy_8(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                       int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    u32x4 v[8];
    if (KIND != kCopyWrite) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = NTL ? __builtin_nontemporal_load(src + i + k * stride) : src[i + k * stride];
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = u32x4{(uint32_t)i, (uint32_t)k, 0u, 0u};
    }
    if (KIND == kCopyRead) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (NTS) __builtin_nontemporal_store(v[k], dst + i + k * stride);
        else dst[i + k * stride] = v[k];
      }
    }
  }
  for (; i < n16; i += stride) {
    if (KIND == kCopyRead) acc ^= src[i].x;
    else if (KIND == kCopyWrite) dst[i] = u32x4{(uint32_t)i, 0u, 0u, 0u};
    else dst[i] = src[i];
  }
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (KIND == kCopyRead && acc == 0x9E3779B9u && j < n16) dst[j] = u32x4{acc, 0u, 0u, 0u};
}

// ---------------------------------------------------------------------------
// Synthetic generator (oracle/pdp_oracle.py:synth_rows)
// ---------------------------------------------------------------------------

__global__ void k_generate(int64_t* __restrict__ pid, int64_t* __restrict__ pk, double* __restrict__ value, int64_t n,
                           int64_t row_offset, int64_t U, int64_t P, double zipf_s, int value_kind, double lo,
                           double hi, uint64_t seed) {
  const int pkb = P > 1 ? pdp::ceil_log2_u64((uint64_t)P) : 1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t gi = (uint64_t)(row_offset + i);
    pdp::u32x4 c{(uint32_t)gi, (uint32_t)(gi >> 32), pdp::kStreamSynth, 0u};
    const pdp::u32x4 x = pdp::philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const double inv = 1.0 / 4294967296.0;
    const double u0 = ((double)x.x + 0.5) * inv, u1 = ((double)x.y + 0.5) * inv, u2 = ((double)x.z + 0.5) * inv;
    int64_t a = (int64_t)(u0 * (double)U);
    if (a > U - 1) a = U - 1;
    int64_t b;
    if (zipf_s > 0.0) {
      const double tt = 1.0 - zipf_s;
      const double top = pow((double)P + 1.0, tt);
      const double xr = pow(1.0 + u1 * (top - 1.0), 1.0 / tt);
      int64_t rank = (int64_t)floor(xr) - 1;
      rank = rank < 0 ? 0 : (rank > P - 1 ? P - 1 : rank);
      uint32_t y = pdp::perm_bits((uint32_t)rank, pkb, 0x5A495046ull);
      while ((int64_t)y >= P) y = pdp::perm_bits(y, pkb, 0x5A495046ull);
      b = y;
    } else {
      b = (int64_t)(u1 * (double)P);
      if (b > P - 1) b = P - 1;
    }
    pid[i] = a;
    pk[i] = b;
    if (value) {
      if (value_kind == 1) {
        int64_t rr = (int64_t)(u2 * 5.0);
        rr = rr > 4 ? 4 : rr;
        value[i] = 1.0 + (double)rr;
      } else {
        value[i] = lo + u2 * (hi - lo);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) return fail(PDP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

int grid_for(int64_t n, int threads, int cap = 4096) {
  int64_t g = (n + threads - 1) / threads;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// hipMemsetAsync(p, 0, bytes) as a kernel, so a captured call holds kernel nodes only: k_zero64 for
// 8-byte aligned buffers of whole words, k_zero_bytes otherwise (no hipMemsetAsync fallback).
hipError_t zero_async(void* p, size_t bytes, hipStream_t stream) {
  if (bytes == 0) return hipSuccess;
  if (((uintptr_t)p & 7u) || (bytes & 7u)) {
    hipLaunchKernelGGL(k_zero_bytes, dim3(grid_for((int64_t)bytes, kThreads, 1024)), dim3(kThreads), 0, stream,
                       (unsigned char*)p, (int64_t)bytes);
    return hipGetLastError();
  }
  const int64_t words = (int64_t)(bytes / 8);
  hipLaunchKernelGGL(k_zero64, dim3(grid_for(words, kThreads, 4096)), dim3(kThreads), 0, stream,
                     (unsigned long long*)p, words);
  return hipGetLastError();
}

struct Layout {
  size_t recs_a, recs_b, recs_c, hist, off, counters, status, ranges, big, tags, tag_lo, keep, k4rep, k4s, grp, total;
  int64_t tiles;
  uint64_t big_cap;
};

// k4p > 0: room for the K4 reduction over k4p partitions (pdp_reduce.inc): the
// digit histogram replicas, the fixed-point scratch (lo, hi, flags per
// partition), the look-back status of a pair pass over up to 2n records, and
// with `variance` the y slots (in recs_c).
Layout layout_for(int64_t n, bool sweep = false, int64_t k4p = 0, bool variance = false) {
  Layout L{};
  size_t o = 0;
  const size_t rb = align_up((size_t)std::max<int64_t>(n, 1) * sizeof(Rec), 256);
  L.recs_a = o; o += rb;
  L.recs_b = o; o += rb;
  L.recs_c = o; o += (sweep || (k4p > 0 && variance)) ? rb : 0;  // sweep: generic-path scratch; K4: y slots
  L.hist = o; o += align_up(kMaxPasses * kHist * 8, 256);
  L.off = o; o += align_up(kMaxPasses * kHist * 8, 256);
  L.counters = o; o += align_up(kNumCounters * 8, 256);
  L.tiles = (std::max<int64_t>(n, 1) + kTile - 1) / kTile;
  L.status = o; o += align_up((size_t)L.tiles * (k4p > 0 ? 2 : 1) * kStatusStride * 8, 256);
  L.ranges = o; o += align_up((size_t)kOverflowCap * 16, 256);
  L.big_cap = (uint64_t)std::max<int64_t>(n, 1) / 129 + 64;  // segments / batches of > 128 rows
  L.big = o; o += align_up((size_t)L.big_cap * 16, 256);
  L.tags = o; o += sweep ? 0 : align_up((size_t)std::max<int64_t>(n, 1) * 4, 256);  // L0 pre-filter tags
  L.tag_lo = o; o += 256 * 4;
  L.keep = o; o += sweep ? 0 : align_up((size_t)std::max<int64_t>(n, 1) / 4 + 64, 256);  // k_filter keep bytes
  // survivor grouping (pdp_group.inc): per-bucket low-byte histogram, claimed run bases, sub-run table, ctl
  L.grp = o; o += sweep ? 0 : align_up((size_t)kGrpSubruns * 8 + 32, 256);
  L.k4rep = o; o += k4p > 0 ? align_up((size_t)kK4Rep * kK4MaxPasses * 256 * 4, 256) : 0;
  L.k4s = o; o += k4p > 0 ? align_up((size_t)k4p * 20, 256) : 0;
  L.total = o;
  return L;
}

struct Plan {
  int pidb, pkb, low, passes;
  int bits[kMaxPasses];
};

Plan make_plan(int64_t n, int64_t U, int64_t P) {
  Plan p{};
  p.pidb = std::max(1, pdp::ceil_log2_u64((uint64_t)U));
  p.pkb = std::max(1, pdp::ceil_log2_u64((uint64_t)P));
  const double rows_per_pid = (double)n / (double)U;
  p.low = 0;  // full sort by pid: segments are contiguous (k_segments)
  (void)rows_per_pid;
  const int kb = p.pidb - p.low;
  p.passes = std::max(1, (kb + 7) / 8);
  int rem = kb;
  for (int i = 0; i < p.passes; ++i) {
    const int w = (rem + (p.passes - i) - 1) / (p.passes - i);
    p.bits[i] = w;
    rem -= w;
  }
  return p;
}

SegParams make_seg(const pdp_bound_params* bp, int low, int pkb, bool has_value) {
  SegParams sp{};
  sp.k4cb = -1;
  sp.low = low;
  sp.pkb = pkb;
  sp.seed = bp->sampling_seed;
  sp.pid_base = (uint64_t)bp->pid_base;
  sp.l0 = bp->max_partitions_contributed;
  sp.linf = bp->max_contributions_per_partition;
  const int m = bp->metrics;
  sp.want_count = (m & (PDP_METRIC_COUNT | PDP_METRIC_MEAN | PDP_METRIC_VARIANCE)) != 0;
  sp.has_value = has_value;
  sp.xmode = kXNone;
  sp.want_y = 0;
  if (m & (PDP_METRIC_MEAN | PDP_METRIC_VARIANCE)) {
    sp.xmode = kXNsum;
    sp.want_y = (m & PDP_METRIC_VARIANCE) != 0;
  } else if (m & PDP_METRIC_SUM) {
    sp.xmode = bp->has_value_bounds ? kXClipSum : kXRawSum;
  }
  sp.a = bp->min_value;
  sp.b = bp->max_value;
  sp.mid = bp->min_value + (bp->max_value - bp->min_value) / 2;  // dp_computations.py:65-69
  sp.smin = bp->min_sum_per_partition;
  sp.smax = bp->max_sum_per_partition;
  sp.packed = 0;
  sp.debug = bp->reserved;
  return sp;
}

}  // namespace

struct pdp_ctx {
  int device = 0;
  int debug = 0;  // pdp_ctx_set_debug: alternative-form flags OR-ed into every call (testing)
  int cur_debug = 0;  // the running call's flags (ctx->debug | pdp_bound_params.reserved)
  // device status block of the last pdp_bound_accumulate(_partials) (k_latch, kStatWords words)
  unsigned long long* dstat = nullptr;
  bool dstat_pending = false;  // an asynchronous call wrote it: pdp_get_status / pdp_get_stats decode it
  bool last_filter = false, last_k4 = false;
  // the last call needed the generic path (overflowing / tied segments): the next one syncs after K2
  // instead of running K4 first and redoing the call
  bool careful = false;
  unsigned int tile_slot = kCtrTile0;  // next free onesweep tile-claim counter
  bool prof = false;
  struct ProfRec {
    int stage;
    hipEvent_t a, b;
  };
  std::vector<ProfRec> pending;
  std::vector<hipEvent_t> pool;
  double prof_ms[PDP_NUM_STAGES] = {};
  int64_t prof_n[PDP_NUM_STAGES] = {};
  void* status_at = nullptr;  // look-back status region cleared for the current epoch run (next_epoch)
  size_t status_ok = 0;  // bytes of the look-back status region cleared for the current epoch run
  uint32_t epoch = 0;
  pdp_stats stats{};
  // Truncated-geometric keep tables, one per (eps, delta, L0), built outside any stream capture
  // (selection_table / pdp_prepare_release) and immutable until pdp_ctx_destroy: a hipGraph that captured
  // pdp_release keeps their device pointer.  (Round 5 rewrote one table in place, or freed it for a
  // larger one: a graph captured earlier then replayed the wrong keep probabilities or a dangling
  // pointer.)
  struct SelTable {
    double eps, delta;
    int64_t k;
    double* dev;
    int64_t len;
  };
  std::vector<SelTable> tables;
};

namespace {

// Makes the context's device current for the duration of an entry point and
// restores the caller's device afterwards (HipBackend(device=k) while another
// device is current).
struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Stream-ordered frees of the generic path's scratch at scope exit, on every
// return path (HIP_TRY returns early).
struct AsyncFrees {
  hipStream_t stream;
  std::vector<void*> ptrs;
  explicit AsyncFrees(hipStream_t s) : stream(s) {}
  hipError_t alloc(void** p, size_t bytes) {
    const hipError_t e = hipMallocAsync(p, bytes, stream);
    if (e == hipSuccess) ptrs.push_back(*p);
    return e;
  }
  ~AsyncFrees() {
    for (void* p : ptrs) (void)hipFreeAsync(p, stream);
  }
};

hipEvent_t prof_event(pdp_ctx* ctx) {
  if (!ctx->pool.empty()) {
    hipEvent_t e = ctx->pool.back();
    ctx->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

// Records hipEvents around a stage on `stream` when profiling is enabled.
struct ProfScope {
  pdp_ctx* ctx;
  int stage;
  hipStream_t stream;
  hipEvent_t a = nullptr;
  ProfScope(pdp_ctx* c, int s, hipStream_t st) : ctx(c), stage(s), stream(st) {
    if (ctx->prof) {
      a = prof_event(ctx);
      (void)hipEventRecord(a, stream);
    }
  }
  ~ProfScope() {
    if (ctx->prof && a) {
      hipEvent_t b = prof_event(ctx);
      (void)hipEventRecord(b, stream);
      ctx->pending.push_back({stage, a, b});
    }
  }
};

int env_int(const char* name, int def);
int dev_occ(int debug);

// Look-back status words carry the epoch of their pass, so a region cleared
// once serves 0xFFFE passes.  The region is cleared again when a pass needs
// more of it, when it moves (another layout of the workspace: the bytes held
// records or other scratch), and on the first pass of every API call
// (ctx->status_at reset on entry: the caller owns the workspace between calls).
// Round 4: the check was keyed on the workspace base, so a utility analysis
// after a larger aggregate on the same workspace met stale record bytes that
// read as published status words -> wrong digit bases -> out-of-range scatter.
int next_epoch(pdp_ctx* ctx, hipStream_t stream, unsigned long long* status, size_t status_bytes) {
  if (ctx->status_at != (void*)status || ctx->epoch >= 0xFFFE || status_bytes > ctx->status_ok) {
    HIP_TRY(zero_async(status, status_bytes, stream));
    ctx->status_at = status;
    ctx->status_ok = status_bytes;
    ctx->epoch = 0;
  }
  ++ctx->epoch;
  return 0;
}

// next_epoch for passes whose row count lives in device memory (*rows_dev + add): the clear is a
// kernel sized by that count.  `fresh`: the first pass of a group (its tiles may exceed what earlier
// passes of this call cleared).
#ifndef PDP_PERSIST_GRID
#define PDP_PERSIST_GRID 2048
#endif
constexpr unsigned kPersistGrid = PDP_PERSIST_GRID;  // look-back launches over a device row count: blocks loop over tiles
void next_epoch_dev(pdp_ctx* ctx, hipStream_t stream, unsigned long long* status, const unsigned long long* rows_dev,
                    int64_t add, bool fresh) {
  if (fresh || ctx->status_at != (void*)status || ctx->epoch >= 0xFFFE) {
    hipLaunchKernelGGL(k_status_clear, dim3(1024), dim3(kThreads), 0, stream, status, rows_dev, add);
    ctx->status_at = status;
    ctx->status_ok = 0;  // a later host-sized pass clears what it needs
    ctx->epoch = 0;
  }
  ++ctx->epoch;
}

int scan_inplace(long long* a, int64_t n, hipStream_t stream) {
  if (n <= 0) return 0;
  const int64_t nb = (n + 2047) / 2048;
  AsyncFrees scratch(stream);
  long long* sums = nullptr;
  HIP_TRY(scratch.alloc((void**)&sums, (size_t)nb * sizeof(long long)));
  hipLaunchKernelGGL(k_scan_chunks, dim3((unsigned)nb), dim3(kThreads), 0, stream, a, n, sums);
  if (nb > 1) {
    int rc = scan_inplace(sums, nb, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(kThreads), 0, stream, a, n, sums);
  }
  HIP_TRY(hipGetLastError());
  return 0;
}

// Reduce-then-scan radix passes: tile digit counts (written by K0 for pass 0,
// by k_tile_counts otherwise) -> per-tile global digit bases in place.
// `tile_cnt` and the chunk sums live in the look-back status region (so the
// next look-back use re-zeroes it).  Needs rows < 2^32 (u32 bases).
struct TileScan {
  unsigned int* tile_cnt;
  unsigned int* chunk;
  int64_t tiles;
};

TileScan tile_scan_bufs(pdp_ctx* ctx, unsigned long long* status, int64_t tiles) {
  ctx->status_at = nullptr;
  TileScan ts;
  ts.tile_cnt = (unsigned int*)status;
  ts.chunk = ts.tile_cnt + (size_t)tiles * 256;
  ts.tiles = tiles;
  return ts;
}

bool use_tile_scan(int64_t n, int debug) { return n < (1ll << 32) && !(debug & kDebugLookback); }

void tile_scan(const TileScan& ts, const unsigned long long* off_pass, hipStream_t stream) {
  const int64_t nchunks = (ts.tiles + kScanTiles - 1) / kScanTiles;
  hipLaunchKernelGGL(k_tile_chunk_sums, dim3((unsigned)nchunks), dim3(kThreads), 0, stream, ts.tile_cnt, ts.tiles,
                     ts.chunk);
  hipLaunchKernelGGL(k_tile_chunk_scan, dim3(256), dim3(kThreads), 0, stream, ts.chunk, nchunks, off_pass);
  hipLaunchKernelGGL(k_tile_bases, dim3((unsigned)nchunks), dim3(kThreads), 0, stream, ts.tile_cnt, ts.tiles,
                     ts.chunk);
}

// LSD sort of `m` records (a <-> b ping-pong) by the passes of `ks`; the
// sorted array pointer is returned in *out.  m_dev != null: the record count
// is *m_dev (device memory, e.g. the pre-filter's survivors) and m an upper
// bound -- no host round trip; the passes run on a persistent look-back grid.
int sort_recs(pdp_ctx* ctx, Rec* a, Rec* b, int64_t m, const KeySpec& ks, unsigned long long* hist,
              unsigned long long* off, unsigned long long* counters, unsigned long long* status, size_t status_bytes,
              void* ws, hipStream_t stream, Rec** out, int stage = PDP_STAGE_GENERIC,
              const int64_t* soa_pid = nullptr, const int64_t* soa_pk = nullptr, const double* soa_val = nullptr,
              const unsigned long long* m_dev = nullptr, int run_passes = -1, bool hist_ready = false) {
  // hist_ready: the caller filled `hist` (no histogram pass; unused since k_filter orders the survivors)
  // run_passes >= 0: histogram and offsets for all ks.passes, but only the first run_passes passes run
  // (the survivor grouping finishes the last one in LDS, pdp_group.inc)
  // soa_pk != null: the utility analysis' rows, packed by the histogram and the first pass themselves
  // (k_histogram<2>, k_ana_sort_first); `a` is not read
  if (m <= 0 || ks.passes == 0) {
    *out = a;
    return 0;
  }
  if (ks.passes > kMaxPasses) return fail(PDP_ERR_INTERNAL, "too many radix passes");
  if (ctx->tile_slot + ks.passes > kNumCounters) {
    HIP_TRY(zero_async(counters + kCtrTile0, (kNumCounters - kCtrTile0) * 8, stream));
    ctx->tile_slot = kCtrTile0;
  }
  if (!hist_ready) HIP_TRY(zero_async(hist, kMaxPasses * kHist * 8, stream));
  ProfScope prof_generic(ctx, stage, stream);
  if (hist_ready) {
  } else if (soa_pk) {
    hipLaunchKernelGGL(k_histogram<2>, dim3(grid_for(m, kThreads, 2048)), dim3(kThreads), 0, stream, soa_pid, soa_pk,
                       (const Rec*)nullptr, m, ks, hist, counters, m_dev);
  } else {
    hipLaunchKernelGGL(k_histogram<0>, dim3(grid_for(m, kThreads, 2048)), dim3(kThreads), 0, stream,
                       (const int64_t*)nullptr, (const int64_t*)nullptr, a, m, ks, hist, counters, m_dev);
  }
  hipLaunchKernelGGL(k_offsets, dim3(1), dim3(kThreads), 0, stream, hist, off, ks.passes, m, counters,
                     (int)kCtrNGeneric, m_dev);
  Rec* src = a;
  Rec* dst = b;
  const int64_t tiles = (m + kTile - 1) / kTile;
  // decoupled look-back passes (no tile-count upsweeps): c3 survivor sort 2.15 -> 2.02 ms, c5 (pk, pid)
  // sort 7.26 -> 6.48 ms (same box); PDP_SORT_TILESCAN=1 restores reduce-then-scan
  const bool rts = use_tile_scan(m, 0) && (ctx->cur_debug & kDebugSortTileScan) != 0 && !m_dev;
  const unsigned grid = m_dev ? (unsigned)std::min<int64_t>(tiles, kPersistGrid) : (unsigned)tiles;
  const int npass = run_passes >= 0 ? std::min(run_passes, ks.passes) : ks.passes;
  for (int p = 0; p < npass; ++p) {
    const unsigned int* bases = nullptr;
    // the fused first pass of the utility analysis reads the SoA columns: its tile counts would need
    // them too, so it always runs by look-back (k_tile_counts reads records)
    if (m_dev) {
      next_epoch_dev(ctx, stream, status, m_dev, 0, p == 0);
    } else if (rts && !(soa_pk && p == 0)) {
      const TileScan ts = tile_scan_bufs(ctx, status, tiles);
      hipLaunchKernelGGL(k_tile_counts, dim3(grid_for(tiles, 1, 4096)), dim3(kThreads), 0, stream, src, counters,
                         (int)kCtrNGeneric, ks, p, tiles, ts.tile_cnt);
      tile_scan(ts, off + p * kHist, stream);
      bases = ts.tile_cnt;
    } else {
      int rc = next_epoch(ctx, stream, status, std::min(status_bytes, (size_t)tiles * kStatusStride * 8));
      if (rc) return rc;
    }
    const bool soa = soa_pk && p == 0;
    const int occ = dev_occ(ctx->cur_debug);
    auto dev_kern = occ == 2 ? k_onesweep_dev<2> : occ == 4 ? k_onesweep_dev<4> : k_onesweep_dev<3>;
    hipLaunchKernelGGL(soa ? k_ana_sort_first : m_dev ? dev_kern : k_onesweep, dim3(grid), dim3(kThreads), 0, stream,
                       soa ? soa_pid : (const int64_t*)nullptr, soa ? soa_pk : (const int64_t*)nullptr,
                       soa ? soa_val : (const double*)nullptr, soa ? (const Rec*)nullptr : src, dst, m,
                       counters, (int)kCtrNGeneric, ks, p, off + p * kHist, status, ctx->epoch, counters,
                       (int)ctx->tile_slot++, bases, (uint32_t*)nullptr, (const uint32_t*)nullptr,
                       (const Rec*)nullptr, (int64_t)INT64_MAX);
    std::swap(src, dst);
  }
  HIP_TRY(hipGetLastError());
  *out = src;
  return 0;
}

KeySpec composite_spec(int mode, int hi_bits, int lo_bits, int pkb, uint64_t U, uint32_t P) {
  KeySpec ks{};
  ks.xcd_remap = 1;
  ks.mode = mode;
  ks.low = 0;
  ks.pkb = pkb;
  ks.num_pids = U;
  ks.num_parts = P;
  // digits of 8 bits; mode 3: lo = 64 bits of val, hi = pid field starting at bit 64
  int sh = 0, p = 0;
  const int lo_total = mode == 3 ? 64 : lo_bits + hi_bits;
  while (sh < lo_total && p < kMaxPasses) {
    ks.shift[p] = sh;
    ks.bits[p] = std::min(8, lo_total - sh);
    sh += ks.bits[p];
    ++p;
  }
  if (mode == 3) {
    for (int h = 0; h < hi_bits; h += 8) {
      ks.shift[p] = 64 + h;
      ks.bits[p] = std::min(8, hi_bits - h);
      ++p;
    }
  }
  ks.passes = p;
  return ks;
}

// Every wait of pdp_bound_accumulate for its stream goes through here (pdp_stats.host_waits).
hipError_t host_wait(pdp_ctx* ctx, hipStream_t stream) {
  ++ctx->stats.host_waits;
  return hipStreamSynchronize(stream);
}

// `sorted` is only read (gather); `alt` is the generic sort's second buffer
// (== sorted on the single-config path, a third buffer in a sweep so the
// sorted rows survive for the next configuration).  K4 (sp.k4x != null): the
// slots buffer (`spare`) must not be touched, so the gather / sort buffers
// are allocated here, and the kept groups' pair records go to an array of
// one slot per group allocated in `keep` (*kf_x / *kf_y, *kf_n slots).
int run_generic(pdp_ctx* ctx, const Rec* sorted, Rec* spare, Rec* alt, const std::vector<unsigned long long>& ranges,
                const Plan& plan, const SegParams& sp_in, const pdp_bound_params* bp, uint64_t U, uint32_t P,
                AccPtrs acc, unsigned long long* hist, unsigned long long* off, unsigned long long* counters,
                unsigned long long* status, size_t status_bytes, void* ws, hipStream_t stream, AsyncFrees* keep,
                Rec** kf_x, Rec** kf_y, int64_t* kf_n) {
  SegParams sp = sp_in;
  const int nr = (int)(ranges.size() / 2);
  std::vector<long long> rsrc(nr), rdst(nr);
  int64_t total = 0;
  for (int i = 0; i < nr; ++i) {
    rsrc[i] = (long long)ranges[2 * i];
    rdst[i] = total;
    total += (int64_t)(ranges[2 * i + 1] - ranges[2 * i]);
  }
  ctx->stats.fallback_rows = total;
  ctx->stats.fallback_ranges = nr;
  if (kf_n) *kf_n = 0;
  if (total == 0) return 0;
  AsyncFrees scratch(stream);
  if (sp.k4x) {
    HIP_TRY(scratch.alloc((void**)&spare, (size_t)total * sizeof(Rec)));
    HIP_TRY(scratch.alloc((void**)&alt, (size_t)total * sizeof(Rec)));
  }
  long long *d_rsrc = nullptr, *d_rdst = nullptr;
  HIP_TRY(scratch.alloc((void**)&d_rsrc, nr * sizeof(long long)));
  HIP_TRY(scratch.alloc((void**)&d_rdst, nr * sizeof(long long)));
  HIP_TRY(hipMemcpyAsync(d_rsrc, rsrc.data(), nr * sizeof(long long), hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemcpyAsync(d_rdst, rdst.data(), nr * sizeof(long long), hipMemcpyHostToDevice, stream));
  hipLaunchKernelGGL(k_gather_ranges, dim3(grid_for(total, kThreads)), dim3(kThreads), 0, stream, sorted, spare,
                     d_rsrc, d_rdst, nr, total);
  HIP_TRY(host_wait(ctx, stream));  // host vectors go out of scope

  // 1) rows by (pid, pk), stable (input order within a group)
  Rec* r = nullptr;
  int rc = sort_recs(ctx, spare, alt, total, composite_spec(1, plan.pidb, plan.pkb, plan.pkb, U, P), hist, off,
                     counters, status, status_bytes, ws, stream, &r);
  if (rc) return rc;
  Rec* r_other = (r == spare) ? alt : spare;

  const size_t m8 = (size_t)total * 8;
  long long *gsc, *psc, *gpos, *pfirst;
  HIP_TRY(scratch.alloc((void**)&gsc, m8));
  HIP_TRY(scratch.alloc((void**)&psc, m8));
  HIP_TRY(scratch.alloc((void**)&gpos, m8 + 8));
  HIP_TRY(scratch.alloc((void**)&pfirst, m8));
  const int gr = grid_for(total, kThreads);
  hipLaunchKernelGGL(k_stream_flags, dim3(gr), dim3(kThreads), 0, stream, r, total, gsc, psc);
  if ((rc = scan_inplace(gsc, total, stream))) return rc;
  if ((rc = scan_inplace(psc, total, stream))) return rc;
  hipLaunchKernelGGL(k_stream_starts, dim3(gr), dim3(kThreads), 0, stream, gsc, psc, r, total, gpos, pfirst);
  long long ngroups = 0, npids = 0;
  HIP_TRY(hipMemcpyAsync(&ngroups, gsc + (total - 1), 8, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipMemcpyAsync(&npids, psc + (total - 1), 8, hipMemcpyDeviceToHost, stream));
  HIP_TRY(host_wait(ctx, stream));

  // 2) L_inf ranks: sort (group, row priority, row) -> rank within group.
  Rec *x1, *x2;
  HIP_TRY(scratch.alloc((void**)&x1, (size_t)total * sizeof(Rec)));
  HIP_TRY(scratch.alloc((void**)&x2, (size_t)total * sizeof(Rec)));
  uint8_t* row_keep;
  int32_t* grank;
  HIP_TRY(scratch.alloc((void**)&row_keep, (size_t)total));
  HIP_TRY(scratch.alloc((void**)&grank, (size_t)ngroups * 4));
  hipLaunchKernelGGL(k_stream_row_prio, dim3(gr), dim3(kThreads), 0, stream, r, total, gsc, gpos, sp.seed, sp.pid_base,
                     x1);
  Rec* xs = nullptr;
  const int gbits = std::max(1, pdp::ceil_log2_u64((uint64_t)ngroups));
  if ((rc = sort_recs(ctx, x1, x2, total, composite_spec(3, gbits, 64, plan.pkb, U, P), hist, off, counters, status,
                      status_bytes, ws, stream, &xs)))
    return rc;
  hipLaunchKernelGGL(k_stream_ranks, dim3(gr), dim3(kThreads), 0, stream, xs, total, gpos, (int64_t)sp.linf,
                     row_keep, (int32_t*)nullptr);
  // 3) L0 ranks: sort (pid, group priority, group) -> rank within pid.
  const int ggr = grid_for(ngroups, kThreads);
  hipLaunchKernelGGL(k_stream_group_prio, dim3(ggr), dim3(kThreads), 0, stream, r, psc, gpos, (int64_t)ngroups,
                     sp.seed, sp.pid_base, x1);
  const int pbits = std::max(1, pdp::ceil_log2_u64((uint64_t)npids));
  if ((rc = sort_recs(ctx, x1, x2, ngroups, composite_spec(3, pbits, 64, plan.pkb, U, P), hist, off, counters,
                      status, status_bytes, ws, stream, &xs)))
    return rc;
  hipLaunchKernelGGL(k_stream_ranks, dim3(ggr), dim3(kThreads), 0, stream, xs, (int64_t)ngroups, pfirst,
                     (int64_t)sp.l0, (uint8_t*)nullptr, grank);
  // 4) kept groups: sums of the kept rows, then accumulators / pair records.
  if (sp.k4x) {
    // 16 bytes per group also hold split slots (k4_soa_offset(ngroups) + 8 ngroups <= 12 ngroups + 12)
    HIP_TRY(keep->alloc((void**)&sp.k4x, (size_t)ngroups * sizeof(Rec) + 16));
    sp.k4y = nullptr;
    if (sp.want_y) HIP_TRY(keep->alloc((void**)&sp.k4y, (size_t)ngroups * sizeof(Rec) + 16));
    if (sp.k4soa) sp.k4soa = k4_soa_offset(ngroups);
    *kf_x = sp.k4x;
    *kf_y = sp.k4y;
    *kf_n = ngroups;
  }
  unsigned long long* big = nullptr;  // [count, group ids]: kept groups over kBigGroupRows rows
  HIP_TRY(scratch.alloc((void**)&big, (size_t)(total / kBigGroupRows + 2) * 8));
  HIP_TRY(zero_async(big, 8, stream));
  hipLaunchKernelGGL(k_stream_groups, dim3(ggr), dim3(kThreads), 0, stream, r, gpos, grank, row_keep,
                     (int64_t)ngroups, sp, acc, big);
  hipLaunchKernelGGL(k_stream_big_groups, dim3((unsigned)std::min<int64_t>(total / kBigGroupRows + 1, 1024)),
                     dim3(kThreads), 0, stream, r, gpos, row_keep, sp, acc, big);
  HIP_TRY(hipGetLastError());
  (void)r_other;
  return 0;
}

double std_normal_cdf(double x) { return 0.5 * std::erfc(-x / std::sqrt(2.0)); }

double gaussian_delta(double sigma, double eps) {
  const double a = 1.0 / (2.0 * sigma), b = eps * sigma;
  return std_normal_cdf(a - b) - std::exp(eps) * std_normal_cdf(-a - b);
}

// Acklam's inverse normal CDF refined by one Halley step.
double norm_ppf(double p) {
  static const double a[] = {-3.969683028665376e+01, 2.209460984245205e+02, -2.759285104469687e+02,
                             1.383577518672690e+02, -3.066479806614716e+01, 2.506628277459239e+00};
  static const double b[] = {-5.447609879822406e+01, 1.615858368580409e+02, -1.556989798598866e+02,
                             6.680131188771972e+01, -1.328068155288572e+01};
  static const double c[] = {-7.784894002430293e-03, -3.223964580411365e-01, -2.400758277161838e+00,
                             -2.549732539343734e+00, 4.374664141464968e+00, 2.938163982698783e+00};
  static const double d[] = {7.784695709041462e-03, 3.224671290700398e-01, 2.445134137142996e+00,
                             3.754408661907416e+00};
  double x;
  if (p < 0.02425) {
    const double q = std::sqrt(-2 * std::log(p));
    x = (((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
        ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1);
  } else if (p > 1 - 0.02425) {
    const double q = std::sqrt(-2 * std::log(1 - p));
    x = -(((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
        ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1);
  } else {
    const double q = p - 0.5, r = q * q;
    x = (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * q /
        (((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1);
  }
  const double e = std_normal_cdf(x) - p;
  const double u = e * std::sqrt(2 * M_PI) * std::exp(x * x / 2);
  return x - u / (1 + x * u / 2);
}

// Per-partition delta of a selection strategy over k = max_partitions_contributed
// partitions: 1 - (1 - delta)^(1/k), so that k independent per-partition
// decisions compose to delta; eps is split as eps / k.  One adjustment for all
// three strategies (truncated geometric, Laplace and Gaussian thresholding).
// PyDP's (partition_selection.py:24-33) is parity unpinned for k > 1: the
// reference pins only k = 1 (analysis/tests/combiners_test.py:197-224), where
// this is delta.  It differs from delta / k by less than delta^2 / 2.
double adjusted_delta(double delta, int64_t k) {
  if (k <= 1) return delta;
  return -std::expm1(std::log1p(-delta) / (double)k);
}

double noise_scale(int kind, double eps, double delta, double l0, double linf) {
  // dp_computations.py:146-175
  if (kind == PDP_NOISE_LAPLACE) return l0 * linf / eps;
  return pdp_gaussian_sigma(eps, delta, std::sqrt(l0) * linf);
}

bool k4_enabled(int64_t n, bool sweep, int debug = 0, int64_t linf = 1);
int decode_status(pdp_ctx* ctx, const unsigned long long* h);

}  // namespace

namespace {

// The truncated-geometric keep table of (eps, delta, k) on the device: found in the context's immutable
// cache, or built there.  Building needs a host copy and an allocation, which a stream capture must not
// contain: under capture an uncached table is PDP_ERR_NEEDS_SYNC (call pdp_prepare_release first).
int selection_table(pdp_ctx* ctx, double eps, double delta, int64_t k, hipStream_t stream, const double** dev,
                    int64_t* len) {
  for (const auto& t : ctx->tables) {
    if (t.eps == eps && t.delta == delta && t.k == k) {
      *dev = t.dev;
      *len = t.len;
      return 0;
    }
  }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIP_TRY(hipStreamIsCapturing(stream, &cs));
  if (cs != hipStreamCaptureStatusNone)
    return fail(PDP_ERR_NEEDS_SYNC, "pdp_release under stream capture needs its selection table prepared first "
                                    "(pdp_prepare_release before the capture)");
  int64_t n = 0;
  if (int rc = pdp_truncated_geometric_table(eps, delta, k, nullptr, 0, &n)) return rc;
  std::vector<double> host((size_t)n, 0.0);
  int64_t n2 = 0;
  if (int rc = pdp_truncated_geometric_table(eps, delta, k, host.data(), n, &n2)) return rc;
  double* d = nullptr;
  HIP_TRY(hipMalloc((void**)&d, (size_t)std::max<int64_t>(n, 1) * 8));
  if (n > 0) {
    const hipError_t e = hipMemcpy(d, host.data(), (size_t)n * 8, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(d);
      return fail(PDP_ERR_HIP, std::string("selection table copy: ") + hipGetErrorString(e));
    }
  }
  ctx->tables.push_back({eps, delta, k, d, n});
  *dev = d;
  *len = n;
  return 0;
}

}  // namespace

extern "C" {

int pdp_abi_version(void) { return PDP_ABI_VERSION; }

const char* pdp_last_error(void) { return g_err.c_str(); }

pdp_ctx* pdp_ctx_create(int device) {
  pdp_ctx* c = new pdp_ctx();
  c->device = device;
  DeviceGuard dg(device);
  if (!dg.ok || hipMalloc((void**)&c->dstat, kStatWords * 8) != hipSuccess) c->dstat = nullptr;
  return c;
}

void pdp_ctx_destroy(pdp_ctx* ctx) {
  if (!ctx) return;
  for (auto& r : ctx->pending) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  for (auto e : ctx->pool) (void)hipEventDestroy(e);
  for (auto& t : ctx->tables) (void)hipFree(t.dev);
  if (ctx->dstat) (void)hipFree(ctx->dstat);
  delete ctx;
}

int pdp_metric_fields(int32_t metrics, int32_t* fields) {
  int n = 0;
  if (metrics & PDP_METRIC_VARIANCE) {
    fields[n++] = PDP_FIELD_VARIANCE;  // VarianceCombiner dict order, combiners.py:386-392
    if (metrics & PDP_METRIC_COUNT) fields[n++] = PDP_FIELD_COUNT;
    if (metrics & PDP_METRIC_SUM) fields[n++] = PDP_FIELD_SUM;
    if (metrics & PDP_METRIC_MEAN) fields[n++] = PDP_FIELD_MEAN;
  } else if (metrics & PDP_METRIC_MEAN) {
    fields[n++] = PDP_FIELD_MEAN;  // combiners.py:323-328
    if (metrics & PDP_METRIC_COUNT) fields[n++] = PDP_FIELD_COUNT;
    if (metrics & PDP_METRIC_SUM) fields[n++] = PDP_FIELD_SUM;
  } else {
    if (metrics & PDP_METRIC_COUNT) fields[n++] = PDP_FIELD_COUNT;
    if (metrics & PDP_METRIC_SUM) fields[n++] = PDP_FIELD_SUM;
  }
  if (metrics & PDP_METRIC_PRIVACY_ID_COUNT) fields[n++] = PDP_FIELD_PRIVACY_ID_COUNT;
  return n;
}

double pdp_gaussian_sigma(double eps, double delta, double l2) {
  // PyDP GaussianMechanism std (see oracle/pdp_oracle.py:gaussian_sigma).
  if (!(eps > 0) || !(delta > 0)) return NAN;
  double lo = 0.0, hi = 1.0;
  while (gaussian_delta(hi, eps) > delta) {
    lo = hi;
    hi *= 2.0;
  }
  while (hi - lo > 1e-3 * lo) {
    const double mid = lo + (hi - lo) / 2.0;
    if (gaussian_delta(mid, eps) > delta)
      lo = mid;
    else
      hi = mid;
  }
  return hi * l2;
}

int pdp_truncated_geometric_table(double eps, double delta, int64_t k, double* out, int64_t cap, int64_t* length) {
  if (!(eps > 0) || delta < 0 || k <= 0 || !length) return fail(PDP_ERR_INVALID_ARG, "bad truncated geometric args");
  const double e = eps / (double)k, d = adjusted_delta(delta, k);
  const double ee = std::exp(e), eme = std::exp(-e);
  double prev = 0.0;
  int64_t len = 1;
  if (out && cap > 0) out[0] = 0.0;
  while (prev < 1.0) {
    double nxt = std::min(std::min(ee * prev + d, 1.0 - eme * (1.0 - prev - d)), 1.0);
    if (nxt <= prev) return fail(PDP_ERR_INVALID_ARG, "truncated geometric selection cannot keep partitions");
    if (out && len < cap) out[len] = nxt;
    ++len;
    prev = nxt;
    if (len > (1ll << 24)) return fail(PDP_ERR_INVALID_ARG, "truncated geometric table too long");
  }
  *length = len;
  return 0;
}

int pdp_selection_threshold(int32_t selection, double eps, double delta, int64_t k, double* thr, double* scale) {
  if (!(eps > 0) || k <= 0) return fail(PDP_ERR_INVALID_ARG, "bad selection args");
  if (selection == PDP_SELECTION_LAPLACE_THRESHOLDING) {
    const double adj = adjusted_delta(delta, k);
    const double b = (double)k / eps;
    *scale = b;
    *thr = adj > 0.5 ? 1.0 + b * std::log(2.0 * (1.0 - adj)) : 1.0 - b * std::log(2.0 * adj);
    return 0;
  }
  if (selection == PDP_SELECTION_GAUSSIAN_THRESHOLDING) {
    if (!(delta > 0)) return fail(PDP_ERR_INVALID_ARG, "Gaussian thresholding needs delta > 0");
    const double td = delta / 2.0, nd = delta - td;
    const double sigma = pdp_gaussian_sigma(eps, nd, std::sqrt((double)k));
    const double adj = adjusted_delta(td, k);
    *scale = sigma;
    *thr = 1.0 + sigma * norm_ppf(1.0 - adj);
    return 0;
  }
  return fail(PDP_ERR_INVALID_ARG, "selection has no threshold");
}

int pdp_workspace_size(const pdp_columns* cols, const pdp_bound_params* bp, size_t* bytes) {
  if (!cols || !bp || !bytes) return fail(PDP_ERR_INVALID_ARG, "null argument");
  if (cols->num_rows < 0) return fail(PDP_ERR_INVALID_ARG, "num_rows < 0");
  const bool k4 = k4_enabled(cols->num_rows, false);
  *bytes = layout_for(cols->num_rows, false, k4 ? std::max<int64_t>(cols->num_partitions, 1) : 0,
                      (bp->metrics & PDP_METRIC_VARIANCE) != 0)
               .total;
  return 0;
}

int pdp_sweep_workspace_size(const pdp_columns* cols, size_t* bytes) {
  if (!cols || !bytes) return fail(PDP_ERR_INVALID_ARG, "null argument");
  if (cols->num_rows < 0) return fail(PDP_ERR_INVALID_ARG, "num_rows < 0");
  *bytes = layout_for(cols->num_rows, true).total;
  return 0;
}

int pdp_ctx_set_debug(pdp_ctx* ctx, int32_t flags) {
  if (!ctx) return fail(PDP_ERR_INVALID_ARG, "null argument");
  if ((flags & kAblationFlags) && !kDebugBuild)
    return fail(PDP_ERR_INVALID_ARG, "timing-ablation debug flags need a -DPDP_DEBUG_BUILD library");
  ctx->debug = flags;
  return 0;
}

int pdp_get_status(pdp_ctx* ctx, int32_t* call_status) {
  if (!ctx || !call_status) return fail(PDP_ERR_INVALID_ARG, "null argument");
  *call_status = 0;
  if (!ctx->dstat_pending) return 0;
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return fail(PDP_ERR_HIP, "hipSetDevice failed");
  unsigned long long h[kStatWords];
  HIP_TRY(hipMemcpy(h, ctx->dstat, sizeof(h), hipMemcpyDeviceToHost));
  ctx->dstat_pending = false;
  const std::string prev = g_err;
  int rc = decode_status(ctx, h);
  if (!rc && (h[kStatRanges] || h[kStatFull])) {
    rc = fail(PDP_ERR_NEEDS_SYNC, "the input needs the generic path: call again without PDP_BOUND_ASYNC");
    ctx->careful = true;
  }
  *call_status = rc;
  if (!rc) g_err = prev;
  return 0;
}

int pdp_get_stats(pdp_ctx* ctx, pdp_stats* out) {
  if (!ctx || !out) return fail(PDP_ERR_INVALID_ARG, "null argument");
  if (ctx->dstat_pending) {
    int32_t st = 0;
    if (int rc = pdp_get_status(ctx, &st)) return rc;
    ctx->dstat_pending = true;  // the status stays readable by pdp_get_status
  }
  *out = ctx->stats;
  return 0;
}

namespace {

// When the L0 pre-filter runs (pdp_filter.inc): small L0, enough rows per
// privacy id for most of them to fall outside the kept partitions, and
// buckets of at most 2 x kFiltWords privacy ids (U up to ~20e6; beyond
// kFiltWords per bucket the sketch is 16 bits per pid).
struct FilterPlan {
  bool on;
  bool half;      // buckets of up to 2 x kFiltWords pids: two 16-bit sketches per LDS word
  uint64_t mult;  // bucket digit = (pid * mult) >> 32
  int low_bits;   // pid bits that tell the ids of one bucket apart
};

// Environment knobs exist only in -DPDP_DEBUG_BUILD libraries (experiment builds,
// tools/copy_probe.py): the shipped library reads no environment.
int env_int(const char* name, int def) {
  if (!kDebugBuild) return def;
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : def;
}

// Blocks per CU of the device-sized look-back passes (PDP_ONESWEEP_LOOP kernels).
int dev_occ(int debug) {
  if (debug & kDebugDevOcc2) return 2;
  return env_int("PDP_DEV_OCC", 3);
}

FilterPlan filter_plan(int64_t n, int64_t U, const pdp_bound_params* bp, int debug, bool sweep, bool rts) {
  FilterPlan f{};
  if (sweep || !rts || bp->bounds_already_enforced || (debug & kDebugNoFilter)) return f;
  const int64_t l0 = bp->max_partitions_contributed;
  if (l0 > kFiltMaxL0 || U < 1 || U > (1ll << 32)) return f;
  if (!(debug & kDebugForceFilter) && (n < (1ll << 22) || n < 4 * l0 * U)) return f;
  const uint64_t mult = (1ull << 40) / (uint64_t)U;  // floor: every digit <= 255
  uint64_t width = 0;
  for (uint64_t b = 0; b < 256; ++b) {
    const uint64_t lo = filt_bucket_lo(b, mult);
    const uint64_t hi = std::min<uint64_t>(filt_bucket_lo(b + 1, mult), (uint64_t)U);
    if (hi > lo) width = std::max(width, hi - lo);
  }
  if (width > 2ull * kFiltWords) return f;
  f.on = true;
  f.half = width > (uint64_t)kFiltWords;
  f.mult = mult;
  f.low_bits = std::max(1, pdp::ceil_log2_u64(width));
  return f;
}

// K4 plan (pdp_reduce.inc): partition-block digits of the pair passes and the
// fixed-point scales.  Off for the parameter sweep (and with debug flag NO_K4; the
// packed per-block counts) and with PDP_K4=0 (A/B experiments): the
// accumulators then take fp64 atomics, as in round 2.
struct K4Plan {
  bool on;
  int sh;  // partition block = pk >> sh (LDS window of the reduction: 2^sh partitions)
  int passes;
  int shift[kK4MaxPasses], bits[kK4MaxPasses];
  int fx, fy;  // fixed-point exponents: q = rint(x * 2^f)
  int cb;      // count bits of a 12-byte pair record's key
  bool p12;    // pair passes move 12-byte records {pk << cb | count - 1, x} (pk and count fit 31 bits)
  bool soa;    // (p12) K2 writes split slots (keys, values); the first pass reads a 4-byte key per empty slot
};

// F = 62 - ceil(log2 M): |q| <= 2^62 for |x| <= M; sums of < 2^32 records stay exact in (lo, hi).
int k4_exponent(double M) {
  if (!(M > 0.0) || !std::isfinite(M)) return 0;
  int e = 0;
  (void)std::frexp(M, &e);  // M < 2^e
  return std::max(-1000, std::min(1000, 62 - e));
}

// Any row count (round 5; round 4 fell back to fp64 atomics at >= 2^32 rows).  What bounds K4 is per
// reduce chunk (<= kK4Chunk pair records): a partition's (count << 32 | pairs) LDS word needs the
// chunk's kept rows of one partition < 2^32, i.e. L_inf < 2^32 / kK4Chunk when rows >= 2^32 (below 2^32
// rows the whole input is smaller); the fixed-point (lo, hi) sums hold <= 2^32 pairs per partition (U <=
// 2^32, one pair per privacy id) exactly.
bool k4_enabled(int64_t n, bool sweep, int debug, int64_t linf) {
  if (sweep || (debug & kDebugNoK4)) return false;
  return n < (1ll << 32) || linf < (1ll << 32) / kK4Chunk;
}

K4Plan k4_plan(const pdp_bound_params* bp, const SegParams& sp, int64_t n, int64_t P, bool sweep) {
  K4Plan k{};
  k.on = k4_enabled(n, sweep, sp.debug, bp->max_contributions_per_partition);
  if (!k.on) return k;
  const int pkb = std::max(1, pdp::ceil_log2_u64((uint64_t)std::max<int64_t>(P, 1)));
  // the 2048-partition window (56 KiB of LDS: 2 reduce workgroups per CU) unless the 4096 one saves a pass
  auto npasses = [&](int sh) { return (std::max(1, pkb - sh) + 7) / 8; };
  k.sh = npasses(kK4ShMax) < npasses(kK4ShMax - 1) ? kK4ShMax : kK4ShMax - 1;
  const int kb = std::max(1, pkb - k.sh);
  k.passes = (kb + 7) / 8;
  int rem = kb, sh = 0;
  for (int i = 0; i < k.passes; ++i) {
    const int w = (rem + (k.passes - i) - 1) / (k.passes - i);
    k.shift[i] = sh;
    k.bits[i] = w;
    sh += w;
    rem -= w;
  }
  // largest |x| of one pair record: at most L_inf kept rows (one row when the bounds are already enforced)
  const double linf = bp->bounds_already_enforced ? 1.0 : (double)bp->max_contributions_per_partition;
  const double half = std::fabs(sp.b - sp.a) / 2.0;
  double mx = 0.0;
  if (sp.xmode == kXNsum) mx = linf * half;
  else if (sp.xmode == kXClipSum) mx = linf * std::max(std::fabs(sp.a), std::fabs(sp.b));
  else if (sp.xmode == kXRawSum) mx = std::max(std::fabs(sp.smin), std::fabs(sp.smax));
  k.fx = k4_exponent(mx);
  k.fy = k4_exponent(linf * half * half);
  // a pair's count is at most L_inf (1 when the bounds are already enforced): 12-byte pair records when
  // the partition id and count - 1 fit 31 bits (c4: 26 + 2) -- a quarter fewer pair-pass bytes than 16
  // the count is used only by COUNT / MEAN / VARIANCE; without it K2 does not sample rows (the slot's count
  // is the group's row count, unbounded), so the key carries no count bits
  k.cb = sp.want_count ? pdp::ceil_log2_u64((uint64_t)std::max(1.0, linf)) : 0;
  k.p12 = pkb + k.cb <= 31 && !(sp.debug & kDebugK4P16);
  // split slots (PDP_K4_SOA=1; parity-green): look-back passes only (k_pair_tile_counts reads 12-byte
  // slots).  Off: c4 pair passes 8.40 / 8.63 ms against 8.35 / 8.34 with 12-byte slots, c3 0.65 against
  // 0.62 (the values wait for their keys), for 1 % fewer pair-pass bytes (r04z7)
  k.soa = k.p12 && (sp.debug & kDebugK4Soa);
  return k;
}

K4Red k4_red(const K4Plan& k, const SegParams& sp, int64_t P, bool y) {
  K4Red r{};
  const int f = y ? k.fy : k.fx;
  r.sh = k.sh;
  r.want_count = sp.want_count;
  r.want_x = sp.xmode != kXNone;
  r.P = P;
  r.q = std::ldexp(1.0, f);
  r.inv_hi = std::ldexp(1.0, 32 - f);
  r.inv_lo = std::ldexp(1.0, -f);
  r.chunk = kK4Chunk;
  r.cb = k.p12 ? k.cb : 0;
  return r;
}

// One K4 run: pair passes over [in_a | in_b (len_b)] (ping-pong in buf1 /
// buf2), then the chunked reduction into `acc` (y = the VARIANCE run).  The
// number of records of in_a lives in device memory (counters[a_slot]: K2's
// slots; a_slot < 0: none) and upper_a bounds it, so nothing here waits for
// the host: k4_total sets the first pass's input count and the reduce chunk,
// the passes run on a persistent look-back grid and the reduction kernels
// stride over their chunks.
int k4_run(pdp_ctx* ctx, hipStream_t stream, const K4Plan& k, const K4Red& kr, bool y, const Rec* in_a, int a_slot,
           int64_t upper_a, const Rec* in_b, int64_t len_b, Rec* buf1, Rec* buf2, AccPtrs acc,
           unsigned long long* off, unsigned long long* counters, unsigned long long* status, void* ws,
           unsigned long long* s_lo, unsigned long long* s_hi, unsigned int* s_fl, int64_t buf_cap,
           int64_t soa_a = 0, int64_t soa_b = 0) {
  const int64_t upper = upper_a + len_b;
  // K2's hot-partition tables: every partition's sum from their scratch first (k4_reduce rewrites the
  // partitions it sees with the complete sums)
  if (kr.addg && kr.want_x && !y)
    hipLaunchKernelGGL(k4_convert_all, dim3(grid_for(kr.P, kThreads, 4096)), dim3(kThreads), 0, stream, kr, acc,
                       s_lo, s_hi, s_fl);
  if (upper == 0) return 0;
  // in_a's count: counters[a_slot], or exactly upper_a (a host count) when a_slot < 0
  hipLaunchKernelGGL(k4_total, dim3(1), dim3(64), 0, stream, counters, a_slot,
                     (unsigned long long)((a_slot < 0 ? upper_a : 0) + len_b));
  KeySpec ks{};
  ks.xcd_remap = 1;
  ks.mode = 6;
  ks.cap = buf_cap;  // the pairs (<= records) land in buf1 / buf2
  ks.soa_a = soa_a;
  ks.soa_b = soa_b;
  ks.low = kr.sh + (k.p12 ? k.cb : 0);  // 12-byte records: the block digit sits above the count bits
  ks.passes = k.passes;
  for (int i = 0; i < k.passes; ++i) {
    ks.shift[i] = k.shift[i];
    ks.bits[i] = k.bits[i];
  }
  const int64_t tiles = (upper + kTile - 1) / kTile;
  const unsigned grid = (unsigned)std::min<int64_t>(tiles, kPersistGrid);
  const Rec* src = in_a;
  Rec* dst = buf1;
  {
    ProfScope ps(ctx, PDP_STAGE_PAIR_PASS, stream);
    for (int p = 0; p < k.passes; ++p) {
      if (ctx->tile_slot >= kNumCounters) {
        HIP_TRY(zero_async(counters + kCtrTile0, (kNumCounters - kCtrTile0) * 8, stream));
        ctx->tile_slot = kCtrTile0;
      }
      const int n_slot = p == 0 ? (int)kCtrK4In : (int)kCtrK4Pairs;
      const Rec* src2 = p == 0 ? in_b : (const Rec*)nullptr;
      // in_a's records come first and their count is device-side: -(len_b) - 1 makes the pass split at
      // n_eff - len_b (onesweep_body); without in_b nothing is read from rin2
      const int64_t split = p == 0 && in_b ? -len_b - 1 : (int64_t)INT64_MAX;
      next_epoch_dev(ctx, stream, status, counters + kCtrK4In, 0, p == 0);
      const int occ = dev_occ(ctx->cur_debug);
      auto pass_kern = k.p12 ? (p == 0 && k.soa ? (occ == 2 ? k_pair_pass12s<2> : occ == 4 ? k_pair_pass12s<4> : k_pair_pass12s<3>)
                                                : (occ == 2 ? k_pair_pass12<2> : occ == 4 ? k_pair_pass12<4> : k_pair_pass12<3>))
                             : (occ == 2 ? k_pair_pass<2> : occ == 4 ? k_pair_pass<4> : k_pair_pass<3>);
      hipLaunchKernelGGL(pass_kern, dim3(grid), dim3(kThreads), 0, stream, (const int64_t*)nullptr,
                         (const int64_t*)nullptr, (const double*)nullptr, src, dst, (int64_t)0, counters, n_slot,
                         ks, p, off + p * kHist, status, ctx->epoch, counters, (int)ctx->tile_slot++,
                         (const unsigned int*)nullptr, (uint32_t*)nullptr, (const uint32_t*)nullptr, src2, split);
      src = dst;
      dst = (dst == buf1) ? buf2 : buf1;
    }
  }
  HIP_TRY(hipGetLastError());
  ProfScope ps(ctx, PDP_STAGE_REDUCE, stream);
  K4Red kd = kr;
  kd.chunk = 0;  // counters[kCtrK4Chunk] (k4_total)
  const unsigned cgrid = (unsigned)std::min<int64_t>((upper + 4095) / 4096, 1024);
  const bool scratch = y || kr.want_x;
  if (scratch && !kr.addg)  // (with the hot tables the scratch was zeroed for the whole call)
    hipLaunchKernelGGL(k.p12 ? k4_zero_shared<1> : k4_zero_shared<0>, dim3(cgrid), dim3(kThreads), 0, stream, src,
                       counters, kr.sh, kr.P, (int64_t)0, s_lo, s_hi, s_fl, kr.cb);
  auto pick = [&](auto k12, auto k11) { return kr.sh == kK4ShMax ? k12 : k11; };
  decltype(&k4_reduce<true, kK4ShMax, 0>) kern;
  if (k.p12)
    kern = y ? pick(k4_reduce<true, kK4ShMax, 1>, k4_reduce<true, kK4ShMax - 1, 1>)
             : pick(k4_reduce<false, kK4ShMax, 1>, k4_reduce<false, kK4ShMax - 1, 1>);
  else
    kern = y ? pick(k4_reduce<true, kK4ShMax, 0>, k4_reduce<true, kK4ShMax - 1, 0>)
             : pick(k4_reduce<false, kK4ShMax, 0>, k4_reduce<false, kK4ShMax - 1, 0>);
  hipLaunchKernelGGL(kern, dim3(cgrid), dim3(kK4Threads), 0, stream, src, counters, kd, acc, s_lo, s_hi, s_fl);
  if (scratch) {
    auto fin = y ? (k.p12 ? k4_finalize<true, 1> : k4_finalize<true, 0>)
                 : (k.p12 ? k4_finalize<false, 1> : k4_finalize<false, 0>);
    hipLaunchKernelGGL(fin, dim3(cgrid), dim3(kThreads), 0, stream, src, counters, kd, acc, s_lo, s_hi, s_fl);
  }
  HIP_TRY(hipGetLastError());
  return 0;
}

// Status block (k_latch) -> ctx->stats and the call's return code.  The generic-path request
// (ranges / full) is not an error here: the caller decides (redo the call, or PDP_ERR_NEEDS_SYNC).
int decode_status(pdp_ctx* ctx, const unsigned long long* h) {
  ctx->stats.kept_rows_in = (int64_t)h[kStatKeptRows];
  ctx->stats.filter_rows = ctx->last_filter ? (int64_t)h[kStatSurvivors] : 0;
  ctx->stats.k4_slots = ctx->last_k4 ? (int64_t)h[kStatK4Slots] : 0;
  ctx->stats.k4_pairs = ctx->last_k4 ? (int64_t)h[kStatK4Pairs] : 0;
  for (int i = 0; i < 4; ++i) ctx->stats.sweep_cycles[i] = (int64_t)h[kStatSweep0 + i];
  ctx->stats.sweep_tiles = (int64_t)h[kStatSweepTiles];
  if (h[kStatInvalid]) return fail(PDP_ERR_OUT_OF_RANGE, "privacy id or partition id out of range");
  const unsigned long long err = h[kStatErr];
  if (err & 4) return fail(PDP_ERR_INTERNAL, "K4 pair histogram disagrees with the pair records");
  if (err & 2) return fail(PDP_ERR_INTERNAL, "K4 pair records not grouped by partition block");
  if (err) return fail(PDP_ERR_INTERNAL, "radix look-back timed out");
  return 0;
}

// pdp_bound_accumulate (nconf == 1, sweep == false) and
// pdp_bound_accumulate_sweep: K0/K1 sort the rows by privacy id ONCE (the
// order does not depend on L0 / L_inf / clipping), then K2 (+ KF) runs per
// configuration over the same sorted rows.
//
// Host round trips (stream-ordered, no host sync inside).  Every
// count the kernels need lives in device memory (survivors, K2's slots, K4's
// pairs and chunk) and every grid is sized from a host upper bound, so the
// common path -- no privacy id routed to the generic path -- enqueues K0 ..
// K4 without waiting, then copies the status block back ONCE at the end
// (errors, statistics).  PDP_BOUND_ASYNC skips even that copy (the call can be
// captured in a hipGraph; pdp_get_status reports afterwards).  The generic
// path (KF: privacy ids of > 1024 rows in a wave kernel, tied priorities that
// k_segments_big does not take) needs the host: when the final status asks
// for it, the call is redone "careful" -- one sync after K2, KF, then K4 --
// and the context remembers to start careful next time (ctx->careful).
int bound_impl(pdp_ctx* ctx, const pdp_columns* cols, const pdp_bound_params* bps, int nconf,
               const pdp_accumulators* accps, void* workspace, size_t workspace_bytes, void* stream_, bool sweep,
               const pdp_partials* parts = nullptr, int force_careful = 0) {
  if (!ctx || !cols || !bps || !accps) return fail(PDP_ERR_INVALID_ARG, "null argument");
  if (parts && (sweep || nconf != 1)) return fail(PDP_ERR_INVALID_ARG, "partials: one configuration, no sweep");
  if (nconf < 1) return fail(PDP_ERR_INVALID_ARG, "num_configs must be >= 1");
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return fail(PDP_ERR_HIP, "hipSetDevice failed");
  hipStream_t stream = (hipStream_t)stream_;
  const pdp_bound_params* bp = &bps[0];
  const int64_t n = cols->num_rows, U = cols->num_privacy_ids, P = cols->num_partitions;
  if (n < 0 || P < 1 || P > (1ll << 31)) return fail(PDP_ERR_INVALID_ARG, "num_partitions must be in [1, 2^31]");
  if (!bp->bounds_already_enforced && (U < 1 || U > (1ll << 32)))
    return fail(PDP_ERR_INVALID_ARG, "num_privacy_ids must be in [1, 2^32]");
  const Plan plan = make_plan(n, std::max<int64_t>(U, 1), P);
  std::vector<SegParams> sps(nconf);
  std::vector<AccPtrs> accs(nconf);
  for (int c = 0; c < nconf; ++c) {
    const pdp_bound_params* b = &bps[c];
    const pdp_accumulators* a = &accps[c];
    if (sweep && b->bounds_already_enforced)
      return fail(PDP_ERR_INVALID_ARG, "a sweep cannot use contribution_bounds_already_enforced");
    if (b->max_partitions_contributed < 1 || b->max_contributions_per_partition < 1)
      return fail(PDP_ERR_INVALID_ARG, "contribution bounds must be positive");
    if (b->pid_base < 0 || b->pid_base != bps[0].pid_base)
      return fail(PDP_ERR_INVALID_ARG, "pid_base must be >= 0 (and the same for every configuration)");
    const bool need_value = (b->metrics & (PDP_METRIC_SUM | PDP_METRIC_MEAN | PDP_METRIC_VARIANCE)) != 0;
    if (need_value && n > 0 && !cols->value)
      return fail(PDP_ERR_INVALID_ARG, "value column required for SUM/MEAN/VARIANCE");
    if (!a->row_count) return fail(PDP_ERR_INVALID_ARG, "row_count accumulator required");
    sps[c] = make_seg(b, plan.low, plan.pkb, cols->value != nullptr);
    sps[c].debug |= ctx->debug;
    if ((sps[c].debug & kAblationFlags) && !kDebugBuild)
      return fail(PDP_ERR_INVALID_ARG, "timing-ablation debug flags need a -DPDP_DEBUG_BUILD library");
    if (sps[c].want_count && !a->count) return fail(PDP_ERR_INVALID_ARG, "count accumulator required");
    if (parts) {
      if (sps[c].xmode != kXNone && (!parts->x_hi || !parts->x_lo || !parts->nan))
        return fail(PDP_ERR_INVALID_ARG, "x_hi / x_lo / nan partials required");
      if (sps[c].want_y && (!parts->y_hi || !parts->y_lo))
        return fail(PDP_ERR_INVALID_ARG, "y_hi / y_lo partials required");
      accs[c] = AccPtrs{(unsigned long long*)a->row_count, (unsigned long long*)a->count, nullptr, nullptr};
      continue;
    }
    if (sps[c].xmode != kXNone && !a->x) return fail(PDP_ERR_INVALID_ARG, "x accumulator required");
    if (sps[c].want_y && !a->y) return fail(PDP_ERR_INVALID_ARG, "y accumulator required");
    accs[c] = AccPtrs{(unsigned long long*)a->row_count, (unsigned long long*)a->count, a->x, a->y};
  }
  if (n > 0 && !cols->pk) return fail(PDP_ERR_INVALID_ARG, "pk column required");
  if (!bp->bounds_already_enforced && n > 0 && !cols->pid) return fail(PDP_ERR_INVALID_ARG, "pid column required");
  SegParams sp = sps[0];
  AccPtrs acc = accs[0];
  const bool async = (bp->flags & PDP_BOUND_ASYNC) != 0;
  ctx->cur_debug = sp.debug;
  if (async && sweep) return fail(PDP_ERR_INVALID_ARG, "PDP_BOUND_ASYNC: one configuration, no sweep");
  if (!ctx->dstat) return fail(PDP_ERR_HIP, "context status block not allocated (hipMalloc failed)");
  const bool careful = !async && (force_careful || sweep || ctx->careful || bp->debug_force_fallback != 0);
  const int32_t waits = force_careful ? ctx->stats.host_waits : 0;  // a redone call counts both passes
  ctx->stats = pdp_stats{};
  ctx->stats.host_waits = waits;
  ctx->stats.bucket_low_bits = plan.low;
  ctx->dstat_pending = false;

  for (const AccPtrs& a : accs) {
    HIP_TRY(zero_async(a.row_count, (size_t)P * 8, stream));
    if (a.count) HIP_TRY(zero_async(a.count, (size_t)P * 8, stream));
    if (a.x) HIP_TRY(zero_async(a.x, (size_t)P * 8, stream));
    if (a.y) HIP_TRY(zero_async(a.y, (size_t)P * 8, stream));
  }
  if (parts) {
    for (int64_t* t : {parts->x_hi, parts->x_lo, parts->y_hi, parts->y_lo, parts->nan})
      if (t) HIP_TRY(zero_async(t, (size_t)P * 8, stream));
  }
  if (n == 0) {
    HIP_TRY(zero_async(ctx->dstat, kStatWords * 8, stream));
    ctx->dstat_pending = async;
    return 0;
  }

  const K4Plan k4 = k4_plan(bp, sp, n, P, sweep);
  ctx->last_k4 = k4.on;
  ctx->last_filter = false;
  if (parts && !k4.on)
    return fail(PDP_ERR_INVALID_ARG, "partials need the K4 reduction (not with debug flag NO_K4, nor with >= 2^32 "
                                     "rows and L_inf >= 131072)");
  const Layout L = layout_for(n, sweep, k4.on ? P : 0, sp.want_y != 0);
  if (!workspace || workspace_bytes < L.total) return fail(PDP_ERR_WORKSPACE, "workspace too small");
  char* ws = (char*)workspace;
  Rec* recs_a = (Rec*)(ws + L.recs_a);
  Rec* recs_b = (Rec*)(ws + L.recs_b);
  unsigned long long* hist = (unsigned long long*)(ws + L.hist);
  unsigned long long* off = (unsigned long long*)(ws + L.off);
  unsigned long long* counters = (unsigned long long*)(ws + L.counters);
  unsigned long long* status = (unsigned long long*)(ws + L.status);
  unsigned long long* ranges = (unsigned long long*)(ws + L.ranges);
  const size_t status_bytes = (size_t)L.tiles * kStatusStride * 8;
  HIP_TRY(zero_async(ws + L.hist, L.status - L.hist, stream));  // hist, off, counters
  ctx->tile_slot = kCtrTile0;
  // End of the call: the status block, then (unless PDP_BOUND_ASYNC) ONE copy to the host.
  // *redo: the generic path was needed and this pass did not run it.
  auto finish = [&](bool generic_done, bool* redo) -> int {
    hipLaunchKernelGGL(k_latch, dim3(1), dim3(64), 0, stream, counters, ctx->dstat);
    HIP_TRY(hipGetLastError());
    if (async) {
      ctx->dstat_pending = true;
      return 0;
    }
    unsigned long long h[kStatWords];
    HIP_TRY(hipMemcpyAsync(h, ctx->dstat, sizeof(h), hipMemcpyDeviceToHost, stream));
    HIP_TRY(host_wait(ctx, stream));
    if (int rc = decode_status(ctx, h)) return rc;
    const bool generic = h[kStatRanges] != 0 || h[kStatFull] != 0;
    if (redo) *redo = generic && !generic_done;
    ctx->careful = generic;
    return 0;
  };
  ctx->status_at = nullptr;  // first look-back pass of this call clears its status words (next_epoch)
  // K4 (pdp_reduce.inc): pair records into `slots` (+ the y slots), then pair passes + reduction
  unsigned int* k4rep = (unsigned int*)(ws + L.k4rep);
  unsigned long long* k4lo = (unsigned long long*)(ws + L.k4s);
  unsigned long long* k4hi = k4lo + P;
  unsigned int* k4fl = (unsigned int*)(k4hi + P);
  Rec* k4y = sp.want_y ? (Rec*)(ws + L.recs_c) : nullptr;
  // compacted pair records from K2 (round 5): only the kept groups reach K4's first pair pass
  // (c3: 40M records instead of 67.7M slots); debug flag K4_SLOT_FORM restores the slot form
  bool k4_compact = false;  // per configuration, with the K2 kernel (below)
  auto k4_attach = [&](SegParams& q, Rec* slots, bool compact) {
    if (!k4.on) return;
    q.packed = 0;
    q.k4ctr = compact ? counters + kCtrK4Slots : nullptr;
    q.k4x = slots;
    q.k4y = k4y;
    q.k4hist = k4rep;
    q.k4sh = k4.sh;
    q.k4cb = k4.p12 ? k4.cb : -1;
    q.k4soa = k4.soa ? k4_soa_offset(n) : 0;  // slot indices < n (sorted rows / survivors / rows)
    q.k4passes = k4.passes;
    for (int i = 0; i < kK4MaxPasses; ++i) {
      q.k4shift[i] = k4.shift[i];
      q.k4bits[i] = k4.bits[i];
    }
  };
  // after K2 (+ KF): x run over [slots | generic-path pairs], then the y run (VARIANCE).  The slot
  // count is counters[slot] (device; slot < 0: exactly `upper` slots), at most `upper`.
  auto k4_finish = [&](const SegParams& q, const Rec* slots, int slot, int64_t upper, const Rec* kfx, const Rec* kfy,
                       int64_t nkf, Rec* buf1, Rec* buf2) -> int {
    hipLaunchKernelGGL(k4_offsets, dim3(1), dim3(kThreads), 0, stream, k4rep, k4.passes, off, counters);
    ctx->stats.k4_passes = k4.passes;
    // records per reduce chunk: counters[kCtrK4Chunk] (k4_total: ~1024 chunks, 4096 .. 32768)
    K4Red krx = k4_red(k4, q, P, false), kry = k4_red(k4, q, P, true);
    krx.addg = q.k4hot;  // the hot tables' fixed-point scratch (x run; not with VARIANCE)
    if (parts) {  // fixed-point export (multi-GPU partials)
      krx.fxh = (long long*)parts->x_hi;
      krx.fxl = (long long*)parts->x_lo;
      krx.fxn = (unsigned long long*)parts->nan;
      krx.nan_inc = 1ull;
      kry.fxh = (long long*)parts->y_hi;
      kry.fxl = (long long*)parts->y_lo;
      kry.fxn = (unsigned long long*)parts->nan;
      kry.nan_inc = 1ull << 32;
    }
    const int64_t soa_a = q.k4soa, soa_b = k4.soa ? k4_soa_offset(nkf) : 0;
    if (int rc = k4_run(ctx, stream, k4, krx, false, slots, slot, upper, kfx, nkf, buf1, buf2, acc, off, counters,
                        status, workspace, k4lo, k4hi, k4fl, n, soa_a, soa_b))
      return rc;
    if (q.want_y) {
      if (int rc = k4_run(ctx, stream, k4, kry, true, k4y, slot, upper, kfy, nkf, buf1, buf2, acc, off, counters,
                          status, workspace, k4lo, k4hi, k4fl, n, soa_a, soa_b))
        return rc;
    }
    return 0;
  };
  if (k4.on) HIP_TRY(zero_async(k4rep, (size_t)kK4Rep * kK4MaxPasses * 256 * 4, stream));

  if (bp->bounds_already_enforced) {
    k4_attach(sp, recs_a, false);  // row i -> slot i
    {
      ProfScope ps(ctx, PDP_STAGE_ENFORCED, stream);
      hipLaunchKernelGGL(k_enforced, dim3(grid_for(n, kThreads, 8192)), dim3(kThreads), 0, stream, cols->pk,
                       cols->value, n, P, sp, acc, counters);
    }
    HIP_TRY(hipGetLastError());
    if (k4.on) {
      if (int rc = k4_finish(sp, recs_a, -1, n, nullptr, nullptr, 0, recs_b, recs_a)) return rc;
    }
    if (int rc = finish(true, nullptr)) {
      if (rc == PDP_ERR_OUT_OF_RANGE) return fail(rc, "partition id >= num_partitions in input");
      return rc;
    }
    return 0;
  }

  sp.packed = !k4.on && sp.want_count && n < (1ll << 32);
  KeySpec ks{};
  ks.xcd_remap = 1;
  ks.mode = 0;
  ks.low = plan.low;
  ks.pkb = plan.pkb;
  ks.seed = bp->sampling_seed;
  ks.pid_base = (uint64_t)bp->pid_base;
  ks.num_pids = (uint64_t)U;
  ks.num_parts = (uint32_t)P;
  ks.passes = plan.passes;
  {
    int sh = 0;
    for (int i = 0; i < plan.passes; ++i) {
      ks.shift[i] = sh;
      ks.bits[i] = plan.bits[i];
      sh += plan.bits[i];
    }
  }
  ks.prof = (sp.debug & kDebugSweepStamps) != 0;
  ks.ablate = (sp.debug & kDebugSortOnly) ? (sp.debug & (kDebugNoLookback | kDebugLinearWrite | kDebugNoScatter)) : 0;
  const bool rts = use_tile_scan(n, sp.debug);
  const TileScan ts = rts ? tile_scan_bufs(ctx, status, L.tiles) : TileScan{};
  // L0 pre-filter (pdp_filter.inc): one pass on the bucket digit instead of the full pid sort
  const FilterPlan fpl = filter_plan(n, U, bp, sp.debug, sweep, rts);
  uint32_t* tags = (uint32_t*)(ws + L.tags);
  uint32_t* tag_lo = (uint32_t*)(ws + L.tag_lo);
  const bool rec16 = (bp->reserved2 & kDebug2FilterRec8) == 0;  // 16-byte bucket records (default)
  ctx->last_filter = fpl.on;
  if (fpl.on) {
    ks.mode = 4;
    ks.mult = fpl.mult;
    // Rows likely to survive (sketch level <= tau) first within each tile's bucket run: the survivors then
    // sit densely in the record array and k_filter's gather reads far fewer lines (c3: ~10 % of the rows
    // are class 0 and hold most survivors).  tau ~ the level of the 3 L0 / (rows per pid) quantile of the
    // priorities; a poor tau costs only speed (a (pid, pk) group has one level, so its rows keep their
    // input order whatever tau is).
    {
      const double slack = (double)env_int("PDP_TAU_SLACK10", 30) / 10.0;  // experiment builds only
      const double q = slack * (double)bp->max_partitions_contributed * (double)U / (double)std::max<int64_t>(n, 1);
      int tau = q >= 1.0 ? 31 : (int)std::floor(31.0 + 4.0 * std::log2(q));
      tau = std::min(31, std::max(0, tau));
      ks.tau = (bp->reserved2 & kDebug2NoClassSplit) ? 31 : tau;
      ks.flip = env_int("PDP_CLASS_FLIP", 1) ? 1 : 0;  // experiment builds only (the shipped library: 1)
    }
    ks.passes = 1;
    ks.shift[0] = 64;
    ks.bits[0] = 8;
    hipLaunchKernelGGL(k_bucket_lo, dim3(1), dim3(256), 0, stream, fpl.mult, tag_lo);
  }
  ctx->stats.sort_passes = ks.passes;
  {
    ProfScope ps(ctx, PDP_STAGE_HISTOGRAM, stream);
    if (rts)
      hipLaunchKernelGGL(fpl.on ? k_histogram_tiles<true> : k_histogram_tiles<false>, dim3(grid_for(L.tiles, 1, 4096)),
                         dim3(kThreads), 0, stream, cols->pid, cols->pk, n, ks, hist, ts.tile_cnt, counters);
    else
      hipLaunchKernelGGL(k_histogram<1>, dim3(grid_for(n, kThreads, 2048)), dim3(kThreads), 0, stream,
                         cols->pid, cols->pk, (const Rec*)nullptr, n, ks, hist, counters,
                         (const unsigned long long*)nullptr);
  }
  hipLaunchKernelGGL(k_offsets, dim3(1), dim3(kThreads), 0, stream, hist, off, ks.passes, n, counters,
                     (int)kCtrNKept, (const unsigned long long*)nullptr);
  Rec* src = nullptr;
  Rec* dst = recs_a;
  // Passes >= 1 reduce-then-scan too (round 4): at c4 the two later passes took 2 x 5.03 ms by
  // decoupled look-back against 2 x 3.22 ms + 1.06 ms per pass of tile counts with the XCD-contiguous
  // tile runs (step 38.31 -> 37.81 ms, same box r04h; round 3, before the loads-ahead passes, had
  // measured the reverse).  PDP_PASS_TILESCAN=0: look-back.
  const bool rest_tile_scan = true;
  for (int p = 0; p < ks.passes; ++p) {
    const unsigned int* bases = nullptr;
    if (rts && (p == 0 || rest_tile_scan)) {
      ProfScope ps(ctx, PDP_STAGE_TILE_COUNTS, stream);
      if (p > 0)
        hipLaunchKernelGGL(k_tile_counts, dim3(grid_for(L.tiles, 1, 4096)), dim3(kThreads), 0, stream, src, counters,
                           (int)kCtrNKept, ks, p, L.tiles, ts.tile_cnt);
      tile_scan(ts, off + p * kHist, stream);
      bases = ts.tile_cnt;
    } else {
      int rc = next_epoch(ctx, stream, status, status_bytes);
      if (rc) return rc;
    }
    ProfScope ps(ctx, p == 0 ? PDP_STAGE_ONESWEEP_FIRST : PDP_STAGE_ONESWEEP_REST, stream);
    if (p == 0 && fpl.on)
      hipLaunchKernelGGL(rec16 ? k_bucket_pass : k_bucket_pass8, dim3((unsigned)L.tiles), dim3(kThreads), 0, stream, cols->pid,
                         cols->pk, cols->value, (const Rec*)nullptr, dst, n, counters, (int)kCtrNKept, ks, p,
                         off + p * kHist, status, ctx->epoch, counters, (int)ctx->tile_slot++, bases, tags, tag_lo,
                         (const Rec*)nullptr, (int64_t)INT64_MAX);
    else if (p == 0)
      hipLaunchKernelGGL(k_sort_first, dim3((unsigned)L.tiles), dim3(kThreads), 0, stream, cols->pid,
                         cols->pk, cols->value, (const Rec*)nullptr, dst, n, counters, (int)kCtrNKept, ks, p,
                         off + p * kHist, status, ctx->epoch, counters, (int)ctx->tile_slot++, bases,
                         (uint32_t*)nullptr, (const uint32_t*)nullptr, (const Rec*)nullptr, (int64_t)INT64_MAX);
    else
      hipLaunchKernelGGL(k_onesweep, dim3((unsigned)L.tiles), dim3(kThreads), 0, stream,
                         (const int64_t*)nullptr, (const int64_t*)nullptr, (const double*)nullptr, src, dst, n,
                         counters, (int)kCtrNKept, ks, p, off + p * kHist, status, ctx->epoch, counters,
                         (int)ctx->tile_slot++, bases, (uint32_t*)nullptr, (const uint32_t*)nullptr,
                         (const Rec*)nullptr, (int64_t)INT64_MAX);
    src = dst;
    dst = (dst == recs_a) ? recs_b : recs_a;
  }
  HIP_TRY(hipGetLastError());
  Rec* sorted = src;
  Rec* spare = dst;
  if (sp.debug & kDebugSortOnly) {
    HIP_TRY(host_wait(ctx, stream));
    return 0;
  }
  int n_slot = kCtrNKept;  // counter holding the number of rows in `sorted`
  uint64_t n_sorted = (uint64_t)n;  // upper bound of that number (grid sizes)
  if (fpl.on) {
    // The survivors' grouping key: the low low_bits bits of the pid.  9..16 bits: a look-back pass on
    // the low (low_bits - 8) bits, then the LDS grouping by the remaining 8 (pdp_group.inc) -- the first
    // pass takes the narrower digit so that the (bucket, digit) sub-runs stay ~1K rows when the buckets
    // are narrow (a rank's share of c3 at 8 GPUs: 13 bits -> 5 + 8, 8192 sub-runs instead of 65536).
    // The first pass widens (up to 8 bits) while the expected survivors (~1.7 rows per kept
    // (pid, partition) pair, U x L0 pairs: measured 1.66-1.7 at c2/c3) would make the average sub-run
    // longer than ~1050 rows, near k_group's 1152-row register/LDS stage (c2: 12 bits -> 6 + 6, not 4 + 8).
    // Otherwise 8-bit look-back passes.
    KeySpec k2 = ks;
    k2.passes = 0;
    // (the sub-run table holds 32-bit starts: inputs of 2^32 rows or more -- as many possible survivors --
    // take the look-back passes)
    const bool group = fpl.low_bits >= 9 && fpl.low_bits <= 16 && n < (1ll << 32) && !(bp->reserved2 & kDebug2NoGroup);
    if (group) {
      const double est = std::min((double)n, 1.7 * (double)U * (double)bp->max_partitions_contributed);
      int b1 = fpl.low_bits - 8;
      while (b1 < 8 && est > 1050.0 * 256.0 * (double)(1 << b1)) ++b1;
      k2.shift[0] = 0;
      k2.bits[0] = b1;
      k2.shift[1] = b1;
      k2.bits[1] = fpl.low_bits - b1;
      k2.passes = 2;
    } else {
      for (int sh = 0; sh < fpl.low_bits; sh += 8) {
        k2.shift[k2.passes] = sh;
        k2.bits[k2.passes] = std::min(8, fpl.low_bits - sh);
        ++k2.passes;
      }
    }
    const int nd0 = 1 << k2.bits[0];  // the filter's digits d0 (sub-runs: nd0 x 256 buckets)
    // K1f: survivors of the bucket-sorted rows -> spare, each bucket's run ordered by d0 = the first
    // grouping step (input order per pid kept)
    HIP_TRY(zero_async(counters + kCtrNSurv, 8, stream));
    uint2* subruns = (uint2*)(ws + L.grp);
    unsigned long long* grp_ctl = (unsigned long long*)(subruns + kGrpSubruns);
    HIP_TRY(zero_async(grp_ctl, 24, stream));
    {
      ProfScope ps(ctx, PDP_STAGE_FILTER, stream);
      hipLaunchKernelGGL(fpl.half ? (rec16 ? k_filter<true, false> : k_filter<true, true>)
                                  : (rec16 ? k_filter<false, false> : k_filter<false, true>),
                         dim3(256), dim3(kFiltThreads), 0, stream, sorted, cols->value, tags, tag_lo, spare,
                         (uint8_t*)(ws + L.keep), off, counters,
                         (int)kCtrNKept, (int)kCtrNSurv, (int)bp->max_partitions_contributed,
                         (sp.debug & kDebugFilterTiming) != 0, group ? subruns : (uint2*)nullptr, grp_ctl,
                         (bp->reserved2 & kDebug2GroupFallback) ? 1u : kGrpBig, (uint32_t)U, (uint32_t)(nd0 - 1));
    }
    HIP_TRY(hipGetLastError());
    // Survivors stably by pid & (2^low_bits - 1) only.  That groups every pid: within a bucket the
    // ids are distinct mod 2^low_bits (a bucket spans <= 2^low_bits ids), and rows of equal low bits
    // from different buckets stay in the order of their buckets' runs, because k_filter writes each
    // bucket's survivors as ONE contiguous run.  (No bucket-digit pass: the order of the pids does
    // not matter to K2, only their grouping.)  The filter did the first step (d0); the rest is k_group
    // (9..16 low bits) or look-back passes on the remaining bytes.
    ctx->stats.sort_passes += k2.passes;
    Rec* sa = spare;
    Rec* sb = sorted;
    Rec* out = sa;
    // K2's row count (the survivors), and the fallback pass's (the survivors if a sub-run was too long)
    hipLaunchKernelGGL(k_grp_count, dim3(1), dim3(64), 0, stream, counters, grp_ctl);
    if (group) {
      ProfScope ps(ctx, PDP_STAGE_SURVIVOR_GROUP, stream);
      Rec* dst = sb;
      hipLaunchKernelGGL(k_group, dim3(4096), dim3(64 * kGrpBlockWaves), 0, stream, (const Rec*)out, dst,
                         (const uint2*)subruns, nd0 * 256, k2.shift[1], k2.bits[1],
                         (const unsigned long long*)grp_ctl);
      // the look-back pass over grp_ctl[1] rows: 0 unless a sub-run was too long for k_group (then its
      // digit histogram and offsets first; the row count k_offsets derives goes to grp_ctl[2], not to K2's
      // counter)
      HIP_TRY(zero_async(hist, kMaxPasses * kHist * 8, stream));
      hipLaunchKernelGGL(k_histogram<0>, dim3(grid_for(n, kThreads, 2048)), dim3(kThreads), 0, stream,
                         (const int64_t*)nullptr, (const int64_t*)nullptr, (const Rec*)out, n, k2, hist, counters,
                         (const unsigned long long*)(grp_ctl + 1));
      hipLaunchKernelGGL(k_offsets, dim3(1), dim3(kThreads), 0, stream, hist, off, k2.passes, n, grp_ctl, 2,
                         (const unsigned long long*)(grp_ctl + 1));
      next_epoch_dev(ctx, stream, status, grp_ctl + 1, 0, true);
      const int occ = dev_occ(ctx->cur_debug);
      auto dev_kern = occ == 2 ? k_onesweep_dev<2> : occ == 4 ? k_onesweep_dev<4> : k_onesweep_dev<3>;
      const int64_t tiles = (n + kTile - 1) / kTile;
      hipLaunchKernelGGL(dev_kern, dim3((unsigned)std::min<int64_t>(tiles, kPersistGrid)), dim3(kThreads), 0, stream,
                         (const int64_t*)nullptr, (const int64_t*)nullptr, (const double*)nullptr, (const Rec*)out,
                         dst, n, (const unsigned long long*)grp_ctl, 1, k2, 1, off + kHist, status, ctx->epoch,
                         counters, (int)ctx->tile_slot++, (const unsigned int*)nullptr, (uint32_t*)nullptr,
                         (const uint32_t*)nullptr, (const Rec*)nullptr, (int64_t)INT64_MAX);
      HIP_TRY(hipGetLastError());
      out = dst;
    } else if (k2.passes > 1) {  // look-back passes on the bytes above d0
      KeySpec k3 = k2;
      k3.passes = k2.passes - 1;
      for (int p = 0; p < k3.passes; ++p) {
        k3.shift[p] = k2.shift[p + 1];
        k3.bits[p] = k2.bits[p + 1];
      }
      int rc = sort_recs(ctx, sa, sb, n, k3, hist, off, counters, status, status_bytes, workspace, stream, &out,
                         PDP_STAGE_SURVIVOR_SORT, nullptr, nullptr, nullptr, counters + kCtrNSurv, -1, false);
      if (rc) return rc;
    }
    sorted = out;
    spare = (out == sa) ? sb : sa;
    n_slot = kCtrNGeneric;
  }

  OvList ov{ranges, counters, (bp->reserved2 & kDebug2OverflowFull1) ? 1ull : 0ull};
  BigList big{(unsigned long long*)(ws + L.big), L.big_cap};
  const int64_t seg_grid = (n + kSegTile - 1) / kSegTile;
  Rec* alt = sweep ? (Rec*)(ws + L.recs_c) : sorted;
  unsigned long long n_kept = 0;
  for (int c = 0; c < nconf; ++c) {
  bp = &bps[c];
  sp = sps[c];
  acc = accs[c];
  sp.packed = !k4.on && sp.want_count && n < (1ll << 32);
  const bool thin = fpl.on && bp->max_partitions_contributed <= kThinMaxL0 &&
                    bp->max_contributions_per_partition <= kThinMaxLinf &&
                    !(sp.debug & (kDebugBatchKernel | kDebugNoThin));
  // debug flag THIN2: the LDS-staged k_thin2 (round 5 experiment, slower: DESIGN.md 3.2)
  const bool thin2 = thin && k4.on && (sp.debug & kDebugThin2);
  // debug flag K4_COMPACT: K2 claims compacted pair slots (k4_claim) instead of writing a slot per row
  // with empties.  Measured slower: the claims are atomics on ONE counter, which serialise (r05f: c3
  // k_thin2 +1.3 ms for a 0.26 ms shorter first pair pass; c4 k_lean 8.56 -> 150 ms).
  k4_compact = k4.on && (sp.debug & kDebugK4Compact);
  k4_attach(sp, spare, k4_compact);
  const bool lean = !thin && bp->max_partitions_contributed <= kLeanMaxL0 && !(sp.debug & kDebugBatchKernel);
  // K4 hot-partition tables (pdp_reduce.inc, K4Hot) in k_thin / k_lean: not with VARIANCE (one
  // fixed-point scratch), the sweep or the debug forms; debug flag NO_HOT_CACHE turns them off
  // k_lean only: in k_thin (L0 <= 8: few pairs per privacy id) the tables cost the kernel about what they
  // save K4 (r05j c3: K2 +0.20 ms, K4 -0.15 ms); at c4 (L0 = 32) they pay (K2 +1.1, K4 -2.2 ms)
  const bool k4hot = k4.on && !sweep && !k4_compact && !thin2 && !sp.want_y &&
                     (lean || (thin && env_int("PDP_K4_HOT_THIN", 0))) && !(sp.debug & kDebugNoHotCache);
  sp.k4hot = k4hot ? 1 : 0;
  if (k4hot) {
    sp.k4q = std::ldexp(1.0, k4.fx);
    sp.k4glo = k4lo;
    sp.k4ghi = k4hi;
    sp.k4gfl = k4fl;
    HIP_TRY(zero_async(k4lo, (size_t)P * 16, stream));  // lo, hi
    HIP_TRY(zero_async(k4fl, ((size_t)P * 4 + 7) / 8 * 8, stream));
  }
  if (c > 0) {
    // fresh K2/KF counters; the kept-row count of the shared sort stays
    unsigned long long reset[kCtrSweepCycles] = {};
    reset[kCtrNKept] = n_kept;
    HIP_TRY(hipMemcpyAsync(counters, reset, sizeof(reset), hipMemcpyHostToDevice, stream));
    HIP_TRY(host_wait(ctx, stream));
  }
  {
    ProfScope ps(ctx, PDP_STAGE_BUCKETS, stream);
    if (thin) {
      const bool v2 = thin2;
      // 2048-row chunks when many survivors are expected (c3: K2 1.88 -> 1.73 ms), 1024 for a rank's share
      // (8-way: 0.35 vs 0.38 ms); the estimate is the survivor grouping's (1.7 rows per kept pair)
      const double est_surv = std::min((double)n, 1.7 * (double)U * (double)bp->max_partitions_contributed);
      const int64_t chunk = v2 ? kThin2Chunk : (est_surv >= 3e7 || (bp->reserved2 & kDebug2ThinChunk2048)
                                                          ? kThinChunkMax : kThinChunk);
      const int64_t waves = ((int64_t)n_sorted + chunk - 1) / chunk;
      // LDS partition cache on: the Zipf-head pairs' HBM atomics otherwise dominate (c3: K2 8.1 -> 3.4 ms);
      // K4 writes pair records instead of atomics, no cache
      const bool tcache = !k4.on;
      const int64_t blocks =
          std::max<int64_t>(1, std::min<int64_t>((waves + 3) / 4, (sp.debug & kDebugOddGrid) ? 7 : kThinMaxBlocks));
      const int64_t l0 = bp->max_partitions_contributed;
      auto kern2 = l0 <= 1 ? k_thin2<1> : l0 <= 2 ? k_thin2<2> : l0 <= 4 ? k_thin2<4> : k_thin2<8>;
      auto kern = k4hot ? (l0 <= 1 ? k_thin<false, 1, false, true> : l0 <= 2 ? k_thin<false, 2, false, true>
                           : l0 <= 4 ? k_thin<false, 4, false, true> : k_thin<false, 8, false, true>)
                : k4_compact ? (l0 <= 1 ? k_thin<false, 1, true> : l0 <= 2 ? k_thin<false, 2, true>
                                : l0 <= 4 ? k_thin<false, 4, true> : k_thin<false, 8, true>)
                : l0 <= 1 ? (tcache ? k_thin<true, 1> : k_thin<false, 1>)
                : l0 <= 2 ? (tcache ? k_thin<true, 2> : k_thin<false, 2>)
                : l0 <= 4 ? (tcache ? k_thin<true, 4> : k_thin<false, 4>)
                          : (tcache ? k_thin<true, 8> : k_thin<false, 8>);
      if (v2)
        hipLaunchKernelGGL(kern2, dim3((unsigned)blocks), dim3(256), 0, stream, sorted, counters, n_slot, sp, acc, ov,
                           big, (int)bp->debug_force_fallback);
      else
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, stream, sorted, counters, n_slot, sp, acc, ov,
                           big, (int)bp->debug_force_fallback, (int)chunk);
    } else if (lean) {
      const int64_t waves = ((int64_t)n_sorted + kLeanChunk - 1) / kLeanChunk;
      int64_t max_blocks = kLeanMaxBlocks;
      if (sp.debug & kDebugOddGrid) max_blocks = 5;
      const int64_t blocks = std::max<int64_t>(1, (waves + 3) / 4 < max_blocks ? (waves + 3) / 4 : max_blocks);
      const bool sorted_l0 = bp->max_partitions_contributed >= kSortMinL0 && !(sp.debug & kDebugLeanMinSearch);
      // the LDS partition cache pays when many privacy ids keep the same hot partitions, which grows with
      // L0: c4 (L0 = 32) K2 137 -> 50 ms (round 1); at c3 (L0 = 4) / c2 (L0 = 8) it does not pay
      const bool cache = !k4.on &&
                         (bp->max_partitions_contributed >= kHotMinL0 || (sp.debug & kDebugForceHotCache) ||
                          false) &&
                         !(sp.debug & kDebugNoHotCache);
      const bool two = bp->max_partitions_contributed > 64;
      auto kern = k4hot ? (sorted_l0 ? (two ? k_lean<2, true, false, true> : k_lean<1, true, false, true>)
                                     : (two ? k_lean<2, false, false, true> : k_lean<1, false, false, true>))
                : sorted_l0 ? (two ? (cache ? k_lean<2, true, true> : k_lean<2, true, false>)
                                   : (cache ? k_lean<1, true, true> : k_lean<1, true, false>))
                            : (two ? (cache ? k_lean<2, false, true> : k_lean<2, false, false>)
                                   : (cache ? k_lean<1, false, true> : k_lean<1, false, false>));
      hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, stream, sorted, counters, n_slot, sp, acc,
                         ov, big, (int)bp->debug_force_fallback);
    } else {
      hipLaunchKernelGGL(k_segments, dim3((unsigned)seg_grid), dim3(kThreads), 0, stream, sorted, counters, n_slot,
                         sp, acc, ov, big, (int)bp->debug_force_fallback);
    }
    // tied segments of <= kBigMax rows: from the overflow ranges to k_segments_big (not under
    // debug_force_fallback, which tests the generic path itself)
    if (!bp->debug_force_fallback)
      hipLaunchKernelGGL(k_ranges_to_big, dim3(1), dim3(256), 0, stream, counters, ranges, big);
    hipLaunchKernelGGL(k_segments_big, dim3(1024), dim3(64 * kBigWaves), 0, stream, sorted, counters, sp, acc, big);
  }
  HIP_TRY(hipGetLastError());

  if (!careful) {
    // optimistic: K4 straight after K2 (a segment handed to the generic path leaves empty slots); the
    // final status says whether the generic path was needed
    if (k4.on) {
      if (!k4_compact) hipLaunchKernelGGL(k4_fill_ranges, dim3(64), dim3(kThreads), 0, stream, sp, ranges, counters);
      if (int rc = k4_finish(sp, spare, k4_compact ? (int)kCtrK4Slots : n_slot, (int64_t)n_sorted, nullptr, nullptr, 0,
                             sorted, spare))
        return rc;
    } else if (sp.packed) {
      hipLaunchKernelGGL(k_unpack_counts, dim3(grid_for(P, kThreads, 4096)), dim3(kThreads), 0, stream,
                         acc.row_count, acc.count, P);
    }
    HIP_TRY(hipGetLastError());
    bool redo = false;
    if (int rc = finish(false, &redo)) return rc;
    if (redo)  // the generic path was needed: the same call, careful (its accumulators are zeroed again)
      return bound_impl(ctx, cols, bps, nconf, accps, workspace, workspace_bytes, stream_, sweep, parts, 1);
    return 0;
  }

  unsigned long long host_ctr[kCtrNDropped + 1];
  HIP_TRY(hipMemcpyAsync(host_ctr, counters, sizeof(host_ctr), hipMemcpyDeviceToHost, stream));
  HIP_TRY(host_wait(ctx, stream));
  ctx->stats.kept_rows_in = (int64_t)(host_ctr[kCtrNKept] - host_ctr[kCtrNDropped]);
  n_kept = host_ctr[n_slot];
  for (int i = 0; i < 4; ++i) ctx->stats.sweep_cycles[i] = (int64_t)host_ctr[kCtrSweepCycles + i];
  ctx->stats.sweep_tiles = (int64_t)host_ctr[kCtrSweepTiles];
  if (host_ctr[kCtrErr]) return fail(PDP_ERR_INTERNAL, "radix look-back timed out");
  if (host_ctr[kCtrInvalid]) return fail(PDP_ERR_OUT_OF_RANGE, "privacy id or partition id out of range");
  std::vector<unsigned long long> rg;
  int64_t k4_slots = (int64_t)host_ctr[n_slot];  // K2's slots (K4)
  if (host_ctr[kCtrFull]) {
    // Too many overflowing buckets: redo everything on the generic path.
    if (k4.on) {
      HIP_TRY(zero_async(k4rep, (size_t)kK4Rep * kK4MaxPasses * 256 * 4, stream));  // drop K2's records
      k4_slots = 0;
      if (sp.k4hot) {
        // K2's hot-partition tables already flushed their kept groups: counts into the accumulators, sums
        // into K4's fixed-point scratch (which k4_finish re-emits through krx.addg).  The generic path
        // redoes every row, so drop them too, or those groups count twice (round-5 advisor finding).
        HIP_TRY(zero_async(acc.row_count, (size_t)P * 8, stream));
        if (acc.count) HIP_TRY(zero_async(acc.count, (size_t)P * 8, stream));
        HIP_TRY(zero_async(k4lo, (size_t)P * 16, stream));  // lo, hi
        HIP_TRY(zero_async(k4fl, ((size_t)P * 4 + 7) / 8 * 8, stream));
      }
    } else {
      HIP_TRY(zero_async(acc.row_count, (size_t)P * 8, stream));
      if (acc.count) HIP_TRY(zero_async(acc.count, (size_t)P * 8, stream));
      if (acc.x) HIP_TRY(zero_async(acc.x, (size_t)P * 8, stream));
      if (acc.y) HIP_TRY(zero_async(acc.y, (size_t)P * 8, stream));
    }
    rg = {0ull, host_ctr[n_slot]};
  } else if (host_ctr[kCtrNRanges]) {
    rg.resize(2 * host_ctr[kCtrNRanges]);
    HIP_TRY(hipMemcpyAsync(rg.data(), ranges, rg.size() * 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(host_wait(ctx, stream));
    if (k4.on && !k4_compact) {  // the generic path's pairs come in their own array: empty these slots
      const int nr = (int)host_ctr[kCtrNRanges];
      hipLaunchKernelGGL(k4_fill_ranges, dim3((unsigned)std::min(nr, 4096)), dim3(kThreads), 0, stream, sp, ranges,
                         counters);
    }
  }
  AsyncFrees k4keep(stream);  // the generic path's pair arrays (until the K4 runs are enqueued)
  Rec *kfx = nullptr, *kfy = nullptr;
  int64_t nkf = 0;
  if (!rg.empty()) {
    SegParams gsp = sp;
    if (k4.on) gsp.k4hist = k4rep;  // replica 0: global atomics from the generic path
    gsp.k4ctr = nullptr;            // KF writes one slot per group of its own array
    int rc = run_generic(ctx, sorted, spare, alt, rg, plan, gsp, bp, ks.num_pids, ks.num_parts, acc, hist, off,
                         counters, status, status_bytes, workspace, stream, &k4keep, &kfx, &kfy, &nkf);
    if (rc) return rc;
    unsigned long long err = 0;
    HIP_TRY(hipMemcpyAsync(&err, counters + kCtrErr, 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(host_wait(ctx, stream));
    if (err) return fail(PDP_ERR_INTERNAL, "radix look-back timed out (generic path)");
  }
  if (k4.on) {
    // K2's slots (none when everything went to the generic path: kCtrFull) + the generic path's pairs
    if (int rc = k4_finish(sp, spare, host_ctr[kCtrFull] ? -1 : k4_compact ? (int)kCtrK4Slots : n_slot, k4_slots, kfx,
                           kfy, nkf, sorted, spare))
      return rc;
  } else if (sp.packed) {
    hipLaunchKernelGGL(k_unpack_counts, dim3(grid_for(P, kThreads, 4096)), dim3(kThreads), 0, stream, acc.row_count,
                       acc.count, P);
    HIP_TRY(hipGetLastError());
  }
  }  // configurations
  if (int rc = finish(true, nullptr)) return rc;
  return 0;
}

// ---------------------------------------------------------------------------
// Utility analysis host side (pdp_analysis.inc)
// ---------------------------------------------------------------------------

// Keep probability table of a selection strategy for k = L0 partitions:
// keep[i] for i < len, 1 beyond (PyDP probability_of_keep restated, the
// functions of the utility analysis' PartitionSelectionCalculator,
// analysis/combiners.py:124-141).
int keep_table(int selection, double eps, double delta, int64_t k, std::vector<double>& t) {
  t.clear();
  if (selection == PDP_SELECTION_NONE) return 0;
  if (selection == PDP_SELECTION_TRUNCATED_GEOMETRIC) {
    int64_t len = 0;
    if (int rc = pdp_truncated_geometric_table(eps, delta, k, nullptr, 0, &len)) return rc;
    t.assign((size_t)len, 0.0);
    return pdp_truncated_geometric_table(eps, delta, k, t.data(), len, &len);
  }
  double thr = 0, scale = 0;
  if (int rc = pdp_selection_threshold(selection, eps, delta, k, &thr, &scale)) return rc;
  t.push_back(0.0);  // n = 0 is never kept
  for (int64_t i = 1;; ++i) {
    const double x = thr - (double)i;
    double p;
    if (selection == PDP_SELECTION_LAPLACE_THRESHOLDING)
      p = x >= 0 ? 0.5 * std::exp(-std::fabs(x) / scale) : 1.0 - 0.5 * std::exp(-std::fabs(x) / scale);
    else
      p = 0.5 * std::erfc(x / (scale * std::sqrt(2.0)));
    if (p >= 1.0) break;
    t.push_back(p);
    if (t.size() > (1u << 24)) return fail(PDP_ERR_INVALID_ARG, "selection keep table too long (eps too small)");
  }
  return 0;
}

// keep_table memoised per (selection, eps, delta, k): a configuration sweep
// repeats each L0 for every L_inf, and the truncated-geometric tables cost
// milliseconds of host time per call (bounded process-wide cache).
int keep_table_cached(int selection, double eps, double delta, int64_t k, std::vector<double>& t) {
  using Key = std::tuple<int, double, double, int64_t>;
  static std::mutex mu;
  static std::map<Key, std::vector<double>> cache;
  const Key key{selection, eps, delta, k};
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it == cache.end()) {
    std::vector<double> v;
    if (int rc = keep_table(selection, eps, delta, k, v)) return rc;
    if (cache.size() >= 1024) cache.clear();
    it = cache.emplace(key, std::move(v)).first;
  }
  t = it->second;
  return 0;
}

struct AnaLayout {
  size_t recs_a, recs_b, flags, ppk, pref, pcnt, psum, npart, pbeg, mom, cfg, keep, hist, off, counters, status, slots,
      slots2, total;
  AnaGroups groups{};  // distinct L0 values (G = 0: more than kAnaMaxGroups)
  int64_t tiles;
  std::vector<AnaCfg> cfgs;  // keep pointers are offsets until bound to the workspace
  std::vector<double> keep_all;
};

int ana_layout(int64_t n, int64_t U, int64_t P, const pdp_analysis_config* cfgs, int nconf, AnaLayout& L) {
  size_t o = 0;
  const size_t n1 = (size_t)std::max<int64_t>(n, 1);
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += align_up(std::max<size_t>(bytes, 8), 256);
    return at;
  };
  L.recs_a = take(n1 * sizeof(Rec));
  L.recs_b = take(n1 * sizeof(Rec));
  L.flags = take(n1 * 8);
  L.ppk = take(n1 * 4);
  L.pref = take(n1 * 4);
  L.pcnt = take(n1 * 4);
  L.psum = take(n1 * 8);
  L.npart = take((size_t)std::max<int64_t>(U, 1) * 4);
  L.pbeg = take((size_t)(P + 1) * 8);
  const bool priv = nconf > 0 && cfgs[0].selection != PDP_SELECTION_NONE;
  L.mom = take(priv ? (size_t)nconf * 4 * P * 8 : 8);
  L.cfg = take((size_t)nconf * sizeof(AnaCfg));
  L.cfgs.assign((size_t)nconf, AnaCfg{});
  L.keep_all.clear();
  std::map<std::tuple<int, double, double, int64_t>, size_t> shared;  // identical tables share one copy
  std::vector<double> t;
  for (int c = 0; c < nconf; ++c) {
    const pdp_analysis_config& a = cfgs[c];
    if ((a.selection != PDP_SELECTION_NONE) != priv)
      return fail(PDP_ERR_INVALID_ARG, "all configurations must use private selection, or none (public partitions)");
    if (a.max_partitions_contributed < 1 || a.max_contributions_per_partition < 1)
      return fail(PDP_ERR_INVALID_ARG, "contribution bounds must be positive");
    const auto key = std::make_tuple(a.selection, a.selection_eps, a.selection_delta, a.max_partitions_contributed);
    auto sh = shared.find(key);
    if (int rc = keep_table_cached(a.selection, a.selection_eps, a.selection_delta, a.max_partitions_contributed, t))
      return rc;
    if (sh == shared.end()) {
      sh = shared.emplace(key, L.keep_all.size()).first;
      L.keep_all.insert(L.keep_all.end(), t.begin(), t.end());
    }
    AnaCfg& g = L.cfgs[c];
    g.l0 = (double)a.max_partitions_contributed;
    g.linf = (double)a.max_contributions_per_partition;
    g.smin = a.min_sum_per_partition;
    g.smax = a.max_sum_per_partition;
    g.keep = (const double*)(uintptr_t)sh->second;  // offset, bound later
    g.keep_len = (int64_t)t.size();
    g.grp = -1;
    for (int j = 0; j < L.groups.G; ++j)
      if (L.groups.l0[j] == g.l0) g.grp = j;
    if (g.grp < 0 && L.groups.G >= 0) {
      if (L.groups.G < kAnaMaxGroups) {
        g.grp = L.groups.G;
        L.groups.rep[L.groups.G] = c;
        L.groups.kmax[L.groups.G] = 0;
        L.groups.l0[L.groups.G++] = g.l0;
      } else {
        L.groups.G = -1;  // too many distinct L0 values: k_ana_select<true / false>
      }
    }
    if (g.grp >= 0 && L.groups.G > 0) L.groups.kmax[g.grp] = std::max(L.groups.kmax[g.grp], g.keep_len);
  }
  L.keep = take(L.keep_all.size() * 8);
  L.hist = take(kMaxPasses * kHist * 8);
  L.off = take(kMaxPasses * kHist * 8);
  L.counters = take(kNumCounters * 8);
  L.tiles = (int64_t)(n1 + kTile - 1) / kTile;
  L.status = take((size_t)L.tiles * kStatusStride * 8);
  // k_ana_metrics' chunk-boundary partials: [chunk][head, tail][kAnaSlotFields][configurations / 64 * 64]
  const size_t chunk = (size_t)kAnaChunk * (size_t)((nconf + 63) / 64);
  const size_t nchunks = (n1 + chunk - 1) / chunk;
  L.slots = take(nchunks * 2 * kAnaSlotFields * (size_t)((nconf + 63) / 64 * 64) * 8);
  L.slots2 = take((nchunks + kAnaFixGroup - 1) / kAnaFixGroup * 2 * kAnaSlotFields * (size_t)((nconf + 63) / 64 * 64) * 8);
  L.total = o;
  return 0;
}

// Raw rows (pid != null) or pre-aggregated pairs (pre_count != null) ->
// per-partition utility-analysis metrics.
struct PairsOut {  // pdp_preaggregate: stop after the pairs and export them
  int64_t *pk, *count, *n_partitions;
  double* sum;
  int64_t* num_pairs;
};

int analysis_impl(pdp_ctx* ctx, const int64_t* pid, const int64_t* pk, const double* val, const int64_t* pre_count,
                  const int64_t* pre_npart, int64_t n, int64_t U, int64_t P, int64_t num_sampled, int32_t metrics,
                  const pdp_analysis_config* cfgs, int nconf, const pdp_analysis_outputs* out, void* workspace,
                  size_t workspace_bytes, hipStream_t stream, const PairsOut* pairs_out = nullptr) {
  if (!ctx || !cfgs || !out || (!out->metrics && !pairs_out)) return fail(PDP_ERR_INVALID_ARG, "null argument");
  if (nconf < 1) return fail(PDP_ERR_INVALID_ARG, "num_configs must be >= 1");
  if (P < 1 || P > (1ll << 31) - 2) return fail(PDP_ERR_INVALID_ARG, "num_partitions must be in [1, 2^31 - 2]");
  if (U < 1 || U > (1ll << 32) - 2) return fail(PDP_ERR_INVALID_ARG, "num_privacy_ids must be in [1, 2^32 - 2]");
  if (n < 0 || n >= (1ll << 32)) return fail(PDP_ERR_INVALID_ARG, "num_rows must be in [0, 2^32)");
  const int mflags = metrics & (PDP_METRIC_SUM | PDP_METRIC_COUNT | PDP_METRIC_PRIVACY_ID_COUNT);
  if (mflags == 0 || mflags != metrics)
    return fail(PDP_ERR_INVALID_ARG, "utility analysis supports COUNT, SUM and PRIVACY_ID_COUNT");
  if (n > 0 && (!pk || (!pid && !pre_count))) return fail(PDP_ERR_INVALID_ARG, "columns required");
  if ((mflags & PDP_METRIC_SUM) && n > 0 && !val) return fail(PDP_ERR_INVALID_ARG, "value column required for SUM");
  if (num_sampled < 0 || num_sampled > P) num_sampled = P;
  AnaLayout L;
  if (int rc = ana_layout(n, U, P, cfgs, nconf, L)) return rc;
  const bool priv = cfgs[0].selection != PDP_SELECTION_NONE;
  if (priv && !out->prob_keep) return fail(PDP_ERR_INVALID_ARG, "prob_keep output required for private selection");
  if (!workspace || workspace_bytes < L.total) return fail(PDP_ERR_WORKSPACE, "workspace too small");
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return fail(PDP_ERR_HIP, "hipSetDevice failed");
  char* ws = (char*)workspace;
  Rec* ra = (Rec*)(ws + L.recs_a);
  Rec* rb = (Rec*)(ws + L.recs_b);
  long long* flags = (long long*)(ws + L.flags);
  uint32_t* ppk = (uint32_t*)(ws + L.ppk);
  uint32_t* pref = (uint32_t*)(ws + L.pref);
  uint32_t* pcnt = (uint32_t*)(ws + L.pcnt);
  double* psum = (double*)(ws + L.psum);
  uint32_t* npart = (uint32_t*)(ws + L.npart);
  int64_t* pbeg = (int64_t*)(ws + L.pbeg);
  double* mom = priv ? (double*)(ws + L.mom) : nullptr;
  AnaCfg* dcfg = (AnaCfg*)(ws + L.cfg);
  double* dkeep = (double*)(ws + L.keep);
  unsigned long long* hist = (unsigned long long*)(ws + L.hist);
  unsigned long long* off = (unsigned long long*)(ws + L.off);
  unsigned long long* counters = (unsigned long long*)(ws + L.counters);
  unsigned long long* status = (unsigned long long*)(ws + L.status);
  for (AnaCfg& g : L.cfgs) g.keep = dkeep + (uintptr_t)g.keep;
  HIP_TRY(hipMemcpyAsync(dcfg, L.cfgs.data(), L.cfgs.size() * sizeof(AnaCfg), hipMemcpyHostToDevice, stream));
  if (!L.keep_all.empty())
    HIP_TRY(hipMemcpyAsync(dkeep, L.keep_all.data(), L.keep_all.size() * 8, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemsetAsync(ws + L.hist, 0, L.status - L.hist, stream));  // hist, off, counters
  HIP_TRY(hipMemsetAsync(npart, 0, (size_t)U * 4, stream));
  const int nb = ((mflags & PDP_METRIC_SUM) != 0) + ((mflags & PDP_METRIC_COUNT) != 0) +
                 ((mflags & PDP_METRIC_PRIVACY_ID_COUNT) != 0);
  if (out->metrics) HIP_TRY(hipMemsetAsync(out->metrics, 0, (size_t)nconf * nb * 5 * P * 8, stream));
  if (mom) HIP_TRY(hipMemsetAsync(mom, 0, (size_t)nconf * 4 * P * 8, stream));
  ctx->tile_slot = kCtrTile0;
  ctx->status_at = nullptr;  // first look-back pass of this call clears its status words (next_epoch)
  ctx->stats = pdp_stats{};
  ctx->cur_debug = ctx->debug;
  const size_t status_bytes = (size_t)L.tiles * kStatusStride * 8;
  const int pkbits = std::max(1, pdp::ceil_log2_u64((uint64_t)P + 1));
  int64_t M = 0;
  bool np_hist = false;
  int np_sh = 0;
  uint32_t* np_spare = nullptr;
  if (n > 0) {
    ProfScope ps(ctx, PDP_STAGE_ANALYSIS_PAIRS, stream);
    const int g = grid_for(n, kThreads, 8192);
    Rec* sorted = nullptr;
    if (pid) {
      // rows -> (pk, pid)-sorted records -> pairs
      const int pidbits = std::max(1, pdp::ceil_log2_u64((uint64_t)U + 1));
      KeySpec ks = composite_spec(1, pkbits, pidbits, pidbits, (uint32_t)std::min<int64_t>(U, 0xFFFFFFFFll),
                                  (uint32_t)P);
      // round 4: the packing is fused into the histogram and the first pass (c5: -0.94 ms of k_ana_pack,
      // +8 B per row in the first pass); PDP_ANA_PACK=1 restores the separate pack
      const bool fused = ks.passes > 0 && !(ctx->cur_debug & kDebugAnaPack);
      if (!fused)
        hipLaunchKernelGGL(k_ana_pack, dim3(g), dim3(kThreads), 0, stream, pid, pk, val, n, U, P, ra, counters);
      if (int rc = sort_recs(ctx, ra, rb, n, ks, hist, off, counters, status, status_bytes, workspace, stream, &sorted,
                             PDP_STAGE_ANALYSIS_SORT, fused ? pid : nullptr, fused ? pk : nullptr,
                             fused ? val : nullptr))
        return rc;
      if (ctx->cur_debug & kDebugAnaFlags) {  // round-3 form: per-row flags, scan, one thread per group start
        hipLaunchKernelGGL(k_ana_group_flags, dim3(g), dim3(kThreads), 0, stream, sorted, n, flags);
        if (int rc = scan_inplace(flags, n, stream)) return rc;
        hipLaunchKernelGGL(k_ana_pairs, dim3(g), dim3(kThreads), 0, stream, sorted, n, flags, num_sampled, ppk, pref,
                           pcnt, psum, npart);
        hipLaunchKernelGGL(k_ana_count_pairs, dim3(1), dim3(1), 0, stream, sorted, n, flags, num_sampled, counters);
      } else {
        const int64_t tiles = (n + kAnaTile - 1) / kAnaTile;
        hipLaunchKernelGGL(k_ana_tile_groups, dim3((unsigned)tiles), dim3(256), 0, stream, sorted, n, flags);
        if (int rc = scan_inplace(flags, tiles, stream)) return rc;
        // n_partitions of the sampled pairs: bucketed LDS histogram (np_hist) or one atomic per pair
        np_sh = std::max(0, pidbits - 8);
        np_hist = np_sh <= 14 && !(ctx->cur_debug & kDebugAnaNpartAtomics);
        np_spare = (uint32_t*)(sorted == ra ? rb : ra);
        hipLaunchKernelGGL(k_ana_tile_pairs, dim3((unsigned)tiles), dim3(256), 0, stream, sorted, n, flags, num_sampled,
                           ppk, pref, pcnt, psum, npart, counters, (int)!np_hist);
      }
    } else {
      // pre-aggregated pairs -> sorted by pk
      hipLaunchKernelGGL(k_ana_pack_pre, dim3(g), dim3(kThreads), 0, stream, pk, val, n, P, ra, counters);
      KeySpec ks{};
      ks.xcd_remap = 1;
      ks.mode = 0;
      ks.num_pids = 0xFFFFFFFFu;
      ks.num_parts = (uint32_t)P;
      for (int sh = 0; sh < pkbits; sh += 8) {
        ks.shift[ks.passes] = sh;
        ks.bits[ks.passes] = std::min(8, pkbits - sh);
        ++ks.passes;
      }
      if (int rc = sort_recs(ctx, ra, rb, n, ks, hist, off, counters, status, status_bytes, workspace, stream, &sorted,
                             PDP_STAGE_ANALYSIS_SORT))
        return rc;
      hipLaunchKernelGGL(k_ana_pairs_pre, dim3(g), dim3(kThreads), 0, stream, sorted, n, pre_count, pre_npart, ppk,
                         pref, pcnt, psum, npart);
    }
    HIP_TRY(hipGetLastError());
    unsigned long long host_ctr[kCtrAnaPairs + 1];
    HIP_TRY(hipMemcpyAsync(host_ctr, counters, sizeof(host_ctr), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    if (host_ctr[kCtrErr]) return fail(PDP_ERR_INTERNAL, "radix look-back timed out");
    if (host_ctr[kCtrInvalid]) return fail(PDP_ERR_OUT_OF_RANGE, "privacy id or partition id out of range");
    M = (int64_t)host_ctr[kCtrAnaPairs];
    if (np_hist && M > 0) {
      // hist[0, 256): bucket counts, off[0, 256): cursors, off[256, 513): bucket starts (zeroed above)
      unsigned long long* bcnt = hist;
      unsigned long long* cur = off;
      unsigned long long* beg = off + kNpBuckets;
      const unsigned nt = (unsigned)((M + kNpTile - 1) / kNpTile);
      HIP_TRY(hipMemsetAsync(bcnt, 0, kNpBuckets * 8, stream));
      hipLaunchKernelGGL(k_np_bucket_count, dim3(nt), dim3(256), 0, stream, pref, M, np_sh, bcnt);
      hipLaunchKernelGGL(k_np_bucket_scan, dim3(1), dim3(256), 0, stream, bcnt, cur, beg);
      hipLaunchKernelGGL(k_np_bucket_scatter, dim3(nt), dim3(256), 0, stream, pref, M, np_sh, cur, np_spare);
      hipLaunchKernelGGL(k_np_bucket_hist, dim3(kNpBuckets), dim3(1024), (size_t)4 << np_sh, stream, np_spare, beg,
                         np_sh, U, npart);
      HIP_TRY(hipGetLastError());
    }
  }
  ctx->stats.kept_rows_in = M;  // pairs of sampled partitions
  if (pairs_out) {
    *pairs_out->num_pairs = M;
    if (M > 0)
      hipLaunchKernelGGL(k_ana_export, dim3(grid_for(M, kThreads, 8192)), dim3(kThreads), 0, stream, ppk, pref, pcnt,
                         psum, npart, M, pairs_out->pk, pairs_out->count, pairs_out->sum, pairs_out->n_partitions);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  ProfScope ps(ctx, PDP_STAGE_ANALYSIS_METRICS, stream);
  const AnaCfg* cfg_d = dcfg;
  hipLaunchKernelGGL(k_ana_bounds, dim3(grid_for(P + 1, kThreads, 8192)), dim3(kThreads), 0, stream, ppk, M, P, pbeg);
  if (out->privacy_ids)
    hipLaunchKernelGGL(k_ana_pid_counts, dim3(grid_for(P, kThreads, 8192)), dim3(kThreads), 0, stream, pbeg, P,
                       out->privacy_ids);
  if (!priv)
    hipLaunchKernelGGL(k_ana_public_init, dim3(grid_for((int64_t)nconf * P, kThreads, 8192)), dim3(kThreads), 0, stream,
                       cfg_d, nconf, mflags, P, out->metrics);
  const unsigned cgroups = (unsigned)((nconf + 63) / 64);
  if (M > 0) {
    const int64_t chunk = (int64_t)kAnaChunk * cgroups;
    const int64_t waves = (M + chunk - 1) / chunk;
    decltype(&k_ana_metrics<true, true, true>) km = nullptr;
    switch (mflags & (PDP_METRIC_SUM | PDP_METRIC_COUNT | PDP_METRIC_PRIVACY_ID_COUNT)) {
#define PDP_KM(S, C, I)                                                                                    \
  case (S ? PDP_METRIC_SUM : 0) | (C ? PDP_METRIC_COUNT : 0) | (I ? PDP_METRIC_PRIVACY_ID_COUNT : 0): \
    km = k_ana_metrics<S, C, I>;                                                                          \
    break;
      PDP_KM(false, false, false) PDP_KM(true, false, false) PDP_KM(false, true, false) PDP_KM(true, true, false)
      PDP_KM(false, false, true) PDP_KM(true, false, true) PDP_KM(false, true, true) PDP_KM(true, true, true)
#undef PDP_KM
    }
    double* slots = (double*)(ws + L.slots);
    hipLaunchKernelGGL(km, dim3((unsigned)((waves + 3) / 4), cgroups), dim3(256), 0, stream, ppk, pref, pcnt, psum,
                       npart, M, cfg_d, nconf, mflags, P, out->metrics, mom, slots, chunk, (int)!priv);
    // fixed-order merge of the chunk-boundary partials, by levels of kAnaFixGroup units
    double* lvl[2] = {slots, (double*)(ws + L.slots2)};
    int64_t nunits = waves, ulen = chunk;
    for (int level = 0;; ++level) {
      const int G = nunits > kAnaFixGroup ? kAnaFixGroup : 0;
      hipLaunchKernelGGL(k_ana_fix, dim3((unsigned)((nunits + 3) / 4), cgroups), dim3(256), 0, stream, ppk, pbeg, M, ulen,
                         nunits, G, nconf, nb, P, (const double*)lvl[level & 1], lvl[(level + 1) & 1], out->metrics,
                         mom, (int)!priv);
      if (G == 0) break;
      nunits = (nunits + G - 1) / G;
      ulen *= G;
    }
  }
  if (priv) {
    ProfScope ps_sel(ctx, PDP_STAGE_ANALYSIS_SELECT, stream);
    const int64_t blocks = std::min<int64_t>((P + kAnaSelWaves - 1) / kAnaSelWaves, 16384);
    if (L.groups.G > 0 && !(ctx->cur_debug & kDebugAnaSelLds)) {
      hipLaunchKernelGGL(k_ana_select_grouped, dim3((unsigned)std::min<int64_t>(P, 65536), cgroups), dim3(64), 0,
                         stream, pref, npart, pbeg, P, cfg_d, nconf, L.groups, (const double*)mom, out->prob_keep);
    } else {  // round-3 form: one launch per regime, lanes = configurations
      hipLaunchKernelGGL(k_ana_select<true>, dim3((unsigned)blocks, cgroups), dim3(64 * kAnaSelWaves), 0, stream, pref,
                         npart, pbeg, P, cfg_d, nconf, (const double*)mom, out->prob_keep);
      hipLaunchKernelGGL(k_ana_select<false>, dim3((unsigned)blocks, cgroups), dim3(64 * kAnaSelWaves), 0, stream,
                         pref, npart, pbeg, P, cfg_d, nconf, (const double*)mom, out->prob_keep);
    }
  }
  HIP_TRY(hipGetLastError());
  return 0;
}

}  // namespace

int pdp_bound_accumulate(pdp_ctx* ctx, const pdp_columns* cols, const pdp_bound_params* bp,
                         const pdp_accumulators* accp, void* workspace, size_t workspace_bytes, void* stream) {
  return bound_impl(ctx, cols, bp, 1, accp, workspace, workspace_bytes, stream, false);
}

int pdp_bound_accumulate_partials(pdp_ctx* ctx, const pdp_columns* cols, const pdp_bound_params* bp,
                                  const pdp_partials* parts, void* workspace, size_t workspace_bytes, void* stream) {
  if (!parts) return fail(PDP_ERR_INVALID_ARG, "null argument");
  const pdp_accumulators a{parts->row_count, parts->count, nullptr, nullptr};
  return bound_impl(ctx, cols, bp, 1, &a, workspace, workspace_bytes, stream, false, parts);
}

int pdp_finalize_partials(pdp_ctx* ctx, const pdp_partials* parts, int64_t P, const pdp_bound_params* bp,
                          const pdp_accumulators* acc, void* stream_) {
  if (!ctx || !parts || !bp || !acc) return fail(PDP_ERR_INVALID_ARG, "null argument");
  if (P < 0) return fail(PDP_ERR_INVALID_ARG, "num_partitions < 0");
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return fail(PDP_ERR_HIP, "hipSetDevice failed");
  hipStream_t stream = (hipStream_t)stream_;
  const SegParams sp = make_seg(bp, 0, 1, true);
  if (!parts->row_count || !acc->row_count) return fail(PDP_ERR_INVALID_ARG, "row_count required");
  if (sp.want_count && (!parts->count || !acc->count)) return fail(PDP_ERR_INVALID_ARG, "count required");
  if (sp.xmode != kXNone && (!parts->x_hi || !parts->x_lo || !acc->x)) return fail(PDP_ERR_INVALID_ARG, "x required");
  if (sp.want_y && (!parts->y_hi || !parts->y_lo || !acc->y)) return fail(PDP_ERR_INVALID_ARG, "y required");
  if (P == 0) return 0;
  if (acc->row_count != parts->row_count)
    HIP_TRY(hipMemcpyAsync(acc->row_count, parts->row_count, (size_t)P * 8, hipMemcpyDeviceToDevice, stream));
  if (sp.want_count && acc->count != parts->count)
    HIP_TRY(hipMemcpyAsync(acc->count, parts->count, (size_t)P * 8, hipMemcpyDeviceToDevice, stream));
  // the exponents K4 used: k4_plan depends on the bounds and metrics only
  const K4Plan k4 = k4_plan(bp, sp, 1, std::max<int64_t>(P, 1), false);
  if (!k4.on) return fail(PDP_ERR_INVALID_ARG, "partials need the K4 reduction (PDP_K4 on)");
  const unsigned grid = (unsigned)grid_for(P, kThreads, 4096);
  if (sp.xmode != kXNone)
    hipLaunchKernelGGL(k4_partials_to_double, dim3(grid), dim3(kThreads), 0, stream, (const long long*)parts->x_hi,
                       (const long long*)parts->x_lo, (const unsigned long long*)parts->nan, 0,
                       k4_red(k4, sp, P, false), acc->x, P);
  if (sp.want_y)
    hipLaunchKernelGGL(k4_partials_to_double, dim3(grid), dim3(kThreads), 0, stream, (const long long*)parts->y_hi,
                       (const long long*)parts->y_lo, (const unsigned long long*)parts->nan, 32,
                       k4_red(k4, sp, P, true), acc->y, P);
  HIP_TRY(hipGetLastError());
  return 0;
}

int pdp_bound_accumulate_sweep(pdp_ctx* ctx, const pdp_columns* cols, const pdp_bound_params* bps, int32_t num_configs,
                               const pdp_accumulators* accs, void* workspace, size_t workspace_bytes, void* stream) {
  return bound_impl(ctx, cols, bps, num_configs, accs, workspace, workspace_bytes, stream, true);
}

int pdp_release(pdp_ctx* ctx, const pdp_accumulators* accp, int64_t P, int64_t pk_offset,
                const pdp_release_params* rp, const pdp_outputs* out, void* stream_) {
  if (!ctx || !accp || !rp || !out || !out->keep || !out->metrics) return fail(PDP_ERR_INVALID_ARG, "null argument");
  if (P < 0) return fail(PDP_ERR_INVALID_ARG, "num_partitions < 0");
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return fail(PDP_ERR_HIP, "hipSetDevice failed");
  hipStream_t stream = (hipStream_t)stream_;
  RelParams q{};
  q.metrics = rp->metrics;
  q.kind = rp->noise_kind;
  q.selection = rp->selection;
  q.add_noise = rp->add_noise;
  q.seed = rp->noise_seed;
  q.max_rows = rp->max_rows_per_privacy_id > 0 ? rp->max_rows_per_privacy_id : 1;
  int32_t fields[5];
  q.nfields = pdp_metric_fields(rp->metrics, fields);
  for (int i = 0; i < q.nfields; ++i) q.field[i] = fields[i];
  const double l0 = (double)rp->max_partitions_contributed, linf = (double)rp->max_contributions_per_partition;
  const int kind = rp->noise_kind;
  const int m = rp->metrics;
  if (kind != PDP_NOISE_LAPLACE && kind != PDP_NOISE_GAUSSIAN)
    return fail(PDP_ERR_INVALID_ARG, "Noise kind must be either Laplace or Gaussian.");
  auto need = [&](int mech) -> int {
    if (!(rp->eps[mech] > 0)) return fail(PDP_ERR_INVALID_ARG, "mechanism epsilon must be positive");
    if (kind == PDP_NOISE_GAUSSIAN && !(rp->delta[mech] > 0))
      return fail(PDP_ERR_INVALID_ARG, "Gaussian mechanism needs delta > 0");
    return 0;
  };
  const double a = rp->min_value, b = rp->max_value;
  q.a = a;
  q.mid = a + (b - a) / 2;
  if (m & (PDP_METRIC_VARIANCE | PDP_METRIC_MEAN)) {
    if (!rp->has_value_bounds) return fail(PDP_ERR_INVALID_ARG, "MEAN/VARIANCE need min_value/max_value");
    const bool var = (m & PDP_METRIC_VARIANCE) != 0;
    const int mech = var ? PDP_MECH_VARIANCE : PDP_MECH_MEAN;
    if (int rc = need(mech)) return rc;
    const int parts = var ? 3 : 2;
    // equally_split_budget, dp_computations.py:224-252
    const double e = rp->eps[mech], d = rp->delta[mech];
    double eu = 0, du = 0, be[3], bd[3];
    for (int i = 0; i < parts - 1; ++i) {
      be[i] = e / parts;
      bd[i] = d / parts;
      eu += be[i];
      du += bd[i];
    }
    be[parts - 1] = e - eu;
    bd[parts - 1] = d - du;
    q.s_mean_count = noise_scale(kind, be[0], bd[0], l0, linf);
    q.mean_degenerate = (a == b);
    q.s_mean_nsum = q.mean_degenerate ? 0.0 : noise_scale(kind, be[1], bd[1], l0, linf * std::fabs(q.mid - a));
    if (var) {
      double sa, sb;  // compute_squares_interval, dp_computations.py:58-62
      if (a < 0 && 0 < b) {
        sa = 0;
        sb = std::max(a * a, b * b);
      } else {
        sa = a * a;
        sb = b * b;
      }
      q.sq_a = sa;
      q.sq_degenerate = (sa == sb);
      q.sq_mid = sa + (sb - sa) / 2;
      q.s_var_nsq = q.sq_degenerate ? 0.0 : noise_scale(kind, be[2], bd[2], l0, linf * std::fabs(q.sq_mid - sa));
    }
  } else {
    if (m & PDP_METRIC_COUNT) {
      if (int rc = need(PDP_MECH_COUNT)) return rc;
      q.s_count = noise_scale(kind, rp->eps[PDP_MECH_COUNT], rp->delta[PDP_MECH_COUNT], l0, linf);
    }
    if (m & PDP_METRIC_SUM) {
      double slinf;
      if (rp->has_value_bounds)
        slinf = linf * std::max(std::fabs(a), std::fabs(b));
      else if (rp->has_partition_bounds)
        slinf = std::max(std::fabs(rp->min_sum_per_partition), std::fabs(rp->max_sum_per_partition));
      else
        return fail(PDP_ERR_INVALID_ARG, "SUM needs value or partition bounds");
      q.sum_zero = (slinf == 0.0);
      if (!q.sum_zero) {
        if (int rc = need(PDP_MECH_SUM)) return rc;
        q.s_sum = noise_scale(kind, rp->eps[PDP_MECH_SUM], rp->delta[PDP_MECH_SUM], l0, slinf);
      }
    }
  }
  if (m & PDP_METRIC_PRIVACY_ID_COUNT) {
    if (int rc = need(PDP_MECH_PRIVACY_ID_COUNT)) return rc;
    q.s_pid = noise_scale(kind, rp->eps[PDP_MECH_PRIVACY_ID_COUNT], rp->delta[PDP_MECH_PRIVACY_ID_COUNT], l0, linf);
  }
  if (rp->selection != PDP_SELECTION_NONE) {
    const double se = rp->eps[PDP_MECH_SELECTION], sd = rp->delta[PDP_MECH_SELECTION];
    if (rp->selection == PDP_SELECTION_TRUNCATED_GEOMETRIC) {
      if (int rc = selection_table(ctx, se, sd, rp->max_partitions_contributed, stream, &q.table, &q.tlen)) return rc;
    } else if (rp->selection == PDP_SELECTION_LAPLACE_THRESHOLDING ||
               rp->selection == PDP_SELECTION_GAUSSIAN_THRESHOLDING) {
      if (int rc = pdp_selection_threshold(rp->selection, se, sd, rp->max_partitions_contributed, &q.sel_thr,
                                           &q.sel_scale))
        return rc;
    } else {
      return fail(PDP_ERR_INVALID_ARG, "Unknown partition selection strategy");
    }
  }
  if (P == 0) return 0;
  ProfScope ps(ctx, PDP_STAGE_RELEASE, stream);
  hipLaunchKernelGGL(k_release, dim3(grid_for(P, kThreads, 8192)), dim3(kThreads), 0, stream,
                     (const unsigned long long*)accp->row_count, (const unsigned long long*)accp->count, accp->x,
                     accp->y, P, pk_offset, q, out->keep, out->metrics);
  HIP_TRY(hipGetLastError());
  return 0;
}

int pdp_prepare_release(pdp_ctx* ctx, const pdp_release_params* rp) {
  if (!ctx || !rp) return fail(PDP_ERR_INVALID_ARG, "null argument");
  if (rp->selection != PDP_SELECTION_TRUNCATED_GEOMETRIC) return 0;
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return fail(PDP_ERR_HIP, "hipSetDevice failed");
  const double* dev = nullptr;
  int64_t len = 0;
  return selection_table(ctx, rp->eps[PDP_MECH_SELECTION], rp->delta[PDP_MECH_SELECTION],
                         rp->max_partitions_contributed, nullptr, &dev, &len);
}

int pdp_profile_enable(pdp_ctx* ctx, int enable) {
  if (!ctx) return fail(PDP_ERR_INVALID_ARG, "null ctx");
  ctx->prof = enable != 0;
  return 0;
}

int pdp_profile_read(pdp_ctx* ctx, double* ms_out, int64_t* launches_out, int reset) {
  if (!ctx) return fail(PDP_ERR_INVALID_ARG, "null ctx");
  for (auto& r : ctx->pending) {
    HIP_TRY(hipEventSynchronize(r.b));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, r.a, r.b));
    ctx->prof_ms[r.stage] += ms;
    ctx->prof_n[r.stage] += 1;
    ctx->pool.push_back(r.a);
    ctx->pool.push_back(r.b);
  }
  ctx->pending.clear();
  for (int i = 0; i < PDP_NUM_STAGES; ++i) {
    if (ms_out) ms_out[i] = ctx->prof_ms[i];
    if (launches_out) launches_out[i] = ctx->prof_n[i];
    if (reset) {
      ctx->prof_ms[i] = 0;
      ctx->prof_n[i] = 0;
    }
  }
  return 0;
}

int pdp_analysis_workspace_size(int64_t num_rows, int64_t num_privacy_ids, int64_t num_partitions,
                                const pdp_analysis_config* cfgs, int32_t num_configs, size_t* bytes) {
  if (!cfgs || !bytes || num_rows < 0 || num_partitions < 1 || num_configs < 1)
    return fail(PDP_ERR_INVALID_ARG, "bad analysis workspace args");
  AnaLayout L;
  if (int rc = ana_layout(num_rows, std::max<int64_t>(num_privacy_ids, 1), num_partitions, cfgs, num_configs, L))
    return rc;
  *bytes = L.total;
  return 0;
}

int pdp_utility_analysis(pdp_ctx* ctx, const pdp_columns* cols, int64_t num_sampled_partitions, int32_t metrics,
                         const pdp_analysis_config* cfgs, int32_t num_configs, const pdp_analysis_outputs* out,
                         void* workspace, size_t workspace_bytes, void* stream) {
  if (!cols) return fail(PDP_ERR_INVALID_ARG, "null argument");
  if (cols->num_rows > 0 && !cols->pid) return fail(PDP_ERR_INVALID_ARG, "pid column required");
  return analysis_impl(ctx, cols->pid, cols->pk, cols->value, nullptr, nullptr, cols->num_rows,
                       cols->num_privacy_ids, cols->num_partitions, num_sampled_partitions, metrics, cfgs, num_configs,
                       out, workspace, workspace_bytes, (hipStream_t)stream);
}

int pdp_utility_aggregate(pdp_ctx* ctx, const double* metrics, const double* prob_keep, const int64_t* privacy_ids,
                          int64_t num_partitions, const pdp_aggregate_params* ap, double* out_errors,
                          double* out_selection, void* stream_) {
  if (!ctx || !ap || !out_errors) return fail(PDP_ERR_INVALID_ARG, "null argument");
  const int C = ap->num_configs, Q = ap->num_quantiles;
  const int mflags = ap->metrics & (PDP_METRIC_SUM | PDP_METRIC_COUNT | PDP_METRIC_PRIVACY_ID_COUNT);
  const int nb = ((mflags & PDP_METRIC_SUM) != 0) + ((mflags & PDP_METRIC_COUNT) != 0) +
                 ((mflags & PDP_METRIC_PRIVACY_ID_COUNT) != 0);
  if (C < 1 || nb < 1 || mflags != ap->metrics) return fail(PDP_ERR_INVALID_ARG, "bad configuration / metric count");
  if (Q < 0 || Q > PDP_AGG_MAX_QUANTILES || (Q > 0 && !ap->quantiles))
    return fail(PDP_ERR_INVALID_ARG, "num_quantiles must be in [0, 8]");
  if (!ap->std_noise || !ap->noise_kind) return fail(PDP_ERR_INVALID_ARG, "std_noise / noise_kind required");
  if (num_partitions < 0 || (num_partitions > 0 && !metrics)) return fail(PDP_ERR_INVALID_ARG, "metrics required");
  if (prob_keep && !out_selection) return fail(PDP_ERR_INVALID_ARG, "out_selection required with prob_keep");
  for (int j = 0; j < Q; ++j)
    if (!(ap->quantiles[j] > 0.0 && ap->quantiles[j] < 1.0)) return fail(PDP_ERR_INVALID_ARG, "quantiles in (0, 1)");
  for (int c = 0; c < C; ++c)
    if (ap->noise_kind[c] != PDP_NOISE_LAPLACE && ap->noise_kind[c] != PDP_NOISE_GAUSSIAN)
      return fail(PDP_ERR_INVALID_ARG, "Noise kind must be either Laplace or Gaussian.");
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return fail(PDP_ERR_HIP, "hipSetDevice failed");
  hipStream_t stream = (hipStream_t)stream_;
  const int K = kAggFields + 2 * Q;
  const int64_t P = num_partitions;
  // metric blocks in pdp_utility_analysis order: SUM, COUNT, PRIVACY_ID_COUNT (those present)
  int is_sum[3], b = 0;
  for (int m : {PDP_METRIC_SUM, PDP_METRIC_COUNT, PDP_METRIC_PRIVACY_ID_COUNT})
    if (mflags & m) is_sum[b++] = m == PDP_METRIC_SUM;
  std::vector<AggRow> rows;
  for (int c = 0; c < C; ++c)
    for (int k = 0; k < nb; ++k) {
      AggRow r{};
      r.m = metrics + ((size_t)c * nb + k) * 5 * (size_t)P;
      r.prob = prob_keep;  // configuration 0's (combiners.py:470-480)
      r.std_noise = ap->std_noise[(size_t)c * nb + k];
      r.kind = ap->noise_kind[c];
      r.is_sum = is_sum[k];
      double* base = out_errors + ((size_t)c * nb + k) * K;
      r.dst = base;
      r.stride = 1;
      r.nf = kAggFields;
      rows.push_back(r);
      for (int j = 0; j < Q; ++j) {  // error_quantiles[j], rel_error_quantiles[j]
        r.qrow = 1;
        r.q = 1.0 - ap->quantiles[j];  // _invert_error_quantiles
        r.dst = base + kAggFields + j;
        r.stride = Q;
        r.nf = 2;
        rows.push_back(r);
      }
    }
  if (prob_keep)
    for (int c = 0; c < C; ++c) {
      AggRow r{};
      r.prob = prob_keep + (size_t)c * P;
      r.dst = out_selection + (size_t)c * 3;
      r.stride = 1;
      r.nf = 3;
      rows.push_back(r);
    }
  const int nrows = (int)rows.size();
  AggParams prm{};
  prm.privacy_ids = privacy_ids;
  prm.P = P;
  prm.nrows = nrows;
  const int nblocks = (int)std::max<int64_t>(1, std::min<int64_t>((P + kAggThreads - 1) / kAggThreads, kAggMaxBlocks));
  AsyncFrees scratch(stream);
  AggRow* d_rows = nullptr;
  double* partials = nullptr;
  HIP_TRY(scratch.alloc((void**)&d_rows, rows.size() * sizeof(AggRow)));
  HIP_TRY(scratch.alloc((void**)&partials, (size_t)nrows * nblocks * kAggFields * sizeof(double)));
  HIP_TRY(hipMemcpyAsync(d_rows, rows.data(), rows.size() * sizeof(AggRow), hipMemcpyHostToDevice, stream));
  prm.rows = d_rows;
  {
    ProfScope ps(ctx, PDP_STAGE_ANALYSIS_AGGREGATE, stream);
    hipLaunchKernelGGL(k_agg_partials, dim3((unsigned)nblocks, (unsigned)std::min(nrows, 65535)), dim3(kAggThreads), 0,
                       stream, prm,
                       partials);
    const int tot = nrows * kAggFields;
    hipLaunchKernelGGL(k_agg_final, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, partials, d_rows, nrows,
                       nblocks);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(stream));  // `rows` (host) is read by the copy above
  return 0;
}

int pdp_utility_analysis_preaggregated(pdp_ctx* ctx, const int64_t* pk, const int64_t* count, const double* sum,
                                       const int64_t* n_partitions, int64_t num_pairs, int64_t num_partitions,
                                       int32_t metrics, const pdp_analysis_config* cfgs, int32_t num_configs,
                                       const pdp_analysis_outputs* out, void* workspace, size_t workspace_bytes,
                                       void* stream) {
  if (num_pairs > 0 && (!count || !n_partitions)) return fail(PDP_ERR_INVALID_ARG, "count / n_partitions required");
  return analysis_impl(ctx, nullptr, pk, sum, count, n_partitions, num_pairs, std::max<int64_t>(num_pairs, 1),
                       num_partitions, num_partitions, metrics, cfgs, num_configs, out, workspace, workspace_bytes,
                       (hipStream_t)stream);
}

int pdp_preaggregate(pdp_ctx* ctx, const pdp_columns* cols, int64_t num_sampled_partitions, int64_t* out_pk,
                     int64_t* out_count, double* out_sum, int64_t* out_n_partitions, int64_t* num_pairs,
                     void* workspace, size_t workspace_bytes, void* stream) {
  if (!cols || !num_pairs) return fail(PDP_ERR_INVALID_ARG, "null argument");
  if (cols->num_rows > 0 && (!cols->pid || !out_pk || !out_count || !out_sum || !out_n_partitions))
    return fail(PDP_ERR_INVALID_ARG, "pid column and outputs required");
  *num_pairs = 0;
  pdp_analysis_config cfg{};
  cfg.max_partitions_contributed = 1;
  cfg.max_contributions_per_partition = 1;
  pdp_analysis_outputs none{};
  const PairsOut po{out_pk, out_count, out_n_partitions, out_sum, num_pairs};
  return analysis_impl(ctx, cols->pid, cols->pk, cols->value, nullptr, nullptr, cols->num_rows,
                       cols->num_privacy_ids, cols->num_partitions, num_sampled_partitions,
                       cols->value ? PDP_METRIC_SUM | PDP_METRIC_COUNT : PDP_METRIC_COUNT, &cfg, 1, &none, workspace,
                       workspace_bytes, (hipStream_t)stream, &po);
}

int pdp_shard_workspace_size(int64_t num_rows, int32_t world_size, size_t* bytes) {
  if (!bytes || num_rows < 0 || world_size < 1 || world_size > kShardMax)
    return fail(PDP_ERR_INVALID_ARG, "bad shard workspace args");
  const int64_t nb = std::max<int64_t>(1, (num_rows + kShardChunk - 1) / kShardChunk);
  *bytes = align_up((size_t)nb * world_size * 8, 256) + align_up((size_t)kShardMax * 8, 256);
  return 0;
}

int pdp_shard_rows(pdp_ctx* ctx, const pdp_columns* cols, int32_t world_size, int64_t* out_pid, int64_t* out_pk,
                   double* out_value, int64_t* rows_per_rank, void* workspace, size_t workspace_bytes,
                   void* stream_) {
  if (!ctx || !cols || !rows_per_rank) return fail(PDP_ERR_INVALID_ARG, "null argument");
  if (world_size < 1 || world_size > kShardMax) return fail(PDP_ERR_INVALID_ARG, "world_size must be in [1, 64]");
  const int64_t n = cols->num_rows;
  if (n < 0) return fail(PDP_ERR_INVALID_ARG, "num_rows < 0");
  for (int d = 0; d < world_size; ++d) rows_per_rank[d] = 0;
  if (n == 0) return 0;
  if (!cols->pid || !cols->pk || !out_pid || !out_pk) return fail(PDP_ERR_INVALID_ARG, "pid / pk columns required");
  if ((cols->value == nullptr) != (out_value == nullptr))
    return fail(PDP_ERR_INVALID_ARG, "value and out_value must both be set or both be null");
  size_t need = 0;
  if (int rc = pdp_shard_workspace_size(n, world_size, &need)) return rc;
  if (!workspace || workspace_bytes < need) return fail(PDP_ERR_WORKSPACE, "workspace too small");
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return fail(PDP_ERR_HIP, "hipSetDevice failed");
  hipStream_t stream = (hipStream_t)stream_;
  const int64_t nb = (n + kShardChunk - 1) / kShardChunk;
  unsigned long long* counts = (unsigned long long*)workspace;
  unsigned long long* totals = (unsigned long long*)((char*)workspace + align_up((size_t)nb * world_size * 8, 256));
  hipLaunchKernelGGL(k_shard_count, dim3((unsigned)nb), dim3(kThreads), 0, stream, cols->pid, n, (int)world_size,
                     counts);
  hipLaunchKernelGGL(k_shard_scan, dim3(1), dim3(kThreads), 0, stream, counts, nb, (int)world_size, totals);
  hipLaunchKernelGGL(k_shard_scatter, dim3((unsigned)nb), dim3(kThreads), 0, stream, cols->pid, cols->pk,
                     cols->value, n, (int)world_size, (const unsigned long long*)counts, out_pid, out_pk, out_value);
  HIP_TRY(hipGetLastError());
  unsigned long long host[kShardMax];
  HIP_TRY(hipMemcpyAsync(host, totals, (size_t)world_size * 8, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  for (int d = 0; d < world_size; ++d) rows_per_rank[d] = (int64_t)host[d];
  return 0;
}

int pdp_generate_synthetic(int64_t* pid, int64_t* pk, double* value, int64_t n, int64_t row_offset, int64_t U,
                           int64_t P, double zipf_s, int32_t value_kind, double lo, double hi, uint64_t seed,
                           void* stream) {
  if (n < 0 || U < 1 || P < 1 || !pid || !pk) return fail(PDP_ERR_INVALID_ARG, "bad generator args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_generate, dim3(grid_for(n, kThreads, 16384)), dim3(kThreads), 0, (hipStream_t)stream, pid, pk,
                     value, n, row_offset, U, P, zipf_s, value_kind, lo, hi, seed);
  HIP_TRY(hipGetLastError());
  return 0;
}

int pdp_fp64_probe(double* tflops, void* stream_) {
  if (!tflops) return fail(PDP_ERR_INVALID_ARG, "null argument");
  hipStream_t stream = (hipStream_t)stream_;
  const int blocks = 256 * 16, iters = 4096;
  double* out = nullptr;
  HIP_TRY(hipMallocAsync((void**)&out, blocks * sizeof(double), stream));
  hipLaunchKernelGGL(k_fp64_probe, dim3(blocks), dim3(256), 0, stream, out, iters, 0.999999, 1e-7);  // warm-up
  hipEvent_t e0 = nullptr, e1 = nullptr;
  HIP_TRY(hipEventCreate(&e0));
  HIP_TRY(hipEventCreate(&e1));
  HIP_TRY(hipEventRecord(e0, stream));
  hipLaunchKernelGGL(k_fp64_probe, dim3(blocks), dim3(256), 0, stream, out, iters, 0.999999, 1e-7);
  HIP_TRY(hipEventRecord(e1, stream));
  HIP_TRY(hipEventSynchronize(e1));
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  HIP_TRY(hipFreeAsync(out, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  *tflops = 2.0 * 8.0 * iters * (double)blocks * 256.0 / (ms * 1e-3) / 1e12;
  return 0;
}

int pdp_stream_copy(const void* src, void* dst, int64_t bytes, void* stream) {
  if (bytes < 0 || (bytes & 15) || (bytes && (!src || !dst))) return fail(PDP_ERR_INVALID_ARG, "bad copy args");
  if (bytes == 0) return 0;
  // default: non-temporal, 8 x 16 B in flight per lane, 32768 blocks (5.32 TB/s against 5.11 for the plain
  // 4-deep form on the same box, tools/copy_probe.py).  PDP_COPY_VARIANT: 0 plain 4-deep; 1 nt loads + nt
  // stores; 2 nt loads, default stores; 3 default loads + stores; 4 default loads, nt stores (8-deep);
  // 5 read only (nt), 6 read only (default); 7 write only (nt), 8 write only (default) -- for 5-8 `bytes`
  // is the bytes read or written
  const int variant = env_int("PDP_COPY_VARIANT", 1);
  const unsigned grid = (unsigned)env_int("PDP_COPY_GRID", 32768);
  auto kern = variant == 1 ? k_stream_copy_8<true, true, kCopyRW>
            : variant == 2 ? k_stream_copy_8<true, false, kCopyRW>
            : variant == 3 ? k_stream_copy_8<false, false, kCopyRW>
            : variant == 4 ? k_stream_copy_8<false, true, kCopyRW>
            : variant == 5 ? k_stream_copy_8<true, true, kCopyRead>
            : variant == 6 ? k_stream_copy_8<false, false, kCopyRead>
            : variant == 7 ? k_stream_copy_8<true, true, kCopyWrite>
            : variant == 8 ? k_stream_copy_8<false, false, kCopyWrite>
                           : nullptr;
  if (kern)
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src, (u32x4*)dst,
                       bytes / 16);
  else
    hipLaunchKernelGGL(k_stream_copy, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src, (u32x4*)dst,
                       bytes / 16);
  HIP_TRY(hipGetLastError());
  return 0;
}

}  // extern "C"
