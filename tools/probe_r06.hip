// Round-6 probes (measurement only, not part of the library):
//  (1) graph: hipMemsetAsync and stream-ordered allocation nodes inside a captured hipGraph, replayed
//      several times, checked byte for byte -- the evidence for or against round 5's claim that "a
//      memset node in a captured graph faulted on replay" (DESIGN.md 3.5).  Sizes and alignments are
//      the ones the aggregate path cleared with hipMemsetAsync before round 5 moved to k_zero64.
//  (2) atomics: random 32-bit atomicOr into a per-privacy-id table of U words (c3: U = 1e7, 40 MB,
//      Infinity-Cache resident), 1e9 operations -- the rate that decides whether a global per-pid
//      sketch can replace the bucket pass.  Also random 4-byte gathers from
//      the same table, and a streaming read of the same bytes as a reference.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_r06 tools/probe_r06.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::printf("HIP error %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__, __LINE__, #x); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_fill(unsigned char* p, int64_t n, unsigned char v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// counts the non-zero bytes of [p, p + n) into *bad (one atomic per thread that saw any)
__global__ void k_count_nonzero(const unsigned char* p, int64_t n, unsigned long long* bad) {
  unsigned long long c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    c += p[i] != 0;
  if (c) atomicAdd(bad, c);
}

__global__ void k_write_pattern(unsigned long long* p, int64_t words) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 0x0123456789ABCDEFull ^ (unsigned long long)i;
}

__global__ void k_check_pattern(const unsigned long long* p, int64_t words, unsigned long long* bad) {
  unsigned long long c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x)
    c += p[i] != (0x0123456789ABCDEFull ^ (unsigned long long)i);
  if (c) atomicAdd(bad, c);
}

__global__ void k_atomic_or(unsigned int* table, uint64_t U, int64_t ops, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ops; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = mix64(seed ^ (uint64_t)i);
    const uint32_t idx = (uint32_t)(((h >> 32) * U) >> 32);
    atomicOr(&table[idx], 1u << (h & 31u));
  }
}

__global__ void k_gather(const unsigned int* table, uint64_t U, int64_t ops, uint64_t seed, unsigned int* out) {
  unsigned int acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ops; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = mix64(seed ^ (uint64_t)i);
    const uint32_t idx = (uint32_t)(((h >> 32) * U) >> 32);
    acc ^= table[idx];
  }
  if (acc == 0x12345678u) out[threadIdx.x] = acc;  // keeps the loads alive
}

__global__ void k_stream_read(const uint4* p, int64_t n16, unsigned int* out) {
  unsigned int acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

// (3) sparse gathers: the L0 pre-filter's survivors (6.8 % of 1e9 rows) gathered from the ORIGINAL pk / value
// columns by row index instead of being carried through the bucket pass.  256 workgroups (one per privacy-id
// bucket), each with a sorted list of ~265K row indices spread over the whole column (survivors keep input
// order within a bucket): read the list (4 B), gather pk (8 B) and value (8 B), write a 16-B record.
__global__ void k_make_lists(uint32_t* list, int64_t per, int64_t stride) {
  const int64_t b = blockIdx.y;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < per; k += (int64_t)gridDim.x * blockDim.x)
    list[b * per + k] = (uint32_t)(k * stride + (int64_t)(mix64(((uint64_t)b << 40) ^ (uint64_t)k) % (uint64_t)stride));
}

template <int G>
__global__ __launch_bounds__(1024) void k_sparse_gather(const uint32_t* list, int64_t per, const int64_t* pk,
                                                         const double* val, uint4* out) {
  const int64_t b = blockIdx.x;
  const uint32_t* l = list + b * per;
  for (int64_t k0 = threadIdx.x; k0 < per; k0 += 1024 * G) {
    uint32_t idx[G];
    int64_t p[G];
    double v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) idx[g] = k0 + g * 1024 < per ? l[k0 + g * 1024] : 0u;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      p[g] = pk[idx[g]];
      v[g] = val[idx[g]];
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (k0 + g * 1024 < per) {
        const uint64_t vb = (uint64_t)__double_as_longlong(v[g]);
        out[b * per + k0 + g * 1024] = uint4{idx[g], (uint32_t)p[g], (uint32_t)vb, (uint32_t)(vb >> 32)};
      }
    }
  }
}

static void sparse_probe() {
  const int64_t N = 1000000000ll, per = 265000, stride = N / per;
  int64_t* pk = nullptr;
  double* val = nullptr;
  uint32_t* list = nullptr;
  uint4* out = nullptr;
  CK(hipMalloc(&pk, N * 8));
  CK(hipMalloc(&val, N * 8));
  CK(hipMalloc(&list, 256 * per * 4));
  CK(hipMalloc(&out, 256 * per * 16));
  CK(hipMemset(pk, 1, N * 8));
  CK(hipMemset(val, 2, N * 8));
  hipLaunchKernelGGL(k_make_lists, dim3(64, 256), dim3(256), 0, 0, list, per, stride);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep) {
    for (int G : {1, 4, 8}) {
      CK(hipEventRecord(a, 0));
      if (G == 1) hipLaunchKernelGGL(k_sparse_gather<1>, dim3(256), dim3(1024), 0, 0, list, per, pk, val, out);
      if (G == 4) hipLaunchKernelGGL(k_sparse_gather<4>, dim3(256), dim3(1024), 0, 0, list, per, pk, val, out);
      if (G == 8) hipLaunchKernelGGL(k_sparse_gather<8>, dim3(256), dim3(1024), 0, 0, list, per, pk, val, out);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      std::printf("SPARSE_GATHER %lld survivors (256 x %lld, 1e9-row columns), %d in flight/lane: %.3f ms\n",
                  (long long)(256 * per), (long long)per, G, ms);
    }
  }
  CK(hipFree(pk));
  CK(hipFree(val));
  CK(hipFree(list));
  CK(hipFree(out));
}

static int graph_probe() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int64_t P = 1000000;
  const size_t total = 64ull << 20;
  unsigned char* buf = nullptr;
  CK(hipMalloc(&buf, total));
  unsigned long long* bad = nullptr;
  CK(hipMalloc(&bad, 64 * 8));
  // (offset, bytes) pairs: the round-4/5 aggregate path's hipMemsetAsync calls (counters word,
  // tile-claim counters, hist 12 x 257 x 8, accumulators P x 8, K4 replicas, fixed-point scratch P x 16
  // and flags P x 4 rounded, an 8-byte counter at an odd word), plus unaligned and odd sizes
  struct Seg {
    size_t off, bytes;
  };
  const std::vector<Seg> segs = {{0, 8},
                                 {256, 44 * 8},
                                 {4096, 12 * 257 * 8},
                                 {1 << 20, (size_t)P * 8},
                                 {10 << 20, 64 * 3 * 256 * 4},
                                 {12 << 20, (size_t)P * 16},
                                 {30 << 20, ((size_t)P * 4 + 7) / 8 * 8},
                                 {40 << 20, 8 + 8},
                                 {41 << 20, 3},
                                 {(41 << 20) + 5, 1001},
                                 {42 << 20, (20ull << 20) + 4}};
  hipGraph_t g;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, s, buf, (int64_t)total, (unsigned char)0xAB);
  for (const Seg& q : segs) CK(hipMemsetAsync(buf + q.off, 0, q.bytes, s));
  CK(hipMemsetAsync(bad, 0, 64 * 8, s));
  for (size_t i = 0; i < segs.size(); ++i)
    hipLaunchKernelGGL(k_count_nonzero, dim3(256), dim3(256), 0, s, buf + segs[i].off, (int64_t)segs[i].bytes,
                       bad + i);
  // stream-ordered allocation inside the capture (graph memory nodes), written and checked, then freed
  void* tmp = nullptr;
  CK(hipMallocAsync(&tmp, 16 << 20, s));
  hipLaunchKernelGGL(k_write_pattern, dim3(512), dim3(256), 0, s, (unsigned long long*)tmp, (int64_t)(2 << 20));
  hipLaunchKernelGGL(k_check_pattern, dim3(512), dim3(256), 0, s, (const unsigned long long*)tmp,
                     (int64_t)(2 << 20), bad + 63);
  CK(hipFreeAsync(tmp, s));
  CK(hipStreamEndCapture(s, &g));
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  int fails = 0;
  for (int r = 0; r < 5; ++r) {
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    unsigned long long h[64];
    CK(hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost));
    unsigned long long nb = 0;
    for (size_t i = 0; i < segs.size(); ++i) nb += h[i];
    std::printf("graph replay %d: memset-node ranges with non-zero bytes: %llu, graph-allocated buffer mismatches: %llu\n",
                r, nb, h[63]);
    fails += (nb != 0) + (h[63] != 0);
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipFree(buf));
  CK(hipFree(bad));
  CK(hipStreamDestroy(s));
  std::printf("GRAPH_PROBE %s\n", fails ? "FAIL" : "OK");
  return fails;
}

static void atomic_probe() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  unsigned int* out = nullptr;
  CK(hipMalloc(&out, 4096));
  for (uint64_t U : {10000000ull, 1000000ull}) {
    unsigned int* table = nullptr;
    CK(hipMalloc(&table, U * 4));
    CK(hipMemsetAsync(table, 0, U * 4, s));
    const int64_t ops = 1000000000ll;
    for (int grid : {4096, 16384}) {
      hipLaunchKernelGGL(k_atomic_or, dim3(grid), dim3(256), 0, s, table, U, ops / 16, 1ull);  // warm
      CK(hipEventRecord(a, s));
      hipLaunchKernelGGL(k_atomic_or, dim3(grid), dim3(256), 0, s, table, U, ops, 2ull);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      std::printf("ATOMIC_OR U=%llu (%.0f MB table) ops=%lld grid=%d: %.2f ms = %.2f e9 ops/s\n",
                  (unsigned long long)U, U * 4 / 1e6, (long long)ops, grid, ms, ops / (ms * 1e6));
      CK(hipEventRecord(a, s));
      hipLaunchKernelGGL(k_gather, dim3(grid), dim3(256), 0, s, table, U, ops, 3ull, out);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      std::printf("GATHER4 U=%llu ops=%lld grid=%d: %.2f ms = %.2f e9 loads/s\n", (unsigned long long)U,
                  (long long)ops, grid, ms, ops / (ms * 1e6));
    }
    CK(hipFree(table));
  }
  // streaming read of 16 GB (the pid + pk columns of 1e9 rows) for comparison
  const int64_t bytes = 16ll << 30;
  uint4* big = nullptr;
  CK(hipMalloc(&big, bytes));
  CK(hipMemsetAsync(big, 1, bytes, s));
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipEventRecord(a, s));
    hipLaunchKernelGGL(k_stream_read, dim3(32768), dim3(256), 0, s, big, bytes / 16, out);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("STREAM_READ 16 GiB: %.2f ms = %.2f TB/s\n", ms, bytes / (ms * 1e9));
  }
  CK(hipFree(big));
  CK(hipFree(out));
  CK(hipStreamDestroy(s));
}

int main(int argc, char** argv) {
  const bool graph = argc < 2 || argv[1][0] == 'g' || argv[1][0] == 'a';
  const bool atom = argc < 2 || argv[1][0] == 't' || argv[1][0] == 'a';
  const bool sparse = argc >= 2 && (argv[1][0] == 's' || argv[1][0] == 'a');
  int rc = 0;
  if (graph) rc = graph_probe();
  if (atom) atomic_probe();
  if (sparse) sparse_probe();
  return rc;
}
