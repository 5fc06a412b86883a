// ubench_random.hip — the MI355X random-read roofline for the Bloom probe's
// access pattern: independent 4-byte (and 8-byte) reads at uniformly random
// word positions of a table, every lane keeping R reads in flight. Reports
// reads/s and the HBM bytes they imply at 64 B and 128 B per read, for plain
// hipMalloc memory, non-temporal loads, and hipDeviceMallocUncached memory;
// plus a dwordx4 streaming read for reference. Output: one JSON object.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

template <int R, bool NT>
__global__ __launch_bounds__(256) void k_gather(const uint32_t* __restrict__ t, uint64_t mask,
                                                uint64_t iters, uint32_t* out) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (uint64_t it = 0; it < iters; ++it) {
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t idx = mix(tid * 1315423911ull + it * R + r) & mask;
      v[r] = NT ? __builtin_nontemporal_load(&t[idx]) : t[idx];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) acc ^= v[r];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_stream(const uint4* __restrict__ t, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = t[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <class F>
static float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  uint32_t* out;
  CHECK(hipMalloc(&out, 4));
  printf("{\"random_reads\": [");
  const size_t sizes[] = {16ull << 20, 256ull << 20, 1ull << 30};
  bool first = true;
  for (size_t bytes : sizes) {
    for (int kind = 0; kind < 3; ++kind) {  // 0 plain, 1 nt loads, 2 uncached memory
      uint32_t* t;
      if (kind == 2)
        CHECK(hipExtMallocWithFlags((void**)&t, bytes, hipDeviceMallocUncached));
      else
        CHECK(hipMalloc(&t, bytes));
      CHECK(hipMemset(t, 1, bytes));
      const uint64_t mask = bytes / 4 - 1;
      const uint32_t grid = 256 * 32;  // 32 blocks per CU slot budget
      const uint64_t iters = 16;
      const double reads = (double)grid * 256 * iters * 8;
      float ms;
      if (kind == 1)
        ms = time_ms([&] { hipLaunchKernelGGL((k_gather<8, true>), dim3(grid), dim3(256), 0, 0, t, mask, iters, out); }, 5);
      else
        ms = time_ms([&] { hipLaunchKernelGGL((k_gather<8, false>), dim3(grid), dim3(256), 0, 0, t, mask, iters, out); }, 5);
      const double rps = reads / (ms * 1e-3);
      printf("%s{\"table_MiB\": %zu, \"mem\": \"%s\", \"reads_per_s\": %.4g, \"GBps_at_64B\": %.1f, \"GBps_at_128B\": %.1f, \"ms\": %.3f}",
             first ? "" : ", ", bytes >> 20, kind == 0 ? "hipMalloc" : kind == 1 ? "hipMalloc+nt" : "uncached",
             rps, rps * 64 / 1e9, rps * 128 / 1e9, ms);
      first = false;
      CHECK(hipFree(t));
    }
  }
  printf("], ");
  {
    const size_t bytes = 1ull << 30;
    uint4* t;
    CHECK(hipMalloc(&t, bytes));
    CHECK(hipMemset(t, 1, bytes));
    const uint64_t n = bytes / 16;
    float ms = time_ms([&] { hipLaunchKernelGGL(k_stream, dim3(256 * 16), dim3(256), 0, 0, t, n, out); }, 10);
    printf("\"stream_read\": {\"table_MiB\": 1024, \"GBps\": %.1f}}\n", bytes / (ms * 1e-3) / 1e9);
    CHECK(hipFree(t));
  }
  return 0;
}
