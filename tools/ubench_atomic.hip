// ubench_atomic.hip — what a one-pass Bloom build (src/bloom.rs:40-44, two
// bit-sets per key) can reach on MI355X: random 32-bit atomicOr into a filter
// of the C2 shape (2^27 bits = 16 MiB, 2^21 bit-sets), compared with
//   direct   — every lane ORs both of its key's bits wherever they fall;
//   xcd      — each workgroup reads its XCD (HW_REG_XCC_ID) and ORs only the
//              bits of that XCD's 1/8 slice of the filter, so every 128-B line
//              is touched from one L2 only; each XCD walks all keys through its
//              own chunk counter;
//   store    — plain (non-atomic, racy) stores of the same words: the scatter
//              rate without RMW;
// plus the workgroup → XCD histogram. Tables are compared for equality.
// Output: one JSON object.
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

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7u;
}

__global__ __launch_bounds__(256) void k_direct(uint32_t* __restrict__ w, uint32_t mbits_log2,
                                                uint32_t n) {
  const uint32_t k = blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  const uint64_t h = mix(k);
  const uint32_t msk = (1u << mbits_log2) - 1u;
  const uint32_t a = (uint32_t)h & msk, b = (uint32_t)(h >> 32) & msk;
  atomicOr(&w[a >> 5], 1u << (a & 31));
  atomicOr(&w[b >> 5], 1u << (b & 31));
}

__global__ __launch_bounds__(256) void k_store(uint32_t* __restrict__ w, uint32_t mbits_log2,
                                               uint32_t n) {
  const uint32_t k = blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  const uint64_t h = mix(k);
  const uint32_t msk = (1u << mbits_log2) - 1u;
  const uint32_t a = (uint32_t)h & msk, b = (uint32_t)(h >> 32) & msk;
  w[a >> 5] = 1u << (a & 31);
  w[b >> 5] = 1u << (b & 31);
}

// chunk = 256 * KPT keys; ctr[x] hands out chunks to XCD x's workgroups.
template <int KPT>
__global__ __launch_bounds__(256) void k_xcd(uint32_t* __restrict__ w, uint32_t mbits_log2,
                                             uint32_t n, uint32_t* ctr, uint32_t* xhist) {
  __shared__ uint32_t s_chunk;
  const uint32_t x = xcc_id();
  if (threadIdx.x == 0) atomicAdd(&xhist[x], 1u);
  const uint32_t nchunks = (n + 256 * KPT - 1) / (256 * KPT);
  const uint32_t msk = (1u << mbits_log2) - 1u;
  const uint32_t sh = mbits_log2 - 3;  // slice = top 3 bits of the position
  for (;;) {
    if (threadIdx.x == 0) s_chunk = atomicAdd(&ctr[x], 1u);
    __syncthreads();
    const uint32_t c = s_chunk;
    __syncthreads();
    if (c >= nchunks) break;
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const uint32_t k = c * 256 * KPT + j * 256 + threadIdx.x;
      if (k < n) {
        const uint64_t h = mix(k);
        const uint32_t a = (uint32_t)h & msk, b = (uint32_t)(h >> 32) & msk;
        if ((a >> sh) == x)
          __hip_atomic_fetch_or(&w[a >> 5], 1u << (a & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if ((b >> sh) == x)
          __hip_atomic_fetch_or(&w[b >> 5], 1u << (b & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
}

template <class F>
static float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  float tot = 0;
  for (int i = 0; i < reps; ++i) {
    CHECK(hipEventRecord(a));
    f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    tot += ms;
  }
  return tot / reps;
}

int main() {
  const uint32_t L = 27, n = 1u << 20;
  const size_t bytes = (size_t(1) << L) / 8;
  uint32_t *w1, *w2, *ctr, *xh;
  CHECK(hipMalloc(&w1, bytes));
  CHECK(hipMalloc(&w2, bytes));
  CHECK(hipMalloc(&ctr, 64));
  CHECK(hipMalloc(&xh, 64));
  const int reps = 20;
  const uint32_t grid = (n + 255) / 256;
  float t_direct = time_ms([&] {
    CHECK(hipMemsetAsync(w1, 0, bytes));
    hipLaunchKernelGGL(k_direct, dim3(grid), dim3(256), 0, 0, w1, L, n);
  }, reps);
  float t_memset = time_ms([&] { CHECK(hipMemsetAsync(w1, 0, bytes)); }, reps);
  float t_store = time_ms([&] {
    CHECK(hipMemsetAsync(w2, 0, bytes));
    hipLaunchKernelGGL(k_store, dim3(grid), dim3(256), 0, 0, w2, L, n);
  }, reps);
  printf("{\"shape\": \"2^20 keys, 2^21 atomicOr into 2^27 bits (16 MiB)\", \"memset_ms\": %.4f, "
         "\"direct_ms\": %.4f, \"store_ms\": %.4f", t_memset, t_direct, t_store);
  for (uint32_t g : {512u, 1024u, 2048u}) {
    float t_x = time_ms([&] {
      CHECK(hipMemsetAsync(w2, 0, bytes));
      CHECK(hipMemsetAsync(ctr, 0, 64));
      CHECK(hipMemsetAsync(xh, 0, 64));
      hipLaunchKernelGGL((k_xcd<4>), dim3(g), dim3(256), 0, 0, w2, L, n, ctr, xh);
    }, reps);
    printf(", \"xcd_g%u_ms\": %.4f", g, t_x);
  }
  // correctness: direct and xcd tables must agree
  hipLaunchKernelGGL(k_direct, dim3(grid), dim3(256), 0, 0, w1, L, n);
  CHECK(hipDeviceSynchronize());
  std::vector<uint32_t> h1(bytes / 4), h2(bytes / 4), hx(16);
  CHECK(hipMemcpy(h1.data(), w1, bytes, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(h2.data(), w2, bytes, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hx.data(), xh, 64, hipMemcpyDeviceToHost));
  size_t diff = 0, pop = 0;
  for (size_t i = 0; i < h1.size(); ++i) {
    diff += h1[i] != h2[i];
    pop += __builtin_popcount(h1[i]);
  }
  printf(", \"xcd_equal\": %s, \"diff_words\": %zu, \"popcount\": %zu, \"xcc_hist\": [", diff ? "false" : "true",
         diff, pop);
  for (int i = 0; i < 8; ++i) printf("%s%u", i ? ", " : "", hx[i]);
  printf("]}\n");
  return 0;
}
