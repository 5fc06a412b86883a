// ubench_fill.hip — what one random 4-byte read costs the memory side, by load
// flavour and memory type: the k_set_probe question of whether a read fills a
// whole 128-B L2 line or only a 64-B (or 32-B) part of it, and whether the
// random-read rate is bound by bytes or by requests. Independent reads at
// uniformly random word positions of a 256 MiB table (the C3 set's size), R in
// flight per lane. Each flavour is its own kernel instance (its own name in a
// rocprofv3 trace), so `rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum
// TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum` over this
// program gives the request sizes per flavour. Diagnostic only.
// Output: one JSON line.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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

// FLAV: 0 plain global load, 1 __builtin_nontemporal_load, 2..5 buffer loads
// with cache-policy aux 0 / 1 (sc0) / 2 (nt) / 16 (sc1) / 17 (sc0 sc1)
template <int FLAV>
__global__ __launch_bounds__(256) void k_fill(const uint32_t* __restrict__ t, uint64_t mask, uint32_t iters,
                                              uint32_t* out) {
  constexpr int R = 8;
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(t), 0, 0x7FFFFFFF, 0x00020000);
  uint32_t acc = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t idx = mix(tid * 1315423911ull + it * R + r) & mask;
      if constexpr (FLAV == 0 || FLAV >= 7) {  // 7, 8: plain loads of the uncached / fine-grained tables
        v[r] = t[idx];
      } else if constexpr (FLAV == 1) {
        v[r] = __builtin_nontemporal_load(&t[idx]);
      } else {
        constexpr int aux = FLAV == 2 ? 0 : FLAV == 3 ? 1 : FLAV == 4 ? 2 : FLAV == 5 ? 16 : 17;
        v[r] = __builtin_amdgcn_raw_buffer_load_b32(rs, (uint32_t)(idx * 4), 0, aux);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) acc ^= v[r];
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

template <int FLAV>
static void run(const char* name, const char* mem, const uint32_t* t, uint64_t bytes, uint32_t* out, bool& first) {
  const uint64_t mask = bytes / 4 - 1;
  const uint32_t grid = 256 * 32, iters = 8;
  const double reads = (double)grid * 256 * iters * 8;
  const float ms = time_ms([&] { hipLaunchKernelGGL(k_fill<FLAV>, dim3(grid), dim3(256), 0, 0, t, mask, iters, out); }, 5);
  const double rps = reads / (ms * 1e-3);
  printf("%s{\"flavour\": \"%s\", \"mem\": \"%s\", \"reads_per_s\": %.4g, \"us\": %.1f}", first ? "" : ", ", name, mem, rps,
         ms * 1e3);
  first = false;
}

int main() {
  uint32_t* out;
  CHECK(hipMalloc(&out, 4));
  const uint64_t bytes = 256ull << 20;
  const int reps = getenv("FILL_REPS") ? atoi(getenv("FILL_REPS")) : 1;
  printf("{\"table_MiB\": 256, \"runs\": [");
  bool first = true;
  for (int rep = 0; rep < reps; ++rep) {
    uint32_t* t;
    CHECK(hipMalloc(&t, bytes));
    CHECK(hipMemset(t, 1, bytes));
    run<0>("plain", "hipMalloc", t, bytes, out, first);
    run<1>("nontemporal", "hipMalloc", t, bytes, out, first);
    run<2>("buffer", "hipMalloc", t, bytes, out, first);
    run<3>("buffer sc0", "hipMalloc", t, bytes, out, first);
    run<4>("buffer nt", "hipMalloc", t, bytes, out, first);
    run<5>("buffer sc1", "hipMalloc", t, bytes, out, first);
    run<6>("buffer sc0 sc1", "hipMalloc", t, bytes, out, first);
    CHECK(hipFree(t));
  }
  {
    uint32_t* t;
    CHECK(hipExtMallocWithFlags((void**)&t, bytes, hipDeviceMallocUncached));
    CHECK(hipMemset(t, 1, bytes));
    // a separate instance name for the uncached table: FLAV 0's code, another template id
    run<7>("plain", "uncached", t, bytes, out, first);
    CHECK(hipFree(t));
  }
  {
    uint32_t* t;
    CHECK(hipExtMallocWithFlags((void**)&t, bytes, hipDeviceMallocFinegrained));
    CHECK(hipMemset(t, 1, bytes));
    run<8>("plain", "finegrained", t, bytes, out, first);
    CHECK(hipFree(t));
  }
  printf("]}\n");
  return 0;
}
