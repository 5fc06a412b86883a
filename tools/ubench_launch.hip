// ubench_launch.hip — the fixed cost of a launch on one stream, by grid
// shape and LDS: back-to-back launches of a kernel that only touches its LDS
// (per-launch time = dispatch + wave launch + drain), the same with a 64 KiB
// tile written back per workgroup (the build's tile write), and single
// launches timed alone. Diagnostic for the C2 build's two launches
// (DESIGN.md §9); not part of the product.
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

template <int NT>
__global__ __launch_bounds__(NT) void k_touch(uint32_t* p) {
  extern __shared__ uint32_t sm[];
  sm[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (sm[NT - 1 - threadIdx.x] == 0xFFFFFFFFu) p[0] = 1;
}

// each workgroup writes `bytes` of zeros from LDS (the tile write-back)
template <int NT>
__global__ __launch_bounds__(NT) void k_tilewrite(uint4* out, uint32_t n4) {
  extern __shared__ uint4 sm4[];
  for (uint32_t i = threadIdx.x; i < n4; i += NT) sm4[i] = make_uint4(0, 0, 0, i);
  __syncthreads();
  uint4* o = out + (size_t)blockIdx.x * n4;
  for (uint32_t i = threadIdx.x; i < n4; i += NT) o[i] = sm4[i];
}

template <class F>
static float per_launch_us(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i) f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / reps;
}

template <int NT>
static void shape(uint32_t* dummy, uint4* big, uint32_t grid, size_t lds, bool first) {
  if (lds > 64 * 1024) {
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_touch<NT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_tilewrite<NT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  }
  const float t = per_launch_us([&] { hipLaunchKernelGGL(k_touch<NT>, dim3(grid), dim3(NT), lds, 0, dummy); }, 200);
  // write-back of 16 MiB over the grid (the C2 filter), when the LDS holds it
  float w = -1;
  const size_t per = (16ull << 20) / grid;
  if (per <= lds && per % 16 == 0)
    w = per_launch_us([&] {
      hipLaunchKernelGGL(k_tilewrite<NT>, dim3(grid), dim3(NT), lds, 0, big, (uint32_t)(per / 16));
    }, 200);
  printf("%s{\"threads\": %d, \"grid\": %u, \"lds\": %zu, \"empty_us\": %.2f, \"write16MiB_us\": %.2f}",
         first ? "" : ", ", NT, grid, lds, t, w);
}

int main() {
  uint32_t* dummy;
  uint4* big;
  CHECK(hipMalloc(&dummy, 64));
  CHECK(hipMalloc(&big, 32ull << 20));
  printf("{\"launch\": [");
  shape<1024>(dummy, big, 256, 64 * 1024, true);
  shape<1024>(dummy, big, 256, 34 * 1024, false);
  shape<1024>(dummy, big, 256, 0, false);
  shape<512>(dummy, big, 256, 64 * 1024, false);
  shape<256>(dummy, big, 256, 64 * 1024, false);
  shape<256>(dummy, big, 256, 0, false);
  shape<256>(dummy, big, 512, 32 * 1024, false);
  shape<256>(dummy, big, 1024, 16 * 1024, false);
  shape<1024>(dummy, big, 128, 128 * 1024, false);
  shape<64>(dummy, big, 256, 0, false);
  printf("]}\n");
  return 0;
}
