// ubench_build.hip — where the C2 build's time goes (2^20
// 16-byte keys -> one 2^27-bit filter). Compiles the library's kernels.hip in
// this translation unit with CB_STAMPS, so the build kernels record
// s_memrealtime (100 MHz) at their phase boundaries. Reports:
//   - back-to-back time per launch of an empty 1024-thread kernel of the
//     same grid and LDS (the launch + drain floor),
//   - the two-kernel build per step, each kernel alone back to back,
//   - per-phase medians across workgroups and each kernel's span (first
//     workgroup start to last workgroup end) from the stamps.
// Output: one JSON object. Diagnostic only; not part of the product.
#define CB_STAMPS 1
#include "../lsmt_amd/csrc/kernels.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__global__ __launch_bounds__(1024) void k_empty(uint32_t* p) {
  extern __shared__ uint32_t sm[];
  sm[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (sm[1023 - threadIdx.x] == 0xFFFFFFFFu) p[0] = 1;
}

__global__ void k_keys(uint4* k, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint64_t x = i * 0x9E3779B97F4A7C15ull + 12345;
  uint32_t w[4];
  for (int j = 0; j < 4; ++j) {
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    w[j] = (uint32_t)(x >> 16);
  }
  k[i] = make_uint4(w[0], w[1], w[2], w[3]);
}

template <class F>
static float per_launch_us(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / reps;
}

static void phases(const char* name, const std::vector<uint64_t>& st, uint32_t nblocks, int nst,
                   bool last) {
  uint64_t t0 = ~0ull, t1 = 0;
  std::vector<std::vector<double>> d(nst);
  for (uint32_t b = 0; b < nblocks; ++b) {
    const uint64_t* r = &st[(size_t)b * 8];
    t0 = std::min(t0, r[0]);
    t1 = std::max(t1, r[nst - 1]);
    for (int i = 1; i < nst; ++i) d[i].push_back((r[i] - r[i - 1]) * 0.01);  // us
  }
  printf("\"%s\": {\"span_us\": %.2f, \"phase_median_us\": [", name, (t1 - t0) * 0.01);
  for (int i = 1; i < nst; ++i) {
    std::sort(d[i].begin(), d[i].end());
    printf("%s%.2f", i > 1 ? ", " : "", d[i][d[i].size() / 2]);
  }
  printf("], \"phase_max_us\": [");
  for (int i = 1; i < nst; ++i) printf("%s%.2f", i > 1 ? ", " : "", d[i].back());
  // spread of workgroup start times
  std::vector<double> starts;
  for (uint32_t b = 0; b < nblocks; ++b) starts.push_back((st[(size_t)b * 8] - t0) * 0.01);
  std::sort(starts.begin(), starts.end());
  printf("], \"start_spread_us\": %.2f}%s", starts.back(), last ? "" : ", ");
}

int main() {
  using namespace cb;
  const uint32_t n = 1u << 20;
  const uint64_t m = 1ull << 27;
  uint4* keys;
  uint32_t *words, *seg, *ent, *dummy;
  CHECK(hipMalloc(&keys, (size_t)n * 16));
  hipLaunchKernelGGL(k_keys, dim3(n / 256), dim3(256), 0, 0, keys, n);
  int mode = 0;
  const ModP mp = make_modp(m, &mode);
  const TilePlan p = plan_build(m, n);
  CHECK(hipMalloc(&words, m / 8));
  CHECK(hipMalloc(&seg, build_seg_bytes(p)));
  CHECK(hipMalloc(&ent, build_ent_bytes(p)));
  CHECK(hipMalloc(&dummy, 64));
  BuildBatch bb{};
  bb.ks[0].bytes = reinterpret_cast<const uint8_t*>(keys);
  bb.ks[0].key_len = 16;
  bb.n[0] = n;
  bb.words[0] = words;
  bb.fresh = 1;
  printf("{\"plan\": {\"tb\": %u, \"T\": %u, \"kpt\": %u, \"C\": %u, \"nblk\": %u}, ",
         p.tb, p.T, p.kpt, p.C, p.nblk);

  const size_t lds1 = ((size_t)((p.T + 4) & ~3u) + 2 * p.C) * 4;
  const size_t lds2 = (size_t)(1u << (p.tb - 5)) * 4;
  allow_lds(k_empty, lds2);
  const float e1 = per_launch_us([&] { hipLaunchKernelGGL(k_empty, dim3(p.nblk), dim3(1024), lds1, 0, dummy); }, 50);
  const float e2 = per_launch_us([&] { hipLaunchKernelGGL(k_empty, dim3(p.T), dim3(1024), lds2, 0, dummy); }, 50);
  const float full = per_launch_us([&] { CHECK(launch_build_batch(KEY_FIXED16, mode, bb, 1, mp, p, seg, ent, 0)); }, 50);
  allow_lds(k_build_tile<16>, lds2);
  allow_lds(k_build_part<KEY_FIXED16, MOD_POW2_32, 4>, lds1);
  auto launch_part = [&] {
    hipLaunchKernelGGL((k_build_part<KEY_FIXED16, MOD_POW2_32, 4>), dim3(p.nblk, 1), dim3(1024), lds1, 0, bb, mp,
                       p.tb, p.T, seg, ent, build_stores());
  };
  const float part = per_launch_us(launch_part, 50);
  const float tile = per_launch_us([&] {
    hipLaunchKernelGGL(k_build_tile<16>, dim3(p.T, 1), dim3(1024), lds2, 0, bb, p.tb, p.T, seg, p.nblk, ent,
                       2 * p.C, build_stores());
  }, 50);
  printf("\"empty_part_grid_us\": %.2f, \"empty_tile_grid_us\": %.2f, \"build_step_us\": %.2f, "
         "\"part_alone_us\": %.2f, \"tile_alone_us\": %.2f, ", e1, e2, full, part, tile);

  uint64_t* st;
  const uint32_t nst_blocks = std::max(p.nblk, p.T);
  CHECK(hipMalloc(&st, (size_t)nst_blocks * 8 * 8));
  CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st)));
  std::vector<uint64_t> h((size_t)nst_blocks * 8);
  CHECK(hipMemset(st, 0, (size_t)nst_blocks * 64));
  launch_part();
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
  phases("part_stamps", h, p.nblk, 6, false);
  CHECK(hipMemset(st, 0, (size_t)nst_blocks * 64));
  hipLaunchKernelGGL(k_build_tile<16>, dim3(p.T, 1), dim3(1024), lds2, 0, bb, p.tb, p.T, seg, p.nblk, ent,
                     2 * p.C, build_stores());
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
  phases("tile_stamps", h, p.T, 5, true);
  printf("}\n");
  return 0;
}
