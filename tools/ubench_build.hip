// ubench_build.hip — where a build's time goes (2^20
// 16-byte keys -> one 2^27-bit filter; or C4's launch pair of 32 filters). Compiles the library's kernels.hip in
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

// Usage: ubench_build [c2|c4]. c2: one build of 2^20 keys into m = 2^27;
// c4: one launch pair of the C4 batch (32 filters of 2^18 keys, m = 2^25).
int main(int argc, char** argv) {
  using namespace cb;
  const bool c4 = argc > 1 && argv[1][0] == 'c' && argv[1][1] == '4';
  const uint32_t n = c4 ? (1u << 18) : (1u << 20);
  const uint64_t m = c4 ? (1ull << 25) : (1ull << 27);
  const uint32_t nb = c4 ? 32 : 1;
  uint4* keys;
  uint32_t *words, *seg, *ent, *dummy;
  CHECK(hipMalloc(&keys, (size_t)n * nb * 16));
  hipLaunchKernelGGL(k_keys, dim3(n * nb / 256), dim3(256), 0, 0, keys, n * nb);
  int mode = 0;
  const ModP mp = make_modp(m, &mode);
  const TilePlan p = plan_build(m, n, nb);
  CHECK(hipMalloc(&words, m / 8 * nb));
  CHECK(hipMalloc(&seg, build_seg_bytes(p) * nb));
  CHECK(hipMalloc(&ent, build_ent_bytes(p) * nb));
  CHECK(hipMalloc(&dummy, 64));
  BuildBatch bb{};
  for (uint32_t f = 0; f < nb; ++f) {
    bb.ks[f].bytes = reinterpret_cast<const uint8_t*>(keys + (size_t)f * n);
    bb.ks[f].key_len = 16;
    bb.n[f] = n;
    bb.words[f] = words + (size_t)f * (m / 32);
  }
  bb.fresh = nb == 64 ? ~0ull : ((1ull << nb) - 1);
  printf("{\"shape\": \"%s\", \"plan\": {\"tb\": %u, \"T\": %u, \"kpt\": %u, \"C\": %u, \"nblk\": %u, \"nb\": %u, \"sub\": %u}, ",
         c4 ? "c4" : "c2", p.tb, p.T, p.kpt, p.C, p.nblk, nb, p.sub);

  const size_t lds1 = ((size_t)((p.T + 4) & ~3u) + 4 + 2 * p.C) * 4;  // hist, discard word, stage
  const size_t lds2 = (size_t)(1u << (p.tb - 5)) * 4;
  allow_lds(k_empty, lds2 > lds1 ? lds2 : lds1);
  const float e1 = per_launch_us([&] { hipLaunchKernelGGL(k_empty, dim3(p.nblk, nb), dim3(1024), lds1, 0, dummy); }, 50);
  const float e2 = per_launch_us([&] { hipLaunchKernelGGL(k_empty, dim3(p.T, nb), dim3(1024), lds2, 0, dummy); }, 50);
  const float full = per_launch_us([&] { CHECK(launch_build_batch(KEY_FIXED16, mode, bb, nb, mp, p, seg, ent, 0)); }, 50);
  if (p.kpt != 4) {
    fprintf(stderr, "plan kpt %u: this tool times the kpt = 4 partition kernel\n", p.kpt);
    return 1;
  }
  if (p.sub && p.sub != 2) {
    fprintf(stderr, "plan sub %u: this tool times sub = 0 or 2\n", p.sub);
    return 1;
  }
  const size_t lds1s = (size_t)((((p.T << p.sub) + 4) & ~3u) + 4) * 4 + 2 * p.C * 2;
  allow_lds(k_build_part<KEY_FIXED16, MOD_POW2_32, 4>, lds1);
  allow_lds(k_build_part<KEY_FIXED16, MOD_POW2_32, 4, uint16_t>, lds1s);
  allow_lds((k_build_tile_sub<8, 2, 2, 512>), lds2);
  auto launch_part = [&] {  // launch_build_batch's partition
    if (p.sub)
      hipLaunchKernelGGL((k_build_part<KEY_FIXED16, MOD_POW2_32, 4, uint16_t>), dim3(p.nblk, nb), dim3(1024), lds1s, 0,
                         bb, mp, 16u, p.T << p.sub, seg, ent, build_stores());
    else
      hipLaunchKernelGGL((k_build_part<KEY_FIXED16, MOD_POW2_32, 4>), dim3(p.nblk, nb), dim3(1024), lds1, 0, bb, mp,
                         p.tb, p.T, seg, ent, build_stores());
  };
  const bool longruns = 2ull * p.C > 48ull * p.T;  // launch_build_batch's choice
  auto launch_tile = [&] {
    if (p.sub)
      hipLaunchKernelGGL((k_build_tile_sub<8, 2, 2, 512>), dim3(p.T, nb), dim3(512), lds2, 0, bb, p.tb, p.T, seg,
                         p.nblk, reinterpret_cast<const uint16_t*>(ent), 2 * p.C, build_stores());
    else if (longruns)
      hipLaunchKernelGGL((k_build_tile<8, 2>), dim3(p.T, nb), dim3(1024), lds2, 0, bb, p.tb, p.T, seg, p.nblk, ent,
                         2 * p.C, build_stores());
    else
      hipLaunchKernelGGL((k_build_tile<16, 1>), dim3(p.T, nb), dim3(1024), lds2, 0, bb, p.tb, p.T, seg, p.nblk, ent,
                         2 * p.C, build_stores());
  };
  allow_lds(k_build_tile<8, 2>, lds2);
  allow_lds(k_build_tile<16, 1>, lds2);
  const float part = per_launch_us(launch_part, 50);
  const float tile = per_launch_us(launch_tile, 50);
  printf("\"empty_part_grid_us\": %.2f, \"empty_tile_grid_us\": %.2f, \"build_step_us\": %.2f, "
         "\"part_alone_us\": %.2f, \"tile_alone_us\": %.2f, ", e1, e2, full, part, tile);

  uint64_t* st;
  const uint32_t nst_blocks = std::max(p.nblk, p.T) * nb;
  CHECK(hipMalloc(&st, (size_t)nst_blocks * 8 * 8));
  CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st)));
  std::vector<uint64_t> h((size_t)nst_blocks * 8);
  CHECK(hipMemset(st, 0, (size_t)nst_blocks * 64));
  launch_part();
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
  phases("part_stamps", h, p.nblk * nb, 6, false);
  CHECK(hipMemset(st, 0, (size_t)nst_blocks * 64));
  launch_tile();
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
  phases("tile_stamps", h, p.T * nb, 5, true);
  printf("}\n");
  return 0;
}
