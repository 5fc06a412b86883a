// zone.hip — ZoneMap bounds of a key batch on gfx950 (see zone.hpp).
//
// Two launches: k_zone_partial (<= 1024 blocks x 256 threads, each thread a
// grid-stride run of keys, then an LDS tree) and k_zone_final (one block over
// the partials). Candidates are key INDICES; a comparison reads both keys'
// bytes (L2-resident after the first pass). Ties keep the smaller index, so
// the result is the first smallest / first largest key, as the reference's
// strict `key < min` / `key > max` updates leave it.
#include <hip/hip_runtime.h>

#include "profile.hpp"
#include "zone.hpp"

namespace cb {
namespace {

constexpr uint64_t kNone = ~0ull;
constexpr uint32_t kZoneThreads = 256;
constexpr uint32_t kZoneMaxBlocks = 1024;

// The better of candidates a and b (min if !MAX else max), ties -> smaller index.
template <int KEYK, bool MAX>
__device__ __forceinline__ uint64_t pick(const KeySrc& ks, uint64_t a, uint64_t b) {
  if (a == kNone) return b;
  if (b == kNone) return a;
  const uint8_t *pa, *pb;
  uint64_t la, lb;
  key_span<KEYK>(ks, a, pa, la);
  key_span<KEYK>(ks, b, pb, lb);
  int c = bytes_cmp(pa, la, pb, lb);
  if (MAX) c = -c;
  if (c != 0) return c < 0 ? a : b;
  return a < b ? a : b;
}

template <int KEYK>
__device__ __forceinline__ void block_pick(const KeySrc& ks, uint64_t& lo, uint64_t& hi) {
  __shared__ uint64_t slo[kZoneThreads], shi[kZoneThreads];
  const uint32_t t = threadIdx.x;
  slo[t] = lo;
  shi[t] = hi;
  __syncthreads();
  for (uint32_t w = kZoneThreads / 2; w > 0; w >>= 1) {
    if (t < w) {
      slo[t] = pick<KEYK, false>(ks, slo[t], slo[t + w]);
      shi[t] = pick<KEYK, true>(ks, shi[t], shi[t + w]);
    }
    __syncthreads();
  }
  lo = slo[0];
  hi = shi[0];
}

template <int KEYK>
__global__ __launch_bounds__(kZoneThreads) void k_zone_partial(KeySrc ks, uint64_t n,
                                                               uint64_t* __restrict__ part) {
  uint64_t lo = kNone, hi = kNone;
  const uint64_t stride = (uint64_t)gridDim.x * kZoneThreads;
  for (uint64_t k = (uint64_t)blockIdx.x * kZoneThreads + threadIdx.x; k < n; k += stride) {
    lo = pick<KEYK, false>(ks, lo, k);
    hi = pick<KEYK, true>(ks, hi, k);
  }
  block_pick<KEYK>(ks, lo, hi);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = lo;
    part[2 * blockIdx.x + 1] = hi;
  }
}

template <int KEYK>
__global__ __launch_bounds__(kZoneThreads) void k_zone_final(KeySrc ks,
                                                             const uint64_t* __restrict__ part,
                                                             uint32_t np, uint64_t* __restrict__ idx) {
  uint64_t lo = kNone, hi = kNone;
  for (uint32_t j = threadIdx.x; j < np; j += kZoneThreads) {
    lo = pick<KEYK, false>(ks, lo, part[2 * j]);
    hi = pick<KEYK, true>(ks, hi, part[2 * j + 1]);
  }
  block_pick<KEYK>(ks, lo, hi);
  if (threadIdx.x == 0) {
    idx[0] = lo;
    idx[1] = hi;
  }
}

template <int KK>
void zone_bounds(const KeySrc& ks, uint64_t n, uint64_t* tmp, uint64_t* idx, hipStream_t s) {
  uint64_t g = (n + kZoneThreads * 8 - 1) / (kZoneThreads * 8);  // >= 8 keys per thread
  const uint32_t grid = (uint32_t)(g < 1 ? 1 : (g > kZoneMaxBlocks ? kZoneMaxBlocks : g));
  hipLaunchKernelGGL((k_zone_partial<KK>), dim3(grid), dim3(kZoneThreads), 0, s, ks, n, tmp);
  hipLaunchKernelGGL((k_zone_final<KK>), dim3(1), dim3(kZoneThreads), 0, s, ks, tmp, grid, idx);
}

}  // namespace

hipError_t launch_zone_bounds(int keyk, const KeySrc& ks, uint64_t n, uint64_t* tmp,
                              uint64_t* idx, hipStream_t s) {
  ProfScope ps("k_zone_bounds", s);
  switch (keyk) {
    case KEY_FIXED16: zone_bounds<KEY_FIXED16>(ks, n, tmp, idx, s); break;
    case KEY_FIXED: zone_bounds<KEY_FIXED>(ks, n, tmp, idx, s); break;
    case KEY_VAR: zone_bounds<KEY_VAR>(ks, n, tmp, idx, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace cb
