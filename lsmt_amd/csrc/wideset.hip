// wideset.hip — wide bit-sliced filter sets (wideset.hpp): set maintenance
// and the hit-row probe for more than 64 slots. The fused read path over a
// wide set (Database::get in one launch) is k_wide_get_many in sstable.hip.
#include <hip/hip_runtime.h>

#include "profile.hpp"
#include "wideset.hpp"

namespace cb {
namespace {

// In-register 32x32 bit transpose (a[i] bit j -> a[j] bit i).
template <int J>
__device__ __forceinline__ void tstep(uint32_t (&a)[32]) {
  constexpr uint32_t m = J == 16 ? 0x0000FFFFu
                         : J == 8 ? 0x00FF00FFu
                         : J == 4 ? 0x0F0F0F0Fu
                         : J == 2 ? 0x33333333u
                                  : 0x55555555u;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    if ((k & J) == 0) {
      const uint32_t t = ((a[k] >> J) ^ a[k | J]) & m;
      a[k] ^= t << J;
      a[k | J] ^= t;
    }
  }
}
__device__ __forceinline__ void transpose32(uint32_t (&a)[32]) {
  tstep<16>(a);
  tstep<8>(a);
  tstep<4>(a);
  tstep<2>(a);
  tstep<1>(a);
}

// One item per (32-position group g, slot word j), j fastest so a warp's
// stores fill whole rows: word g of filters 64 j .. 64 j + 63, transposed into
// the 32 rows' word j.
__global__ __launch_bounds__(256) void k_wide_build(const uint32_t* const* __restrict__ fw, uint32_t nf,
                                                    uint64_t ngroups, uint64_t m, uint32_t R,
                                                    uint64_t* __restrict__ set) {
  const uint64_t items = ngroups * R, stride = (uint64_t)gridDim.x * 256;
  for (uint64_t it = (uint64_t)blockIdx.x * 256 + threadIdx.x; it < items; it += stride) {
    const uint64_t g = it / R;
    const uint32_t j = (uint32_t)(it - g * R);
    uint32_t a[32], c[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const uint32_t f0 = 64 * j + i, f1 = f0 + 32;
      a[i] = f0 < nf ? fw[f0][g] : 0u;
      c[i] = f1 < nf ? fw[f1][g] : 0u;
    }
    transpose32(a);
    transpose32(c);
    const uint64_t p0 = g * 32;
    const uint32_t valid = (uint32_t)min<uint64_t>(32, m - p0);
#pragma unroll
    for (int q = 0; q < 32; ++q)
      if ((uint32_t)q < valid) set[(p0 + q) * R + j] = (uint64_t)a[q] | (uint64_t)c[q] << 32;
  }
}

// slot |= filter, slot known all-zero: only the filter's set bits touch the
// set. Position p belongs to one thread (the owner of filter word p / 32).
__global__ __launch_bounds__(256) void k_wide_or_slot(const uint32_t* __restrict__ words, uint64_t nwords,
                                                      uint32_t slot, uint32_t R, uint64_t* __restrict__ set) {
  const uint64_t stride = (uint64_t)gridDim.x * 256, bit = 1ull << (slot & 63);
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < nwords; w += stride) {
    uint32_t v = words[w];
    while (v) {
      const uint32_t b = __builtin_ctz(v);
      v &= v - 1;
      set[(w * 32 + b) * R + (slot >> 6)] |= bit;
    }
  }
}

// slot := filter (words == nullptr: cleared), every row.
__global__ __launch_bounds__(256) void k_wide_put_slot(const uint32_t* __restrict__ words, uint64_t m,
                                                       uint32_t slot, uint32_t R, uint64_t* __restrict__ set) {
  const uint64_t stride = (uint64_t)gridDim.x * 256, bit = 1ull << (slot & 63);
  for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < m; p += stride) {
    const bool on = words ? ((words[p >> 5] >> (p & 31)) & 1u) : false;
    uint64_t* w = set + p * R + (slot >> 6);
    *w = on ? (*w | bit) : (*w & ~bit);
  }
}

// Hit rows of a wide set: one key per lane, one 64-key hit word per wave, 16
// waves per block (as k_set_probe). For each 64-slot word j of the rows: row
// a's word, row b's word only where a's is non-zero (the reference's `&&`,
// src/bloom.rs:50), the zone gate on the gated candidates, then 64 ballots
// give lane f slot 64 j + f's hit word, staged in LDS so each row leaves as
// one 128-B segment.
constexpr uint32_t kWideWaves = 16, kWideNT = 64 * kWideWaves;
template <int KEYK, int MODE>
__global__ __launch_bounds__(kWideNT) void k_wide_probe(const uint64_t* __restrict__ set, uint32_t R, uint32_t used,
                                                        KeySrc ks, uint64_t n, ModP mp, WideZone z,
                                                        uint64_t* __restrict__ hits, uint64_t hwords) {
  __shared__ uint64_t hb[64][kWideWaves];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t wbase = (uint64_t)blockIdx.x * kWideWaves;
  const uint64_t k = (wbase + wave) * 64 + lane;
  const bool live = k < n;
  uint64_t pa = 0, pb = 0;
  if (live) key_positions<KEYK, MODE>(ks, k, mp, pa, pb);
  const uint64_t* ra = set + pa * R;
  const uint64_t* rb = set + pb * R;
  uint32_t kw[4] = {0, 0, 0, 0};
  const uint8_t* kp = nullptr;
  uint64_t kl = 0;
  if (z.any && live) {
    key_span<KEYK>(ks, k, kp, kl);
    if constexpr (KEYK == KEY_FIXED16) {
      const uint4 v = reinterpret_cast<const uint4*>(ks.bytes)[k];
      kw[0] = be32(v.x);
      kw[1] = be32(v.y);
      kw[2] = be32(v.z);
      kw[3] = be32(v.w);
    }
  }
  const uint64_t nw = (n + 63) / 64;
  const uint32_t nj = (used + 63) / 64;
  uint64_t va_next = live ? ra[0] : 0ull;
  for (uint32_t j = 0; j < nj; ++j) {
    const uint64_t va = va_next;
    if (j + 1 < nj) va_next = live ? ra[j + 1] : 0ull;  // the next word's load in flight
    uint64_t mask = va ? (va & rb[j]) : 0ull;
    if (z.any && mask) {
      uint64_t c = mask & z.gbits[j];
      while (c) {
        const uint32_t i = (uint32_t)__builtin_ctzll(c);
        c &= c - 1;
        if (!wide_zone_ok<KEYK>(z, 64 * j + i, kw, kp, kl)) mask &= ~(1ull << i);
      }
    }
    const uint32_t fn = used - 64 * j < 64 ? used - 64 * j : 64;
    uint64_t mine = 0;
    for (uint32_t f = 0; f < fn; ++f) {
      const uint64_t bal = __ballot((mask >> f) & 1ull);
      mine = lane == f ? bal : mine;
    }
    __syncthreads();  // the previous word's rows have left hb
    if (lane < fn) hb[lane][wave] = mine;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < fn * kWideWaves; i += kWideNT) {
      const uint32_t f = i / kWideWaves, w = i % kWideWaves;
      if (wbase + w < nw) hits[(uint64_t)(64 * j + f) * hwords + wbase + w] = hb[f][w];
    }
  }
}

inline uint32_t grid_cap(uint64_t items, uint32_t cap) {
  uint64_t g = (items + 255) / 256;
  if (g < 1) g = 1;
  return (uint32_t)(g < cap ? g : cap);
}

}  // namespace

hipError_t launch_wide_build(const uint32_t* const* fw, uint32_t nf, uint64_t m, uint32_t R, uint64_t* set,
                             hipStream_t s) {
  if (!m) return hipSuccess;
  if (!R || R > kWideMax / 64 || nf > 64 * R) return hipErrorInvalidValue;
  const uint64_t ng = (m + 31) / 32;
  ProfScope ps("k_wide_build", s);
  hipLaunchKernelGGL(k_wide_build, dim3(grid_cap(ng * R, 16384)), dim3(256), 0, s, fw, nf, ng, m, R, set);
  return hipGetLastError();
}

hipError_t launch_wide_or_slot(const uint32_t* words, uint64_t m, uint32_t slot, uint32_t R, uint64_t* set,
                               hipStream_t s) {
  if (!m) return hipSuccess;
  if (slot >= 64 * R) return hipErrorInvalidValue;
  const uint64_t nw = (m + 31) / 32;
  ProfScope ps("k_wide_or_slot", s);
  hipLaunchKernelGGL(k_wide_or_slot, dim3(grid_cap(nw, 8192)), dim3(256), 0, s, words, nw, slot, R, set);
  return hipGetLastError();
}

hipError_t launch_wide_put_slot(const uint32_t* words, uint64_t m, uint32_t slot, uint32_t R, uint64_t* set,
                                hipStream_t s) {
  if (!m) return hipSuccess;
  if (slot >= 64 * R) return hipErrorInvalidValue;
  ProfScope ps("k_wide_put_slot", s);
  hipLaunchKernelGGL(k_wide_put_slot, dim3(grid_cap(m, 8192)), dim3(256), 0, s, words, m, slot, R, set);
  return hipGetLastError();
}

hipError_t launch_wide_probe(int keyk, int mode, uint32_t R, const uint64_t* set, uint32_t used, const KeySrc& ks,
                             uint64_t n, const ModP& mp, const WideZone* zones, uint64_t* hits, uint64_t hwords,
                             hipStream_t s) {
  if (!n || !used) return hipSuccess;
  if (used > 64 * R) return hipErrorInvalidValue;
  const WideZone z = zones ? *zones : WideZone{nullptr, nullptr, nullptr, nullptr, 0};
  const dim3 g((uint32_t)(((n + 63) / 64 + kWideWaves - 1) / kWideWaves));
  ProfScope ps("k_wide_probe", s);
#define WP(KK, MM) hipLaunchKernelGGL((k_wide_probe<KK, MM>), g, dim3(kWideNT), 0, s, set, R, used, ks, n, mp, z, hits, hwords)
  switch (keyk * 3 + mode) {
    case 0: WP(KEY_FIXED16, MOD_POW2_32); break;
    case 1: WP(KEY_FIXED16, MOD_POW2_64); break;
    case 2: WP(KEY_FIXED16, MOD_GENERIC); break;
    case 3: WP(KEY_FIXED, MOD_POW2_32); break;
    case 4: WP(KEY_FIXED, MOD_POW2_64); break;
    case 5: WP(KEY_FIXED, MOD_GENERIC); break;
    case 6: WP(KEY_VAR, MOD_POW2_32); break;
    case 7: WP(KEY_VAR, MOD_POW2_64); break;
    case 8: WP(KEY_VAR, MOD_GENERIC); break;
    default: return hipErrorInvalidValue;
  }
#undef WP
  return hipGetLastError();
}

}  // namespace cb
