// kernels.hip — gfx950 kernels for the Bloom-filter build and probe paths.
//
// Reference semantics: /root/reference/src/bloom.rs:26-51 (hashes / insert /
// may_contain). Filter layout in HBM: packed uint32 words, bit p at word p>>5,
// bit p&31 (LSB-first).
//
// Two paths per operation:
//   direct — one lane per key: hash, then global atomicOr (build) or word
//            gathers (probe). Latency-optimal for small batches.
//   tiled  — partition the batch by filter tile (k_part_*), then one
//            workgroup per tile stages the tile in LDS (k_tile_*): build ORs
//            bits with ds_or and writes the tile back coalesced; probe streams
//            each filter's tile through LDS, tests bit a from LDS, and reads
//            bit b from HBM only when bit a is set (the reference's `&&`
//            short-circuit, src/bloom.rs:50). Results leave as wave64 ballots.
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "profile.hpp"

namespace cb {

namespace {

constexpr uint32_t kBlock = 256;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// Exclusive scan of arr[0..len) in LDS by the whole 256-thread block; returns
// the total. wsum: 4 words of LDS scratch. Contains barriers: all threads call.
__device__ uint32_t block_exclusive_scan(uint32_t* arr, uint32_t len, uint32_t* wsum) {
  const uint32_t tid = threadIdx.x, lane = lane_id(), wid = tid >> 6;
  const uint32_t per = (len + kBlock - 1) / kBlock;
  const uint32_t beg = min(tid * per, len), end = min(beg + per, len);
  uint32_t s = 0;
  for (uint32_t i = beg; i < end; ++i) s += arr[i];
  uint32_t x = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  uint32_t wpre = 0, total = 0;
#pragma unroll
  for (uint32_t w = 0; w < kBlock / 64; ++w) {
    const uint32_t v = wsum[w];
    wpre += (w < wid) ? v : 0u;
    total += v;
  }
  uint32_t run = wpre + x - s;
  for (uint32_t i = beg; i < end; ++i) {
    const uint32_t v = arr[i];
    arr[i] = run;
    run += v;
  }
  __syncthreads();
  return total;
}

// Segment bookkeeping shared by the tile kernels. For tile t, partition block
// b wrote its entries for t at ent[b*estride + S[b] .. + cnt_b). After the
// scan, P[b] is the exclusive prefix of cnt over b ("tile order").
__device__ __forceinline__ uint32_t seg_find(const uint32_t* P, uint32_t nblk, uint32_t j) {
  uint32_t lo = 0, hi = nblk;  // first b with P[b] > j, minus one
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (P[mid] <= j)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo - 1;
}

// ---------------------------------------------------------------- direct ---

template <int KEYK, int MODE>
__global__ __launch_bounds__(kBlock) void k_insert_direct(uint32_t* __restrict__ words, KeySrc ks,
                                                          uint64_t n, ModP mp) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x; k < n; k += stride) {
    uint64_t a, b;
    key_positions<KEYK, MODE>(ks, k, mp, a, b);
    atomicOr(&words[a >> 5], 1u << (a & 31));  // src/bloom.rs:42
    atomicOr(&words[b >> 5], 1u << (b & 31));  // src/bloom.rs:43
  }
}

// One wave handles 64 consecutive keys (one hits word per filter). Lane f
// collects the ballot for filter f and stores it: one store per wave.
template <int KEYK, int MODE>
__global__ __launch_bounds__(kBlock) void k_probe_direct(FilterPtrs fp, uint32_t nf, KeySrc ks,
                                                         uint64_t n, ModP mp,
                                                         uint64_t* __restrict__ hits,
                                                         uint64_t hwords) {
  const uint32_t lane = lane_id();
  const uint64_t nwaves = ((uint64_t)gridDim.x * kBlock) >> 6;
  for (uint64_t wv = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; wv < hwords;
       wv += nwaves) {
    const uint64_t k = wv * 64 + lane;
    const bool valid = k < n;
    uint64_t a = 0, b = 0;
    if (valid) key_positions<KEYK, MODE>(ks, k, mp, a, b);
    const uint64_t wa = a >> 5, wb = b >> 5;
    const uint32_t sa = (uint32_t)(a & 31), sb = (uint32_t)(b & 31);
    uint64_t mine = 0;
    for (uint32_t f0 = 0; f0 < nf; f0 += 8) {
      uint32_t va[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        va[i] = (valid && f0 + i < nf) ? fp.w[f0 + i][wa] : 0u;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        bool hit = false;
        if ((va[i] >> sa) & 1u) hit = (fp.w[f0 + i][wb] >> sb) & 1u;  // `&&` short-circuit
        const uint64_t bal = __ballot(hit);
        if (lane == f0 + i) mine = bal;
      }
    }
    if (lane < nf) hits[(uint64_t)fp.row[lane] * hwords + wv] = mine;
  }
}

// ---------------------------------------------------------------- tiled ----

// Partition for build: every key contributes two entries (bit a, bit b), each
// bucketed by its tile. Per block: LDS histogram with ranks, block scan,
// LDS staging in tile order, coalesced write of the block's run.
template <int KEYK, int MODE, int KPT>
__global__ __launch_bounds__(kBlock) void k_part_build(KeySrc ks, uint64_t n, ModP mp, uint32_t tb,
                                                       uint32_t T, uint32_t* __restrict__ seg,
                                                       uint32_t nblk, uint32_t* __restrict__ ent) {
  constexpr uint32_t C = kBlock * KPT;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t Tp = (T + 4) & ~3u;
  uint32_t* hist = smem;
  uint32_t* stage = smem + Tp;
  uint32_t* wsum = stage + 2 * C;
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < Tp; i += kBlock) hist[i] = 0;
  __syncthreads();

  const uint64_t kbase = (uint64_t)blockIdx.x * C;
  const uint32_t tmask = (1u << tb) - 1u;
  uint32_t et[2 * KPT], er[2 * KPT], eo[2 * KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint64_t k = kbase + (uint64_t)j * kBlock + tid;
    et[2 * j] = et[2 * j + 1] = 0xFFFFFFFFu;
    if (k < n) {
      uint64_t a, b;
      key_positions<KEYK, MODE>(ks, k, mp, a, b);
      const uint32_t ta = (uint32_t)(a >> tb), tbb = (uint32_t)(b >> tb);
      et[2 * j] = ta;
      eo[2 * j] = (uint32_t)a & tmask;
      er[2 * j] = atomicAdd(&hist[ta], 1u);
      et[2 * j + 1] = tbb;
      eo[2 * j + 1] = (uint32_t)b & tmask;
      er[2 * j + 1] = atomicAdd(&hist[tbb], 1u);
    }
  }
  __syncthreads();
  const uint32_t total = block_exclusive_scan(hist, T, wsum);
  if (tid == 0) hist[T] = total;
  __syncthreads();
  for (uint32_t t = tid; t <= T; t += kBlock) seg[(size_t)t * nblk + blockIdx.x] = hist[t];
#pragma unroll
  for (int e = 0; e < 2 * KPT; ++e)
    if (et[e] != 0xFFFFFFFFu) stage[hist[et[e]] + er[e]] = eo[e];
  __syncthreads();
  uint32_t* out = ent + (size_t)blockIdx.x * (2 * C);
  for (uint32_t i = tid; i < total; i += kBlock) out[i] = stage[i];
}

// One workgroup per tile: stage the tile in LDS (zeros if the filter is known
// empty), OR in every entry of the tile with LDS atomics, write it back.
__global__ __launch_bounds__(kBlock) void k_tile_build(uint32_t* __restrict__ words, uint32_t tb,
                                                       uint32_t T,
                                                       const uint32_t* __restrict__ seg,
                                                       uint32_t nblk,
                                                       const uint32_t* __restrict__ ent,
                                                       uint32_t estride, int fresh) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t tw = 1u << (tb - 5);
  const uint32_t nbp = (nblk + 3) & ~3u;
  uint32_t* tile = smem;
  uint32_t* P = tile + tw;
  uint32_t* S = P + nbp;
  uint32_t* wsum = S + nbp;
  const uint32_t tid = threadIdx.x;
  const uint32_t t = blockIdx.x;

  uint4* gt = reinterpret_cast<uint4*>(words + (size_t)t * tw);
  uint4* lt = reinterpret_cast<uint4*>(tile);
  for (uint32_t i = tid; i < tw / 4; i += kBlock) lt[i] = fresh ? make_uint4(0, 0, 0, 0) : gt[i];
  for (uint32_t b = tid; b < nblk; b += kBlock) {
    const uint32_t s0 = seg[(size_t)t * nblk + b], s1 = seg[(size_t)(t + 1) * nblk + b];
    S[b] = s0;
    P[b] = s1 - s0;
  }
  __syncthreads();
  const uint32_t E = block_exclusive_scan(P, nblk, wsum);
  const uint32_t per = (E + kBlock - 1) / kBlock;
  const uint32_t j0 = min(tid * per, E), j1 = min(j0 + per, E);
  if (j0 < j1) {
    uint32_t b = seg_find(P, nblk, j0);
    uint32_t pnext = (b + 1 < nblk) ? P[b + 1] : E;
    for (uint32_t j = j0; j < j1; ++j) {
      while (j >= pnext) {
        ++b;
        pnext = (b + 1 < nblk) ? P[b + 1] : E;
      }
      const uint32_t off = ent[(size_t)b * estride + S[b] + (j - P[b])];
      atomicOr(&tile[off >> 5], 1u << (off & 31));
    }
  }
  __syncthreads();
  for (uint32_t i = tid; i < tw / 4; i += kBlock) gt[i] = lt[i];
}

// Partition for probe: one entry per key, bucketed by the tile of bit a. The
// entry carries (offset of a in its tile, b, key index, b >> 32).
template <int KEYK, int MODE, int KPT>
__global__ __launch_bounds__(kBlock) void k_part_probe(KeySrc ks, uint64_t n, ModP mp, uint32_t tb,
                                                       uint32_t T, uint32_t* __restrict__ seg,
                                                       uint32_t nblk, uint4* __restrict__ ent) {
  constexpr uint32_t C = kBlock * KPT;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t Tp = (T + 4) & ~3u;
  uint32_t* hist = smem;
  uint4* stage = reinterpret_cast<uint4*>(smem + Tp);
  uint32_t* wsum = reinterpret_cast<uint32_t*>(stage + C);
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < Tp; i += kBlock) hist[i] = 0;
  __syncthreads();

  const uint64_t kbase = (uint64_t)blockIdx.x * C;
  const uint32_t tmask = (1u << tb) - 1u;
  uint32_t et[KPT], er[KPT];
  uint4 rec[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint64_t k = kbase + (uint64_t)j * kBlock + tid;
    et[j] = 0xFFFFFFFFu;
    if (k < n) {
      uint64_t a, b;
      key_positions<KEYK, MODE>(ks, k, mp, a, b);
      et[j] = (uint32_t)(a >> tb);
      er[j] = atomicAdd(&hist[et[j]], 1u);
      rec[j] = make_uint4((uint32_t)a & tmask, (uint32_t)b, (uint32_t)k, (uint32_t)(b >> 32));
    }
  }
  __syncthreads();
  const uint32_t total = block_exclusive_scan(hist, T, wsum);
  if (tid == 0) hist[T] = total;
  __syncthreads();
  for (uint32_t t = tid; t <= T; t += kBlock) seg[(size_t)t * nblk + blockIdx.x] = hist[t];
#pragma unroll
  for (int j = 0; j < KPT; ++j)
    if (et[j] != 0xFFFFFFFFu) stage[hist[et[j]] + er[j]] = rec[j];
  __syncthreads();
  uint4* out = ent + (size_t)blockIdx.x * C;
  for (uint32_t i = tid; i < total; i += kBlock) out[i] = stage[i];
}

// Probe one tile against up to 32 filters (group blockIdx.y). Each filter's
// tile is streamed HBM -> registers -> LDS, double-buffered so the next
// filter's loads are in flight while the current tile is tested. Bit a is
// tested in LDS; bit b is gathered from HBM only for (key, filter) pairs whose
// bit a was set. Output: masks[g*n + key] = per-filter result bits.
template <int EPT>
__global__ __launch_bounds__(kBlock) void k_tile_probe(FilterPtrs fp, uint32_t nf, uint32_t tb,
                                                       const uint32_t* __restrict__ seg,
                                                       uint32_t nblk, const uint4* __restrict__ ent,
                                                       uint32_t estride, uint64_t n,
                                                       uint32_t* __restrict__ masks) {
  constexpr uint32_t RPT = 8;  // uint4 per thread per tile: tiles up to 2^18 bits
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t tw = 1u << (tb - 5);
  const uint32_t nbp = (nblk + 3) & ~3u;
  uint32_t* buf = smem;  // 2 * tw
  uint32_t* P = buf + 2 * tw;
  uint32_t* S = P + nbp;
  uint32_t* wsum = S + nbp;
  const uint32_t** fw = reinterpret_cast<const uint32_t**>(wsum + 4);  // 32 pointers
  const uint32_t tid = threadIdx.x;
  const uint32_t t = blockIdx.x, g = blockIdx.y;
  const uint32_t f0 = g * kFiltersPerGroup;
  const uint32_t nfg = min(kFiltersPerGroup, nf - f0);
  if (tid < nfg) fw[tid] = fp.w[f0 + tid];

  for (uint32_t b = tid; b < nblk; b += kBlock) {
    const uint32_t s0 = seg[(size_t)t * nblk + b], s1 = seg[(size_t)(t + 1) * nblk + b];
    S[b] = s0;
    P[b] = s1 - s0;
  }
  __syncthreads();
  const uint32_t E = block_exclusive_scan(P, nblk, wsum);
  const uint32_t q = tw / 4;  // uint4 per tile
  uint32_t* mg = masks + (size_t)g * n;

  for (uint32_t cbase = 0; cbase < E; cbase += kBlock * EPT) {
    const uint32_t cn = min(E - cbase, kBlock * EPT);
    const uint32_t per = (cn + kBlock - 1) / kBlock;
    const uint32_t j0 = cbase + min(tid * per, cn);
    const uint32_t cnt = cbase + min(tid * per + per, cn) - j0;
    uint32_t off[EPT], pb[EPT], kk[EPT], am[EPT];
    {
      uint32_t b = cnt ? seg_find(P, nblk, j0) : 0;
      uint32_t pnext = (b + 1 < nblk) ? P[b + 1] : E;
#pragma unroll
      for (int i = 0; i < EPT; ++i) {
        am[i] = 0;
        if ((uint32_t)i < cnt) {
          const uint32_t j = j0 + i;
          while (j >= pnext) {
            ++b;
            pnext = (b + 1 < nblk) ? P[b + 1] : E;
          }
          const uint4 r = ent[(size_t)b * estride + S[b] + (j - P[b])];
          off[i] = r.x;
          pb[i] = r.y;
          kk[i] = r.z;
        }
      }
    }

    uint4 pre[RPT];
    {
      const uint4* src = reinterpret_cast<const uint4*>(fw[0] + (size_t)t * tw);
#pragma unroll
      for (uint32_t r = 0; r < RPT; ++r)
        if (tid + r * kBlock < q) pre[r] = src[tid + r * kBlock];
    }
    for (uint32_t f = 0; f < nfg; ++f) {
      uint4* dst = reinterpret_cast<uint4*>(buf + (f & 1) * tw);
#pragma unroll
      for (uint32_t r = 0; r < RPT; ++r)
        if (tid + r * kBlock < q) dst[tid + r * kBlock] = pre[r];
      __syncthreads();
      if (f + 1 < nfg) {
        const uint4* src = reinterpret_cast<const uint4*>(fw[f + 1] + (size_t)t * tw);
#pragma unroll
        for (uint32_t r = 0; r < RPT; ++r)
          if (tid + r * kBlock < q) pre[r] = src[tid + r * kBlock];
      }
      const uint32_t* lb = buf + (f & 1) * tw;
#pragma unroll
      for (int i = 0; i < EPT; ++i)
        if ((uint32_t)i < cnt) am[i] |= ((lb[off[i] >> 5] >> (off[i] & 31)) & 1u) << f;
    }
    __syncthreads();  // buffers are reused by the next chunk

#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      if ((uint32_t)i < cnt) {
        uint32_t mask = 0, x = am[i];
        const uint32_t wb = pb[i] >> 5, sb = pb[i] & 31;
        while (x) {
          const uint32_t f = __builtin_ctz(x);
          x &= x - 1;
          mask |= ((fw[f][wb] >> sb) & 1u) << f;
        }
        mg[kk[i]] = mask;
      }
    }
  }
}

// Transpose per-key masks into the [filter][n/64] hit bitmaps with wave64
// ballots: wave w owns keys [64w, 64w+64), lane f stores filter f's word.
__global__ __launch_bounds__(kBlock) void k_masks_to_hits(const uint32_t* __restrict__ masks,
                                                          FilterPtrs fp, uint32_t nf, uint64_t n,
                                                          uint64_t* __restrict__ hits,
                                                          uint64_t hwords) {
  const uint32_t lane = lane_id();
  const uint64_t nwaves = ((uint64_t)gridDim.x * kBlock) >> 6;
  const uint64_t nw = (n + 63) / 64;
  for (uint64_t wv = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; wv < nw; wv += nwaves) {
    const uint64_t k = wv * 64 + lane;
    uint64_t mine = 0;
    for (uint32_t g = 0; g * kFiltersPerGroup < nf; ++g) {
      const uint32_t mask = k < n ? masks[(size_t)g * n + k] : 0u;
      const uint32_t nfg = min(kFiltersPerGroup, nf - g * kFiltersPerGroup);
      for (uint32_t f = 0; f < nfg; ++f) {
        const uint64_t bal = __ballot((mask >> f) & 1u);
        if (lane == g * kFiltersPerGroup + f) mine = bal;
      }
    }
    if (lane < nf) hits[(uint64_t)fp.row[lane] * hwords + wv] = mine;
  }
}

// ------------------------------------------------------------- codecs ------

// packed words -> m bytes of 0/1 (the Vec<bool> layout). Thread per word.
__global__ __launch_bounds__(kBlock) void k_export_bools(const uint32_t* __restrict__ words,
                                                         uint64_t m, uint8_t* __restrict__ out) {
  const uint64_t nw = (m + 31) / 32;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < nw; w += stride) {
    const uint32_t v = words[w];
    const uint64_t p0 = w * 32;
    if (p0 + 32 <= m && !(reinterpret_cast<uintptr_t>(out + p0) & 15)) {
      uint32_t o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t nib = (v >> (4 * i)) & 15u;
        o[i] = (nib & 1u) | ((nib & 2u) << 7) | ((nib & 4u) << 14) | ((nib & 8u) << 21);
      }
      uint4* dst = reinterpret_cast<uint4*>(out + p0);
      dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
      dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
    } else {
      for (uint64_t p = p0; p < m && p < p0 + 32; ++p) out[p] = (v >> (p - p0)) & 1u;
    }
  }
}

// m bytes (nonzero = set) -> packed words; bits >= m are cleared.
__global__ __launch_bounds__(kBlock) void k_import_bools(uint32_t* __restrict__ words, uint64_t m,
                                                         const uint8_t* __restrict__ in) {
  const uint64_t nw = (m + 31) / 32;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < nw; w += stride) {
    const uint64_t p0 = w * 32;
    uint32_t v = 0;
    if (p0 + 32 <= m && !(reinterpret_cast<uintptr_t>(in + p0) & 15)) {
      const uint4* src = reinterpret_cast<const uint4*>(in + p0);
      const uint4 x0 = src[0], x1 = src[1];
      const uint32_t xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t x = xs[i];
        const uint32_t nib = ((x & 0xFFu) != 0) | (((x >> 8) & 0xFFu) != 0) << 1 |
                             (((x >> 16) & 0xFFu) != 0) << 2 | ((x >> 24) != 0) << 3;
        v |= nib << (4 * i);
      }
    } else {
      for (uint64_t p = p0; p < m && p < p0 + 32; ++p) v |= (uint32_t)(in[p] != 0) << (p - p0);
    }
    words[w] = v;
  }
}

// Clears the bits >= m of the last word (packed imports must not carry bits
// the reference's Vec<bool> of length m cannot hold).
__global__ void k_mask_tail(uint32_t* words, uint64_t m) {
  if (threadIdx.x == 0) words[m >> 5] &= (1u << (m & 31)) - 1u;
}

// Instantiates CALL for the (key source, modulo mode) pair with KK / MM bound
// as compile-time constants.
#define CB_DISPATCH(keyk, mode, CALL)                                  \
  switch ((keyk) * 3 + (mode)) {                                       \
    case 0: { constexpr int KK = KEY_FIXED16, MM = MOD_POW2_32; CALL; } break; \
    case 1: { constexpr int KK = KEY_FIXED16, MM = MOD_POW2_64; CALL; } break; \
    case 2: { constexpr int KK = KEY_FIXED16, MM = MOD_GENERIC; CALL; } break; \
    case 3: { constexpr int KK = KEY_FIXED, MM = MOD_POW2_32; CALL; } break;   \
    case 4: { constexpr int KK = KEY_FIXED, MM = MOD_POW2_64; CALL; } break;   \
    case 5: { constexpr int KK = KEY_FIXED, MM = MOD_GENERIC; CALL; } break;   \
    case 6: { constexpr int KK = KEY_VAR, MM = MOD_POW2_32; CALL; } break;     \
    case 7: { constexpr int KK = KEY_VAR, MM = MOD_POW2_64; CALL; } break;     \
    case 8: { constexpr int KK = KEY_VAR, MM = MOD_GENERIC; CALL; } break;     \
    default: return hipErrorInvalidValue;                              \
  }

inline uint32_t grid_for(uint64_t items, uint32_t cap = 2048) {
  uint64_t g = (items + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  return (uint32_t)(g < cap ? g : cap);
}

template <class K>
inline void allow_lds(K kernel, size_t bytes) {
  if (bytes > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

inline uint32_t ilog2_floor(uint64_t x) { return 63u - (uint32_t)__builtin_clzll(x); }
inline uint32_t ilog2_ceil(uint64_t x) { return x <= 1 ? 0 : ilog2_floor(x - 1) + 1; }

}  // namespace

// ------------------------------------------------------------- plans -------

static uint32_t clamp_u32(int64_t v, int64_t lo, int64_t hi) {
  return (uint32_t)(v < lo ? lo : (v > hi ? hi : v));
}

TilePlan plan_build(uint64_t m, uint64_t n) {
  TilePlan p{};
  // ~512 tiles (2 workgroups per CU), tiles within [2^12, 2^18] bits, T <= 4096.
  int64_t tb = (int64_t)ilog2_floor(m > 512 ? m / 512 : 1);
  tb = clamp_u32(tb, kMinTileBits, kMaxTileBits);
  if (((m + (1ull << tb) - 1) >> tb) > kMaxTiles) tb = ilog2_ceil((m + kMaxTiles - 1) / kMaxTiles);
  p.tb = (uint32_t)tb;
  p.T = (uint32_t)((m + (1ull << tb) - 1) >> tb);
  p.kpt = 4;
  while (p.kpt < 16 && (n + 256ull * p.kpt - 1) / (256ull * p.kpt) > 2048) p.kpt *= 2;
  p.C = 256 * p.kpt;
  p.nblk = (uint32_t)((n + p.C - 1) / p.C);
  return p;
}

TilePlan plan_probe(uint64_t m, uint64_t n) {
  TilePlan p{};
  // ~512 tiles, and about <= 4096 entries (16 per thread) per tile.
  int64_t tb1 = (int64_t)ilog2_floor(m > 512 ? m / 512 : 1);
  const uint64_t want = n ? (m * 4096ull) / n : m;
  int64_t tb2 = (int64_t)ilog2_floor(want ? want : 1);
  int64_t tb = clamp_u32(tb1 < tb2 ? tb1 : tb2, kMinTileBits, kMaxTileBits);
  if (((m + (1ull << tb) - 1) >> tb) > kMaxTiles) tb = ilog2_ceil((m + kMaxTiles - 1) / kMaxTiles);
  p.tb = (uint32_t)tb;
  p.T = (uint32_t)((m + (1ull << tb) - 1) >> tb);
  p.kpt = 4;
  while (p.kpt < 8 && (n + 256ull * p.kpt - 1) / (256ull * p.kpt) > 2048) p.kpt *= 2;
  p.C = 256 * p.kpt;
  p.nblk = (uint32_t)((n + p.C - 1) / p.C);
  return p;
}

size_t build_seg_bytes(const TilePlan& p) { return (size_t)(p.T + 1) * p.nblk * 4; }
size_t build_ent_bytes(const TilePlan& p) { return (size_t)p.nblk * 2 * p.C * 4; }
size_t probe_seg_bytes(const TilePlan& p) { return (size_t)(p.T + 1) * p.nblk * 4; }
size_t probe_ent_bytes(const TilePlan& p) { return (size_t)p.nblk * p.C * 16; }

// ------------------------------------------------------------- launchers ---

hipError_t launch_insert_direct(int keyk, int mode, uint32_t* words, const KeySrc& ks, uint64_t n,
                                const ModP& mp, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint32_t grid = grid_for(n);
  ProfScope ps("k_insert_direct", s);
  CB_DISPATCH(keyk, mode,
              hipLaunchKernelGGL((k_insert_direct<KK, MM>), dim3(grid), dim3(kBlock), 0, s, words,
                                 ks, n, mp));
  return hipGetLastError();
}

hipError_t launch_probe_direct(int keyk, int mode, const FilterPtrs& fp, uint32_t nf,
                               const KeySrc& ks, uint64_t n, const ModP& mp, uint64_t* hits,
                               uint64_t hwords, hipStream_t s) {
  if (!n || !nf) return hipSuccess;
  const uint64_t nw = (n + 63) / 64;
  const uint32_t grid = grid_for(nw * 64, 4096);
  ProfScope ps("k_probe_direct", s);
  CB_DISPATCH(keyk, mode,
              hipLaunchKernelGGL((k_probe_direct<KK, MM>), dim3(grid), dim3(kBlock), 0, s, fp, nf,
                                 ks, n, mp, hits, hwords));
  return hipGetLastError();
}

template <int KK, int MM, int KPT>
static void part_build(const TilePlan& p, const KeySrc& ks, uint64_t n, const ModP& mp,
                       uint32_t* seg, uint32_t* ent, size_t lds, hipStream_t s) {
  allow_lds(k_part_build<KK, MM, KPT>, lds);
  hipLaunchKernelGGL((k_part_build<KK, MM, KPT>), dim3(p.nblk), dim3(kBlock), lds, s, ks, n, mp,
                     p.tb, p.T, seg, p.nblk, ent);
}

template <int KK, int MM, int KPT>
static void part_probe(const TilePlan& p, const KeySrc& ks, uint64_t n, const ModP& mp,
                       uint32_t* seg, uint4* ent, size_t lds, hipStream_t s) {
  allow_lds(k_part_probe<KK, MM, KPT>, lds);
  hipLaunchKernelGGL((k_part_probe<KK, MM, KPT>), dim3(p.nblk), dim3(kBlock), lds, s, ks, n, mp,
                     p.tb, p.T, seg, p.nblk, ent);
}

hipError_t launch_build_tiled(int keyk, int mode, uint32_t* words, bool fresh, const KeySrc& ks,
                              uint64_t n, const ModP& mp, const TilePlan& p, uint32_t* seg,
                              uint32_t* ent, hipStream_t s) {
  if (!n) return hipSuccess;
  const size_t lds1 = ((size_t)((p.T + 4) & ~3u) + 2 * p.C + 8) * 4;
  {
  ProfScope ps("k_part_build", s);
  if (p.kpt == 4) {
    CB_DISPATCH(keyk, mode, (part_build<KK, MM, 4>(p, ks, n, mp, seg, ent, lds1, s)));
  } else if (p.kpt == 8) {
    CB_DISPATCH(keyk, mode, (part_build<KK, MM, 8>(p, ks, n, mp, seg, ent, lds1, s)));
  } else {
    CB_DISPATCH(keyk, mode, (part_build<KK, MM, 16>(p, ks, n, mp, seg, ent, lds1, s)));
  }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint32_t nbp = (p.nblk + 3) & ~3u;
  const size_t lds2 = ((size_t)(1u << (p.tb - 5)) + 2 * nbp + 8) * 4;
  allow_lds(k_tile_build, lds2);
  ProfScope ps("k_tile_build", s);
  hipLaunchKernelGGL(k_tile_build, dim3(p.T), dim3(kBlock), lds2, s, words, p.tb, p.T, seg, p.nblk,
                     ent, 2 * p.C, fresh ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_probe_partition(int keyk, int mode, const KeySrc& ks, uint64_t n,
                                  const ModP& mp, const TilePlan& p, uint32_t* seg, uint4* ent,
                                  hipStream_t s) {
  if (!n) return hipSuccess;
  const size_t lds1 = ((size_t)((p.T + 4) & ~3u) + 4 * p.C + 8) * 4;
  ProfScope ps("k_part_probe", s);
  if (p.kpt == 4) {
    CB_DISPATCH(keyk, mode, (part_probe<KK, MM, 4>(p, ks, n, mp, seg, ent, lds1, s)));
  } else {
    CB_DISPATCH(keyk, mode, (part_probe<KK, MM, 8>(p, ks, n, mp, seg, ent, lds1, s)));
  }
  return hipGetLastError();
}

hipError_t launch_probe_tiles(const FilterPtrs& fp, uint32_t nf, uint64_t n, const TilePlan& p,
                              const uint32_t* seg, const uint4* ent, uint32_t* masks,
                              uint64_t* hits, uint64_t hwords, hipStream_t s) {
  if (!n || !nf) return hipSuccess;
  const uint32_t nbp = (p.nblk + 3) & ~3u;
  const size_t lds2 = ((size_t)2 * (1u << (p.tb - 5)) + 2 * nbp + 4) * 4 + kFiltersPerGroup * 8;
  const uint32_t G = (nf + kFiltersPerGroup - 1) / kFiltersPerGroup;
  allow_lds(k_tile_probe<16>, lds2);
  {
    ProfScope ps("k_tile_probe", s);
    hipLaunchKernelGGL((k_tile_probe<16>), dim3(p.T, G), dim3(kBlock), lds2, s, fp, nf, p.tb, seg,
                       p.nblk, ent, p.C, n, masks);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint64_t nw = (n + 63) / 64;
  ProfScope ps("k_masks_to_hits", s);
  hipLaunchKernelGGL(k_masks_to_hits, dim3(grid_for(nw * 64, 4096)), dim3(kBlock), 0, s, masks,
                     fp, nf, n, hits, hwords);
  return hipGetLastError();
}

hipError_t launch_mask_tail(uint32_t* words, uint64_t m, hipStream_t s) {
  if (!(m & 31)) return hipSuccess;
  hipLaunchKernelGGL(k_mask_tail, dim3(1), dim3(64), 0, s, words, m);
  return hipGetLastError();
}

hipError_t launch_export_bools(const uint32_t* words, uint64_t m, uint8_t* out, hipStream_t s) {
  if (!m) return hipSuccess;
  hipLaunchKernelGGL(k_export_bools, dim3(grid_for((m + 31) / 32, 8192)), dim3(kBlock), 0, s,
                     words, m, out);
  return hipGetLastError();
}

hipError_t launch_import_bools(uint32_t* words, uint64_t m, const uint8_t* in, hipStream_t s) {
  if (!m) return hipSuccess;
  hipLaunchKernelGGL(k_import_bools, dim3(grid_for((m + 31) / 32, 8192)), dim3(kBlock), 0, s,
                     words, m, in);
  return hipGetLastError();
}

}  // namespace cb
