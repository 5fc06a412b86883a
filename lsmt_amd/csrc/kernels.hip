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
//
// Partition layout shared by the tiled kernels: partition block b (C keys)
// writes its entries sorted by tile into ent[b*estride ...] and, in
// seg[b*(T+1) + t], the start of tile t's run inside that region
// (seg[b*(T+1) + T] = the block's total). Tile t's entries are therefore the
// runs [seg[b][t], seg[b][t+1]) of every block b.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "blockscan.hpp"
#include "kernels.hpp"
#include "profile.hpp"

// Phase stamps for diagnostics (tools/ubench_build.hip defines CB_STAMPS and
// provides g_stamps): wall-clock s_memrealtime at phase boundaries, one row of
// 8 per workgroup. Compiled out of the library.
#ifdef CB_STAMPS
__device__ uint64_t* g_stamps;
#define CB_STAMP(i)                                                                   \
  do {                                                                                \
    if (threadIdx.x == 0 && g_stamps)                                                 \
      g_stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] =             \
          __builtin_amdgcn_s_memrealtime();                                           \
  } while (0)
#else
#define CB_STAMP(i) \
  do {              \
  } while (0)
#endif

namespace cb {

namespace {

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// Global (address space 1) pointer types: loads through them are global_load
// with counted vmcnt waits, never flat_load (which also waits on lgkmcnt).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4* gptr_u4;
typedef const __attribute__((address_space(1))) uint32_t* gptr_u32;

// Non-temporal 16-B store, for data written once and read only by later
// launches: no L2 allocation to write back at the kernel's end.
__device__ __forceinline__ void store16_nt(uint4* p, const uint4& v) {
  u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}

// Write-through (sc1) 16-B store at byte offset off of a buffer resource.
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store16_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, const uint4& v) {
  const i32x4 w = {(int)v.x, (int)v.y, (int)v.z, (int)v.w};
  __builtin_amdgcn_raw_buffer_store_b128(w, r, off, 0, 16);
}

// Exclusive scan of arr[0..len) in LDS by a whole NT-thread block; returns the
// total. wsum: NT/64 words of LDS scratch. Contains barriers: all threads call.
template <uint32_t NT>
__device__ uint32_t block_exclusive_scan(uint32_t* arr, uint32_t len, uint32_t* wsum) {
  const uint32_t tid = threadIdx.x, lane = lane_id(), wid = tid >> 6;
  const uint32_t per = (len + NT - 1) / NT;
  const uint32_t beg = min(tid * per, len), end = min(beg + per, len);
  uint32_t s = 0;
  for (uint32_t i = beg; i < end; ++i) s += arr[i];
  const uint32_t x = wave_inclusive_scan(s);
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  uint32_t wpre = 0, total = 0;
#pragma unroll
  for (uint32_t w = 0; w < NT / 64; ++w) {
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

// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs
// (MI355X_MICROARCH.md, "Workgroup dispatch"), so blocks b and b+8 share an
// L2. Giving each XCD a contiguous range of tiles lets the 128-B lines that
// adjacent tiles' runs and run-table entries share be fetched once per XCD
// instead of once per tile. Placement only affects speed, never results.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t bid, uint32_t T) {
  if (T & 7u) return bid;
  return (bid & 7u) * (T >> 3) + (bid >> 3);
}

// Last b with P[b] <= j (P: exclusive prefix of the runs' lengths, P[0] = 0).
__device__ __forceinline__ uint32_t seg_find(const uint32_t* P, uint32_t nblk, uint32_t j) {
  uint32_t lo = 0, hi = nblk;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (P[mid] <= j)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo - 1;
}

// Loads tile t's run table into LDS: S[b] = run start in block b's region,
// P[b] = exclusive prefix of run lengths. Returns the tile's entry count.
template <uint32_t NT>
__device__ uint32_t load_runs(const uint32_t* __restrict__ seg, uint32_t nblk, uint32_t T,
                              uint32_t t, uint32_t* S, uint32_t* P, uint32_t* wsum) {
  for (uint32_t b = threadIdx.x; b < nblk; b += NT) {
    const uint32_t* row = seg + (size_t)b * (T + 1) + t;
    const uint32_t s0 = row[0], s1 = row[1];
    S[b] = s0;
    P[b] = s1 - s0;
  }
  __syncthreads();
  return block_exclusive_scan<NT>(P, nblk, wsum);
}

// ---------------------------------------------------------------- direct ---

constexpr uint32_t kBlock = 256;

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

// Filters of at most 2^19 bits (the product's m = 1024 flushes): the filter
// kept in LDS per block, so 2n ORs land in LDS instead of contending on
// m/32 words of HBM (1024 keys into m = 1024 by global atomics took 27.5 us,
// every word taking ~64 serialised memory-side atomics). store_all: one
// block on a fresh filter writes every allocated word (zeros past nw), so the
// filter needs no fill first; otherwise each block ORs its non-zero words in.
template <int KEYK, int MODE>
__global__ __launch_bounds__(1024) void k_insert_lds(uint32_t* __restrict__ words, uint32_t nw, uint32_t nw_alloc,
                                                    KeySrc ks, uint64_t n, ModP mp, uint32_t store_all) {
  extern __shared__ uint32_t lw[];
  for (uint32_t i = threadIdx.x; i < nw; i += 1024) lw[i] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * 1024;
  for (uint64_t k = (uint64_t)blockIdx.x * 1024 + threadIdx.x; k < n; k += stride) {
    uint64_t a, b;
    key_positions<KEYK, MODE>(ks, k, mp, a, b);
    atomicOr(&lw[a >> 5], 1u << (a & 31));  // src/bloom.rs:42
    atomicOr(&lw[b >> 5], 1u << (b & 31));  // src/bloom.rs:43
  }
  __syncthreads();
  if (store_all) {
    for (uint32_t i = threadIdx.x; i < nw_alloc; i += 1024) words[i] = i < nw ? lw[i] : 0u;
  } else {
    for (uint32_t i = threadIdx.x; i < nw; i += 1024) {
      const uint32_t v = lw[i];
      if (v) atomicOr(&words[i], v);
    }
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
      for (int i = 0; i < 8; ++i) va[i] = (valid && f0 + i < nf) ? fp.w[f0 + i][wa] : 0u;
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

constexpr uint32_t kPartThreads = 256;

// ------------------------------------------------------- build ------------
//
// Two passes. Every key contributes two entries (bit a, bit b), bucketed by
// the filter tile they fall in; then one workgroup per tile ORs its entries
// into the tile in LDS and writes the tile back once. At C2 size a pass over
// 16 MiB is ~3 us of bandwidth, so the dependent steps, not the bytes, set the
// time (tools/ubench_build.hip stamps the phases):
//   k_build_part — 1024-thread blocks of KPT keys per thread (C = 1024*KPT).
//                  All key loads issue before any LDS work; ranks from LDS
//                  atomics; the block's entries leave tile-sorted as one
//                  contiguous region, its run starts as one row of seg.
//   k_build_tile — one 1024-thread workgroup per tile of up to 2^19 bits
//                  (64 KiB of LDS). Wave w reads whole runs (lane i = entry i
//                  of the run, one coalesced load per run), 8 runs in flight
//                  per wave, so the 128-B lines of a run are fetched by one
//                  instruction instead of by 64 lanes' scattered loads.
// Fewer, larger tiles (~256 for C2) and larger blocks make the average run
// ~32 entries = one 128-B line.
constexpr uint32_t kBuildNT = 1024;

// A 16-byte key's two positions packed as partition entries ((bin << 20) |
// offset in the bin, bins of 2^tb bits), 0xFFFFFFFF for both when !live.
// 32-bit arithmetic where the positions are (MOD_POW2_32).
template <int MODE>
__device__ __forceinline__ void pack_positions(const uint4& kv, bool live, const ModP& mp, uint32_t tb, uint32_t& qa,
                                               uint32_t& qb) {
  const uint32_t tmask = (1u << tb) - 1u;
  uint32_t a32, b32, ah, bh;
  if constexpr (MODE == MOD_POW2_32) {
    uint32_t h1, h2;
    hash16_u32(kv, h1, h2);
    const uint32_t mask = static_cast<uint32_t>(mp.mask);
    a32 = h1 & mask;
    b32 = h2 & mask;
    ah = a32 >> tb;
    bh = b32 >> tb;
  } else {
    uint64_t a, b;
    key_positions_u4<MODE>(kv, mp, a, b);
    a32 = (uint32_t)a;
    b32 = (uint32_t)b;
    ah = (uint32_t)(a >> tb);
    bh = (uint32_t)(b >> tb);
  }
  qa = live ? (ah << 20) | (a32 & tmask) : 0xFFFFFFFFu;
  qb = live ? (bh << 20) | (b32 & tmask) : 0xFFFFFFFFu;
}

// A partition block's LDS phases once its entries are in registers (q: packed
// (bin << 20) | offset, 0xFFFFFFFF for none): ranks from LDS atomics, the bin
// scan, the seg row (run starts and the total), the tile-sorted entries into
// LDS and out to `out` as one contiguous region. Barriers inside; the block's
// LDS is free again when it returns except for the final store's reads of
// `stage` (the caller's next LDS write must follow a barrier).
// pol: the store policy bits (build_stores(): bit 0 write-through entries).
template <int KPT, typename E>
__device__ __forceinline__ void part_phases(const uint32_t (&q)[2 * KPT], uint32_t T, uint32_t* smem,
                                            uint32_t* __restrict__ srow, E* __restrict__ out, uint32_t pol) {
  constexpr uint32_t NT = kBuildNT, C = NT * KPT;
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  const uint32_t Tp = (T + 4) & ~3u;
  // hist: T + 1 entries (counts, then run starts and the total), zero to Tp,
  // then a discard word at Tp for the lanes without an entry
  uint32_t* hist = smem;
  E* stage = reinterpret_cast<E*>(smem + Tp + 4);
  const uint32_t tid = threadIdx.x;
  uint32_t er[2 * KPT];
  for (uint32_t i = tid; i < Tp; i += NT) hist[i] = 0;
  __syncthreads();
  CB_STAMP(1);
  // every lane adds (no branch per entry, whose merges cost more VALU than
  // the rare discards on the last block's padding)
#pragma unroll
  for (int e = 0; e < 2 * KPT; ++e) er[e] = atomicAdd(&hist[q[e] != kNone ? q[e] >> 20 : Tp], 1u);
  __syncthreads();
  CB_STAMP(2);
  wave0_exclusive_scan4(hist, Tp);  // Tp >= T + 1: hist[T] = the total
  __syncthreads();
  CB_STAMP(3);
  const uint32_t total = hist[T];
  for (uint32_t t = tid; t <= T; t += NT) srow[t] = hist[t];
#pragma unroll
  for (int e = 0; e < 2 * KPT; ++e)
    if (q[e] != kNone) stage[hist[q[e] >> 20] + er[e]] = (E)(q[e] & 0xFFFFFu);
  __syncthreads();
  CB_STAMP(4);
  constexpr uint32_t PER = 16 / sizeof(E);  // entries per 16-B store (out and stage 16-B aligned)
  const uint32_t n4 = total / PER;
  // write-through (sc1): the entries go on to the memory side at once, so the
  // kernel's end has no dirty L2 lines to write back, and the tile pass (on
  // other XCDs) still finds them there; C2 on four lanes 101 -> 105-107 G
  // keys/s (non-temporal stores instead made the tile pass's reads slower)
  if (pol & 4u) {  // (bit 2: non-temporal entries)
    for (uint32_t i = tid; i < n4; i += NT) store16_nt(reinterpret_cast<uint4*>(out) + i, reinterpret_cast<const uint4*>(stage)[i]);
  } else if (pol & 1u) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, 2 * C * sizeof(E), 0x00020000);
    for (uint32_t i = tid; i < n4; i += NT) store16_wt(r, i * 16, reinterpret_cast<const uint4*>(stage)[i]);
  } else {
    for (uint32_t i = tid; i < n4; i += NT)
      reinterpret_cast<uint4*>(out)[i] = reinterpret_cast<const uint4*>(stage)[i];
  }
  if (tid < total - PER * n4) out[PER * n4 + tid] = stage[PER * n4 + tid];  // the < PER left over
  CB_STAMP(5);
}

// E: the entry type — uint32_t (offsets in tiles of up to 2^20 bits) or
// uint16_t (bins of 2^16 bits, tb = 16 here: the sub-tiles of
// k_build_tile_sub's tiles).
template <int KEYK, int MODE, int KPT, typename E = uint32_t>
__global__ __launch_bounds__(kBuildNT) void k_build_part(BuildBatch bb, ModP mp, uint32_t tb,
                                                         uint32_t T,
                                                         uint32_t* __restrict__ seg_all,
                                                         void* __restrict__ ent_all, uint32_t pol) {
  constexpr uint32_t NT = kBuildNT, C = NT * KPT;
  static_assert(sizeof(E) == 4 || sizeof(E) == 2, "entry type");
  const KeySrc ks = bb.ks[blockIdx.y];
  const uint64_t n = bb.n[blockIdx.y];
  uint32_t* seg = seg_all + (size_t)blockIdx.y * gridDim.x * (T + 1);
  E* ent = reinterpret_cast<E*>(ent_all) + (size_t)blockIdx.y * gridDim.x * (2 * C);
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t tid = threadIdx.x;
  const uint64_t kbase = (uint64_t)blockIdx.x * C;
  CB_STAMP(0);

  // positions first: every key load of the thread is in flight together.
  // Each entry is kept packed as (tile << 20) | offset in the tile (tiles <
  // kMaxTiles = 2^12, offsets < 2^kMaxTileBits <= 2^20), 0xFFFFFFFF for none:
  // one register per entry instead of a 64-bit position and a tile.
  static_assert(kMaxTiles <= 4096 && kMaxTileBits <= 20, "packed entry");
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  uint32_t q[2 * KPT];
  if constexpr (KEYK == KEY_FIXED16) {
    // every lane loads all its keys first (indices clamped to the last key,
    // so no per-key branch serialises the loads behind each other's waits)
    uint4 kv[KPT] = {};  // (a block past this filter's keys hashes zeros, all discarded)
    if (kbase < n) {  // uniform
      const uint4* keys = reinterpret_cast<const uint4*>(ks.bytes);
#pragma unroll
      for (int j = 0; j < KPT; ++j) {
        const uint64_t k = kbase + (uint64_t)j * NT + tid;
        kv[j] = keys[k < n ? k : n - 1];
      }
    }
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const uint64_t k = kbase + (uint64_t)j * NT + tid;
      pack_positions<MODE>(kv[j], k < n, mp, tb, q[2 * j], q[2 * j + 1]);
    }
  } else {
    const uint32_t tmask = (1u << tb) - 1u;
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const uint64_t k = kbase + (uint64_t)j * NT + tid;
      q[2 * j] = q[2 * j + 1] = kNone;
      if (k < n) {
        uint64_t a, b;
        key_positions<KEYK, MODE>(ks, k, mp, a, b);
        q[2 * j] = ((uint32_t)(a >> tb) << 20) | ((uint32_t)a & tmask);
        q[2 * j + 1] = ((uint32_t)(b >> tb) << 20) | ((uint32_t)b & tmask);
      }
    }
  }
  part_phases<KPT, E>(q, T, smem, seg + (size_t)blockIdx.x * (T + 1), ent + (size_t)blockIdx.x * (2 * C), pol);
}

// Wave w owns partition blocks b = w + NW*u. Per group of 16: lanes 0..15
// load the 16 blocks' run bounds (seg[b][t], seg[b][t+1]), shuffles hand each
// run's start and length to the whole wave, and the wave issues the 16 run
// loads back to back (lane i = entry i): two dependent memory round trips per
// group and no LDS run table or barrier before the ORs.
// pol: the store policy bits (build_stores(): bit 1 non-temporal write-back).
template <int G, int R, uint32_t NT = kBuildNT>
__global__ __launch_bounds__(NT) void k_build_tile(BuildBatch bb, uint32_t tb, uint32_t T,
                                                         const uint32_t* __restrict__ seg_all,
                                                         uint32_t nblk,
                                                         const uint32_t* __restrict__ ent_all,
                                                         uint32_t estride, uint32_t pol) {
  constexpr uint32_t NW = NT / 64;
  static_assert(G <= 64, "one lane per run bound");
  uint32_t* __restrict__ words = bb.words[blockIdx.y];
  const bool fresh = (bb.fresh >> blockIdx.y) & 1ull;
  const uint32_t* __restrict__ seg = seg_all + (size_t)blockIdx.y * nblk * (T + 1);
  const uint32_t* __restrict__ ent = ent_all + (size_t)blockIdx.y * nblk * estride;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t tw = 1u << (tb - 5);
  uint32_t* tile = smem;
  const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const uint32_t t = xcd_tile(blockIdx.x, T);
  CB_STAMP(0);

  // first group's run bounds in flight while the tile is cleared / loaded
  uint32_t s0 = 0, s1 = 0;
  {
    const uint32_t b = w + NW * lane;
    if (lane < (uint32_t)G && b < nblk) {
      const uint32_t* row = seg + (size_t)b * (T + 1) + t;
      s0 = row[0];
      s1 = row[1];
    }
  }
  uint4* gt = reinterpret_cast<uint4*>(words + (size_t)t * tw);
  uint4* lt = reinterpret_cast<uint4*>(tile);
  for (uint32_t i = tid; i < tw / 4; i += NT) lt[i] = fresh ? make_uint4(0, 0, 0, 0) : gt[i];
  __syncthreads();
  CB_STAMP(1);

  for (uint32_t g0 = 0; w + NW * g0 < nblk; g0 += G) {
    if (g0) {
      s0 = s1 = 0;
      const uint32_t b = w + NW * (g0 + lane);
      if (lane < (uint32_t)G && b < nblk) {
        const uint32_t* row = seg + (size_t)b * (T + 1) + t;
        s0 = row[0];
        s1 = row[1];
      }
    }
    // R rounds of run loads (lane i = entry i + 64 r): every load of the G
    // runs goes out before any OR. R = 2 for long runs (C4's 64 tiles per
    // filter give ~128 entries per run) with G = 8, so a lane holds G * R =
    // 16 entries either way (62 VGPRs, 8 waves per SIMD: two 16-wave tiles per
    // CU; 32 entries per lane took 80 VGPRs and one tile per CU)
    uint32_t o[R][G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const uint32_t st = __shfl(s0, u, 64), len = __shfl(s1, u, 64) - st;
      const uint32_t b = w + NW * (g0 + u);
#pragma unroll
      for (int q = 0; q < R; ++q) {
        o[q][u] = 0xFFFFFFFFu;
        if (64 * q + lane < len) o[q][u] = ent[(size_t)b * estride + st + 64 * q + lane];
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u)
#pragma unroll
      for (int q = 0; q < R; ++q)
        if (o[q][u] != 0xFFFFFFFFu) atomicOr(&tile[o[q][u] >> 5], 1u << (o[q][u] & 31));
    // runs longer than R waves (skewed inputs, few partition blocks)
    if (__ballot(lane < (uint32_t)G && s1 - s0 > 64u * R)) {
#pragma unroll 1
      for (int u = 0; u < G; ++u) {
        const uint32_t st = __shfl(s0, u, 64), len = __shfl(s1, u, 64) - st;
        const uint32_t* run = ent + (size_t)(w + NW * (g0 + u)) * estride + st;
        for (uint32_t i = 64 * R + lane; i < len; i += 64) {
          const uint32_t v = run[i];
          atomicOr(&tile[v >> 5], 1u << (v & 31));
        }
      }
    }
  }
  CB_STAMP(2);
  __syncthreads();
  CB_STAMP(3);
  // non-temporal: the filter is written once and read by other launches, so
  // no L2 lines to write back at the kernel's end (tile pass alone 8.8 ->
  // 7.5 us, C2 on four lanes 97.8 -> 101 G keys/s; write-through measured
  // the same here)
  if (pol & 2u)
    for (uint32_t i = tid; i < tw / 4; i += NT) store16_nt(gt + i, lt[i]);
  else
    for (uint32_t i = tid; i < tw / 4; i += NT) gt[i] = lt[i];
  CB_STAMP(4);
}

// The tile pass over 16-bit entries (batched builds of long runs, C4): the
// partition binned by sub-tiles of 2^16 bits (S = 2^SUB per tile), so block
// b's entries for tile t are one contiguous super-run [seg[b][S t],
// seg[b][S (t+1)]) and sub-tile j's part of it starts at seg[b][S t + j].
// Lanes 0 .. G (S+1) - 1 load the G blocks' S + 1 bounds; an entry's
// sub-tile is the number of interior bounds at or below its index (uniform
// values taken by readlane, S - 1 compares), its bit (j << 16) | entry. Half
// the entry bytes of k_build_tile for S - 1 compares per entry.
template <int G, int R, int SUB, uint32_t NT = kBuildNT>
__global__ __launch_bounds__(NT) void k_build_tile_sub(BuildBatch bb, uint32_t tb, uint32_t T,
                                                       const uint32_t* __restrict__ seg_all,
                                                       uint32_t nblk,
                                                       const uint16_t* __restrict__ ent_all,
                                                       uint32_t estride, uint32_t pol) {
  constexpr uint32_t NW = NT / 64, S = 1u << SUB, NB = S + 1;
  static_assert(G * NB <= 64, "one lane per bound");
  uint32_t* __restrict__ words = bb.words[blockIdx.y];
  const bool fresh = (bb.fresh >> blockIdx.y) & 1ull;
  const uint32_t TS = T << SUB;  // bins per filter
  const uint32_t* __restrict__ seg = seg_all + (size_t)blockIdx.y * nblk * (TS + 1);
  const uint16_t* __restrict__ ent = ent_all + (size_t)blockIdx.y * nblk * estride;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t tw = 1u << (tb - 5);
  uint32_t* tile = smem;
  const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const uint32_t t = xcd_tile(blockIdx.x, T);
  const uint32_t lu = lane / NB, lk = lane - lu * NB;  // this lane's bound: block lu, bound lk

  uint32_t sb = 0;  // first group's bounds in flight while the tile is cleared / loaded
  {
    const uint32_t b = w + NW * lu;
    if (lane < G * NB && b < nblk) sb = seg[(size_t)b * (TS + 1) + (t << SUB) + lk];
  }
  uint4* gt = reinterpret_cast<uint4*>(words + (size_t)t * tw);
  uint4* lt = reinterpret_cast<uint4*>(tile);
  for (uint32_t i = tid; i < tw / 4; i += NT) lt[i] = fresh ? make_uint4(0, 0, 0, 0) : gt[i];
  __syncthreads();

  for (uint32_t g0 = 0; w + NW * g0 < nblk; g0 += G) {
    if (g0) {
      sb = 0;
      const uint32_t b = w + NW * (g0 + lu);
      if (lane < G * NB && b < nblk) sb = seg[(size_t)b * (TS + 1) + (t << SUB) + lk];
    }
    uint32_t o[R][G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const uint32_t st = __builtin_amdgcn_readlane(sb, u * NB);
      const uint32_t len = __builtin_amdgcn_readlane(sb, u * NB + S) - st;
      const uint32_t b = w + NW * (g0 + u);
#pragma unroll
      for (int q = 0; q < R; ++q) {
        o[q][u] = 0;
        if (64 * q + lane < len) o[q][u] = ent[(size_t)b * estride + st + 64 * q + lane];
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const uint32_t st = __builtin_amdgcn_readlane(sb, u * NB);
      const uint32_t len = __builtin_amdgcn_readlane(sb, u * NB + S) - st;
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const uint32_t i = 64 * q + lane;
        if (i < len) {
          uint32_t j = 0;
#pragma unroll
          for (uint32_t k = 1; k < S; ++k) j += (st + i >= __builtin_amdgcn_readlane(sb, u * NB + k)) ? 1u : 0u;
          const uint32_t v = (j << 16) | o[q][u];
          atomicOr(&tile[v >> 5], 1u << (v & 31));
        }
      }
    }
    // super-runs longer than R waves (skewed inputs)
    bool longrun = false;
#pragma unroll
    for (int u = 0; u < G; ++u)
      longrun |= __builtin_amdgcn_readlane(sb, u * NB + S) - __builtin_amdgcn_readlane(sb, u * NB) > 64u * R;
    if (longrun) {
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const uint32_t st = __builtin_amdgcn_readlane(sb, u * NB);
        const uint32_t len = __builtin_amdgcn_readlane(sb, u * NB + S) - st;
        const uint16_t* run = ent + (size_t)(w + NW * (g0 + u)) * estride + st;
        for (uint32_t i = 64 * R + lane; i < len; i += 64) {
          uint32_t j = 0;
#pragma unroll
          for (uint32_t k = 1; k < S; ++k) j += (st + i >= __builtin_amdgcn_readlane(sb, u * NB + k)) ? 1u : 0u;
          const uint32_t v = (j << 16) | run[i];
          atomicOr(&tile[v >> 5], 1u << (v & 31));
        }
      }
    }
  }
  __syncthreads();
  if (pol & 2u)
    for (uint32_t i = tid; i < tw / 4; i += NT) store16_nt(gt + i, lt[i]);
  else
    for (uint32_t i = tid; i < tw / 4; i += NT) gt[i] = lt[i];
}

// Partition for probe: one 8-byte entry per key, bucketed by the tile of bit
// a: x = (offset of a in its tile) | (key index within the block << tb),
// y = b. Requires tb + log2(C) <= 32 and m <= 2^32 (checked on the host).
// lkey[b*C + i] = the block-local key index of region slot i: k_tile_probe
// writes each key's result mask at its entry's slot, and k_masks_to_hits
// reads a block's region back in order and un-permutes it in LDS.
template <int KEYK, int MODE, int KPT>
__global__ __launch_bounds__(kPartThreads) void k_part_probe(KeySrc ks, uint64_t n, ModP mp,
                                                             uint32_t tb, uint32_t T,
                                                             uint32_t* __restrict__ seg,
                                                             uint2* __restrict__ ent,
                                                             uint16_t* __restrict__ lkey) {
  constexpr uint32_t C = kPartThreads * KPT;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t Tp = (T + 4) & ~3u;
  uint32_t* hist = smem;
  uint2* stage = reinterpret_cast<uint2*>(smem + Tp);
  uint16_t* lstage = reinterpret_cast<uint16_t*>(stage + C);
  uint32_t* wsum = reinterpret_cast<uint32_t*>(lstage + C);
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < Tp; i += kPartThreads) hist[i] = 0;
  __syncthreads();

  const uint64_t kbase = (uint64_t)blockIdx.x * C;
  const uint32_t tmask = (1u << tb) - 1u;
  uint32_t et[KPT], er[KPT];
  uint2 rec[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t local = (uint32_t)j * kPartThreads + tid;
    const uint64_t k = kbase + local;
    et[j] = 0xFFFFFFFFu;
    if (k < n) {
      uint64_t a, b;
      key_positions<KEYK, MODE>(ks, k, mp, a, b);
      et[j] = (uint32_t)(a >> tb);
      er[j] = atomicAdd(&hist[et[j]], 1u);
      rec[j] = make_uint2(((uint32_t)a & tmask) | (local << tb), (uint32_t)b);
    }
  }
  __syncthreads();
  const uint32_t total = block_exclusive_scan<kPartThreads>(hist, T, wsum);
  if (tid == 0) hist[T] = total;
  __syncthreads();
  uint32_t* srow = seg + (size_t)blockIdx.x * (T + 1);
  for (uint32_t t = tid; t <= T; t += kPartThreads) srow[t] = hist[t];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    if (et[j] != 0xFFFFFFFFu) {
      const uint32_t slot = hist[et[j]] + er[j];
      stage[slot] = rec[j];
      lstage[slot] = (uint16_t)(j * kPartThreads + tid);
    }
  }
  __syncthreads();
  uint2* out = ent + (size_t)blockIdx.x * C;
  uint16_t* lout = lkey + (size_t)blockIdx.x * C;
  for (uint32_t i = tid; i < total; i += kPartThreads) {
    out[i] = stage[i];
    lout[i] = lstage[i];
  }
}

constexpr uint32_t kTileProbeThreads = 512;

// Timing-only experiment switches for k_tile_probe (CB_PROBE_XFLAGS; results
// are wrong when set — bench attribution only, never set in production).
constexpr uint32_t kXSkipGather = 1, kXSkipStream = 2, kXSkipStore = 4;

// Probe one tile against up to 32 filters (group blockIdx.y). Each filter's
// tile is streamed HBM -> registers -> LDS through a D-deep register ring, so
// D tiles are in flight while the current one is tested. Bit a is tested in
// LDS; bit b is gathered from HBM only for (key, filter) pairs whose bit a was
// set. Output: masks[g*n + key] = per-filter result bits.
// RPT = uint4 per thread per tile (tile bits = RPT * 16 * 8 * NT).
template <int EPT, int RPT, int D>
__global__ __launch_bounds__(kTileProbeThreads) void k_tile_probe(
    FilterPtrs fp, uint32_t nf, uint32_t tb, uint32_t T, const uint32_t* __restrict__ seg,
    uint32_t nblk, const uint2* __restrict__ ent, uint32_t C, uint64_t n,
    uint32_t* __restrict__ masks, uint32_t xflags) {
  constexpr uint32_t NT = kTileProbeThreads;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t tw = 1u << (tb - 5);  // == RPT * 4 * NT
  const uint32_t nbp = (nblk + 3) & ~3u;
  uint32_t* buf = smem;  // 2 * tw
  uint32_t* P = buf + 2 * tw;
  uint32_t* S = P + nbp;
  uint32_t* wsum = S + nbp;                                                  // NT/64 words
  const uint32_t** fw = reinterpret_cast<const uint32_t**>(wsum + NT / 64);  // 32 pointers
  const uint32_t tid = threadIdx.x;
  const uint32_t t = xcd_tile(blockIdx.x, T), g = blockIdx.y;
  const uint32_t f0 = g * kFiltersPerGroup;
  const uint32_t nfg = min(kFiltersPerGroup, nf - f0);
  const uint32_t tmask = (1u << tb) - 1u;
  if (tid < nfg) fw[tid] = fp.w[f0 + tid];

  // Register ring: slot s holds filter fb+s's tile. Each slot is its own
  // named array so every index is static (no scratch); a slot is refilled
  // right after it is committed to LDS, keeping D tiles in flight. Loads go
  // through address-space-1 pointers (global_load, counted vmcnt waits).
  u32x4 r0[RPT], r1[RPT], r2[RPT], r3[RPT];
#define TP_FETCH(R, F)                                                        \
  if (!(xflags & kXSkipStream)) {                                             \
    const gptr_u4 src = (gptr_u4)(fp.w[f0 + (F)] + (size_t)t * tw);           \
    _Pragma("unroll") for (int q = 0; q < RPT; ++q) R[q] = src[tid + q * NT]; \
  }
#define TP_FETCH_FIRST()                  \
  {                                       \
    TP_FETCH(r0, 0);                      \
    if (1 < nfg) TP_FETCH(r1, 1);         \
    if constexpr (D == 4) {               \
      if (2 < nfg) TP_FETCH(r2, 2);       \
      if (3 < nfg) TP_FETCH(r3, 3);       \
    }                                     \
  }
  // The first D tiles are requested before the run table and entries are
  // read, so their HBM latency overlaps the prologue.
  TP_FETCH_FIRST();

  const uint32_t E = load_runs<NT>(seg, nblk, T, t, S, P, wsum);
  uint32_t* mg = masks + (size_t)g * n;  // results go to each entry's region slot

  for (uint32_t cbase = 0; cbase < E; cbase += NT * EPT) {
    if (cbase) TP_FETCH_FIRST();  // rare extra chunk: stream the tiles again
    const uint32_t cn = min(E - cbase, NT * EPT);
    const uint32_t per = (cn + NT - 1) / NT;
    const uint32_t j0 = cbase + min(tid * per, cn);
    const uint32_t cnt = cbase + min(tid * per + per, cn) - j0;
    uint32_t off[EPT], pb[EPT], am[EPT], slot[EPT];
    {
      uint32_t b = cnt ? seg_find(P, nblk, j0) : 0;
      uint32_t pnext = (b + 1 < nblk) ? P[b + 1] : E;
#pragma unroll
      for (int i = 0; i < EPT; ++i) {
        am[i] = 0;
        off[i] = 0;  // unused slots test bit 0 (branch-free LDS reads) and are dropped
        if ((uint32_t)i < cnt) {
          const uint32_t j = j0 + i;
          while (j >= pnext) {
            ++b;
            pnext = (b + 1 < nblk) ? P[b + 1] : E;
          }
          slot[i] = b * C + S[b] + (j - P[b]);
          const uint2 r = ent[slot[i]];
          off[i] = r.x & tmask;
          pb[i] = r.y;
        }
      }
    }

#define TP_STAGE(R, F)                                                                     \
  {                                                                                        \
    const uint32_t f_ = (F);                                                               \
    u32x4* dst = reinterpret_cast<u32x4*>(buf + (f_ & 1) * tw);                            \
    _Pragma("unroll") for (int q = 0; q < RPT; ++q) dst[tid + q * NT] = R[q];              \
    __syncthreads();                                                                       \
    if (f_ + D < nfg) TP_FETCH(R, f_ + D);                                                 \
    const uint32_t* lb = buf + (f_ & 1) * tw;                                              \
    _Pragma("unroll") for (int i = 0; i < EPT; ++i) am[i] |=                               \
        ((lb[off[i] >> 5] >> (off[i] & 31)) & 1u) << f_;                                   \
  }
    for (uint32_t fb = 0; fb < nfg; fb += D) {
      TP_STAGE(r0, fb);
      if (fb + 1 < nfg) TP_STAGE(r1, fb + 1);
      if constexpr (D == 4) {
        if (fb + 2 < nfg) TP_STAGE(r2, fb + 2);
        if (fb + 3 < nfg) TP_STAGE(r3, fb + 3);
      }
    }
#undef TP_STAGE
    __syncthreads();  // the LDS buffers are rewritten by the next chunk

    // Bit b of every (entry, filter) pair whose bit a was set, gathered from
    // HBM in rounds: each round issues one independent load per entry.
    uint32_t mask[EPT], x[EPT];
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      mask[i] = 0;
      x[i] = ((uint32_t)i < cnt && !(xflags & kXSkipGather)) ? am[i] : 0u;
    }
    for (;;) {
      uint32_t any = 0, v[EPT];
#pragma unroll
      for (int i = 0; i < EPT; ++i) {
        any |= x[i];
        v[i] = x[i] ? ((gptr_u32)fw[__builtin_ctz(x[i])])[pb[i] >> 5] : 0u;
      }
      if (!any) break;
#pragma unroll
      for (int i = 0; i < EPT; ++i) {
        if (x[i]) {
          const uint32_t f = __builtin_ctz(x[i]);
          mask[i] |= ((v[i] >> (pb[i] & 31)) & 1u) << f;
          x[i] &= x[i] - 1;
        }
      }
    }
    if (!(xflags & kXSkipStore)) {
#pragma unroll
      for (int i = 0; i < EPT; ++i)
        if ((uint32_t)i < cnt) mg[slot[i]] = mask[i];
    }
  }
#undef TP_FETCH_FIRST
#undef TP_FETCH
}

constexpr uint32_t kHitsThreads = 512;

// Un-permute one partition block's results and transpose them into the
// [filter][n/64] hit bitmaps. Block b reads its region's masks and local key
// indices in order (coalesced), scatters the masks into LDS by key, then each
// wave turns 64 keys into one word per filter with wave64 ballots; the words
// are staged in LDS so every filter row leaves as whole contiguous segments.
template <int KPT>
__global__ __launch_bounds__(kHitsThreads) void k_masks_to_hits(
    const uint32_t* __restrict__ masks, const uint16_t* __restrict__ lkey, FilterPtrs fp,
    uint32_t nf, uint64_t n, uint64_t* __restrict__ hits, uint64_t hwords) {
  constexpr uint32_t C = kPartThreads * KPT;  // keys per partition block
  constexpr uint32_t W = C / 64;              // hit words per filter row
  constexpr uint32_t G = kMaxFiltersPerLaunch / kFiltersPerGroup;
  __shared__ uint32_t km[G][C];
  __shared__ uint64_t hb[kMaxFiltersPerLaunch][W];
  __shared__ uint32_t rows[kMaxFiltersPerLaunch];
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t ng = (nf + kFiltersPerGroup - 1) / kFiltersPerGroup;
  const uint64_t kbase = (uint64_t)blockIdx.x * C;
  const uint32_t cnt = (uint32_t)min((uint64_t)C, n - kbase);
  if (tid < nf) rows[tid] = fp.row[tid];
  for (uint32_t i = tid; i < cnt; i += kHitsThreads) {
    const uint32_t lk = lkey[kbase + i];
    km[0][lk] = masks[kbase + i];
    if (ng > 1) km[1][lk] = masks[n + kbase + i];
  }
  __syncthreads();
  for (uint32_t w = wave; w < W; w += kHitsThreads / 64) {
    const uint32_t kl = w * 64 + lane;
#pragma unroll
    for (uint32_t g = 0; g < G; ++g) {
      if (g < ng) {
        const uint32_t m = kl < cnt ? km[g][kl] : 0u;
        uint64_t mine = 0;
#pragma unroll
        for (uint32_t f = 0; f < kFiltersPerGroup; ++f) {
          const uint64_t bal = __ballot((m >> f) & 1u);
          mine = (lane == f) ? bal : mine;
        }
        if (lane < min(kFiltersPerGroup, nf - g * kFiltersPerGroup))
          hb[g * kFiltersPerGroup + lane][w] = mine;
      }
    }
  }
  __syncthreads();
  const uint64_t wbase = kbase / 64, nw = (n + 63) / 64;
  for (uint32_t i = tid; i < nf * W; i += kHitsThreads) {
    const uint32_t f = i / W, w = i % W;
    if (wbase + w < nw) hits[(uint64_t)rows[f] * hwords + wbase + w] = hb[f][w];
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
#define CB_DISPATCH(keyk, mode, CALL)                                          \
  switch ((keyk) * 3 + (mode)) {                                               \
    case 0: { constexpr int KK = KEY_FIXED16, MM = MOD_POW2_32; CALL; } break; \
    case 1: { constexpr int KK = KEY_FIXED16, MM = MOD_POW2_64; CALL; } break; \
    case 2: { constexpr int KK = KEY_FIXED16, MM = MOD_GENERIC; CALL; } break; \
    case 3: { constexpr int KK = KEY_FIXED, MM = MOD_POW2_32; CALL; } break;   \
    case 4: { constexpr int KK = KEY_FIXED, MM = MOD_POW2_64; CALL; } break;   \
    case 5: { constexpr int KK = KEY_FIXED, MM = MOD_GENERIC; CALL; } break;   \
    case 6: { constexpr int KK = KEY_VAR, MM = MOD_POW2_32; CALL; } break;     \
    case 7: { constexpr int KK = KEY_VAR, MM = MOD_POW2_64; CALL; } break;     \
    case 8: { constexpr int KK = KEY_VAR, MM = MOD_GENERIC; CALL; } break;     \
    default: return hipErrorInvalidValue;                                      \
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

}  // namespace

// ------------------------------------------------------------- plans -------

static int64_t clamp64(int64_t v, int64_t lo, int64_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Raise tb (up to hi) until the tile count fits the partition histogram.
static uint32_t fit_tiles(uint64_t m, int64_t tb, int64_t hi) {
  while (tb < hi && ((m + (1ull << tb) - 1) >> tb) > kMaxTiles) ++tb;
  return (uint32_t)tb;
}

// Tuning overrides, compiled only into experiment builds (make
// EXTRA=-DCB_EXPERIMENTS): CB_PROBE_TB / CB_BUILD_TB fix the tile bits,
// CB_PROBE_KPT / CB_BUILD_KPT the partition keys per thread, CB_BUILD_STORES
// the build's store policy, CB_PROBE_XFLAGS the tile probe's variant bits.
// The shipped library always takes the defaults.
static int env_int(const char* name, int dflt) {
#ifdef CB_EXPERIMENTS
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
#else
  (void)name;
  return dflt;
#endif
}

TilePlan plan_build(uint64_t m, uint64_t n, uint32_t nb) {
  // ~256 tiles per launch over the whole batch, each as large as the 64 KiB
  // LDS tile allows (fewer tiles = longer runs per partition block);
  // 1024-thread partition blocks of up to 4096 keys, fewer keys per thread
  // only while that leaves under 256 blocks in the launch.
  TilePlan p{};
  static const int env_tb = env_int("CB_BUILD_TB", 0);
  static const int env_kpt = env_int("CB_BUILD_KPT", 0);
  if (nb < 1) nb = 1;
  const uint64_t want_tiles = nb >= 256 ? 1 : 256 / nb;
  int64_t tb = clamp64((int64_t)ilog2_floor(m > want_tiles ? m / want_tiles : 1), kMinTileBits,
                       kMaxTileBits);
  if (env_tb) tb = clamp64(env_tb, kMinTileBits, kMaxTileBits);
  p.tb = fit_tiles(m, tb, kMaxTileBits);
  p.T = (uint32_t)((m + (1ull << p.tb) - 1) >> p.tb);
  p.kpt = 4;
  while (p.kpt > 1 && nb * ((n + kBuildNT * p.kpt - 1) / (kBuildNT * p.kpt)) < 256) p.kpt /= 2;
  if (env_kpt == 1 || env_kpt == 2 || env_kpt == 4) p.kpt = env_kpt;
  p.C = kBuildNT * p.kpt;
  p.nblk = (uint32_t)((n + p.C - 1) / p.C);
  // Batched builds of long runs (C4: 32 filters of 2^18 keys into 2^25 bits,
  // ~128 entries per run) move 16-bit entries in 2^16-bit sub-tiles: the
  // passes are bandwidth-bound there, and the entries are a third of the
  // bytes. Single builds keep 32-bit entries (their tile pass is bound by its
  // dependent loads, where the sub-tile arithmetic cost more than the bytes
  // saved: HISTORY.md, round 3 build notes).
  // Their tiles are 2^18 bits (4 sub-tiles) worked by 512-thread
  // workgroups, four per CU instead of two 1024-thread ones on 2^19-bit
  // tiles: C4 141 -> 128-131 us per step on one lane, 147-151 -> 139-141 on
  // three (profiles/c4_sub_r04.json).
  static const int env_sub = env_int("CB_BUILD_SUB", -1);
  p.sub = 0;
  // (CB_BUILD_SUB=1, experiment builds: every build of tb >= 17 takes them)
  if (env_sub != 0 && p.tb >= 17 && ((nb >= 8 && 2ull * p.C > 48ull * p.T) || env_sub == 1)) {
    if (p.tb == 19 && !env_tb && (2ull * p.C > 48ull * 2 * p.T || env_sub == 1) && ((uint64_t)p.T << 3) <= kMaxTiles) {
      p.tb = 18;
      p.T = (uint32_t)((m + (1ull << 18) - 1) >> 18);
    }
    if (((uint64_t)p.T << (p.tb - 16)) <= kMaxTiles) p.sub = p.tb - 16;
  }
  return p;
}

TilePlan plan_probe(uint64_t m, uint64_t n) {
  TilePlan p{};
  // The probe kernel is instantiated for tiles of 2^16..2^18 bits. Aim for
  // ~512 tiles and <= ~4096 entries per tile.
  int64_t tb1 = (int64_t)ilog2_floor(m > 512 ? m / 512 : 1);
  const uint64_t want = n ? (m * 4096ull) / n : m;
  int64_t tb2 = (int64_t)ilog2_floor(want ? want : 1);
  int64_t tb = clamp64(tb1 < tb2 ? tb1 : tb2, kMinProbeTileBits, kMaxProbeTileBits);
  static const int env_tb = env_int("CB_PROBE_TB", 0);
  if (env_tb) tb = clamp64(env_tb, kMinProbeTileBits, kMaxProbeTileBits);
  p.tb = fit_tiles(m, tb, kMaxProbeTileBits);
  p.T = (uint32_t)((m + (1ull << p.tb) - 1) >> p.tb);
  // Longer runs per (block, tile) with C = 2048 once that still leaves >= 512
  // partition blocks; never more than 4096 blocks (the host chunks keys).
  p.kpt = n >= 512ull * 2048 ? 8 : 4;
  static const int env_kpt = env_int("CB_PROBE_KPT", 0);
  if (env_kpt == 4 || env_kpt == 8) p.kpt = env_kpt;
  p.C = kPartThreads * p.kpt;
  p.nblk = (uint32_t)((n + p.C - 1) / p.C);
  return p;
}

bool plan_ok(const TilePlan& p) { return p.T <= kMaxTiles; }

size_t build_seg_bytes(const TilePlan& p) { return ((size_t)(p.T << p.sub) + 1) * p.nblk * 4; }
size_t build_ent_bytes(const TilePlan& p) { return (size_t)p.nblk * 2 * p.C * (p.sub ? 2 : 4); }
size_t probe_seg_bytes(const TilePlan& p) { return (size_t)(p.T + 1) * p.nblk * 4; }
size_t probe_ent_bytes(const TilePlan& p) { return (size_t)p.nblk * p.C * 8; }
size_t probe_lkey_bytes(const TilePlan& p) { return (size_t)p.nblk * p.C * 2; }

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

template <int KK, int MM>
static void insert_lds(uint32_t* words, uint32_t nw, uint32_t nw_alloc, const KeySrc& ks, uint64_t n, const ModP& mp,
                       bool store_all, uint32_t grid, size_t lds, hipStream_t s) {
  allow_lds(k_insert_lds<KK, MM>, lds);
  hipLaunchKernelGGL((k_insert_lds<KK, MM>), dim3(grid), dim3(1024), lds, s, words, nw, nw_alloc, ks, n, mp,
                     store_all ? 1u : 0u);
}

hipError_t launch_insert_lds(int keyk, int mode, uint32_t* words, uint64_t m, uint64_t nw_alloc, const KeySrc& ks,
                             uint64_t n, const ModP& mp, bool store_all, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t nw = (m + 31) / 32;
  if (m > kInsertLdsMaxBits || nw_alloc < nw) return hipErrorInvalidValue;
  const uint32_t grid = store_all ? 1u : (uint32_t)std::min<uint64_t>(128, (n + 8191) / 8192);
  const size_t lds = nw * 4;
  ProfScope ps("k_insert_lds", s);
  CB_DISPATCH(keyk, mode, (insert_lds<KK, MM>(words, (uint32_t)nw, (uint32_t)nw_alloc, ks, n, mp, store_all, grid, lds, s)));
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
static void part_probe(const TilePlan& p, const KeySrc& ks, uint64_t n, const ModP& mp,
                       uint32_t* seg, uint2* ent, uint16_t* lkey, size_t lds, hipStream_t s) {
  allow_lds(k_part_probe<KK, MM, KPT>, lds);
  hipLaunchKernelGGL((k_part_probe<KK, MM, KPT>), dim3(p.nblk), dim3(kPartThreads), lds, s, ks, n,
                     mp, p.tb, p.T, seg, ent, lkey);
}

// Store cache policy of the build's two outputs (CB_BUILD_STORES, default
// 3): bit 0 write-through partition entries, bit 1 non-temporal tile
// write-back.
static uint32_t build_stores() {
  static const uint32_t v = (uint32_t)env_int("CB_BUILD_STORES", 3);
  return v;
}

template <int KK, int MM, int KPT>
static void build_part(const TilePlan& p, const BuildBatch& bb, uint32_t nb, const ModP& mp,
                       uint32_t* seg, uint32_t* ent, size_t lds, hipStream_t s) {
  if (p.sub) {  // 16-bit entries binned by 2^16-bit sub-tile
    allow_lds(k_build_part<KK, MM, KPT, uint16_t>, lds);
    hipLaunchKernelGGL((k_build_part<KK, MM, KPT, uint16_t>), dim3(p.nblk, nb), dim3(kBuildNT), lds, s, bb, mp,
                       16u, p.T << p.sub, seg, ent, build_stores());
    return;
  }
  allow_lds(k_build_part<KK, MM, KPT>, lds);
  hipLaunchKernelGGL((k_build_part<KK, MM, KPT>), dim3(p.nblk, nb), dim3(kBuildNT), lds, s, bb, mp,
                     p.tb, p.T, seg, ent, build_stores());
}

hipError_t launch_build_batch(int keyk, int mode, const BuildBatch& bb, uint32_t nb,
                              const ModP& mp, const TilePlan& p, uint32_t* seg, uint32_t* ent,
                              hipStream_t s) {
  if (!nb) return hipSuccess;
  if (!plan_ok(p) || nb > kMaxBuildBatch || p.nblk > kMaxBuildBlocks) return hipErrorInvalidValue;
  if (p.sub && (p.sub > 3 || p.tb != 16 + p.sub || ((uint64_t)p.T << p.sub) > kMaxTiles)) return hipErrorInvalidValue;
  const uint32_t TS = p.T << p.sub;  // partition bins
  const size_t lds1 = (size_t)(((TS + 4) & ~3u) + 4) * 4 + 2 * p.C * (p.sub ? 2 : 4);  // part_phases: hist, discard, stage
  {
    ProfScope ps("k_build_part", s);
    if (p.kpt == 1) {
      CB_DISPATCH(keyk, mode, (build_part<KK, MM, 1>(p, bb, nb, mp, seg, ent, lds1, s)));
    } else if (p.kpt == 2) {
      CB_DISPATCH(keyk, mode, (build_part<KK, MM, 2>(p, bb, nb, mp, seg, ent, lds1, s)));
    } else {
      CB_DISPATCH(keyk, mode, (build_part<KK, MM, 4>(p, bb, nb, mp, seg, ent, lds1, s)));
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t lds2 = (size_t)(1u << (p.tb - 5)) * 4;
  ProfScope ps("k_build_tile", s);
  if (p.sub) {
    const uint16_t* e16 = reinterpret_cast<const uint16_t*>(ent);
    if (p.sub == 2) {  // 2^18-bit tiles: 512-thread workgroups, four per CU
      allow_lds(k_build_tile_sub<8, 2, 2, 512>, lds2);
      hipLaunchKernelGGL((k_build_tile_sub<8, 2, 2, 512>), dim3(p.T, nb), dim3(512), lds2, s, bb, p.tb, p.T, seg,
                         p.nblk, e16, 2 * p.C, build_stores());
      return hipGetLastError();
    }
#define CB_TILE_SUB(SUBV)                                                                                 \
  allow_lds(k_build_tile_sub<4, 2, SUBV>, lds2);                                                         \
  hipLaunchKernelGGL((k_build_tile_sub<4, 2, SUBV>), dim3(p.T, nb), dim3(kBuildNT), lds2, s, bb, p.tb, p.T, seg, \
                     p.nblk, e16, 2 * p.C, build_stores())
    if (p.sub == 1) {
      CB_TILE_SUB(1);
    } else {
      CB_TILE_SUB(3);
    }
#undef CB_TILE_SUB
    return hipGetLastError();
  }
  // entries per (partition block, tile): 2 C / T on average (tiles of one
  // filter); two rounds of run loads once that passes ~3/4 of a wave
#ifdef CB_EXPERIMENTS
  static const int tile_nt = env_int("CB_BUILD_TILE_NT", 1024);  // 512: half-size tile workgroups
  if (tile_nt == 512) {
    allow_lds(k_build_tile<8, 2, 512>, lds2);
    hipLaunchKernelGGL((k_build_tile<8, 2, 512>), dim3(p.T, nb), dim3(512), lds2, s, bb, p.tb, p.T, seg, p.nblk,
                       ent, 2 * p.C, build_stores());
    return hipGetLastError();
  }
#endif
  if (2ull * p.C > 48ull * p.T) {
    allow_lds(k_build_tile<8, 2>, lds2);
    hipLaunchKernelGGL((k_build_tile<8, 2>), dim3(p.T, nb), dim3(kBuildNT), lds2, s, bb, p.tb, p.T, seg, p.nblk,
                       ent, 2 * p.C, build_stores());
  } else {
    allow_lds(k_build_tile<16, 1>, lds2);
    hipLaunchKernelGGL((k_build_tile<16, 1>), dim3(p.T, nb), dim3(kBuildNT), lds2, s, bb, p.tb, p.T, seg,
                       p.nblk, ent, 2 * p.C, build_stores());
  }
  return hipGetLastError();
}

hipError_t launch_build_tiled(int keyk, int mode, uint32_t* words, bool fresh, const KeySrc& ks,
                              uint64_t n, const ModP& mp, const TilePlan& p, uint32_t* seg,
                              uint32_t* ent, hipStream_t s) {
  if (!n) return hipSuccess;
  BuildBatch bb{};
  bb.ks[0] = ks;
  bb.n[0] = n;
  bb.words[0] = words;
  bb.fresh = fresh ? 1u : 0u;
  return launch_build_batch(keyk, mode, bb, 1, mp, p, seg, ent, s);
}

hipError_t launch_probe_partition(int keyk, int mode, const KeySrc& ks, uint64_t n,
                                  const ModP& mp, const TilePlan& p, uint32_t* seg, uint2* ent,
                                  uint16_t* lkey, hipStream_t s) {
  if (!n) return hipSuccess;
  if (!plan_ok(p) || p.tb + 12 > 32) return hipErrorInvalidValue;
  const size_t lds1 = ((size_t)((p.T + 4) & ~3u) + 2 * p.C + p.C / 2 + 8) * 4;
  ProfScope ps("k_part_probe", s);
  if (p.kpt == 4) {
    CB_DISPATCH(keyk, mode, (part_probe<KK, MM, 4>(p, ks, n, mp, seg, ent, lkey, lds1, s)));
  } else {
    CB_DISPATCH(keyk, mode, (part_probe<KK, MM, 8>(p, ks, n, mp, seg, ent, lkey, lds1, s)));
  }
  return hipGetLastError();
}

template <int RPT>
static hipError_t tile_probe(const FilterPtrs& fp, uint32_t nf, uint64_t n, const TilePlan& p,
                             const uint32_t* seg, const uint2* ent, uint32_t* masks, size_t lds,
                             uint32_t G, hipStream_t s) {
  static const uint32_t xflags = (uint32_t)env_int("CB_PROBE_XFLAGS", 0);
  // The instantiation must cover the tile exactly: RPT uint4 per thread.
  if ((1u << (p.tb - 5)) != (uint32_t)RPT * 4u * kTileProbeThreads) return hipErrorInvalidValue;
  constexpr int D = RPT >= 4 ? 2 : 4;  // 32-64 KiB of tiles in flight per workgroup
  allow_lds(k_tile_probe<8, RPT, D>, lds);
  hipLaunchKernelGGL((k_tile_probe<8, RPT, D>), dim3(p.T, G), dim3(kTileProbeThreads), lds, s, fp,
                     nf, p.tb, p.T, seg, p.nblk, ent, p.C, n, masks, xflags);
  return hipGetLastError();
}

hipError_t launch_probe_tiles(const FilterPtrs& fp, uint32_t nf, uint64_t n, const TilePlan& p,
                              const uint32_t* seg, const uint2* ent, const uint16_t* lkey,
                              uint32_t* masks, uint64_t* hits, uint64_t hwords, hipStream_t s) {
  if (!n || !nf) return hipSuccess;
  const uint32_t nbp = (p.nblk + 3) & ~3u;
  const size_t lds2 = ((size_t)2 * (1u << (p.tb - 5)) + 2 * nbp + kTileProbeThreads / 64) * 4 +
                      kFiltersPerGroup * 8;
  const uint32_t G = (nf + kFiltersPerGroup - 1) / kFiltersPerGroup;
  hipError_t e;
  {
    ProfScope ps("k_tile_probe", s);
    // tile bits = RPT * 16 B * 8 * 512 threads = RPT * 2^16
    switch (p.tb) {
      case 16: e = tile_probe<1>(fp, nf, n, p, seg, ent, masks, lds2, G, s); break;
      case 17: e = tile_probe<2>(fp, nf, n, p, seg, ent, masks, lds2, G, s); break;
      case 18: e = tile_probe<4>(fp, nf, n, p, seg, ent, masks, lds2, G, s); break;
      default: e = hipErrorInvalidValue;
    }
  }
  if (e != hipSuccess) return e;
  ProfScope ps("k_masks_to_hits", s);
  if (p.kpt == 4)
    hipLaunchKernelGGL((k_masks_to_hits<4>), dim3(p.nblk), dim3(kHitsThreads), 0, s, masks, lkey,
                       fp, nf, n, hits, hwords);
  else
    hipLaunchKernelGGL((k_masks_to_hits<8>), dim3(p.nblk), dim3(kHitsThreads), 0, s, masks, lkey,
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
