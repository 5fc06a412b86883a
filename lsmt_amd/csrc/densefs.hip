// densefs.hip — the FilterSet probe for dense batches: keys partitioned by
// set region, each region of the set streamed through LDS once.
//
// Same answer as k_set_probe (filterset.hip): per key, (a, b) = (h1 % m,
// h2 % m) (/root/reference/src/bloom.rs:26-37) and mask = set[a] & set[b]
// for every slot at once, set[b] read only where set[a] != 0 (the `&&` of
// may_contain, src/bloom.rs:48-51), over Database::get's table fan-out
// (src/lib.rs:129-134). What changes is the order of the reads. At C5's
// density (10M keys against a 256 MiB set of 2M 128-B lines) k_set_probe
// reads every line ~7 times, each a random 128-B fill: 14.3M fills, 1.8 GB
// of fabric traffic for 0.26 GB of distinct sectors. Here:
//
//   k_dense_part  (1024 threads x 3 batches of 4 keys per block): hash, bin
//                 every key by the 64 KiB region of the set holding set[a]
//                 (LDS count atomics, a block scan, LDS cursor atomics),
//                 write the block's entries
//                 region-sorted {b, a's offset in the region << 16 | key index
//                 in the block} as one contiguous run list, its run starts
//                 as one row of a block-major table (u16), and zero the
//                 block's hit words (no separate memset);
//   k_dense_seg_t transposes the run-start table to region-major (LDS tiles);
//   k_dense_probe (one workgroup per region, two per CU): stage the region
//                 (64 KiB, coalesced) in LDS, gather the region's runs from
//                 every partition block (a block scan of their lengths, each
//                 lane finding its entry's run by binary search), set[a] from
//                 LDS, set[b] by one global read only where set[a] != 0, and
//                 the few non-zero masks ORed into the hit rows (atomicOr).
//
// The set is read once as a stream (256 MiB) instead of ~10M random fills;
// the entries cost one 8-B round trip per key, and set[b] stays a random read
// for the ~45 % of keys whose set[a] is non-zero. Regions are dealt to XCDs
// in contiguous ranges, so the run lines adjacent regions share are fetched
// once per XCD. Selected by density (capi.cpp set_probe_*); results are the
// same bits, checked against the oracle (tests/test_dense_probe_gpu.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "blockscan.hpp"
#include "filterset.hpp"
#include "profile.hpp"
#include "setmask.hpp"

namespace cb {
namespace {

constexpr uint32_t kDenseNT = 1024;
// A partition block ranks NB batches of KPT keys per thread (C = 12288 keys):
// batch g + 1's key loads are in flight while batch g's ranks are taken, and
// fewer, larger blocks shorten the probe's per-region run table. One batch
// of 7 keys per thread (C = 7168, 1396 blocks at C5) measured 209-211 us per
// C5 step on three lanes; two of 5 (977 blocks) 194-196; three of 4 (814
// blocks) 190-191 (experiment r05_c5nb, HISTORY.md, same box, alternating).
#if defined(CB_EXPERIMENTS) && defined(CB_DENSE_KPT)
constexpr uint32_t kDenseKPT = CB_DENSE_KPT;  // (experiment builds: keys per partition thread and batch)
#else
constexpr uint32_t kDenseKPT = 4;
#endif
#if defined(CB_EXPERIMENTS) && defined(CB_DENSE_NB)
constexpr uint32_t kDenseNB = CB_DENSE_NB;  // (experiment builds: key batches per partition block)
#else
constexpr uint32_t kDenseNB = 3;
#endif
constexpr uint32_t kDenseC = kDenseNT * kDenseKPT * kDenseNB;  // keys per partition block (a multiple of 64)
static_assert(kDenseC % 64 == 0 && kDenseC < 65536, "block keys: whole hit words, u16 run starts");
constexpr uint32_t kRegionBytes = 65536;  // one region of the set, staged in LDS
constexpr uint32_t kDenseMaxRegions = 4096;  // the partition histogram (16 KiB of LDS)
constexpr uint32_t kDenseMaxBlocks = 2048;   // partition blocks per launch pair (the probe's run table)
constexpr uint32_t kProbeU = 4;              // entries per lane per round of the probe
// The partition pass at its natural 84-89 VGPRs runs five waves per SIMD (one
// 16-wave block per CU, though LDS would take two); the experiment build can
// force eight (two blocks per CU: 80-116 B of spill per lane at 7 keys per
// thread) and fewer keys per thread (CB_DENSE_KPT) for the A/B. Two blocks
// per CU at 5 keys per thread (12 B of spill): this pass 72.5 -> 55.5 us, but
// 1954 partition blocks instead of 1396 cost the probe 9 us, and the C5 step
// on three lanes went 209-211 -> 221-225 us (one lane 249 -> 242); at 4 keys
// per thread (no spill) the batch needs two chunks and the set is streamed
// twice: 265-268 us (experiment r05_c5part, HISTORY.md).
#if defined(CB_EXPERIMENTS) && defined(CB_DENSE_PART_LB8)
#define CB_DENSE_PART_WAVES 8
#elif defined(CB_EXPERIMENTS) && defined(CB_DENSE_PART_W)
#define CB_DENSE_PART_WAVES CB_DENSE_PART_W
#else
#define CB_DENSE_PART_WAVES 1
#endif

// Dynamic LDS of a partition block over R regions: the R + 1 counts (padded)
// and a discard word, then the block's C staged entries.
constexpr size_t dense_part_lds(uint32_t R) { return (size_t)(((R + 4) & ~3u) + 4) * 4 + (size_t)kDenseC * 8; }
constexpr size_t dense_part_lds_max() { return dense_part_lds(kDenseMaxRegions); }

// The partition pass's stores of the entries and of the zeroed hit words:
// non-temporal (written once, read by the probe launch on every XCD; the hit
// words then ORed there): k_dense_probe 150.3-150.7 -> 141.8-142.1 us, C5
// one lane 227.5-228.3 -> 219.9-220.3 us, three lanes 188.9-189.8 -> 177.6-
// 178.1 us, against plain stores; write-through (sc1) buffer stores measured
// as plain, and the entries alone non-temporal 143.4 us (round 6, HISTORY.md).
// Experiment builds: CB_DENSE_ST 0 plain, 1 write-through, 2 non-temporal;
// CB_DENSE_HST 0 the hit words plain.
#if defined(CB_EXPERIMENTS) && defined(CB_DENSE_ST)
constexpr int kDenseSt = CB_DENSE_ST;
#else
constexpr int kDenseSt = 2;
#endif
#if defined(CB_EXPERIMENTS) && defined(CB_DENSE_HST)
constexpr bool kDenseHitsNt = CB_DENSE_HST;
#else
constexpr bool kDenseHitsNt = true;
#endif
typedef uint32_t dense_u32x4 __attribute__((ext_vector_type(4)));
typedef int dense_i32x4 __attribute__((ext_vector_type(4)));

// XCD-aware region order (workgroups are dealt round-robin over the 8 XCDs):
// XCD x takes regions [x R/8, (x+1) R/8) in order.
__device__ __forceinline__ uint32_t xcd_region(uint32_t bid, uint32_t R) {
  if (R & 7u) return bid;
  return (bid & 7u) * (R >> 3) + (bid >> 3);
}

// Keys [k0 + blockIdx.x C, ...) of the chunk: positions, region bins, the
// block's region-sorted entries and its column of the run-start table.
template <int KEYK, int MODE, int W>
__global__ __launch_bounds__(kDenseNT, CB_DENSE_PART_WAVES) void k_dense_part(KeySrc ks, uint64_t k0, uint64_t n, ModP mp,
                                                         uint32_t rshift, uint32_t R,
                                                         uint16_t* __restrict__ seg, uint32_t segstride,
                                                         uint2* __restrict__ ent, uint64_t* __restrict__ hits,
                                                         uint64_t hwords, uint32_t used) {
  constexpr uint32_t NT = kDenseNT, KPT = kDenseKPT, C = kDenseC;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t b = blockIdx.x;
  const uint32_t Rp = (R + 4) & ~3u;  // hist: R + 1 counts (zero-padded to Rp), a discard word at Rp
  uint32_t* hist = smem;
  uint2* stage = reinterpret_cast<uint2*>(smem + Rp + 4);
  const uint32_t tid = threadIdx.x;
  const uint64_t kb = k0 + (uint64_t)b * C;  // the block's first key
  const uint32_t pmask = (1u << rshift) - 1u;
  for (uint32_t i = tid; i < Rp + 4; i += NT) hist[i] = 0;
  // positions first: every key load of a batch in flight together; with
  // NB > 1 batches, batch g + 1's loads go out while batch g's ranks are taken
  constexpr uint32_t NB = kDenseNB, CB = NT * KPT;  // keys per batch
  // no rank is kept per key: the count pass's atomics only count, and the
  // scatter takes each entry's slot from a second atomic on its bin's cursor
  // (two registers per key instead of three; an entry's place inside its run
  // is immaterial to the probe)
  uint32_t pa[NB][KPT], pb[NB][KPT];
  bool live[NB][KPT];
#pragma unroll
  for (uint32_t g = 0; g < NB; ++g) {
    const uint64_t kg = kb + (uint64_t)g * CB;
    if constexpr (KEYK == KEY_FIXED16 && MODE == MOD_POW2_32) {
      uint4 kv[KPT];
      const uint4* keys = reinterpret_cast<const uint4*>(ks.bytes);
#pragma unroll
      for (int j = 0; j < (int)KPT; ++j) {
        const uint64_t k = kg + (uint64_t)j * NT + tid;
        live[g][j] = k < n;
        kv[j] = keys[live[g][j] ? k : n - 1];
      }
#pragma unroll
      for (int j = 0; j < (int)KPT; ++j) {
        uint32_t h1, h2;
        hash16_u32(kv[j], h1, h2);
        pa[g][j] = h1 & (uint32_t)mp.mask;
        pb[g][j] = h2 & (uint32_t)mp.mask;
      }
    } else {
#pragma unroll
      for (int j = 0; j < (int)KPT; ++j) {
        const uint64_t k = kg + (uint64_t)j * NT + tid;
        live[g][j] = k < n;
        uint64_t a = 0, b = 0;
        if (live[g][j]) key_positions<KEYK, MODE>(ks, k, mp, a, b);
        pa[g][j] = (uint32_t)a;  // m <= 2^32: positions fit (dense_ok)
        pb[g][j] = (uint32_t)b;
      }
    }
    if (g == 0) __syncthreads();  // hist zeroed
#pragma unroll
    for (int j = 0; j < (int)KPT; ++j) atomicAdd(&hist[live[g][j] ? pa[g][j] >> rshift : Rp], 1u);
  }
  __syncthreads();
  {
    // exclusive scan of the R + 1 counts by every wave (a wave-0 scan of
    // 4096 bins is a ~2 us chain per block): thread t owns RPT consecutive
    // bins, one block scan of the thread sums, then the prefixes in place
    constexpr uint32_t RPT = (kDenseMaxRegions + 4 + NT - 1) / NT;
    uint32_t c[RPT], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < RPT; ++j) {
      const uint32_t i = tid * RPT + j;
      c[j] = i < Rp ? hist[i] : 0u;
      sum += c[j];
    }
    uint64_t tot;
    uint32_t run = (uint32_t)block_scan<NT>(sum, &tot);
#pragma unroll
    for (uint32_t j = 0; j < RPT; ++j) {
      const uint32_t i = tid * RPT + j;
      if (i < Rp) hist[i] = run;
      run += c[j];
    }
  }
  __syncthreads();  // hist[r] = region r's run start in the block, hist[R] = the block's entry count
  // row blockIdx.x of the block-major run-start table (R + 1 u16, coalesced;
  // the probe reads its two columns, L2-resident per XCD)
  {
    uint16_t* row = seg + (uint64_t)b * segstride;
    for (uint32_t t = tid; t <= R; t += NT) row[t] = (uint16_t)hist[t];
  }
  __syncthreads();  // the run row is out: hist becomes the bins' cursors
#pragma unroll
  for (uint32_t g = 0; g < NB; ++g)
#pragma unroll
    for (int j = 0; j < (int)KPT; ++j)
      if (live[g][j]) {
        const uint32_t at = atomicAdd(&hist[pa[g][j] >> rshift], 1u);
        stage[at] = make_uint2(pb[g][j], ((pa[g][j] & pmask) << 16) | (g * CB + j * NT + tid));
      }
  // the block's hit words (keys kb .. kb + C, whole words) start at zero:
  // the probe only ORs the set bits in
  {
    const uint64_t nw = (n + 63) / 64, w0 = kb / 64;
    constexpr uint32_t WPB = C / 64;
    for (uint32_t i = tid; i < used * WPB; i += NT) {
      const uint32_t f = i / WPB, w = i % WPB;
      if (w0 + w < nw) {
        if constexpr (kDenseHitsNt)
          __builtin_nontemporal_store(0ull, reinterpret_cast<unsigned long long*>(hits) + (uint64_t)f * hwords + w0 + w);
        else
          hits[(uint64_t)f * hwords + w0 + w] = 0ull;
      }
    }
  }
  __syncthreads();
  const uint32_t total = hist[R];
  uint2* out = ent + (uint64_t)b * C;
  const uint32_t n2 = total / 2;
  if constexpr (kDenseSt == 1) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, total * 8, 0x00020000);
    for (uint32_t i = tid; i < n2; i += NT) {
      const uint4 v = reinterpret_cast<const uint4*>(stage)[i];
      const dense_i32x4 w = {(int)v.x, (int)v.y, (int)v.z, (int)v.w};
      __builtin_amdgcn_raw_buffer_store_b128(w, rs, i * 16, 0, 16);
    }
  } else if constexpr (kDenseSt == 2) {
    for (uint32_t i = tid; i < n2; i += NT) {
      const uint4 v = reinterpret_cast<const uint4*>(stage)[i];
      const dense_u32x4 w = {v.x, v.y, v.z, v.w};
      __builtin_nontemporal_store(w, reinterpret_cast<dense_u32x4*>(out) + i);
    }
  } else {
    for (uint32_t i = tid; i < n2; i += NT) reinterpret_cast<uint4*>(out)[i] = reinterpret_cast<const uint4*>(stage)[i];
  }
  if (tid == 0 && (total & 1u)) out[total - 1] = stage[total - 1];
}

// The run-start table, block-major [nblk][R + 1] (the partition pass's
// coalesced rows) -> region-major [R + 1][tstride] (the probe's contiguous
// columns), through 64 x 64 LDS tiles: every load and store is a 128-B row
// piece. (Measured against: each block's column stored scattered from the
// partition pass, 86 against 73 us for that pass; the same with the blocks
// dealt to XCDs in contiguous ranges, 88 us; the probe reading the
// block-major rows scattered, +33 us for the probe. This launch: 12 us.)
__global__ __launch_bounds__(256) void k_dense_seg_t(const uint16_t* __restrict__ in, uint32_t istride,
                                                      uint32_t nblk, uint32_t nrow, uint16_t* __restrict__ out,
                                                      uint32_t ostride) {
  __shared__ uint16_t tile[64][66];
  const uint32_t tx = threadIdx.x & 63u, ty = threadIdx.x >> 6;
  const uint32_t b0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
  for (uint32_t i = ty; i < 64; i += 4) {
    const uint32_t b = b0 + i, r = r0 + tx;
    tile[i][tx] = (b < nblk && r < nrow) ? in[(uint64_t)b * istride + r] : (uint16_t)0;
  }
  __syncthreads();
  for (uint32_t i = ty; i < 64; i += 4) {
    const uint32_t r = r0 + i, b = b0 + tx;
    if (r < nrow && b < nblk) out[(uint64_t)r * ostride + b] = tile[tx][i];
  }
}

// Last b with P[b] <= j (P: exclusive prefix of the runs' lengths, P[0] = 0).
__device__ __forceinline__ uint32_t run_of(const uint32_t* P, uint32_t nblk, uint32_t j) {
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

template <int W>
__global__ __launch_bounds__(kDenseNT, 8) void k_dense_probe(const void* __restrict__ setp, uint64_t m,
                                                             uint32_t rshift, uint32_t R,
                                                             const uint16_t* __restrict__ seg, uint32_t segstride,
                                                             uint32_t nblk, const uint2* __restrict__ ent,
                                                             uint64_t k0, uint64_t* __restrict__ hits,
                                                             uint64_t hwords, uint32_t used, uint32_t xflags) {
  typedef typename std::conditional<W == 32, uint32_t, uint64_t>::type word_t;
  constexpr uint32_t NT = kDenseNT, C = kDenseC, P = kRegionBytes / sizeof(word_t);
  __shared__ __attribute__((aligned(16))) word_t stage[P];
  __shared__ uint32_t scan[kDenseMaxBlocks + 1];
  __shared__ uint16_t starts[kDenseMaxBlocks];
  const word_t* __restrict__ set = reinterpret_cast<const word_t*>(setp);
  // rows exist for the used slots only (hits is used x hwords): slots past
  // them are never written, whatever their set words hold
  const word_t usedm = used >= W ? ~(word_t)0 : (((word_t)1 << used) - 1);
  const uint32_t tid = threadIdx.x;
  const uint32_t r = xcd_region(blockIdx.x, R);
  const uint64_t p0 = (uint64_t)r << rshift;
  // the region's words in flight (64 KiB: four 16-B loads per lane) with the
  // run table's two rows
  constexpr uint32_t PER4 = 16 / sizeof(word_t), N4 = P / PER4;
  uint4 v[N4 / NT];
#pragma unroll
  for (uint32_t j = 0; j < N4 / NT; ++j) {
    const uint64_t p = p0 + (uint64_t)(j * NT + tid) * PER4;
    if (p + PER4 <= m) {
      v[j] = reinterpret_cast<const uint4*>(set + p)[0];
    } else {  // the last region's tail (m not a multiple of the region)
      word_t t[PER4];
#pragma unroll
      for (uint32_t q = 0; q < PER4; ++q) t[q] = p + q < m ? set[p + q] : (word_t)0;
      v[j] = *reinterpret_cast<const uint4*>(t);
    }
  }
  uint32_t s0[2] = {0, 0}, len[2] = {0, 0};
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const uint32_t b = 2 * tid + u;
    if (b < nblk) {  // rows r and r + 1 of the region-major table: contiguous over the blocks
      s0[u] = seg[(uint64_t)r * segstride + b];
      len[u] = (uint32_t)seg[(uint64_t)(r + 1) * segstride + b] - s0[u];
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < N4 / NT; ++j) reinterpret_cast<uint4*>(stage)[j * NT + tid] = v[j];
  uint64_t total64;
  const uint32_t pre = (uint32_t)block_scan<NT>((uint64_t)(len[0] + len[1]), &total64);
  const uint32_t E = (uint32_t)total64;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const uint32_t b = 2 * tid + u;
    if (b < nblk) {
      scan[b] = pre + (u ? len[0] : 0u);
      starts[b] = (uint16_t)s0[u];
    }
  }
  if (tid == 0) scan[nblk] = E;
  __syncthreads();
  for (uint32_t base = 0; base < E; base += kProbeU * NT) {
    // a round of kProbeU entries per lane: every load of the round in
    // flight together (entries, then the set[b] reads)
    uint2 e[kProbeU];
    uint32_t blk[kProbeU];
#pragma unroll
    for (uint32_t u = 0; u < kProbeU; ++u) {
      const uint32_t i = base + u * NT + tid;
      blk[u] = 0;
      e[u] = make_uint2(0, 0xFFFFFFFFu);
      if (i < E) {
        blk[u] = run_of(scan, nblk, i);
        e[u] = ent[(uint64_t)blk[u] * C + starts[blk[u]] + (i - scan[blk[u]])];
      }
    }
    word_t va[kProbeU], vb[kProbeU];
#pragma unroll
    for (uint32_t u = 0; u < kProbeU; ++u) va[u] = e[u].y != 0xFFFFFFFFu ? stage[e[u].y >> 16] : (word_t)0;
#pragma unroll
    for (uint32_t u = 0; u < kProbeU; ++u)
      vb[u] = va[u] ? ((xflags & 1u) ? va[u] : set[e[u].x]) : (word_t)0;  // src/bloom.rs:50's &&
#pragma unroll
    for (uint32_t u = 0; u < kProbeU; ++u) {
      word_t mask = va[u] & vb[u] & usedm;
      if (mask && !(xflags & 2u)) {
        const uint64_t key = k0 + (uint64_t)blk[u] * C + (e[u].y & 0xFFFFu);
        const unsigned long long bit = 1ull << (key & 63u);
        unsigned long long* row = reinterpret_cast<unsigned long long*>(hits) + key / 64;
        while (mask) {
          const uint32_t f = (uint32_t)__builtin_ctzll((uint64_t)mask);
          mask &= mask - 1;
          atomicOr(row + (uint64_t)f * hwords, bit);
        }
      }
    }
  }
}

template <int KK, int MM, int WW>
void dense_part(uint32_t nblk, size_t lds, hipStream_t s, const KeySrc& ks, uint64_t k0, uint64_t kend,
                const ModP& mp, uint32_t rshift, uint32_t R, uint16_t* seg, uint32_t stride, uint2* ent,
                uint64_t* hits, uint64_t hwords, uint32_t used) {
  // ~115 KiB of dynamic LDS at C5: past the 64 KiB a launch gets without
  // asking, set once per instantiation
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(k_dense_part<KK, MM, WW>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)dense_part_lds_max());
  (void)attr;
  hipLaunchKernelGGL((k_dense_part<KK, MM, WW>), dim3(nblk), dim3(kDenseNT), lds, s, ks, k0, kend, mp, rshift, R,
                     seg, stride, ent, hits, hwords, used);
}

}  // namespace

uint32_t dense_regions(uint32_t width, uint64_t m) {
  const uint64_t P = kRegionBytes / (width / 8);
  return (uint32_t)((m + P - 1) / P);
}

// The device's LDS per workgroup (queried once; the current device is the
// set's, every caller holds a DeviceGuard): the partition block needs
// dense_part_lds(R), the probe 64 KiB + its run tables.
static size_t device_lds_limit() {
  static thread_local int dev = -1;
  static thread_local size_t lim = 0;
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return 0;
  if (d != dev) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, d) != hipSuccess) v = 0;
    dev = d;
    lim = (size_t)v;
  }
  return lim;
}

bool set_dense_shape_ok(uint32_t width, uint64_t m) {
  if (!((width == 32 || width == 64) && m && m <= (1ull << 32) && dense_regions(width, m) <= kDenseMaxRegions))
    return false;
  // a device with less LDS than the passes need takes k_set_probe instead
  const size_t probe_lds = kRegionBytes + (kDenseMaxBlocks + 1) * 4 + kDenseMaxBlocks * 2;
  const size_t need = std::max(dense_part_lds(dense_regions(width, m)), probe_lds);
  return device_lds_limit() >= need;
}

bool set_probe_dense_ok(uint32_t width, uint64_t m, uint64_t n) {
  if (!set_dense_shape_ok(width, m)) return false;
  // keys per 128-B line of the set: the streamed region pays for itself once
  // each line would take ~2 random fills (C3: 0.5 per line, C5: 4.8)
  const uint64_t lines = (m * (width / 8) + 127) / 128;
  return n >= 2 * lines;
}

uint64_t dense_scratch_bytes(uint32_t width, uint64_t m, uint64_t n) {
  const uint64_t chunk = (uint64_t)kDenseMaxBlocks * kDenseC;
  const uint64_t nk = n < chunk ? n : chunk;
  const uint64_t nblk = (nk + kDenseC - 1) / kDenseC;
  const uint64_t R1 = (uint64_t)dense_regions(width, m) + 1;
  const uint64_t stride = (R1 + 63) & ~63ull, tstride = (nblk + 63) & ~63ull;  // u16, 128-B rows
  const uint64_t segb = nblk * stride * 2 + R1 * tstride * 2;
  return nblk * kDenseC * 8 + ((segb + 255) & ~255ull);
}

hipError_t launch_set_probe_dense(int keyk, int mode, uint32_t width, const void* set, uint32_t used,
                                  const KeySrc& ks, uint64_t n, const ModP& mp, uint64_t* hits, uint64_t hwords,
                                  void* scratch, hipStream_t s) {
  if (!n || !used) return hipSuccess;
  if (!set_dense_shape_ok(width, mp.m)) return hipErrorInvalidValue;
  const uint32_t R = dense_regions(width, mp.m);
  const uint32_t rshift = width == 32 ? 14 : 13;  // 64 KiB of 4-B or 8-B words
  const uint64_t chunk = (uint64_t)kDenseMaxBlocks * kDenseC;
  const uint64_t nk0 = n < chunk ? n : chunk;
  const uint32_t nblk0 = (uint32_t)((nk0 + kDenseC - 1) / kDenseC);
  const uint32_t stride = (R + 1 + 63) & ~63u, tstride = (nblk0 + 63) & ~63u;
  uint2* ent = reinterpret_cast<uint2*>(scratch);
  uint16_t* seg = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(scratch) + (uint64_t)nblk0 * kDenseC * 8);
  uint16_t* segT = seg + (uint64_t)nblk0 * stride;
  const size_t lds1 = dense_part_lds(R);
  uint32_t xflags = 0;
#ifdef CB_EXPERIMENTS
  // timing-only A/B (the hits are wrong): CB_DENSE_X bit 0 skips the set[b]
  // gathers, bit 1 the hit atomics
  static const uint32_t env_x = getenv("CB_DENSE_X") ? (uint32_t)atoi(getenv("CB_DENSE_X")) : 0u;
  xflags = env_x;
#endif
  for (uint64_t k0 = 0; k0 < n; k0 += chunk) {
    const uint64_t nk = n - k0 < chunk ? n - k0 : chunk;
    const uint32_t nblk = (uint32_t)((nk + kDenseC - 1) / kDenseC);
    {
      ProfScope ps("k_dense_part", s);
      // the keys of this chunk: k in [k0, k0 + nk), indices global
      CB_SET_DISPATCH(keyk, mode, width,
                      (dense_part<KK, MM, WW>(nblk, lds1, s, ks, k0, k0 + nk, mp, rshift, R, seg, stride, ent, hits,
                                              hwords, used)));
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    {
      ProfScope ps("k_dense_seg_t", s);
      hipLaunchKernelGGL(k_dense_seg_t, dim3((nblk + 63) / 64, (R + 1 + 63) / 64), dim3(256), 0, s, seg, stride, nblk,
                         R + 1, segT, tstride);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    {
      ProfScope ps("k_dense_probe", s);
      if (width == 32)
        hipLaunchKernelGGL((k_dense_probe<32>), dim3(R), dim3(kDenseNT), 0, s, set, mp.m, rshift, R, segT, tstride,
                           nblk, ent, k0, hits, hwords, used, xflags);
      else
        hipLaunchKernelGGL((k_dense_probe<64>), dim3(R), dim3(kDenseNT), 0, s, set, mp.m, rshift, R, segT, tstride,
                           nblk, ent, k0, hits, hwords, used, xflags);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

}  // namespace cb
