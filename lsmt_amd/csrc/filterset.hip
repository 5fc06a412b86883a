// filterset.hip — bit-sliced filter sets for the read-path fan-out.
//
// A FilterSet holds up to W (32 or 64) Bloom filters of one size m in a
// position-major layout: word p (uint32 for W = 32, uint64 for W = 64) has
// bit s = bit p of the filter in slot s. Database::get probes every SSTable
// for each key (/root/reference/src/lib.rs:129-134); with m uniform across
// tables (src/sstable.rs:44,59) one key's answer for ALL slots is
//   set[a] & set[b],  (a, b) = (h1 % m, h2 % m)            (src/bloom.rs:26-51)
// i.e. two random word reads per key instead of one per (key, filter). The
// reference's `&&` short-circuit is kept per key: set[b] is read only when
// set[a] has any slot bit set.
//
// Compulsory HBM bytes per probe batch (SURVEY.md §8d alternative layout):
// 64 B x distinct sectors touched by the a/b reads + 16 B/key + the hit bitmap.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "blockscan.hpp"
#include "filterset.hpp"
#include "profile.hpp"
#include "setmask.hpp"
#include "zone.hpp"

namespace cb {
namespace {

typedef const __attribute__((address_space(1))) uint64_t* gsp64;

// In-register 32x32 bit transpose: on entry a[i] bit j = element (i, j); on
// exit a[j] bit i = element (i, j). Every index is static after unrolling.
template <int J>
__device__ __forceinline__ void transpose_step(uint32_t (&a)[32]) {
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
  transpose_step<16>(a);
  transpose_step<8>(a);
  transpose_step<4>(a);
  transpose_step<2>(a);
  transpose_step<1>(a);
}

// Rebuild slots 0..nf-1 from packed filters (slots >= nf become zero). One
// thread per 32-position group g: reads word g of every filter (coalesced
// across threads), transposes, writes the 32 set words of the group.
template <int W>
__global__ __launch_bounds__(256) void k_set_build(FilterPtrs fp, uint32_t nf, uint64_t ngroups,
                                                   uint64_t m, void* __restrict__ set,
                                                   uint32_t* __restrict__ any) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < ngroups; g += stride) {
    uint32_t a[32], u = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      a[i] = (uint32_t)i < nf ? fp.w[i][g] : 0u;
      u |= a[i];
    }
    transpose32(a);
    const uint64_t p0 = g * 32;
    const uint32_t valid = (uint32_t)min<uint64_t>(32, m - p0);
    if constexpr (W == 32) {
      uint32_t* out = reinterpret_cast<uint32_t*>(set) + p0;
      if (valid == 32) {
#pragma unroll
        for (int q = 0; q < 8; ++q)
          reinterpret_cast<uint4*>(out)[q] = make_uint4(a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]);
      } else {
#pragma unroll
        for (int j = 0; j < 32; ++j)
          if ((uint32_t)j < valid) out[j] = a[j];
      }
    } else {
      uint32_t c[32];
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        c[i] = (uint32_t)(32 + i) < nf ? fp.w[32 + i][g] : 0u;
        u |= c[i];
      }
      transpose32(c);
      uint32_t* out = reinterpret_cast<uint32_t*>(set) + 2 * p0;  // (lo, hi) per position
      if (valid == 32) {
#pragma unroll
        for (int q = 0; q < 16; ++q)
          reinterpret_cast<uint4*>(out)[q] = make_uint4(a[2 * q], c[2 * q], a[2 * q + 1], c[2 * q + 1]);
      } else {
#pragma unroll
        for (int j = 0; j < 32; ++j)
          if ((uint32_t)j < valid) {
            out[2 * j] = a[j];
            out[2 * j + 1] = c[j];
          }
      }
    }
    any[g] = u;
  }
}

// OR a packed filter into a slot known to be all-zero: only the set bits
// (~1.5% at BASELINE densities) touch the set. Position p belongs to exactly
// one thread (the one owning word p/32), so a plain read-modify-write is safe.
template <int W>
__global__ __launch_bounds__(256) void k_set_or_slot(const uint32_t* __restrict__ words,
                                                     uint64_t nwords, uint32_t slot,
                                                     void* __restrict__ set,
                                                     uint32_t* __restrict__ any) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < nwords; w += stride) {
    uint32_t v = words[w];
    if (v) any[w] |= v;
    while (v) {
      const uint32_t j = __builtin_ctz(v);
      v &= v - 1;
      const uint64_t p = w * 32 + j;
      if constexpr (W == 32)
        reinterpret_cast<uint32_t*>(set)[p] |= 1u << slot;
      else
        reinterpret_cast<uint64_t*>(set)[p] |= 1ull << slot;
    }
  }
}

// Replace a slot's bits wholesale (slot possibly non-zero): every position is
// rewritten. words == nullptr clears the slot.
template <int W>
__global__ __launch_bounds__(256) void k_set_put_slot(const uint32_t* __restrict__ words,
                                                      uint64_t m, uint32_t slot,
                                                      void* __restrict__ set,
                                                      uint32_t* __restrict__ any) {
  const uint64_t ngroups = (m + 31) / 32;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < ngroups; g += stride) {
    const uint32_t v = words ? words[g] : 0u;
    const uint32_t valid = (uint32_t)min<uint64_t>(32, m - g * 32);
    uint32_t u = 0;
    for (uint32_t j = 0; j < valid; ++j) {
      const uint64_t p = g * 32 + j;
      if constexpr (W == 32) {
        uint32_t* s = reinterpret_cast<uint32_t*>(set) + p;
        const uint32_t nv = (*s & ~(1u << slot)) | (((v >> j) & 1u) << slot);
        *s = nv;
        u |= (uint32_t)(nv != 0) << j;
      } else {
        uint64_t* s = reinterpret_cast<uint64_t*>(set) + p;
        const uint64_t nv = (*s & ~(1ull << slot)) | ((uint64_t)((v >> j) & 1u) << slot);
        *s = nv;
        u |= (uint32_t)(nv != 0) << j;
      }
    }
    any[g] = u;
  }
}

constexpr uint32_t kSetProbeThreads = 64 * kSetWords;  // one 64-key hit word per wave
#ifdef CB_EXPERIMENTS
constexpr uint32_t kFlowThreads = 256;  // k_set_probe_flow: 4 waves per block
constexpr uint32_t kFlowWaves = kFlowThreads / 64;
#endif

// set_key_mask for a 16-byte key already in registers (no union pre-test).
template <int MODE, int W, bool SC>
__device__ __forceinline__ typename std::conditional<W == 32, uint32_t, uint64_t>::type set_key_mask_u4(
    const void* __restrict__ set, const uint4& kv, bool ok, const ModP& mp, const ZoneView& zv,
    const BoundPrefix* zp) {
  typedef typename std::conditional<W == 32, uint32_t, uint64_t>::type word_t;
  typedef const __attribute__((address_space(1))) word_t* gptr;
  const gptr sp = (gptr)set;
  uint64_t pa = 0, pb = 0;
  if (ok) key_positions_u4<MODE>(kv, mp, pa, pb);
  const word_t va = ok ? sp[pa] : (word_t)0;
  word_t vb;
  if constexpr (!SC)
    vb = ok ? sp[pb] : (word_t)0;
  else
    vb = va ? sp[pb] : (word_t)0;
  word_t mask = va & vb;
  word_t c = zv.gated ? mask & (word_t)zv.gated : (word_t)0;
  if (c) {
    const uint32_t kw[4] = {be32(kv.x), be32(kv.y), be32(kv.z), be32(kv.w)};
    while (c) {
      const uint32_t s = (uint32_t)__builtin_ctzll((uint64_t)c);
      c &= c - 1;
      if (cmp16(kw, zp[2 * s]) < 0 || cmp16(kw, zp[2 * s + 1]) > 0) mask &= ~((word_t)1 << s);
    }
  }
  return mask;
}

// The wave's 64 keys' masks -> lane f holds slot f's 64-key hit word.
template <int W, class word_t>
__device__ __forceinline__ uint64_t slot_words(word_t mask, uint32_t used, uint32_t lane) {
  uint64_t mine = 0;
#pragma unroll
  for (uint32_t f = 0; f < (uint32_t)W; ++f) {
    if (f < used) {
      const uint64_t bal = __ballot((mask >> f) & 1u);
      mine = (lane == f) ? bal : mine;
    }
  }
  return mine;
}

// The block's hit positions into the exchange pack (PackSink): the block's
// set bits are counted (one entry per thread: thread i = slot i / 16, word
// i % 16), one relaxed atomic add claims their slots (low half: slots, high
// half: finished blocks, so the last block writes the total), and each
// thread writes its word's positions in order. Words past the batch are zero
// (their keys were never probed), so they add nothing.
__device__ __forceinline__ void emit_positions(const PackSink& sink, const uint64_t (&hb)[64][kSetWords],
                                               uint32_t used, uint64_t wbase, uint64_t hwords) {
  __shared__ uint32_t s_base;
  const uint32_t i = threadIdx.x;
  const uint64_t v = i < used * kSetWords ? hb[i / kSetWords][i % kSetWords] : 0ull;
  uint64_t total;
  const uint64_t excl = block_scan<kSetProbeThreads>((uint64_t)__popcll(v), &total);
  uint32_t* dir = sink.pack + 2 + sink.cap;
  if (i == 0) {
    const unsigned long long old = atomicAdd(sink.ctl + sink.par, (1ull << 32) | total);
    s_base = (uint32_t)old;
    if ((uint32_t)(old >> 32) == gridDim.x - 1) {  // the last claim: every block is counted
      sink.pack[0] = (uint32_t)old + (uint32_t)total;
      sink.pack[1] = 0;
    }
    if (blockIdx.x == 0)
      __hip_atomic_store(sink.ctl + (sink.par ^ 1u), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    dir[2 * (uint64_t)blockIdx.x] = (uint32_t)old;
    dir[2 * (uint64_t)blockIdx.x + 1] = (uint32_t)total;
  }
  __syncthreads();
  uint64_t slot = (uint64_t)s_base + excl, bits = v;
  const uint64_t pos0 = ((uint64_t)(i / kSetWords) * hwords + wbase + i % kSetWords) * 64;
  while (bits) {
    const uint32_t b = (uint32_t)__builtin_ctzll(bits);
    bits &= bits - 1;
    if (slot < sink.cap) sink.pack[2 + slot] = (uint32_t)(pos0 + b);
    ++slot;
  }
}

// One key per lane, one 64-key hit word per wave, 16 waves per block. Ballots
// turn each 64-key word into one hit word per slot, staged in LDS so every
// slot row leaves as a contiguous 128-byte segment. (Two or four keys per
// lane, to keep more independent reads in flight, measured no faster: the
// wave count already saturates the memory pipeline. Non-temporal key loads
// and hit stores, to keep the streamed bytes out of the set's cache lines,
// measured no different: 40.4 us. 512-thread blocks (8 hit words) measured
// 40.9-41.1 us.)
template <int KEYK, int MODE, int W, bool SC>
__global__ __launch_bounds__(kSetProbeThreads) void k_set_probe(const void* __restrict__ set,
                                                                const uint32_t* __restrict__ any,
                                                                uint32_t used, KeySrc ks,
                                                                uint64_t n, ModP mp, ZoneView zv,
                                                                uint64_t* __restrict__ hits,
                                                                uint64_t hwords, PackSink sink) {
  __shared__ uint64_t hb[64][kSetWords];
  __shared__ BoundPrefix zp[2 * W];  // gated 16-byte keys: the bounds' prefixes, staged
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  stage_zone_prefixes<KEYK, W>(zv, zp, kSetProbeThreads);  // issued alongside the key loads
  const uint64_t wbase = (uint64_t)blockIdx.x * kSetWords;
  const uint64_t k = (wbase + wave) * 64 + lane;
  const auto mask = set_key_mask<KEYK, MODE, W, SC, true>(set, any, ks, k, k < n, mp, zv, zp);
  const uint64_t mine = slot_words<W>(mask, used, lane);
  if (lane < used) hb[lane][wave] = mine;
  __syncthreads();
  const uint64_t nw = (n + 63) / 64;
  for (uint32_t i = threadIdx.x; i < used * kSetWords; i += kSetProbeThreads) {
    const uint32_t f = i / kSetWords, w = i % kSetWords;
    if (wbase + w < nw) hits[(uint64_t)f * hwords + wbase + w] = hb[f][w];
  }
  if (sink.pack) emit_positions(sink, hb, used, wbase, hwords);
}

#ifdef CB_EXPERIMENTS
// Persistent form: a grid sized to the chip (blocks per CU x CUs), each wave
// striding over 64-key hit words on its own, with no block barrier after the
// start: a wave whose random reads came back early starts its next word at
// once instead of waiting for the block's slowest wave, so the launch has no
// block-round tail. Lane f stores slot f's word directly (one store
// instruction per wave and word; the 8-byte pieces of a row's 128-byte
// segment meet in L2).
template <int KEYK, int MODE, int W, bool SC>
__global__ __launch_bounds__(kFlowThreads) void k_set_probe_flow(const void* __restrict__ set,
                                                                 const uint32_t* __restrict__ any,
                                                                 uint32_t used, KeySrc ks,
                                                                 uint64_t n, ModP mp, ZoneView zv,
                                                                 uint64_t* __restrict__ hits,
                                                                 uint64_t hwords) {
  __shared__ BoundPrefix zp[2 * W];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  stage_zone_prefixes<KEYK, W>(zv, zp, kFlowThreads);
  if (KEYK == KEY_FIXED16 && zv.gated) __syncthreads();
  const uint64_t nw = (n + 63) / 64;
  const uint64_t stride = (uint64_t)gridDim.x * kFlowWaves;
  uint64_t w = (uint64_t)blockIdx.x * kFlowWaves + wave;
  if constexpr (KEYK == KEY_FIXED16) {
    // software-pipelined: the next word's key load is in flight while this
    // word's random set reads are outstanding
    const uint4* kp = reinterpret_cast<const uint4*>(ks.bytes);
    uint4 next = make_uint4(0, 0, 0, 0);
    if (w < nw && w * 64 + lane < n) next = kp[w * 64 + lane];
    for (; w < nw; w += stride) {
      const uint64_t k = w * 64 + lane;
      const uint4 kv = next;
      const uint64_t kn = (w + stride) * 64 + lane;
      if (w + stride < nw && kn < n) next = kp[kn];
      const auto mask = set_key_mask_u4<MODE, W, SC>(set, kv, k < n, mp, zv, zp);
      const uint64_t mine = slot_words<W>(mask, used, lane);
      if (lane < used) hits[(uint64_t)lane * hwords + w] = mine;
    }
  } else {
    for (; w < nw; w += stride) {
      const uint64_t k = w * 64 + lane;
      const auto mask = set_key_mask<KEYK, MODE, W, SC, false>(set, any, ks, k, k < n, mp, zv, zp);
      const uint64_t mine = slot_words<W>(mask, used, lane);
      if (lane < used) hits[(uint64_t)lane * hwords + w] = mine;
    }
  }
}
#endif  // CB_EXPERIMENTS

inline uint32_t grid_cap(uint64_t items, uint32_t cap) {
  uint64_t g = (items + 255) / 256;
  if (g < 1) g = 1;
  return (uint32_t)(g < cap ? g : cap);
}

}  // namespace

hipError_t launch_set_build(const FilterPtrs& fp, uint32_t nf, uint64_t m, uint32_t width,
                            void* set, uint32_t* any, hipStream_t s) {
  if (!m) return hipSuccess;
  const uint64_t ngroups = (m + 31) / 32;
  ProfScope ps("k_set_build", s);
  if (width == 32)
    hipLaunchKernelGGL((k_set_build<32>), dim3(grid_cap(ngroups, 8192)), dim3(256), 0, s, fp, nf,
                       ngroups, m, set, any);
  else
    hipLaunchKernelGGL((k_set_build<64>), dim3(grid_cap(ngroups, 8192)), dim3(256), 0, s, fp, nf,
                       ngroups, m, set, any);
  return hipGetLastError();
}

hipError_t launch_set_or_slot(const uint32_t* words, uint64_t m, uint32_t slot, uint32_t width,
                              void* set, uint32_t* any, hipStream_t s) {
  if (!m) return hipSuccess;
  const uint64_t nw = (m + 31) / 32;
  ProfScope ps("k_set_or_slot", s);
  if (width == 32)
    hipLaunchKernelGGL((k_set_or_slot<32>), dim3(grid_cap(nw, 8192)), dim3(256), 0, s, words, nw,
                       slot, set, any);
  else
    hipLaunchKernelGGL((k_set_or_slot<64>), dim3(grid_cap(nw, 8192)), dim3(256), 0, s, words, nw,
                       slot, set, any);
  return hipGetLastError();
}

hipError_t launch_set_put_slot(const uint32_t* words, uint64_t m, uint32_t slot, uint32_t width,
                               void* set, uint32_t* any, hipStream_t s) {
  if (!m) return hipSuccess;
  const uint64_t ng = (m + 31) / 32;
  ProfScope ps("k_set_put_slot", s);
  if (width == 32)
    hipLaunchKernelGGL((k_set_put_slot<32>), dim3(grid_cap(ng, 8192)), dim3(256), 0, s, words, m,
                       slot, set, any);
  else
    hipLaunchKernelGGL((k_set_put_slot<64>), dim3(grid_cap(ng, 8192)), dim3(256), 0, s, words, m,
                       slot, set, any);
  return hipGetLastError();
}

template <int KK, int MM, int WW>
static void set_probe(bool flow, const void* set, const uint32_t* any, uint32_t used, const KeySrc& ks,
                      uint64_t n, const ModP& mp, const ZoneView& zv, uint64_t* hits, uint64_t hwords,
                      uint32_t grid, hipStream_t s, const PackSink& sink) {
#ifdef CB_EXPERIMENTS
  if (flow) {
    hipLaunchKernelGGL((k_set_probe_flow<KK, MM, WW, true>), dim3(grid), dim3(kFlowThreads), 0, s, set, any,
                       used, ks, n, mp, zv, hits, hwords);
    return;
  }
#else
  (void)flow;
#endif
  // the reference's short-circuit (src/bloom.rs:50): set[b] only where set[a] != 0
  hipLaunchKernelGGL((k_set_probe<KK, MM, WW, true>), dim3(grid), dim3(kSetProbeThreads), 0, s, set, any, used,
                     ks, n, mp, zv, hits, hwords, sink);
}

#ifdef CB_EXPERIMENTS
// Compute units of the current device (cached per device).
static uint32_t device_cus() {
  static uint32_t cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cus[dev] = (uint32_t)v;
  }
  return cus[dev];
}
#endif

hipError_t launch_set_probe(int keyk, int mode, uint32_t width, const void* set,
                            const uint32_t* any, uint32_t used, const KeySrc& ks, uint64_t n,
                            const ModP& mp, const ZoneView* zones, uint64_t* hits,
                            uint64_t hwords, hipStream_t s, const PackSink* sink) {
  if (!n || !used) return hipSuccess;
  const PackSink nosink{nullptr, 0, nullptr, 0};
  const ZoneView zv = zones ? *zones : ZoneView{nullptr, nullptr, nullptr, 0};
  const uint64_t nw = (n + 63) / 64;
  uint32_t grid = (uint32_t)((nw + kSetWords - 1) / kSetWords);
  bool use_any = false, flow = false;
#ifdef CB_EXPERIMENTS
  // A/B knobs, compiled only into experiment builds (make EXTRA=-DCB_EXPERIMENTS):
  // CB_SET_ANY=1 the union pre-test (measured on C3: 52.8 vs 40.0 us, the 2
  // extra random reads per key into any[] cost as much as the set reads they
  // avoid); CB_SET_FLOW=1 the persistent k_set_probe_flow (38.6-39.3 us, no
  // better; slower at the C5 shape), CB_SET_FLOW_BPC its blocks per CU.
  static const bool env_any = [] {
    const char* v = getenv("CB_SET_ANY");
    return v && v[0] == '1';
  }();
  static const int env_flow_bpc = [] {
    const char* v = getenv("CB_SET_FLOW");
    if (!(v && v[0] == '1')) return 0;
    const char* b = getenv("CB_SET_FLOW_BPC");
    return b && atoi(b) > 0 ? atoi(b) : 8;
  }();
  use_any = env_any;
  flow = env_flow_bpc && !use_any && !sink;  // no union pre-test or pack in the flow form
  if (flow) {
    const uint64_t want = (nw + kFlowWaves - 1) / kFlowWaves;
    const uint64_t cap = (uint64_t)device_cus() * (uint32_t)env_flow_bpc;
    grid = (uint32_t)(want < cap ? want : cap);
  }
#endif
  ProfScope ps(zv.gated ? "k_set_probe_gated" : "k_set_probe", s);
  CB_SET_DISPATCH(keyk, mode, width,
                  (set_probe<KK, MM, WW>(flow, set, use_any ? any : nullptr, used, ks, n, mp, zv, hits, hwords,
                                         grid, s, sink ? *sink : nosink)));
  return hipGetLastError();
}

}  // namespace cb
