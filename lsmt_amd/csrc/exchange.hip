// exchange.hip — sparse form of the multi-GPU hit-bitmap exchange (SURVEY.md
// §8e). Each rank probes the replicated key batch against its filter subset
// and holds hit rows [rows][words]; Database::get (/root/reference/src/
// lib.rs:129-134) needs every table's answer per key, so the rows are
// all-gathered. At BASELINE densities the rows are sparse (a present key hits
// one table, false positives ~(1.55 %)^2 per (key, table)), so a rank ships
// the POSITIONS of its set bits instead of its dense rows:
//   k_hits_count / k_hits_emit — pack = {count, 0, positions...} with the
//       positions (row*words*64 + bit, u32) in ascending order: per-block
//       popcounts, then each block's base from the blocks before it and an
//       in-order block scan per pass. count may exceed cap (then only the
//       first cap positions are stored).
//   k_hits_expand — after the all-gather of packs: each workgroup owns a
//       32 KiB chunk of the global [total_rows][words] map, finds the
//       positions that fall in it by wave-wide 64-ary searches in the (sorted) packs of
//       the ranks it overlaps, ORs them into the chunk in LDS and writes the
//       chunk once: the map is written exactly once, with no memset and no
//       global atomics. A rank whose count exceeds cap contributes nothing and
//       clears *ok (asynchronous overflow report: the caller checks ok before
//       using the map and redoes that exchange densely).
// The expanded map is bit-identical to the dense all-gather's.
#include <hip/hip_runtime.h>

#include "exchange.hpp"
#include "profile.hpp"

namespace cb {
namespace {

constexpr uint32_t kCT = 1024, kCW = 4;      // compress: threads per block, words per thread per pass
constexpr uint64_t kPass = (uint64_t)kCT * kCW;
constexpr uint32_t kXT = 512;                // expand: threads per block
constexpr uint32_t kChunkWords = 4096;       // expand: map words per block (32 KiB of LDS)

// Inclusive block scan of one uint32 per thread; *total = block sum.
// wsum: NT/64 words of LDS. Barriers inside: call uniformly.
template <uint32_t NT>
__device__ __forceinline__ uint32_t block_incl_scan(uint32_t c, uint32_t* wsum, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  uint32_t x = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  __syncthreads();  // wsum may still be read by a previous call
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < NT / 64; ++k) {
    const uint32_t v = wsum[k];
    before += k < wid ? v : 0u;
    tot += v;
  }
  *total = tot;
  return before + x;
}

// sums[b] = set bits in block b's word range [b*per, min((b+1)*per, nw)).
__global__ __launch_bounds__(kCT) void k_hits_count(const uint64_t* __restrict__ hits, uint64_t nw,
                                                    uint64_t per, uint32_t* __restrict__ sums) {
  __shared__ uint32_t wsum[kCT / 64];
  const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = b0 + per < nw ? b0 + per : nw;
  uint32_t c = 0;
  for (uint64_t i = b0 + threadIdx.x; i < b1; i += kCT) c += (uint32_t)__popcll(hits[i]);
  uint32_t total;
  block_incl_scan<kCT>(c, wsum, &total);
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(kCT) void k_hits_emit(const uint64_t* __restrict__ hits, uint64_t nw,
                                                   uint64_t per, const uint32_t* __restrict__ sums,
                                                   uint32_t* __restrict__ pack, uint64_t cap) {
  __shared__ uint32_t wsum[kCT / 64];
  const uint32_t tid = threadIdx.x;
  // base = set bits of all earlier blocks; the last block also publishes the count
  uint32_t mine = 0;
  for (uint32_t j = tid; j < blockIdx.x; j += kCT) mine += sums[j];
  uint32_t base;
  block_incl_scan<kCT>(mine, wsum, &base);
  if (blockIdx.x == gridDim.x - 1 && tid == 0) {
    pack[0] = base + sums[blockIdx.x];
    pack[1] = 0;
  }
  const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = b0 + per < nw ? b0 + per : nw;
  uint64_t run = base;
  for (uint64_t p0 = b0; p0 < b1; p0 += kPass) {
    uint64_t w[kCW];
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < (int)kCW; ++j) {
      const uint64_t i = p0 + (uint64_t)tid * kCW + j;
      w[j] = i < b1 ? hits[i] : 0ull;
      c += (uint32_t)__popcll(w[j]);
    }
    uint32_t total;
    const uint32_t incl = block_incl_scan<kCT>(c, wsum, &total);
    uint64_t slot = run + incl - c;
#pragma unroll
    for (int j = 0; j < (int)kCW; ++j) {
      uint64_t v = w[j];
      const uint64_t pos0 = (p0 + (uint64_t)tid * kCW + j) * 64;  // row * words * 64 + col * 64
      while (v) {
        const uint32_t b = (uint32_t)__builtin_ctzll(v);
        v &= v - 1;
        if (slot < cap) pack[2 + slot] = (uint32_t)(pos0 + b);
        ++slot;
      }
    }
    run += total;
  }
}

// First index in p[0..n) with p[i] >= x (p ascending), by one whole wave:
// each round the 64 lanes probe 64 evenly spaced entries and the ballot of
// "< x" (a prefix of the lanes) narrows the range 64-fold, so a 70K-entry
// pack takes 3 rounds of one parallel load instead of 17 dependent ones.
__device__ __forceinline__ uint64_t wave_lower_bound(const uint32_t* p, uint64_t n, uint64_t x) {
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t lo = 0, hi = n;  // the answer is in [lo, hi]
  while (hi - lo > 64) {
    const uint64_t step = (hi - lo + 63) / 64;
    const uint64_t i = lo + lane * step;
    const bool below = i < hi && (uint64_t)p[i] < x;
    const uint32_t c = (uint32_t)__popcll(__ballot(below));
    const uint64_t nlo = c ? lo + (uint64_t)(c - 1) * step + 1 : lo;
    const uint64_t nhi = lo + (uint64_t)c * step < hi ? lo + (uint64_t)c * step : hi;
    lo = nlo;
    hi = nhi;
  }
  const uint64_t i = lo + lane;
  const bool below = i < hi && (uint64_t)p[i] < x;
  return lo + (uint64_t)__popcll(__ballot(below));
}

__global__ __launch_bounds__(kXT) void k_hits_expand(const uint32_t* __restrict__ packs,
                                                     uint32_t nranks, uint64_t cap, RankRows rr,
                                                     uint64_t words, uint64_t total_words,
                                                     uint64_t* __restrict__ full,
                                                     uint32_t* __restrict__ ok) {
  __shared__ uint64_t chunk[kChunkWords];
  __shared__ uint64_t seg[kMaxRanks][3];  // per overlapped rank: first entry, end entry, base word
  __shared__ uint64_t job[kMaxRanks][3];  // per overlapped rank: pack offset, count, first local word
  __shared__ uint32_t nseg;
  const uint32_t tid = threadIdx.x;
  const uint64_t w0 = (uint64_t)blockIdx.x * kChunkWords;
  const uint64_t w1 = w0 + kChunkWords < total_words ? w0 + kChunkWords : total_words;
  for (uint32_t i = tid; i < kChunkWords; i += kXT) chunk[i] = 0;
  if (tid == 0) {
    uint32_t ns = 0;
    for (uint32_t r = 0; r < nranks; ++r) {
      const uint64_t rb = rr.row_off[r] * words;
      const uint64_t re = (r + 1 < nranks ? rr.row_off[r + 1] : total_words / words) * words;
      if (re <= w0 || rb >= w1) continue;
      const uint32_t* pk = packs + (size_t)r * (2 + cap);
      const uint64_t count = pk[0];
      if (count > cap) {  // this rank's positions do not all fit: the map is incomplete
        if (ok) atomicAnd(ok, 0u);
        continue;
      }
      const uint64_t lw0 = (w0 > rb ? w0 : rb) - rb, lw1 = (w1 < re ? w1 : re) - rb;
      job[ns][0] = (uint64_t)r * (2 + cap) + 2;
      job[ns][1] = count;
      job[ns][2] = lw0 | (lw1 << 32);  // local words < 2^32 (positions are u32)
      seg[ns][2] = rb;
      ++ns;
    }
    nseg = ns;
  }
  __syncthreads();
  // the chunk's entry range in each overlapped pack: two wave-wide searches
  // per rank, one per wave
  for (uint32_t j = tid >> 6; j < 2 * nseg; j += kXT / 64) {
    const uint32_t s = j >> 1;
    const uint64_t lw = (j & 1) ? job[s][2] >> 32 : job[s][2] & 0xFFFFFFFFull;
    const uint64_t e = wave_lower_bound(packs + job[s][0], job[s][1], lw * 64);
    if ((tid & 63) == 0) seg[s][j & 1] = job[s][0] + e;
  }
  __syncthreads();
  for (uint32_t s = 0; s < nseg; ++s) {
    const uint64_t e0 = seg[s][0], e1 = seg[s][1], rb = seg[s][2];
    for (uint64_t e = e0 + tid; e < e1; e += kXT) {
      const uint64_t p = packs[e];
      atomicOr(reinterpret_cast<unsigned long long*>(&chunk[rb + (p >> 6) - w0]), 1ull << (p & 63));
    }
  }
  __syncthreads();
  for (uint64_t i = w0 + tid; i < w1; i += kXT) full[i] = chunk[i - w0];
}

inline uint64_t compress_plan(uint64_t nw, uint32_t* grid) {
  uint64_t g = (nw + kPass - 1) / kPass;
  if (g > kMaxCompressBlocks) g = kMaxCompressBlocks;
  if (g < 1) g = 1;
  const uint64_t per = ((nw + g - 1) / g + kPass - 1) / kPass * kPass;
  *grid = (uint32_t)((nw + per - 1) / per);
  if (*grid < 1) *grid = 1;
  return per;
}

}  // namespace

hipError_t launch_hits_compress(const uint64_t* hits, uint64_t rows, uint64_t words,
                                uint32_t* pack, uint64_t cap, uint32_t* sums, hipStream_t s) {
  const uint64_t nw = rows * words;
  if (!nw) return hipMemsetAsync(pack, 0, 8, s);
  uint32_t grid = 1;
  const uint64_t per = compress_plan(nw, &grid);
  ProfScope ps("k_hits_compress", s);
  hipLaunchKernelGGL(k_hits_count, dim3(grid), dim3(kCT), 0, s, hits, nw, per, sums);
  hipLaunchKernelGGL(k_hits_emit, dim3(grid), dim3(kCT), 0, s, hits, nw, per, sums, pack, cap);
  return hipGetLastError();
}

hipError_t launch_hits_expand(const uint32_t* packs, uint32_t nranks, uint64_t cap,
                              const RankRows& rr, uint64_t words, uint64_t total_rows,
                              uint64_t* full, uint32_t* ok, hipStream_t s) {
  const uint64_t tw = total_rows * words;
  if (!tw) return hipSuccess;
  if (!nranks) return hipMemsetAsync(full, 0, tw * 8, s);
  const uint64_t g = (tw + kChunkWords - 1) / kChunkWords;
  ProfScope ps("k_hits_expand", s);
  hipLaunchKernelGGL(k_hits_expand, dim3((uint32_t)g), dim3(kXT), 0, s, packs, nranks, cap, rr, words,
                     tw, full, ok);
  return hipGetLastError();
}

}  // namespace cb
