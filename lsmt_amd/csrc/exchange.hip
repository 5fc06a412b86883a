// exchange.hip — sparse form of the multi-GPU hit-bitmap exchange (SURVEY.md
// §8e). Each rank probes the replicated key batch against its filter subset
// and holds hit rows [rows][words]; Database::get (/root/reference/src/
// lib.rs:129-134) needs every table's answer per key, so the rows are
// all-gathered. At BASELINE densities the rows are sparse (a present key hits
// one table, false positives ~(1.55 %)^2 per (key, table)), so a rank ships
// the POSITIONS of its set bits instead of its dense rows.
//
// Pack layout (uint32; exchange.hpp): {count, 0, positions[cap], dir[2*D]}.
// The rank's words are cut into D = ceil(rows*words / 2048) blocks; block b's
// positions (row*words*64 + bit, ascending inside the block) sit at
// positions[dir[2b] .. dir[2b] + dir[2b+1]). Blocks claim their slots with
// one atomic add each, so no block ever waits for another:
//   k_hits_compress — one block per 2048 words: count, claim, write the
//       block's positions in order and its directory entry; the last block
//       to finish writes count. count may exceed cap (the pack is then
//       unusable: every rank must fall back to the dense exchange).
//   k_hits_expand — after the all-gather of packs: one block per (rank,
//       compress block), i.e. per 2048 words of the global map: ORs that
//       block's positions into the chunk in LDS and writes the chunk once.
//       The map is written exactly once, with no memset, no search and no
//       global atomics. A rank whose count exceeds cap writes zeros and
//       clears *ok (asynchronous overflow report: the caller checks ok before
//       using the map and redoes that exchange densely).
// The expanded map is bit-identical to the dense all-gather's.
#include <hip/hip_runtime.h>

#include "blockscan.hpp"
#include "exchange.hpp"
#include "profile.hpp"

namespace cb {
namespace {

constexpr uint32_t kCT = 256, kCW = 8;  // compress: threads per block, words per thread
static_assert((uint64_t)kCT * kCW == kCompressWords, "one block = kCompressWords words");
constexpr uint32_t kXT = 256;           // expand: threads per block (one chunk of kCompressWords)

// Inclusive block scan of one uint32 per thread; *total = block sum.
// wsum: NT/64 words of LDS. Barriers inside: call uniformly.
template <uint32_t NT>
__device__ __forceinline__ uint32_t block_incl_scan(uint32_t c, uint32_t* wsum, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  const uint32_t x = wave_inclusive_scan(c);
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

// ctl: two uint64 claim words, one per launch parity: a block adds
// (1 << 32) | its set bits, so the low half hands out slots and the high half
// counts finished claims (the block that draws gridDim.x - 1 is the last and
// knows the total). One relaxed atomic per block, no fence: the only value
// read across blocks is the atomic word itself. A launch uses word `par` and
// clears the other for the next launch on the stream.
__global__ __launch_bounds__(kCT) void k_hits_compress(const uint64_t* __restrict__ hits, uint64_t nw,
                                                       uint32_t* __restrict__ pack, uint64_t cap,
                                                       unsigned long long* __restrict__ ctl, uint32_t par) {
  __shared__ uint32_t wsum[kCT / 64];
  __shared__ uint32_t s_base;
  const uint32_t tid = threadIdx.x, b = blockIdx.x;
  const uint64_t i0 = (uint64_t)b * kCompressWords + (uint64_t)tid * kCW;
  uint64_t w[kCW];
  if (i0 + kCW <= nw && !((uintptr_t)hits & 15)) {
    const ulonglong2* v = reinterpret_cast<const ulonglong2*>(hits + i0);
#pragma unroll
    for (uint32_t j = 0; j < kCW / 2; ++j) {
      const ulonglong2 a = v[j];
      w[2 * j] = a.x;
      w[2 * j + 1] = a.y;
    }
  } else {
#pragma unroll
    for (uint32_t j = 0; j < kCW; ++j) w[j] = i0 + j < nw ? hits[i0 + j] : 0ull;
  }
  uint32_t c = 0;
#pragma unroll
  for (uint32_t j = 0; j < kCW; ++j) c += (uint32_t)__popcll(w[j]);
  uint32_t total;
  const uint32_t incl = block_incl_scan<kCT>(c, wsum, &total);
  if (tid == 0) {
    const unsigned long long old = atomicAdd(ctl + par, (1ull << 32) | total);
    s_base = (uint32_t)old;
    if ((uint32_t)(old >> 32) == gridDim.x - 1) {  // the last claim: every block's bits are counted
      pack[0] = (uint32_t)old + total;
      pack[1] = 0;
    }
    if (b == 0) __hip_atomic_store(ctl + (par ^ 1u), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const uint64_t base = s_base;
  uint32_t* dir = pack + 2 + cap;
  if (tid == 0) {
    dir[2 * (uint64_t)b] = (uint32_t)base;
    dir[2 * (uint64_t)b + 1] = total;
  }
  uint64_t slot = base + incl - c;
#pragma unroll
  for (uint32_t j = 0; j < kCW; ++j) {
    uint64_t v = w[j];
    const uint64_t pos0 = (i0 + j) * 64;  // row * words * 64 + col * 64
    while (v) {
      const uint32_t bit = (uint32_t)__builtin_ctzll(v);
      v &= v - 1;
      if (slot < cap) pack[2 + slot] = (uint32_t)(pos0 + bit);
      ++slot;
    }
  }
}

__global__ __launch_bounds__(kXT) void k_hits_expand(const uint32_t* __restrict__ packs, uint32_t nranks,
                                                     uint64_t cap, uint64_t stride, ExpandPlan plan,
                                                     uint64_t words, uint64_t* __restrict__ full,
                                                     uint32_t* __restrict__ ok) {
  __shared__ uint64_t chunk[kCompressWords];
  const uint32_t tid = threadIdx.x;
  // this block's rank: the last r with blk_off[r] <= blockIdx.x (ranks with
  // no rows have no blocks and are skipped by the ballot)
  uint32_t r = 0;
  for (uint32_t r0 = 0; r0 < nranks; r0 += 64) {
    const uint32_t rr = r0 + (tid & 63u);
    const uint64_t m = __ballot(rr < nranks && plan.blk_off[rr] <= blockIdx.x);
    if (m) r = r0 + 63u - (uint32_t)__builtin_clzll(m);
  }
  const uint64_t b = blockIdx.x - plan.blk_off[r];
  const uint64_t rows_r = plan.row_off[r + 1] - plan.row_off[r];
  const uint64_t lw0 = b * kCompressWords;
  const uint64_t lw1 = lw0 + kCompressWords < rows_r * words ? lw0 + kCompressWords : rows_r * words;
  const uint32_t* pk = packs + (uint64_t)r * stride;
  const uint64_t count = pk[0];
  for (uint32_t i = tid; i < kCompressWords; i += kXT) chunk[i] = 0;
  __syncthreads();
  if (count > cap) {  // this rank's positions do not all fit: the map is incomplete
    if (ok && tid == 0 && b == 0) atomicAnd(ok, 0u);
  } else {
    const uint32_t* dir = pk + 2 + cap;
    const uint64_t e0 = dir[2 * b], ne = dir[2 * b + 1];
    for (uint64_t e = tid; e < ne; e += kXT) {
      const uint64_t p = pk[2 + e0 + e];
      atomicOr(reinterpret_cast<unsigned long long*>(&chunk[(p >> 6) - lw0]), 1ull << (p & 63));
    }
  }
  __syncthreads();
  uint64_t* out = full + plan.row_off[r] * words + lw0;
  const uint64_t n = lw1 - lw0;
  for (uint64_t i = tid; i < n; i += kXT) out[i] = chunk[i];
}

constexpr uint32_t kBlkRows = 64, kBlkWordsMax = 16;

__global__ __launch_bounds__(kXT) void k_hits_expand_blocks(const uint32_t* __restrict__ packs, uint64_t cap,
                                                            uint64_t stride, ExpandPlan plan, uint64_t hwords,
                                                            uint32_t nblk, uint32_t bw,
                                                            uint64_t* __restrict__ full,
                                                            uint32_t* __restrict__ ok) {
  __shared__ uint64_t chunk[kBlkRows * kBlkWordsMax];
  const uint32_t tid = threadIdx.x;
  const uint32_t r = blockIdx.x / nblk, b = blockIdx.x % nblk;
  const uint32_t rows = (uint32_t)(plan.row_off[r + 1] - plan.row_off[r]);
  const uint64_t w0 = (uint64_t)b * bw;
  for (uint32_t i = tid; i < rows * bw; i += kXT) chunk[i] = 0;
  __syncthreads();
  const uint32_t* pk = packs + (uint64_t)r * stride;
  if (pk[0] > cap) {  // this rank's positions do not all fit: its rows stay zero
    if (ok && tid == 0 && b == 0) atomicAnd(ok, 0u);
  } else {
    const uint32_t* dir = pk + 2 + cap;
    const uint64_t e0 = dir[2 * (uint64_t)b], ne = dir[2 * (uint64_t)b + 1];
    for (uint64_t e = tid; e < ne; e += kXT) {
      const uint32_t p = pk[2 + e0 + e];
      const uint32_t wl = p >> 6;  // row * hwords + word (< 2^26)
      const uint32_t row = (uint32_t)(wl / (uint32_t)hwords), word = wl - row * (uint32_t)hwords;
      atomicOr(reinterpret_cast<unsigned long long*>(&chunk[row * bw + (word - (uint32_t)w0)]), 1ull << (p & 63));
    }
  }
  __syncthreads();
  for (uint32_t i = tid; i < rows * bw; i += kXT) {
    const uint32_t f = i / bw, w = i % bw;
    if (w0 + w < hwords) full[(plan.row_off[r] + f) * hwords + w0 + w] = chunk[i];
  }
}

}  // namespace

hipError_t launch_hits_compress(const uint64_t* hits, uint64_t rows, uint64_t words,
                                uint32_t* pack, uint64_t cap, CompressState& st, hipStream_t s) {
  const uint64_t nw = rows * words;
  if (!nw) return hipMemsetAsync(pack, 0, 8, s);
  if (nw > kMaxCompressWords) return hipErrorInvalidValue;
  const uint32_t g = (uint32_t)pack_blocks(nw);
  ProfScope ps("k_hits_compress", s);
  hipLaunchKernelGGL(k_hits_compress, dim3(g), dim3(kCT), 0, s, hits, nw, pack, cap,
                     reinterpret_cast<unsigned long long*>(st.ctl), st.parity);
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) {
    st.parity ^= 1u;  // the launch cleared the other pair for the next one
  } else {
    // the kernel may still have been queued (an earlier sticky error): clear
    // both claim words behind it, so the next launch never reuses a dirty one
    (void)hipMemsetAsync(st.ctl, 0, 16, s);
  }
  return e;
}

hipError_t launch_hits_expand(const uint32_t* packs, uint32_t nranks, uint64_t cap,
                              const RankRows& rr, uint64_t words, uint64_t total_rows,
                              uint64_t* full, uint32_t* ok, hipStream_t s) {
  const uint64_t tw = total_rows * words;
  if (!tw) return hipSuccess;
  if (!nranks) return hipMemsetAsync(full, 0, tw * 8, s);
  ExpandPlan plan{};
  uint64_t max_rows = 0, nblk = 0;
  for (uint32_t r = 0; r < nranks; ++r) {
    const uint64_t end = r + 1 < nranks ? rr.row_off[r + 1] : total_rows;
    if (end < rr.row_off[r] || end > total_rows) return hipErrorInvalidValue;
    plan.row_off[r] = rr.row_off[r];
    plan.blk_off[r] = nblk;
    nblk += pack_blocks((end - rr.row_off[r]) * words);
    max_rows = end - rr.row_off[r] > max_rows ? end - rr.row_off[r] : max_rows;
  }
  if (rr.row_off[0] != 0) return hipErrorInvalidValue;
  plan.row_off[nranks] = total_rows;
  for (uint32_t r = nranks; r < kMaxRanks; ++r) plan.blk_off[r] = ~0ull;
  if (!nblk) return hipSuccess;
  ProfScope ps("k_hits_expand", s);
  hipLaunchKernelGGL(k_hits_expand, dim3((uint32_t)nblk), dim3(kXT), 0, s, packs, nranks, cap,
                     pack_words(max_rows * words, cap), plan, words, full, ok);
  return hipGetLastError();
}

}  // namespace cb

namespace cb {

hipError_t launch_hits_expand_blocks(const uint32_t* packs, uint32_t nranks, uint64_t cap, uint64_t stride,
                                     const RankRows& rr, uint64_t hwords, uint64_t total_rows, uint32_t nblk,
                                     uint32_t block_words, uint64_t* full, uint32_t* ok, hipStream_t s) {
  if (!total_rows || !hwords || !nranks || !nblk) return hipSuccess;
  if (block_words > kBlkWordsMax || rr.row_off[0] != 0) return hipErrorInvalidValue;
  ExpandPlan plan{};
  for (uint32_t r = 0; r < nranks; ++r) {
    const uint64_t end = r + 1 < nranks ? rr.row_off[r + 1] : total_rows;
    // a rank's rows fit one workgroup's chunk, and its positions fit 32 bits
    if (end < rr.row_off[r] || end - rr.row_off[r] > kBlkRows || (end - rr.row_off[r]) * hwords * 64 >= (1ull << 32))
      return hipErrorInvalidValue;
    plan.row_off[r] = rr.row_off[r];
  }
  plan.row_off[nranks] = total_rows;
  ProfScope ps("k_hits_expand_blocks", s);
  hipLaunchKernelGGL(k_hits_expand_blocks, dim3(nranks * nblk), dim3(kXT), 0, s, packs, cap, stride, plan, hwords,
                     nblk, block_words, full, ok);
  return hipGetLastError();
}

}  // namespace cb
