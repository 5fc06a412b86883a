// flush.hip — SsTable::create's data file on the device.
//
// /root/reference/src/sstable.rs:56-72: the flushed entries are stably sorted
// by key (`sort_by(|a, b| a.0.cmp(&b.0))`) and written as one line per entry,
// `key \t STANDARD.encode(value) \n`. Memtable flushes arrive sorted already
// (the memtable is a BTreeMap, src/memtable.rs:6-8), so a sortedness check
// runs first and the sort is skipped when it passes. Otherwise entries are
// sorted by rocPRIM's stable merge sort on 24-byte records (16-byte key
// prefix + length + index) with a full compare only for prefix ties. Line
// lengths are known up front (key + 1 + 4*ceil(value/3) + 1), so an
// exclusive scan gives every line's offset and one lane formats each line.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_merge_sort.hpp>

#include "flush.hpp"
#include "profile.hpp"
#include "zone.hpp"

namespace cb {
namespace {

constexpr uint32_t kNT = 256;

inline uint32_t blocks_for(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }

__device__ __forceinline__ uint64_t prefix_word(const uint8_t* p, uint64_t len, uint64_t at) {
  return at < len ? be_chunk(p + at, len - at < 8 ? len - at : 8) : 0;
}

__global__ __launch_bounds__(kNT) void k_sort_keys(const uint8_t* __restrict__ kb,
                                                   const uint64_t* __restrict__ ko, uint64_t n,
                                                   SortKey* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  if (i >= n) return;
  const uint8_t* p = kb + ko[i];
  const uint64_t len = ko[i + 1] - ko[i];
  SortKey s;
  s.w0 = prefix_word(p, len, 0);
  s.w1 = prefix_word(p, len, 8);
  s.len = len > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)len;
  s.idx = (uint32_t)i;
  out[i] = s;
}

// *ok &= key[i-1] <= key[i] for all i (already in stable-sorted order).
__global__ __launch_bounds__(kNT) void k_sorted_check(const uint8_t* __restrict__ kb,
                                                      const uint64_t* __restrict__ ko, uint64_t n,
                                                      uint32_t* ok) {
  const uint64_t i = (uint64_t)blockIdx.x * kNT + threadIdx.x + 1;
  const bool bad =
      i < n && bytes_cmp(kb + ko[i - 1], ko[i] - ko[i - 1], kb + ko[i], ko[i + 1] - ko[i]) > 0;
  // one atomic per block, and none once the flag is down: a fully unsorted
  // batch would otherwise serialise up to a million atomics on one word
  if (__syncthreads_or(bad) && threadIdx.x == 0 && *(volatile uint32_t*)ok) atomicAnd(ok, 0u);
}

// Rust str order on the records: the 16-byte zero-padded prefixes, then (when
// either key fits in 16 bytes) the length, else the bytes past 16. Equal keys
// compare equal, so the merge sort's stability keeps their input order.
struct KeyLess {
  const uint8_t* kb;
  const uint64_t* ko;
  __device__ bool operator()(const SortKey& a, const SortKey& b) const {
    if (a.w0 != b.w0) return a.w0 < b.w0;
    if (a.w1 != b.w1) return a.w1 < b.w1;
    if (a.len <= 16 || b.len <= 16) return a.len < b.len;
    const uint64_t al = ko[a.idx + 1] - ko[a.idx], bl = ko[b.idx + 1] - ko[b.idx];
    return bytes_cmp(kb + ko[a.idx] + 16, al - 16, kb + ko[b.idx] + 16, bl - 16) < 0;
  }
};

__global__ __launch_bounds__(kNT) void k_line_lens(const SortKey* __restrict__ order,
                                                   const uint64_t* __restrict__ ko,
                                                   const uint64_t* __restrict__ vo, uint64_t n,
                                                   uint64_t* __restrict__ lens) {
  const uint64_t p = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  if (p >= n) return;
  const uint64_t i = order ? order[p].idx : p;
  const uint64_t vl = vo[i + 1] - vo[i];
  lens[p] = (ko[i + 1] - ko[i]) + 1 + (vl + 2) / 3 * 4 + 1;
}

__device__ __forceinline__ uint8_t b64c(uint32_t v) {
  return (uint8_t)(v < 26 ? 'A' + v : v < 52 ? 'a' + (v - 26) : v < 62 ? '0' + (v - 52) : v == 62 ? '+' : '/');
}

// One lane per line: key, TAB, STANDARD.encode(value), NL, through put(j, b).
template <class Put>
__device__ __forceinline__ void format_line(const uint8_t* k, uint64_t kl, const uint8_t* v,
                                            uint64_t vl, Put put) {
  uint64_t o = 0;
  for (uint64_t j = 0; j < kl; ++j) put(o++, k[j]);
  put(o++, '\t');
  for (uint64_t j = 0; j < vl; j += 3) {
    const uint64_t r = vl - j;
    const uint32_t w = (uint32_t)v[j] << 16 | (r > 1 ? (uint32_t)v[j + 1] << 8 : 0u) |
                       (r > 2 ? (uint32_t)v[j + 2] : 0u);
    put(o++, b64c(w >> 18));
    put(o++, b64c((w >> 12) & 63));
    put(o++, r > 1 ? b64c((w >> 6) & 63) : (uint8_t)'=');
    put(o++, r > 2 ? b64c(w & 63) : (uint8_t)'=');
  }
  put(o, '\n');
}

constexpr uint32_t kFormatLds = 32768;  // staged output bytes per block

// A block's 256 lines are one contiguous output range [loff[p0], loff[p0+256]).
// When it fits in LDS the lanes format into LDS and the block writes the
// range with aligned dword stores; otherwise lanes write bytes directly.
__global__ __launch_bounds__(kNT) void k_format(const SortKey* __restrict__ order,
                                                const uint8_t* __restrict__ kb,
                                                const uint64_t* __restrict__ ko,
                                                const uint8_t* __restrict__ vb,
                                                const uint64_t* __restrict__ vo,
                                                const uint64_t* __restrict__ loff, uint64_t n,
                                                uint8_t* __restrict__ out) {
  __shared__ uint8_t stage[kFormatLds];
  const uint64_t p0 = (uint64_t)blockIdx.x * kNT;
  const uint64_t p = p0 + threadIdx.x;
  const uint64_t pend = p0 + kNT < n ? p0 + kNT : n;
  const uint64_t base = loff[p0], total = loff[pend] - base;
  const bool live = p < n;
  const uint64_t i = live ? (order ? order[p].idx : p) : 0;
  const uint8_t* k = kb + (live ? ko[i] : 0);
  const uint64_t kl = live ? ko[i + 1] - ko[i] : 0;
  const uint8_t* v = vb + (live ? vo[i] : 0);
  const uint64_t vl = live ? vo[i + 1] - vo[i] : 0;
  const uint64_t o = live ? loff[p] : 0;
  if (total > kFormatLds) {  // uniform: long lines, direct byte stores
    if (live) format_line(k, kl, v, vl, [&](uint64_t j, uint8_t c) { out[o + j] = c; });
    return;
  }
  if (live) format_line(k, kl, v, vl, [&](uint64_t j, uint8_t c) { stage[o - base + j] = c; });
  __syncthreads();
  uint8_t* g = out + base;
  const uint64_t mis = (4 - ((uintptr_t)g & 3)) & 3;
  const uint64_t head = mis < total ? mis : total;
  if (threadIdx.x < head) g[threadIdx.x] = stage[threadIdx.x];
  const uint64_t body = (total - head) / 4;
  uint32_t* gw = reinterpret_cast<uint32_t*>(g + head);
  for (uint64_t j = threadIdx.x; j < body; j += kNT) {
    const uint64_t q = head + 4 * j;
    gw[j] = (uint32_t)stage[q] | (uint32_t)stage[q + 1] << 8 | (uint32_t)stage[q + 2] << 16 |
            (uint32_t)stage[q + 3] << 24;
  }
  const uint64_t tail0 = head + 4 * body;
  if (tail0 + threadIdx.x < total) g[tail0 + threadIdx.x] = stage[tail0 + threadIdx.x];
}

}  // namespace

hipError_t launch_sort_keys(const uint8_t* kb, const uint64_t* ko, uint64_t n, SortKey* out,
                            hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("k_sort_keys", s);
  hipLaunchKernelGGL(k_sort_keys, dim3(blocks_for(n, kNT)), dim3(kNT), 0, s, kb, ko, n, out);
  return hipGetLastError();
}

hipError_t launch_sorted_check(const uint8_t* kb, const uint64_t* ko, uint64_t n, uint32_t* ok,
                               hipStream_t s) {
  if (n < 2) return hipSuccess;
  ProfScope ps("k_sorted_check", s);
  hipLaunchKernelGGL(k_sorted_check, dim3(blocks_for(n - 1, kNT)), dim3(kNT), 0, s, kb, ko, n, ok);
  return hipGetLastError();
}

hipError_t entry_sort(void* tmp, size_t& tmp_bytes, const SortKey* in, SortKey* out, uint64_t n,
                      const uint8_t* kb, const uint64_t* ko, hipStream_t s) {
  if (!tmp) return rocprim::merge_sort(tmp, tmp_bytes, in, out, (size_t)n, KeyLess{kb, ko}, s);
  ProfScope ps("rocprim_merge_sort", s);
  return rocprim::merge_sort(tmp, tmp_bytes, in, out, (size_t)n, KeyLess{kb, ko}, s);
}

hipError_t launch_line_lens(const SortKey* order, const uint64_t* ko, const uint64_t* vo, uint64_t n,
                            uint64_t* lens, hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("k_line_lens", s);
  hipLaunchKernelGGL(k_line_lens, dim3(blocks_for(n, kNT)), dim3(kNT), 0, s, order, ko, vo, n, lens);
  return hipGetLastError();
}

hipError_t launch_format(const SortKey* order, const uint8_t* kb, const uint64_t* ko,
                         const uint8_t* vb, const uint64_t* vo, const uint64_t* loff, uint64_t n,
                         uint8_t* out, hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("k_format", s);
  hipLaunchKernelGGL(k_format, dim3(blocks_for(n, kNT)), dim3(kNT), 0, s, order, kb, ko, vb, vo, loff,
                     n, out);
  return hipGetLastError();
}

}  // namespace cb
