// sort.hip — the stable key sort of SsTable::create (/root/reference/src/
// sstable.rs:57-58: `entries.sort_by(|a, b| a.0.cmp(&b.0))`, a stable sort on
// the keys' bytes) for unsorted flush batches, as an LDS merge sort of the
// 24-byte SortKey records {w0, w1 = key bytes 0..15 big-endian, len, idx}.
//
// Order: (w0, w1), then length when either key is <= 16 bytes (the shorter
// is a prefix of the other), then the bytes past 16 for two longer keys, then
// idx — a strict total order whose ties on the key are broken by input
// position, i.e. exactly the stable order.
//
//   k_sort_block — one 1024-thread block per tile of kTile = 4096 records
//       (built from the key batch itself): each thread sorts its 4 records in
//       registers, then log2(1024) merge passes inside LDS (each thread finds
//       its 4 outputs' merge-path split by binary search and merges them
//       sequentially). At 1M entries 1024 x 4 (8 merge rounds) took 192 us,
//       512 x 4 (9 rounds) 207 us and 256 x 8 223 us: a round costs one
//       block's latency chain, so fewer, fatter rounds win.
//   k_sort_merge — log2(tiles) rounds of pairwise run merges: each block
//       owns 4096 outputs, finds its two splits with wave-wide 64-ary
//       merge-path searches in global memory (3-4 dependent rounds for runs
//       of up to 2^20 records), stages the two input pieces in LDS and merges
//       them as in the block sort; loads and stores are coalesced through LDS.
// Records make (1 + rounds) round trips through HBM: 48 MB per round at 1M
// entries. The last launch also writes what k_format needs in sorted order
// (value spans and line-tile sums), from the records in its registers, so
// no separate pass gathers them through the permutation.
#include <hip/hip_runtime.h>

#include "flush.hpp"
#include "profile.hpp"
#include "zone.hpp"

namespace cb {
namespace {

constexpr uint32_t kST = 1024;          // threads per block
constexpr uint32_t kIPT = 4;            // records per thread
constexpr uint32_t kTile = kST * kIPT;  // records per block
constexpr uint32_t kSentinel = 0xFFFFFFFFu;

// Two keys longer than 16 bytes that agree on their first 16: compare the
// rest from the key bytes. Rare, and kept out of line so the many inlined
// comparisons stay small (inlined, the byte loop made k_sort_block's code
// several times the instruction cache).
__device__ __noinline__ int tail_cmp(const uint8_t* kb, const uint64_t* ko, uint32_t ia, uint32_t ib) {
  const uint64_t ao = ko[ia], bo = ko[ib];
  return bytes_cmp(kb + ao + 16, ko[ia + 1] - ao - 16, kb + bo + 16, ko[ib + 1] - bo - 16);
}

struct RecLess {
  const uint8_t* kb;
  const uint64_t* ko;
  __device__ __forceinline__ bool operator()(const SortKey& a, const SortKey& b) const {
    if (a.w0 != b.w0) return a.w0 < b.w0;
    if (a.w1 != b.w1) return a.w1 < b.w1;
    if (a.len != b.len && (a.len <= 16 || b.len <= 16)) return a.len < b.len;
    if (a.len > 16 && b.len > 16 && a.idx != kSentinel && b.idx != kSentinel) {
      const int c = tail_cmp(kb, ko, a.idx, b.idx);
      if (c) return c < 0;
    }
    return a.idx < b.idx;
  }
};

__device__ __forceinline__ SortKey sentinel() {
  SortKey s;
  s.w0 = ~0ull;
  s.w1 = ~0ull;
  s.len = kSentinel;
  s.idx = kSentinel;
  return s;
}

// A tile of records in LDS as three padded arrays of 8-byte words (w0, w1,
// and len | idx << 32, the record's third word), so that a thread walking
// its own 8 consecutive records and its neighbours walking theirs hit
// different banks (record i sits at word i + i/8 of each array).
constexpr uint32_t kPadBits = 3;
constexpr uint32_t kPadded = kTile + (kTile >> kPadBits);
__device__ __forceinline__ uint32_t pad(uint32_t i) { return i + (i >> kPadBits); }

struct LdsTile {
  uint64_t* w;  // 3 * kPadded words
  __device__ __forceinline__ SortKey get(uint32_t i) const {
    const uint32_t j = pad(i);
    const uint64_t li = w[2 * kPadded + j];
    SortKey r;
    r.w0 = w[j];
    r.w1 = w[kPadded + j];
    r.len = (uint32_t)li;
    r.idx = (uint32_t)(li >> 32);
    return r;
  }
  __device__ __forceinline__ void set(uint32_t i, const SortKey& r) const {
    const uint32_t j = pad(i);
    w[j] = r.w0;
    w[kPadded + j] = r.w1;
    w[2 * kPadded + j] = (uint64_t)r.len | (uint64_t)r.idx << 32;
  }
  // global record words -> LDS: word g of the records is field g % 3 of record g / 3
  __device__ __forceinline__ void put_word(uint32_t g, uint64_t v) const { w[(g % 3) * kPadded + pad(g / 3)] = v; }
  __device__ __forceinline__ uint64_t word(uint32_t g) const { return w[(g % 3) * kPadded + pad(g / 3)]; }
};

// What the last launch of a sort also writes (vo == nullptr: nothing): per
// output p, vsp[p] = {value offset, value length} of its entry, and per
// kFormatTile outputs the sum of their line lengths (k_format's tile sums).
struct SortTail {
  const uint64_t* vo;
  ulonglong2* vsp;
  uint64_t* tsum;
};
static_assert(kFormatTile % kIPT == 0 && kFormatTile / kIPT <= 64 && kTile % kFormatTile == 0, "tile sums by shuffles");

// This thread's kIPT outputs r (at output position p0, count valid) into the
// tail: their value spans, and the line-length sum of each format tile (the
// kFormatTile / kIPT threads of a tile are consecutive lanes of one wave).
// Every lane of the block calls it.
__device__ __forceinline__ void emit_tail(const SortTail& tl, const SortKey (&r)[kIPT], uint64_t p0, uint32_t valid,
                                          const uint64_t* ko) {
  uint64_t sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kIPT; ++k) {
    if (k < valid) {
      const uint32_t i = r[k].idx;
      const uint64_t v0 = tl.vo[i], vl = tl.vo[i + 1] - v0;
      const uint64_t kl = r[k].len != 0xFFFFFFFFu ? r[k].len : ko[i + 1] - ko[i];
      ulonglong2 e;
      e.x = v0;
      e.y = vl;
      tl.vsp[p0 + k] = e;
      sum += line_len(kl, vl);
    }
  }
  constexpr uint32_t W = kFormatTile / kIPT;  // threads per tile
#pragma unroll
  for (uint32_t o = W / 2; o; o >>= 1) sum += __shfl_xor(sum, (int)o, 64);
  if ((threadIdx.x & (W - 1)) == 0 && valid) tl.tsum[p0 / kFormatTile] = sum;
}

// Records move between global memory and LDS as 8-byte words (3 per record),
// consecutive threads on consecutive words; past cnt the tile holds
// sentinels (greater than every record).
__device__ __forceinline__ void tile_load(const SortKey* __restrict__ g, uint32_t cnt, const LdsTile& t) {
  const uint64_t* gw = reinterpret_cast<const uint64_t*>(g);
  for (uint32_t i = threadIdx.x; i < 3 * cnt; i += kST) t.put_word(i, gw[i]);
  for (uint32_t i = cnt + threadIdx.x; i < kTile; i += kST) t.set(i, sentinel());
}

__device__ __forceinline__ void tile_store(const LdsTile& t, SortKey* __restrict__ g, uint32_t cnt) {
  uint64_t* gw = reinterpret_cast<uint64_t*>(g);
  for (uint32_t i = threadIdx.x; i < 3 * cnt; i += kST) gw[i] = t.word(i);
}

// Merge-path split of diagonal d between sorted a[0..la) and b[0..lb): the
// number of a-records among the first d outputs (a-records first on ties,
// which the total order never has).
template <class A, class B>
__device__ __forceinline__ uint32_t merge_split(const A& a, uint32_t la, const B& b, uint32_t lb, uint32_t d,
                                                const RecLess& less) {
  uint32_t lo = d > lb ? d - lb : 0, hi = d < la ? d : la;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (less(b[d - mid - 1], a[mid]))
      hi = mid;
    else
      lo = mid + 1;
  }
  return lo;
}

// A run of records inside the LDS tile, starting at record `base`.
struct LdsRun {
  LdsTile t;
  uint32_t base;
  __device__ __forceinline__ SortKey operator[](uint32_t i) const { return t.get(base + i); }
};

// Up to kIPT outputs from a[i..la) and b[j..lb), in order; sentinels once
// both are exhausted.
template <class A, class B>
__device__ __forceinline__ void merge_seq(const A& a, uint32_t la, const B& b, uint32_t lb, uint32_t i,
                                          uint32_t j, SortKey (&r)[kIPT], const RecLess& less) {
  SortKey x = i < la ? a[i] : sentinel(), y = j < lb ? b[j] : sentinel();
#pragma unroll
  for (uint32_t k = 0; k < kIPT; ++k) {
    const bool take_b = i >= la || (j < lb && less(y, x));
    if (take_b) {
      r[k] = y;
      ++j;
      y = j < lb ? b[j] : sentinel();
    } else {
      r[k] = x;
      ++i;
      x = i < la ? a[i] : sentinel();
    }
  }
}

__device__ __forceinline__ void cas(SortKey& x, SortKey& y, const RecLess& less) {
  if (less(y, x)) {
    const SortKey t = x;
    x = y;
    y = t;
  }
}

__global__ __launch_bounds__(kST) void k_sort_block(const SortKey* __restrict__ in, SortKey* __restrict__ out,
                                                    uint64_t n, RecLess less, SortTail tl) {
  __shared__ uint64_t lds[3 * kPadded];
  const LdsTile tile{lds};
  const uint64_t base = (uint64_t)blockIdx.x * kTile;
  const uint32_t cnt = (uint32_t)(n - base < kTile ? n - base : kTile);
  if (in) {
    tile_load(in + base, cnt, tile);
  } else {  // the records straight from the key batch
    for (uint32_t i = threadIdx.x; i < kTile; i += kST) tile.set(i, i < cnt ? sort_record(less.kb, less.ko, base + i) : sentinel());
  }
  __syncthreads();
  SortKey r[kIPT];
  const uint32_t t0 = threadIdx.x * kIPT;
#pragma unroll
  for (uint32_t k = 0; k < kIPT; ++k) r[k] = tile.get(t0 + k);
  // odd-even transposition network on the thread's 8 records
#pragma unroll
  for (uint32_t p = 0; p < kIPT; ++p) {
#pragma unroll
    for (uint32_t k = p & 1; k + 1 < kIPT; k += 2) cas(r[k], r[k + 1], less);
  }
  for (uint32_t w = kIPT; w < kTile; w <<= 1) {
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kIPT; ++k) tile.set(t0 + k, r[k]);
    __syncthreads();
    const uint32_t pb = t0 & ~(2 * w - 1), d = t0 - pb;  // pair base and this thread's diagonal
    const LdsRun a{tile, pb}, b{tile, pb + w};
    const uint32_t i = merge_split(a, w, b, w, d, less);
    merge_seq(a, w, b, w, i, d - i, r, less);
  }
  if (tl.vo) emit_tail(tl, r, base + t0, t0 < cnt ? (cnt - t0 < kIPT ? cnt - t0 : kIPT) : 0, less.ko);
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kIPT; ++k) tile.set(t0 + k, r[k]);
  __syncthreads();
  tile_store(tile, out + base, cnt);
}

// Merge-path split in global memory by one wave: 64 lanes test 64 evenly
// spaced candidates per round (the predicate "b[d-i-1] < a[i]" is monotone in
// i), narrowing the range 64-fold per round.
__device__ __forceinline__ uint64_t wave_merge_split(const SortKey* a, uint64_t la, const SortKey* b, uint64_t lb,
                                                     uint64_t d, const RecLess& less) {
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t lo = d > lb ? d - lb : 0, hi = d < la ? d : la;  // the split is in [lo, hi]
  while (lo < hi) {
    const uint64_t span = hi - lo;
    if (span <= 64) {  // last round: every remaining candidate at once
      const uint64_t i = lo + lane;
      const uint64_t m = __ballot(i < hi && less(b[d - i - 1], a[i]));
      return m ? lo + (uint64_t)__builtin_ctzll(m) : hi;
    }
    const uint64_t step = (span + 63) / 64;
    const uint64_t i = lo + (uint64_t)lane * step;
    const uint64_t m = __ballot(i < hi && less(b[d - i - 1], a[i]));
    if (m) {  // the first true candidate bounds the split from above
      const uint64_t f = (uint64_t)__builtin_ctzll(m);
      hi = lo + f * step;
      lo = f ? lo + (f - 1) * step + 1 : lo;
    } else {  // every candidate false: the split is past the last one
      lo += ((span + step - 1) / step - 1) * step + 1;
    }
  }
  return lo;
}

__global__ __launch_bounds__(kST) void k_sort_merge(const SortKey* __restrict__ in, SortKey* __restrict__ out,
                                                    uint64_t n, uint64_t w, RecLess less, SortTail tl) {
  __shared__ uint64_t lds[3 * kPadded];
  __shared__ uint64_t split[2];
  const LdsTile tile{lds};
  const uint64_t o0 = (uint64_t)blockIdx.x * kTile;
  const uint64_t pb = o0 / (2 * w) * (2 * w);
  const uint64_t la = n - pb < w ? n - pb : w;
  const uint64_t lb = n - pb > w ? (n - pb - w < w ? n - pb - w : w) : 0;
  const SortKey* a = in + pb;
  const SortKey* b = a + la;
  const uint64_t d0 = o0 - pb;
  const uint64_t d1 = d0 + kTile < la + lb ? d0 + kTile : la + lb;
  const uint32_t wave = threadIdx.x >> 6;
  if (wave < 2) {
    const uint64_t sp = wave_merge_split(a, la, b, lb, wave ? d1 : d0, less);
    if ((threadIdx.x & 63u) == 0) split[wave] = sp;
  }
  __syncthreads();
  const uint64_t i0 = split[0], i1 = split[1];
  const uint64_t j0 = d0 - i0, j1 = d1 - i1;
  const uint32_t na = (uint32_t)(i1 - i0), nb = (uint32_t)(j1 - j0);
  // stage a[i0..i1) then b[j0..j1) contiguously
  {
    const uint64_t* ga = reinterpret_cast<const uint64_t*>(a + i0);
    const uint64_t* gb = reinterpret_cast<const uint64_t*>(b + j0);
    for (uint32_t i = threadIdx.x; i < 3 * na; i += kST) tile.put_word(i, ga[i]);
    for (uint32_t i = threadIdx.x; i < 3 * nb; i += kST) tile.put_word(3 * na + i, gb[i]);
  }
  __syncthreads();
  const uint32_t t0 = threadIdx.x * kIPT;
  const uint32_t tot = na + nb;
  SortKey r[kIPT];
  if (t0 < tot) {
    const LdsRun sa{tile, 0}, sb{tile, na};
    const uint32_t i = merge_split(sa, na, sb, nb, t0, less);
    merge_seq(sa, na, sb, nb, i, t0 - i, r, less);
  }
  if (tl.vo) emit_tail(tl, r, o0 + t0, t0 < tot ? (tot - t0 < kIPT ? tot - t0 : kIPT) : 0, less.ko);
  __syncthreads();
  if (t0 < tot) {
#pragma unroll
    for (uint32_t k = 0; k < kIPT; ++k)
      if (t0 + k < tot) tile.set(t0 + k, r[k]);
  }
  __syncthreads();
  tile_store(tile, out + o0, tot);
}

}  // namespace

uint64_t entry_sort_tmp_bytes(uint64_t n) { return n * sizeof(SortKey); }

hipError_t launch_entry_sort(const SortKey* in, SortKey* out, SortKey* tmp, uint64_t n, const uint8_t* kb,
                             const uint64_t* ko, hipStream_t s, const uint64_t* vo, ulonglong2* vsp,
                             uint64_t* tsum) {
  if (!n) return hipSuccess;
  const uint64_t tiles = (n + kTile - 1) / kTile;
  uint32_t rounds = 0;
  while ((uint64_t)kTile << rounds < n) ++rounds;
  // the last round writes `out`: rounds alternate tmp/out backwards from it
  SortKey* bufs[2] = {out, tmp};
  const RecLess less{kb, ko};
  ProfScope ps("k_entry_sort", s);
  const SortTail none{nullptr, nullptr, nullptr}, tail{vo, vsp, tsum};
  hipLaunchKernelGGL(k_sort_block, dim3((uint32_t)tiles), dim3(kST), 0, s, in, bufs[rounds & 1], n, less,
                     rounds ? none : tail);
  for (uint32_t r = 0; r < rounds; ++r) {
    const uint64_t w = (uint64_t)kTile << r;
    hipLaunchKernelGGL(k_sort_merge, dim3((uint32_t)tiles), dim3(kST), 0, s, bufs[(rounds - r) & 1],
                       bufs[(rounds - r - 1) & 1], n, w, less, r + 1 == rounds ? tail : none);
  }
  return hipGetLastError();
}

}  // namespace cb
