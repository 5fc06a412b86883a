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
// entries. cb_sstable_create uses it for batches the bin sort below cannot
// take (a bin larger than one LDS tile, or too few entries). The last launch also writes what k_format needs in sorted order
// (value spans and line-tile sums), from the records in its registers, so
// no separate pass gathers them through the permutation.
#include <hip/hip_runtime.h>

#include "blockscan.hpp"
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

// P: words per field array; PAD: record i at word i + i / 8 (else i).
template <uint32_t P, bool PAD>
struct LdsTileT {
  uint64_t* w;  // 3 * P words
  static __device__ __forceinline__ uint32_t pad(uint32_t i) { return PAD ? i + (i >> kPadBits) : i; }
  __device__ __forceinline__ SortKey get(uint32_t i) const {
    const uint32_t j = pad(i);
    const uint64_t li = w[2 * P + j];
    SortKey r;
    r.w0 = w[j];
    r.w1 = w[P + j];
    r.len = (uint32_t)li;
    r.idx = (uint32_t)(li >> 32);
    return r;
  }
  __device__ __forceinline__ void set(uint32_t i, const SortKey& r) const {
    const uint32_t j = pad(i);
    w[j] = r.w0;
    w[P + j] = r.w1;
    w[2 * P + j] = (uint64_t)r.len | (uint64_t)r.idx << 32;
  }
  // global record words -> LDS: word g of the records is field g % 3 of record g / 3
  __device__ __forceinline__ void put_word(uint32_t g, uint64_t v) const { w[(g % 3) * P + pad(g / 3)] = v; }
  __device__ __forceinline__ uint64_t word(uint32_t g) const { return w[(g % 3) * P + pad(g / 3)]; }
};
using LdsTile = LdsTileT<kPadded, true>;

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
template <uint32_t NT = kST, uint32_t TILE = kTile, class Tile = LdsTile>
__device__ __forceinline__ void tile_load(const SortKey* __restrict__ g, uint32_t cnt, const Tile& t) {
  const uint64_t* gw = reinterpret_cast<const uint64_t*>(g);
  for (uint32_t i = threadIdx.x; i < 3 * cnt; i += NT) t.put_word(i, gw[i]);
  for (uint32_t i = cnt + threadIdx.x; i < TILE; i += NT) t.set(i, sentinel());
}

template <uint32_t NT = kST, class Tile = LdsTile>
__device__ __forceinline__ void tile_store(const Tile& t, SortKey* __restrict__ g, uint32_t cnt) {
  uint64_t* gw = reinterpret_cast<uint64_t*>(g);
  for (uint32_t i = threadIdx.x; i < 3 * cnt; i += NT) gw[i] = t.word(i);
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
    // the first key words decide almost every step: the rest of the two
    // records is read only on a tie (a third of the LDS reads)
    const uint64_t x = b.w0(d - mid - 1), y = a.w0(mid);
    if (x != y ? x < y : less(b[d - mid - 1], a[mid]))
      hi = mid;
    else
      lo = mid + 1;
  }
  return lo;
}

// A run of records inside the LDS tile, starting at record `base`.
template <class Tile = LdsTile>
struct LdsRunT {
  Tile t;
  uint32_t base;
  __device__ __forceinline__ SortKey operator[](uint32_t i) const { return t.get(base + i); }
  __device__ __forceinline__ uint64_t w0(uint32_t i) const { return t.w[Tile::pad(base + i)]; }
};
using LdsRun = LdsRunT<>;

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
                                                    uint64_t n, RecLess less, SortTail tl,
                                                    const uint32_t* __restrict__ run_if) {
  if (run_if && !*run_if) return;  // (uniform) the batch needs no sort
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
                                                    uint64_t n, uint64_t w, RecLess less, SortTail tl,
                                                    const uint32_t* __restrict__ run_if) {
  if (run_if && !*run_if) return;  // (uniform) the batch needs no sort
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

// ---- bin sort: one pass to bin the records, one LDS sort per group of bins ----
//
// The bins are the buckets of a DirMap over the keys' 8-byte prefixes (its
// byte masks sampled by k_sorted_check; sstable.hpp), at most kBins of them:
// a monotone function of the key, so every record of bin b sorts before
// every record of bin b + 1. As in a radix sort pass, without global
// atomics: k_bin_count leaves each block's bin histogram (LDS) in cnt;
// k_bin_offsets turns every bin's column into the blocks' exclusive offsets
// and the bins' starts inside 64-bin blocks plus each block's sum;
// k_bin_scatter writes each record into its bin's range (LDS cursors; any
// order inside a bin); k_bin_sort sorts one group of ~T records in LDS by
// the full record order (index last: the stable order) and writes what
// k_format needs. Groups are cut at bin boundaries: group g starts at the
// first bin starting at or after g * T, which each group-sort block finds
// itself from the 64-bin blocks' sums. A group larger than an LDS tile (a bin holding more than
// tile - T records: keys sharing a long prefix) sets
// CreateResult::flags[3] and the caller redoes the sort with the merge sort.
// Records make 2 round trips through HBM instead of 9, and the group sorts
// run as one wave at 1M entries.

constexpr uint32_t kBins = 8192;         // bins at most (one 32-KiB LDS histogram)
constexpr uint32_t kBinNT = 1024;        // count / scatter threads (16 waves: loads in flight)
constexpr uint32_t kBinPer = 4;          // records per count / scatter thread
constexpr uint32_t kBinChunk = kBinNT * kBinPer;  // records per count / scatter block
// Group sorts: 256 threads x 4 records (26 KiB of LDS, six blocks per CU)
// for groups of <= 1024 records, 512 x 4 (51 KiB, three per CU) up to 2048.
// A CU's share of the sort is what sets the time (the blocks all run in one
// wave): at 1M entries 1536 groups of ~683 fill 6 x 256 slots evenly, where
// 683 groups of ~1536 left a third of the CUs with two groups and the rest
// with three.
constexpr uint32_t kBinTileMax = 2048;    // records per group sort, at most
// LDS tiles padded by 1/16 (record i at word i + i / 16): 3 x 2176 x 8 B =
// 51 KiB for 2048 records (1/8 padding would leave room for two per CU)
template <uint32_t TILE>
struct LdsTile16 {
  static constexpr uint32_t P = TILE + TILE / 16;
  uint64_t* w;
  static __device__ __forceinline__ uint32_t pad(uint32_t i) { return i + (i >> 4); }
  __device__ __forceinline__ SortKey get(uint32_t i) const {
    const uint32_t j = pad(i);
    const uint64_t li = w[2 * P + j];
    SortKey r;
    r.w0 = w[j];
    r.w1 = w[P + j];
    r.len = (uint32_t)li;
    r.idx = (uint32_t)(li >> 32);
    return r;
  }
  __device__ __forceinline__ void set(uint32_t i, const SortKey& r) const {
    const uint32_t j = pad(i);
    w[j] = r.w0;
    w[P + j] = r.w1;
    w[2 * P + j] = (uint64_t)r.len | (uint64_t)r.idx << 32;
  }
  __device__ __forceinline__ void put_word(uint32_t g, uint64_t v) const { w[(g % 3) * P + pad(g / 3)] = v; }
  __device__ __forceinline__ uint64_t word(uint32_t g) const { return w[(g % 3) * P + pad(g / 3)]; }
};

// The bins' map and whether the bin sort runs at all, from r (every bin
// launch derives them itself: the host enqueues the sort before it knows the
// batch): it runs when the batch is unsorted and the sampled prefixes give at
// least two bins; an unsorted batch of one bin is left to the merge sort
// (flags[3], set by the first block of k_bin_count). Thread 0, into LDS.
__device__ __forceinline__ bool bin_plan(const CreateResult* r, uint64_t n, DirMap& sdm) {
  if (!r->flags[0]) return false;  // sorted: no sort at all
  sdm = make_dirmap(r->dmask, n, kBins);
  return sdm.nbuckets >= 2;
}

__global__ __launch_bounds__(kBinNT) void k_bin_count(const uint8_t* __restrict__ kb, const uint64_t* __restrict__ ko,
                                                      uint64_t n, CreateResult* r, uint32_t* __restrict__ cnt,
                                                      uint64_t* __restrict__ tsum, uint64_t ntiles) {
  __shared__ DirMap sdm;
  __shared__ uint32_t hist[kBins];
  __shared__ uint32_t go;
  if (threadIdx.x == 0) {
    go = bin_plan(r, n, sdm);
    if (!go && r->flags[0] && blockIdx.x == 0) r->flags[3] = 1u;  // unsorted, one bin: the merge sort's
  }
  __syncthreads();
  if (!go) return;
  const uint64_t p0 = (uint64_t)blockIdx.x * kBinChunk + threadIdx.x;
  uint64_t w0[kBinPer];
#pragma unroll
  for (uint32_t k = 0; k < kBinPer; ++k) {  // every key load in flight together
    const uint64_t p = p0 + (uint64_t)k * kBinNT;
    uint64_t w1;
    w0[k] = 0;
    if (p < n) load16(kb + ko[p], ko[p + 1] - ko[p], w0[k], w1);
  }
  // k_bin_sort adds the sorted line tiles into tsum (k_sorted_check left the
  // input order's there)
  for (uint64_t i = (uint64_t)blockIdx.x * kBinNT + threadIdx.x; i < ntiles; i += (uint64_t)gridDim.x * kBinNT)
    tsum[i] = 0;
  for (uint32_t b = threadIdx.x; b < kBins; b += kBinNT) hist[b] = 0;
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kBinPer; ++k)
    if (p0 + (uint64_t)k * kBinNT < n) atomicAdd(&hist[dir_bucket(sdm, w0[k])], 1u);
  __syncthreads();
  const uint32_t nb = (uint32_t)sdm.nbuckets;
  for (uint32_t b = threadIdx.x; b < nb; b += kBinNT) cnt[(uint64_t)blockIdx.x * nb + b] = hist[b];
}

// cnt[blk][b] := the blocks' exclusive offsets inside bin b; lstart[b] :=
// the exclusive prefix of the bin totals inside its 64-bin block; bsum[j] :=
// block j's total. A block takes 64 bins (the lanes: each row of cnt is read
// 256 B at a time) and splits the nblk rows among its 16 waves, each wave
// loading its first 16 rows together and keeping them for the rewrite; the
// waves' row sums are joined in LDS. The bins' global starts are never
// written: k_bin_scatter and k_bin_sort add the 64-bin blocks' prefix (a
// wave scan of <= 128 sums) to lstart themselves, so no single-block plan
// launch sits between the passes (one took 9 us).
constexpr uint32_t kOffW = 16;  // waves per k_bin_offsets block
constexpr uint32_t kOffR = 16;  // rows per wave held in registers
constexpr uint32_t kBinBlocks = kBins / 64;  // 64-bin blocks at most
__global__ __launch_bounds__(kOffW * 64) void k_bin_offsets(uint32_t* __restrict__ cnt, uint32_t nblk, uint64_t n,
                                                            const CreateResult* r, uint32_t* __restrict__ lstart,
                                                            uint32_t* __restrict__ bsum) {
  __shared__ uint32_t part[kOffW][64];
  __shared__ DirMap sdm;
  __shared__ uint32_t go;
  if (threadIdx.x == 0) go = bin_plan(r, n, sdm) && blockIdx.x * 64 < sdm.nbuckets;
  __syncthreads();
  if (!go) return;  // (the grid covers the most bins; blocks past this map's return)
  const uint32_t nb = (uint32_t)sdm.nbuckets;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, b = blockIdx.x * 64 + lane;
  const uint32_t per = (nblk + kOffW - 1) / kOffW, k0 = min(wv * per, nblk), k1 = min(k0 + per, nblk);
  const bool live = b < nb;
  uint32_t v[kOffR], sum = 0;
#pragma unroll
  for (uint32_t j = 0; j < kOffR; ++j) {  // every load in flight together
    v[j] = live && k0 + j < k1 ? cnt[(uint64_t)(k0 + j) * nb + b] : 0u;
    sum += v[j];
  }
  for (uint32_t k = k0 + kOffR; k < k1; ++k) sum += live ? cnt[(uint64_t)k * nb + b] : 0u;  // > 4M entries
  part[wv][lane] = sum;
  __syncthreads();
  uint32_t run = 0, tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < kOffW; ++w) {
    const uint32_t x = part[w][lane];
    run += w < wv ? x : 0u;
    tot += x;
  }
  if (wv == 0) {  // the bins' prefix inside this 64-bin block, and its total
    const uint32_t x = wave_inclusive_scan(tot);
    if (live) lstart[b] = x - tot;
    if (lane == 63) bsum[blockIdx.x] = x;
  }
  if (!live) return;
#pragma unroll
  for (uint32_t j = 0; j < kOffR; ++j) {
    if (k0 + j < k1) {
      cnt[(uint64_t)(k0 + j) * nb + b] = run;
      run += v[j];
    }
  }
  for (uint32_t k = k0 + kOffR; k < k1; ++k) {
    const uint32_t x = cnt[(uint64_t)k * nb + b];
    cnt[(uint64_t)k * nb + b] = run;
    run += x;
  }
}

// One wave (all 64 lanes): the 64-bin blocks' exclusive prefix from bsum
// (nbb <= 128 blocks, two per lane). Lane l gets pre0 = prefix of block 2l
// and a0 = its sum, so block 2l spans [pre0, pre0 + a0) and block 2l + 1
// [pre0 + a0, pre0 + s).
struct BinPrefix {
  uint32_t pre0, a0, s;
};
__device__ __forceinline__ BinPrefix bin_block_prefix(const uint32_t* __restrict__ bsum, uint32_t nbb) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t a = 2 * lane < nbb ? bsum[2 * lane] : 0u, c = 2 * lane + 1 < nbb ? bsum[2 * lane + 1] : 0u;
  const uint32_t s = a + c;
  const uint32_t x = wave_inclusive_scan(s);
  return BinPrefix{x - s, a, s};
}

__global__ __launch_bounds__(kBinNT) void k_bin_scatter(const uint8_t* __restrict__ kb,
                                                        const uint64_t* __restrict__ ko, uint64_t n,
                                                        const CreateResult* res,
                                                        const uint32_t* __restrict__ cnt,
                                                        const uint32_t* __restrict__ lstart,
                                                        const uint32_t* __restrict__ bsum,
                                                        SortKey* __restrict__ out) {
  __shared__ DirMap sdm;
  __shared__ uint32_t cur[kBins];
  __shared__ uint32_t bpre[kBinBlocks];
  __shared__ uint32_t go;
  if (threadIdx.x == 0) go = bin_plan(res, n, sdm);
  __syncthreads();
  if (!go) return;
  const uint32_t nbb = (uint32_t)((sdm.nbuckets + 63) / 64);
  const uint64_t p0 = (uint64_t)blockIdx.x * kBinChunk + threadIdx.x;
  SortKey r[kBinPer];
#pragma unroll
  for (uint32_t k = 0; k < kBinPer; ++k) {
    const uint64_t p = p0 + (uint64_t)k * kBinNT;
    if (p < n) r[k] = sort_record(kb, ko, p);
  }
  if (threadIdx.x < 64) {
    const BinPrefix bp = bin_block_prefix(bsum, nbb);
    const uint32_t l = threadIdx.x;
    if (2 * l < nbb) bpre[2 * l] = bp.pre0;
    if (2 * l + 1 < nbb) bpre[2 * l + 1] = bp.pre0 + bp.a0;
  }
  __syncthreads();
  const uint32_t nb = (uint32_t)sdm.nbuckets;
  for (uint32_t b = threadIdx.x; b < nb; b += kBinNT)
    cur[b] = bpre[b >> 6] + lstart[b] + cnt[(uint64_t)blockIdx.x * nb + b];
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kBinPer; ++k)
    if (p0 + (uint64_t)k * kBinNT < n) out[atomicAdd(&cur[dir_bucket(sdm, r[k].w0)], 1u)] = r[k];
}

// The start of group g: 0 for g = 0, n for g >= G, else the start of the
// first bin starting at or after g * T (bins never split). One wave: the
// first 64-bin block j whose end reaches g * T, then the first of its bins
// starting there (or, if its last bin straddles g * T, the next block's
// start).
__device__ __forceinline__ uint32_t bin_group_start(uint32_t g, uint32_t G, uint32_t T, uint32_t n,
                                                    const uint32_t* __restrict__ lstart,
                                                    const uint32_t* __restrict__ bsum, uint32_t nb,
                                                    uint32_t nbb) {
  if (g == 0) return 0;
  if (g >= G) return n;
  const uint32_t X = g * T, lane = threadIdx.x & 63u;
  const BinPrefix bp = bin_block_prefix(bsum, nbb);
  const uint32_t e0 = bp.pre0 + bp.a0, e1 = bp.pre0 + bp.s;  // ends of blocks 2l, 2l + 1
  const uint64_t m0 = __ballot(2 * lane < nbb && e0 >= X), m1 = __ballot(2 * lane + 1 < nbb && e1 >= X);
  // block nbb - 1 ends at n > X, so one of the masks is non-zero
  const uint32_t j0 = m0 ? 2 * (uint32_t)__builtin_ctzll(m0) : ~0u;
  const uint32_t j1 = m1 ? 2 * (uint32_t)__builtin_ctzll(m1) + 1 : ~0u;
  const uint32_t j = min(j0, j1), src = j >> 1;
  const uint32_t p = __shfl(bp.pre0, src, 64), a = __shfl(bp.a0, src, 64), sj = __shfl(bp.s, src, 64);
  const uint32_t bj = (j & 1) ? p + a : p, ej = (j & 1) ? p + sj : p + a;
  const uint32_t b = j * 64 + lane;
  const uint32_t st = b < nb ? bj + lstart[b] : ej;
  const uint64_t m = __ballot(st >= X);
  return m ? __shfl(st, (int)__builtin_ctzll(m), 64) : ej;
}

// One group [start(g), start(g + 1)) per block (bin_group_start): the k_sort_block network
// on the group's records, then vsp / tsum for k_format (tsum zeroed by the
// caller: a group's outputs are not aligned to format tiles, so each wave
// adds its share of the (at most two) tiles its 256 outputs touch) and the
// sorted records.
template <uint32_t NT>
__global__ __launch_bounds__(NT) void k_bin_sort(const SortKey* __restrict__ in, SortKey* __restrict__ out,
                                                 const uint32_t* __restrict__ lstart,
                                                 const uint32_t* __restrict__ bsum, CreateResult* res,
                                                 uint32_t T, uint32_t G, uint32_t n, RecLess less,
                                                 const uint64_t* __restrict__ vo, ulonglong2* __restrict__ vsp,
                                                 uint64_t* __restrict__ tsum) {
  static_assert(kFormatTile == 64 * kIPT, "a wave's outputs span at most two format tiles");
  constexpr uint32_t TILE = NT * kIPT;
  using BinTile = LdsTile16<TILE>;
  __shared__ uint64_t lds[3 * BinTile::P];
  const BinTile tile{lds};
  __shared__ uint32_t gb[2];
  __shared__ DirMap sdm;
  __shared__ uint32_t go;
  if (threadIdx.x == 0) go = bin_plan(res, n, sdm);
  __syncthreads();
  if (!go) return;
  const uint32_t nb = (uint32_t)sdm.nbuckets, nbb = (nb + 63) / 64;
  if (threadIdx.x < 128) {  // waves 0 and 1: the group's start and end
    const uint32_t v = bin_group_start(blockIdx.x + (threadIdx.x >> 6), G, T, n, lstart, bsum, nb, nbb);
    if ((threadIdx.x & 63u) == 0) gb[threadIdx.x >> 6] = v;
  }
  __syncthreads();
  const uint64_t beg = gb[0], end = gb[1];
  if (end <= beg) return;
  if (end - beg > TILE) {  // a bin too large for one tile: the table falls back to the merge sort
    if (threadIdx.x == 0) res->flags[3] = 1u;  // (every writer stores the same value)
    return;
  }
  const uint32_t cnt = (uint32_t)(end - beg);
  tile_load<NT, TILE>(in + beg, cnt, tile);
  __syncthreads();
  SortKey r[kIPT];
  const uint32_t t0 = threadIdx.x * kIPT;
#pragma unroll
  for (uint32_t k = 0; k < kIPT; ++k) r[k] = tile.get(t0 + k);
#pragma unroll
  for (uint32_t q = 0; q < kIPT; ++q) {
#pragma unroll
    for (uint32_t k = q & 1; k + 1 < kIPT; k += 2) cas(r[k], r[k + 1], less);
  }
  uint32_t span = kIPT;  // the network only as wide as the group
  while (span < cnt) span <<= 1;
  for (uint32_t w = kIPT; w < span; w <<= 1) {
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kIPT; ++k) tile.set(t0 + k, r[k]);
    __syncthreads();
    const uint32_t pb = t0 & ~(2 * w - 1), d = t0 - pb;
    const LdsRunT<BinTile> a{tile, pb}, b{tile, pb + w};
    const uint32_t i = merge_split(a, w, b, w, d, less);
    merge_seq(a, w, b, w, i, d - i, r, less);
  }
  // value spans, and the line lengths of this wave's outputs into the two
  // format tiles they can touch
  const uint64_t wbase = beg + (uint64_t)(threadIdx.x & ~63u) * kIPT;
  const uint64_t tlo = wbase / kFormatTile;
  uint64_t s_lo = 0, s_hi = 0;
#pragma unroll
  for (uint32_t k = 0; k < kIPT; ++k) {
    if (t0 + k < cnt) {
      const uint32_t i = r[k].idx;
      const uint64_t v0 = vo[i], vl = vo[i + 1] - v0;
      const uint64_t kl = r[k].len != 0xFFFFFFFFu ? r[k].len : less.ko[i + 1] - less.ko[i];
      const uint64_t p = beg + t0 + k;
      vsp[p] = make_ulonglong2(v0, vl);
      (p / kFormatTile == tlo ? s_lo : s_hi) += line_len(kl, vl);
    }
  }
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    s_lo += __shfl_xor(s_lo, o, 64);
    s_hi += __shfl_xor(s_hi, o, 64);
  }
  if ((threadIdx.x & 63u) == 0) {
    if (s_lo) atomicAdd((unsigned long long*)&tsum[tlo], (unsigned long long)s_lo);
    if (s_hi) atomicAdd((unsigned long long*)&tsum[tlo + 1], (unsigned long long)s_hi);
  }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kIPT; ++k) tile.set(t0 + k, r[k]);
  __syncthreads();
  tile_store<NT>(tile, out + beg, cnt);
}

}  // namespace

uint64_t entry_sort_tmp_bytes(uint64_t n) { return n * sizeof(SortKey); }

uint64_t bin_sort_tmp_bytes(uint64_t n, uint32_t T) {
  const uint64_t nblk = (n + kBinChunk - 1) / kBinChunk;
  (void)T;
  // the bins are known only on the device: room for the most of them
  return n * sizeof(SortKey) + (nblk * kBins + kBins + kBinBlocks) * 4;
}

uint32_t bin_sort_max_group() { return kBinTileMax; }

hipError_t launch_bin_sort(const uint8_t* kb, const uint64_t* ko, uint64_t n, uint32_t T, SortKey* out, void* tmp,
                           hipStream_t s, const uint64_t* vo, ulonglong2* vsp, uint64_t* tsum, CreateResult* r) {
  if (!n) return hipSuccess;
  if (!T || T > kBinTileMax || n >= (1ull << 32)) return hipErrorInvalidValue;
  const uint32_t G = (uint32_t)((n + T - 1) / T);
  const uint32_t nblk = (uint32_t)((n + kBinChunk - 1) / kBinChunk);
  SortKey* binned = (SortKey*)tmp;
  // cnt is nblk x nb for the device's nb; lstart and bsum sit past the most
  uint32_t* cnt = (uint32_t*)(binned + n);
  uint32_t* lstart = cnt + (uint64_t)nblk * kBins;
  uint32_t* bsum = lstart + kBins;
  {
    ProfScope ps("k_bin_count", s);
    hipLaunchKernelGGL(k_bin_count, dim3(nblk), dim3(kBinNT), 0, s, kb, ko, n, r, cnt, tsum, format_tiles(n));
  }
  {
    ProfScope ps("k_bin_offsets", s);
    hipLaunchKernelGGL(k_bin_offsets, dim3(kBinBlocks), dim3(kOffW * 64), 0, s, cnt, nblk, n, r, lstart, bsum);
  }
  {
    ProfScope ps("k_bin_scatter", s);
    hipLaunchKernelGGL(k_bin_scatter, dim3(nblk), dim3(kBinNT), 0, s, kb, ko, n, r, cnt, lstart, bsum, binned);
  }
  ProfScope ps("k_bin_sort", s);
  if (T <= 768)  // 1024-record tiles: room for bins of up to 1024 - T records past the target
    hipLaunchKernelGGL(k_bin_sort<256>, dim3(G), dim3(256), 0, s, binned, out, lstart, bsum, r, T, G,
                       (uint32_t)n, RecLess{kb, ko}, vo, vsp, tsum);
  else
    hipLaunchKernelGGL(k_bin_sort<512>, dim3(G), dim3(512), 0, s, binned, out, lstart, bsum, r, T, G,
                       (uint32_t)n, RecLess{kb, ko}, vo, vsp, tsum);
  return hipGetLastError();
}

hipError_t launch_entry_sort(const SortKey* in, SortKey* out, SortKey* tmp, uint64_t n, const uint8_t* kb,
                             const uint64_t* ko, hipStream_t s, const uint64_t* vo, ulonglong2* vsp,
                             uint64_t* tsum, const uint32_t* run_if) {
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
                     rounds ? none : tail, run_if);
  for (uint32_t r = 0; r < rounds; ++r) {
    const uint64_t w = (uint64_t)kTile << r;
    hipLaunchKernelGGL(k_sort_merge, dim3((uint32_t)tiles), dim3(kST), 0, s, bufs[(rounds - r) & 1],
                       bufs[(rounds - r - 1) & 1], n, w, less, r + 1 == rounds ? tail : none, run_if);
  }
  return hipGetLastError();
}

}  // namespace cb
