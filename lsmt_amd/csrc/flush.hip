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


#include "blockscan.hpp"
#include "flush.hpp"
#include "profile.hpp"
#include "zone.hpp"

namespace cb {
namespace {

constexpr uint32_t kNT = 256;  // = kFormatTile

inline uint32_t blocks_for(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }


// The first 16 bytes of key p (output order) as zero-padded big-endian words,
// and its length. Unsorted input: the sort record already holds them; sorted
// input: load16 of the key's bytes.
__device__ __forceinline__ void key_words(const SortKey* order, const uint8_t* kb,
                                          const uint64_t* ko, uint64_t p, uint64_t& i,
                                          uint64_t& kl, uint64_t& w0, uint64_t& w1) {
  if (order) {  // the record holds the words and (unless clamped) the length
    const SortKey sk = order[p];
    i = sk.idx;
    w0 = sk.w0;
    w1 = sk.w1;
    kl = sk.len != 0xFFFFFFFFu ? sk.len : ko[i + 1] - ko[i];
    return;
  }
  i = p;
  const uint64_t o0 = ko[i];
  kl = ko[i + 1] - o0;
  load16(kb + o0, kl, w0, w1);
}

// Does a big-endian word hold byte c among its first m (<= 8) bytes?
__device__ __forceinline__ bool has_byte(uint64_t w, uint64_t m, uint32_t c) {
  if (!m) return false;
  const uint64_t keep = m >= 8 ? ~0ull : ~(~0ull >> (8 * m));  // the first m bytes
  const uint64_t x = (w ^ (0x0101010101010101ull * c)) | ~keep;  // 0x00 where byte == c
  return ((x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull) != 0;
}

// Sort records in input order (the key's first 16 bytes read as words).
__global__ __launch_bounds__(kNT) void k_sort_keys(const uint8_t* __restrict__ kb,
                                                   const uint64_t* __restrict__ ko, uint64_t n,
                                                   SortKey* __restrict__ out) {
  const uint64_t p = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  if (p >= n) return;
  out[p] = sort_record(kb, ko, p);
}

// Rust str order of keys q and p (q, p index the key batch) given their first
// 16 bytes as words: from the words alone when both fit in 16 bytes.
__device__ __forceinline__ int key_cmp(const uint8_t* kb, const uint64_t* ko, uint64_t q,
                                       uint64_t ql, uint64_t qw0, uint64_t qw1, uint64_t p,
                                       uint64_t pl, uint64_t pw0, uint64_t pw1) {
  if (ql <= 16 && pl <= 16) {
    if (qw0 != pw0) return qw0 < pw0 ? -1 : 1;
    if (qw1 != pw1) return qw1 < pw1 ? -1 : 1;
    return ql < pl ? -1 : (ql > pl ? 1 : 0);
  }
  return bytes_cmp(kb + ko[q], ql, kb + ko[p], pl);
}


// The sum of each kFormatTile-line tile's lengths (order == nullptr: input
// order), for k_format's offsets. Call uniformly.
__device__ __forceinline__ void tile_sum(const SortKey* order, const uint64_t* ko, const uint64_t* vo,
                                         uint64_t n, uint64_t* tsum) {
  const uint64_t p = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  uint64_t len = 0;
  if (p < n) {
    const uint64_t i = order ? order[p].idx : p;
    len = line_len(ko[i + 1] - ko[i], vo[i + 1] - vo[i]);
  }
  uint64_t total;
  (void)block_scan<kNT>(len, &total);
  if (threadIdx.x == 0) tsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(kNT) void k_line_sums(const SortKey* __restrict__ order,
                                                   const uint64_t* __restrict__ ko,
                                                   const uint64_t* __restrict__ vo, uint64_t n,
                                                   uint64_t* __restrict__ tsum) {
  tile_sum(order, ko, vo, n, tsum);
}

static_assert(offsetof(CreateResult, len) == kCreateHead, "the zeroed head of CreateResult");

// r->flags[0] |= key[i-1] > key[i] for some i (not in stable-sorted order).
// Each lane's key comes in as words; the previous one from the neighbour lane.
__global__ __launch_bounds__(kNT) void k_sorted_check(const uint8_t* __restrict__ kb,
                                                      const uint64_t* __restrict__ ko,
                                                      const uint64_t* __restrict__ vo, uint64_t n,
                                                      CreateResult* r, uint64_t* __restrict__ tsum,
                                                      uint64_t kmax, uint64_t vmax) {
  const uint64_t p = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  tile_sum(nullptr, ko, vo, n, tsum);  // the line tiles if the input is already sorted
  if (p == 0) {
    const uint64_t kt = ko[n], vt = vo[n];
    r->ktot = kt;
    r->vtot = vt;
    // the file buffer was sized from the caller's byte bounds: a batch past
    // them is refused (k_format writes nothing) and reported by the table
    if (kt > kmax || vt > vmax) r->flags[4] = 1u;
  }
  uint64_t i = 0, kl = 0, w0 = 0, w1 = 0;
  if (p < n) key_words(nullptr, kb, ko, p, i, kl, w0, w1);
  if (blockIdx.x < kSampleBlocks)  // the directory's alphabet, from evenly spaced keys (order-free)
    sample_pfx_masks(n, [&](uint64_t q) {
      uint64_t a, b;
      load16(kb + ko[q], ko[q + 1] - ko[q], a, b);
      return a;
    }, &r->dmask[0][0]);
  uint64_t pkl = __shfl_up(kl, 1, 64), pw0 = __shfl_up(w0, 1, 64), pw1 = __shfl_up(w1, 1, 64);
  uint64_t pi = p - 1;
  if (p < n && lane == 0 && p > 0) key_words(nullptr, kb, ko, p - 1, pi, pkl, pw0, pw1);
  const bool bad = p < n && p > 0 && key_cmp(kb, ko, p - 1, pkl, pw0, pw1, p, kl, w0, w1) > 0;
  // one plain store of 1 per block holding an inversion (every writer
  // writes the same value): a fully unsorted batch would otherwise queue a
  // returning load and an atomic per block on one word
  if (__syncthreads_or(bad) && threadIdx.x == 0) r->flags[0] = 1u;
}



// One bound of the ZoneMap (the file's first or last key, w = 0 / 1) into r:
// input index, full length and up to kZoneInline bytes. Whole block.
__device__ __forceinline__ void zone_bound(const SortKey* order, const uint8_t* kb, const uint64_t* ko,
                                           uint64_t p, uint32_t w, CreateResult* r) {
  const uint64_t i = order ? order[p].idx : p;
  const uint64_t o = ko[i], kl = ko[i + 1] - o;
  if (threadIdx.x == 0) {
    (w ? r->idx_max : r->idx_min) = i;
    r->zlen[w] = (uint32_t)min<uint64_t>(kl, 0xFFFFFFFFull);
  }
  for (uint32_t b = threadIdx.x; b < kl && b < kZoneInline; b += kNT) r->zkey[w][b] = kb[o + b];
}

__device__ __forceinline__ uint8_t b64c(uint32_t v) {
  return (uint8_t)(v < 26 ? 'A' + v : v < 52 ? 'a' + (v - 26) : v < 62 ? '0' + (v - 52) : v == 62 ? '+' : '/');
}

// Byte j (< 16) of a string held as two zero-padded big-endian words.
__device__ __forceinline__ uint32_t be_byte(uint64_t w0, uint64_t w1, uint64_t j) {
  return (uint32_t)((j < 8 ? w0 >> (56 - 8 * j) : w1 >> (120 - 8 * j)) & 0xFF);
}

// One lane per line: key, TAB, STANDARD.encode(value), NL, through put(j, b);
// kb(j) / vb(j) give the key's and the value's bytes.
template <class KB, class VB, class Put>
__device__ __forceinline__ void format_line(uint64_t kl, KB kbyte, uint64_t vl, VB vbyte, Put put) {
  uint64_t o = 0;
  for (uint64_t j = 0; j < kl; ++j) put(o++, kbyte(j));
  put(o++, '\t');
  for (uint64_t j = 0; j < vl; j += 3) {
    const uint64_t r = vl - j;
    const uint32_t w = vbyte(j) << 16 | (r > 1 ? vbyte(j + 1) << 8 : 0u) | (r > 2 ? vbyte(j + 2) : 0u);
    put(o++, b64c(w >> 18));
    put(o++, b64c((w >> 12) & 63));
    put(o++, r > 1 ? b64c((w >> 6) & 63) : (uint8_t)'=');
    put(o++, r > 2 ? b64c(w & 63) : (uint8_t)'=');
  }
  put(o, '\n');
}

// Byte t (static) of 16 bytes held in memory order as two little-endian words.
__device__ __forceinline__ uint32_t mem_byte(uint64_t b0, uint64_t b1, uint32_t t) {
  return t < 8 ? (uint32_t)(b0 >> (8 * t)) & 0xFF : t < 16 ? (uint32_t)(b1 >> (8 * (t - 8))) & 0xFF : 0u;
}

// dst[j] = bytes [4j, 4j+4) of src shifted up by s (0..3) bytes: src's byte i
// lands at byte i + s. N output dwords from N-1 input dwords (+ the top one).
template <int N>
__device__ __forceinline__ void shift_bytes(const uint32_t* src, uint32_t s, uint32_t* dst) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const uint64_t hi = j < N - 1 ? src[j] : 0u, lo = j ? src[j - 1] : 0u;
    dst[j] = (uint32_t)(((hi << 32) | lo) >> (32 - 8 * s));
  }
}

// A line whose key and value are both <= 16 bytes (words w0/w1: the key as
// big-endian words; v0/v1: the value's) built in registers: L[0..12) holds
// its bytes in memory order, zero past the end. Static byte positions only,
// so nothing spills: the key's 4 dwords, then '\t' + base64 + '\n' built at
// fixed positions and shifted into place by kl bytes. Returns the length.
__device__ __forceinline__ uint32_t line16(uint64_t w0, uint64_t w1, uint32_t kl, uint64_t v0, uint64_t v1,
                                           uint32_t vl, uint32_t L[12]) {
  const uint64_t k0 = __builtin_bswap64(w0), k1 = __builtin_bswap64(w1);  // memory order
  const uint32_t K[4] = {(uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32)};
  const uint64_t b0 = __builtin_bswap64(v0), b1 = __builtin_bswap64(v1);
  const uint32_t g = (vl + 2) / 3;  // base64 quads
  uint32_t V[8] = {'\t', 0, 0, 0, 0, 0, 0, 0};  // '\t' at 0, quad i at 1+4i, '\n' at 1+4g
#pragma unroll
  for (uint32_t i = 0; i < 6; ++i) {
    if (i < g) {
      const uint32_t t = 3 * i, r = vl - t;
      const uint32_t w = mem_byte(b0, b1, t) << 16 | (r > 1 ? mem_byte(b0, b1, t + 1) << 8 : 0u) |
                         (r > 2 ? mem_byte(b0, b1, t + 2) : 0u);
      const uint32_t c0 = b64c(w >> 18), c1 = b64c((w >> 12) & 63);
      const uint32_t c2 = r > 1 ? b64c((w >> 6) & 63) : '=', c3 = r > 2 ? b64c(w & 63) : '=';
      V[i] |= c0 << 8 | c1 << 16 | c2 << 24;
      V[i + 1] |= c3;
    }
    if (i == g) V[i] |= (uint32_t)'\n' << 8;
  }
  if (g == 6) V[6] |= (uint32_t)'\n' << 8;
  // the key's kl bytes, then V: V shifted up by kl = 4 * (kl >> 2) + (kl & 3)
  uint32_t S[9];
  shift_bytes<9>(V, kl & 3, S);
  const uint32_t ds = kl >> 2;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    uint32_t x = 0;
#pragma unroll
    for (int d = 0; d <= 4; ++d)
      if (j - d >= 0 && j - d < 9 && ds == (uint32_t)d) x = S[j - d];
    L[j] = (j < 4 ? K[j] : 0u) | x;
  }
  return kl + 2 + 4 * g;
}

// Staged output bytes per block: 16 KiB (more resident blocks) when the
// average line is short, else 32 KiB; a block whose lines exceed the stage
// writes its bytes directly.
constexpr uint32_t kFormatLdsSmall = 16384, kFormatLdsLarge = 32768;

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// SsTable::create's file and everything derived from it, one lane per entry p
// (= line p; entries in key order):
// - the line `key \t base64(value) \n` at its offset: the tile sums before
//   the block (tsum from k_sorted_check or k_line_sums, scanned by
//   k_tile_scan) plus the scan of the block's line lengths: no full-length
//   scan pass. A block's 256 lines are one
//   contiguous range; when it fits in LDS the lanes format into LDS (staged at
//   the range's address mod 4, so LDS and global dwords line up) and the block
//   writes it with aligned dword stores, else lanes write bytes directly.
//   Keys and values of <= 16 bytes come in as aligned dword loads.
// - the line index that k_line_finish / k_line_keys would derive by re-reading
//   the file: LineRec, prefix and fence (sstable.hpp layout). flags[1] |= 1 if
//   a key holds '\n' or '\t' (the caller then re-indexes the file the way
//   SsTable::get splits it); flags[2] &= keys strictly increasing.
// - r: the ZoneMap bounds (first / last key); k_tile_scan wrote r->len.
template <uint32_t LDSB>
__global__ __launch_bounds__(kNT) void k_format(const SortKey* __restrict__ order,
                                                const uint8_t* __restrict__ kb,
                                                const uint64_t* __restrict__ ko,
                                                const uint8_t* __restrict__ vb,
                                                const uint64_t* __restrict__ vo,
                                                const uint64_t* __restrict__ tsum, uint64_t n,
                                                uint8_t* __restrict__ out, LineRec* __restrict__ rec,
                                                uint64_t* __restrict__ pfx, uint64_t* __restrict__ fence,
                                                uint32_t* __restrict__ llen_out,
                                                CreateResult* r, const ulonglong2* __restrict__ vsp,
                                                uint32_t* __restrict__ dir, DirMap* dmap_out, uint32_t inline_nt) {
  __shared__ uint32_t stage32[LDSB / 4];
  __shared__ uint64_t s_base;
  __shared__ DirMap sdm;  // the directory's map, indexed per lane
  uint8_t* stage = reinterpret_cast<uint8_t*>(stage32);
  // The byte totals exceed the bounds the file buffer was sized from: nothing
  // here may write at offsets derived from them; the table reports the error
  // when it is finalised. (A batch the bin sort could not place, flags[3],
  // was sorted again by the merge sort enqueued after it.)
  if (r->flags[4]) return;
  if (!r->flags[0]) {  // the batch was sorted: the sort left nothing, format in input order
    order = nullptr;
    vsp = nullptr;
  }
  const uint64_t p0 = (uint64_t)blockIdx.x * kNT;
  const uint64_t p = p0 + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t pend = p0 + kNT < n ? p0 + kNT : n;
  const bool live = p < n;
  uint64_t i = 0, kl = 0, w0 = 0, w1 = 0;
  if (dir && threadIdx.x == 0) {  // the directory's map from the sampled prefix bytes (order-free)
    sdm = make_dirmap(r->dmask, n);
    if (blockIdx.x == 0) *dmap_out = sdm;  // the table's copy, for the read path
  }
  if (live) key_words(order, kb, ko, p, i, kl, w0, w1);
  // the previous entry's key: the neighbour lane's, or loaded by lane 0
  uint64_t pkl = __shfl_up(kl, 1, 64), pw0 = __shfl_up(w0, 1, 64), pw1 = __shfl_up(w1, 1, 64);
  uint64_t pi = __shfl_up(i, 1, 64);
  if (live && lane == 0 && p > 0) key_words(order, kb, ko, p - 1, pi, pkl, pw0, pw1);
  uint64_t vo0 = 0, vl = 0;
  if (live && vsp) {  // sorted by launch_entry_sort: in output order, one coalesced load
    const ulonglong2 e = vsp[p];
    vo0 = e.x;
    vl = e.y;
  } else if (live) {
    vo0 = vo[i];
    vl = vo[i + 1] - vo0;
  }
  // the line's offset: the tiles before this block, then the scan inside it.
  // (Loading the value here, before the barriers, measured slower: 55 vs 52
  // us after a sort.)
  uint64_t total;
  const uint64_t pre = block_scan<kNT>(live ? line_len(kl, vl) : 0, &total);
  uint64_t base;
  if (inline_nt) {
    // small batches (<= 64 tiles): the raw tile sums, scanned here by wave 0
    // instead of by a k_tile_scan launch; block 0 also writes the file length
    if (threadIdx.x < 64) {
      const uint64_t v = threadIdx.x < inline_nt ? tsum[threadIdx.x] : 0;
      const uint64_t before = wave_sum_u64(threadIdx.x < blockIdx.x ? v : 0);
      const uint64_t all = wave_sum_u64(v);
      if (threadIdx.x == 0) {
        s_base = before;
        if (blockIdx.x == 0) r->len = all;
      }
    }
    __syncthreads();
    base = s_base;
  } else {
    base = tsum[blockIdx.x];  // k_tile_scan: the tiles before
  }
  const uint64_t o = base + pre;
  bool special = false, not_inc = false;
  if (live) {
    const uint64_t llen = kl + 1 + (vl + 2) / 3 * 4;  // without the '\n'
    if (kl <= 16) {
      special = has_byte(w0, kl < 8 ? kl : 8, '\n') || has_byte(w0, kl < 8 ? kl : 8, '\t') ||
                (kl > 8 && (has_byte(w1, kl - 8, '\n') || has_byte(w1, kl - 8, '\t')));
    } else {
      const uint8_t* k = kb + ko[i];
      for (uint64_t j = 0; j < kl; ++j) special |= (k[j] == '\n') | (k[j] == '\t');
    }
    special |= llen >= kNoSep;  // the re-index reports it
    LineRec lr;
    lr.start = o;
    lr.pfx2 = w1;  // bytes 8..15 (zero when kl <= 8)
    lr.klen = (uint32_t)kl;
    lr.vdl = (uint32_t)vl;  // canonical STANDARD encoding: always decodes
    lr.pfx0 = w0;
    // the index and the file are written once and read by later launches
    // (the read path): non-temporal, no L2 lines to write back at the
    // kernel's end (k_format 52.3 -> 49.2 us after the bin sort)
    typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
    const u32x4_t ra = {(uint32_t)lr.start, (uint32_t)(lr.start >> 32), (uint32_t)lr.pfx2,
                        (uint32_t)(lr.pfx2 >> 32)};
    const u32x4_t rb = {lr.klen, lr.vdl, (uint32_t)lr.pfx0, (uint32_t)(lr.pfx0 >> 32)};
    __builtin_nontemporal_store(ra, reinterpret_cast<u32x4_t*>(rec + p));
    __builtin_nontemporal_store(rb, reinterpret_cast<u32x4_t*>(rec + p) + 1);
    __builtin_nontemporal_store(w0, pfx + p);
    __builtin_nontemporal_store((uint32_t)llen, llen_out + p);
    fence_put(fence, n, p, w0);
    if (p > 0) not_inc = key_cmp(kb, ko, pi, pkl, pw0, pw1, i, kl, w0, w1) >= 0;
  }
  // plain stores of one value from every block that has one (no atomics)
  if (__syncthreads_or(special) && threadIdx.x == 0) r->flags[1] = 1u;
  if (__syncthreads_or(not_inc) && threadIdx.x == 0) r->flags[2] = 1u;
  if (dir) {
    // the byte-rank directory (sstable.hpp DirMap, dir_fill): line p owns
    // dir[B] for the buckets B in (bucket(line p-1), bucket(line p)]
    const uint64_t b1 = live ? dir_bucket(sdm, w0) : 0;
    uint64_t bp = __shfl_up(b1, 1, 64);  // the previous line's bucket: the neighbour lane's
    if (live && lane == 0 && p > 0) bp = dir_bucket(sdm, pw0);
    dir_fill(dir, sdm.nbuckets, n, p, live, b1, bp);
  }
  if (blockIdx.x == 0) zone_bound(order, kb, ko, 0, 0, r);
  if (pend == n) {
    zone_bound(order, kb, ko, n - 1, 1, r);
    // 16 zero bytes after the file: the readable slack of the table's buffer
    if (threadIdx.x < 16) out[base + total + threadIdx.x] = 0;
  }
  const uint8_t* k = kb + (live && kl > 16 ? ko[i] : 0);  // key bytes: only past 16 (else the words)
  const uint8_t* v = vb + vo0;
  uint64_t v0 = 0, v1 = 0;
  const bool words = kl <= 16 && vl <= 16;
  if (live && vl <= 16) load16(v, vl, v0, v1);
  auto emit = [&](auto put) {  // byte at a time (long lines)
    if (!live) return;
    auto kbyte = [&](uint64_t j) { return kl <= 16 ? be_byte(w0, w1, j) : (uint32_t)k[j]; };
    auto vbyte = [&](uint64_t j) { return vl <= 16 ? be_byte(v0, v1, j) : (uint32_t)v[j]; };
    format_line(kl, kbyte, vl, vbyte, put);
  };
  const uint64_t sh0 = base & 3;
  if (total + sh0 > LDSB) {  // uniform: long lines, direct byte stores
    emit([&](uint64_t j, uint8_t c) { out[o + j] = c; });
    return;
  }
  // Stage the block's range in LDS, ORed into zeroed dwords: the lines of
  // neighbouring lanes share edge dwords, and ds_or keeps both.
  const uint32_t nd = (uint32_t)((sh0 + total + 3) / 4);
  for (uint32_t j = threadIdx.x; j < nd; j += kNT) stage32[j] = 0;
  __syncthreads();
  const uint64_t off = o - base + sh0;  // the line's first byte in the stage
  if (live && words) {
    uint32_t L[12], M[13];
    const uint32_t len = line16(w0, w1, (uint32_t)kl, v0, v1, (uint32_t)vl, L);
    shift_bytes<13>(L, (uint32_t)(off & 3), M);
    const uint32_t nw = (uint32_t)((off & 3) + len + 3) / 4;
    uint32_t* dst = stage32 + off / 4;
#pragma unroll
    for (uint32_t j = 0; j < 13; ++j)
      if (j < nw) atomicOr(dst + j, M[j]);
  } else if (live) {
    emit([&](uint64_t j, uint8_t c) {
      const uint64_t b = off + j;
      atomicOr(stage32 + b / 4, (uint32_t)c << (8 * (b & 3)));
    });
  }
  __syncthreads();
  // out[base .. base+total): bytes up to the first 4-aligned address, then
  // aligned dwords (LDS dword-aligned too), then the tail
  uint8_t* g = out + base;
  const uint64_t head = min<uint64_t>((4 - sh0) & 3, total);
  if (threadIdx.x < head) g[threadIdx.x] = stage[sh0 + threadIdx.x];
  const uint64_t body = (total - head) / 4;
  uint32_t* gw = reinterpret_cast<uint32_t*>(g + head);
  const uint32_t* sw = stage32 + (sh0 + head) / 4;
  for (uint64_t j = threadIdx.x; j < body; j += kNT) __builtin_nontemporal_store(sw[j], gw + j);
  const uint64_t tail0 = head + 4 * body;
  if (tail0 + threadIdx.x < total) g[tail0 + threadIdx.x] = stage[sh0 + tail0 + threadIdx.x];
}

}  // namespace

hipError_t launch_sort_keys(const uint8_t* kb, const uint64_t* ko, uint64_t n, SortKey* out,
                            hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("k_sort_keys", s);
  hipLaunchKernelGGL(k_sort_keys, dim3(blocks_for(n, kNT)), dim3(kNT), 0, s, kb, ko, n, out);
  return hipGetLastError();
}


hipError_t launch_sorted_check(const uint8_t* kb, const uint64_t* ko, const uint64_t* vo, uint64_t n,
                               CreateResult* r, uint64_t* tsum, uint64_t kmax, uint64_t vmax, hipStream_t s) {
  ProfScope ps("k_sorted_check", s);
  hipLaunchKernelGGL(k_sorted_check, dim3(n ? blocks_for(n, kNT) : 1), dim3(kNT), 0, s, kb, ko, vo, n, r,
                     tsum, kmax, vmax);
  return hipGetLastError();
}

hipError_t launch_line_sums(const SortKey* order, const uint64_t* ko, const uint64_t* vo, uint64_t n,
                            uint64_t* tsum, hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("k_line_sums", s);
  hipLaunchKernelGGL(k_line_sums, dim3(blocks_for(n, kNT)), dim3(kNT), 0, s, order, ko, vo, n, tsum);
  return hipGetLastError();
}




hipError_t launch_format(const SortKey* order, const uint8_t* kb, const uint64_t* ko,
                         const uint8_t* vb, const uint64_t* vo, const uint64_t* tsum, uint64_t n,
                         uint8_t* out, LineRec* rec, uint64_t* pfx, uint64_t* fence, uint32_t* llen,
                         CreateResult* r, uint64_t bytes_bound, hipStream_t s, const ulonglong2* vsp,
                         uint32_t* dir, DirMap* dmap_out, bool inline_scan) {
  if (!n) return hipSuccess;
  if (dir && !dmap_out) return hipErrorInvalidValue;
  const uint64_t nb = blocks_for(n, kNT);
  if (inline_scan && nb > kFormatInlineTiles) return hipErrorInvalidValue;
  const uint32_t inl = inline_scan ? (uint32_t)nb : 0u;
  ProfScope ps("k_format", s);
  const dim3 g((uint32_t)nb);
  if (bytes_bound / n * kNT * 5 / 4 <= kFormatLdsSmall)
    hipLaunchKernelGGL(k_format<kFormatLdsSmall>, g, dim3(kNT), 0, s, order, kb, ko, vb, vo, tsum, n, out,
                       rec, pfx, fence, llen, r, order ? vsp : nullptr, dir, dmap_out, inl);
  else
    hipLaunchKernelGGL(k_format<kFormatLdsLarge>, g, dim3(kNT), 0, s, order, kb, ko, vb, vo, tsum, n, out,
                       rec, pfx, fence, llen, r, order ? vsp : nullptr, dir, dmap_out, inl);
  return hipGetLastError();
}

}  // namespace cb
