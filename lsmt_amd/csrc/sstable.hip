// sstable.hip — line index, batched binary search and base64 for SSTable data
// files in HBM (see sstable.hpp for the reference mapping).
//
// Index build is streaming byte work (HBM-bound): each block owns a 4 KiB
// chunk, each thread 16 contiguous bytes read as one dwordx4. A byte i starts
// a line iff data[i] != '\n' and (i == 0 or data[i-1] == '\n') — exactly the
// non-empty pieces of raw.split('\n') (src/sstable.rs:142-146). Per-line work
// (TAB position, key prefixes, base64 validity of the value) is done once
// here, so the read path only touches the index and, at the end, the value.
//
// Resolution is latency-bound random access: one lane per key. Each lane
// gathers its candidate tables first and then searches its own next
// candidate, so a wave's lanes search different tables concurrently.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdlib>
#include <cstring>

#include "blockscan.hpp"
#include "profile.hpp"
#include "setmask.hpp"
#include "sstable.hpp"
#include "wideset.hpp"
#include "zone.hpp"

namespace cb {
namespace {

constexpr uint32_t kNT = 256;


// ---- byte access helpers ----

// 8 bytes at any address p of a table's data buffer (allocated with 16 bytes
// of slack past the file), little-endian: three aligned dword loads and two
// byte-aligns instead of eight byte loads.
__device__ __forceinline__ uint64_t ld8(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t x = w[0], y = w[1], z = w[2];
  const uint32_t lo = __builtin_amdgcn_alignbyte(y, x, sh);
  const uint32_t hi = __builtin_amdgcn_alignbyte(z, y, sh);
  return (uint64_t)hi << 32 | lo;
}

// Up to 8 data bytes as a big-endian word, zero-padded past m.
__device__ __forceinline__ uint64_t ld8_be(const uint8_t* p, uint64_t m) {
  const uint64_t v = __builtin_bswap64(ld8(p));
  return m >= 8 ? v : (m ? v & ~(~0ull >> (8 * m)) : 0);
}

// Rust str order of a line key (table data, side a) against a query key.
__device__ __forceinline__ int line_cmp(const uint8_t* a, uint64_t al, const uint8_t* b,
                                        uint64_t bl) {
  const uint64_t n = al < bl ? al : bl;
  for (uint64_t i = 0; i < n; i += 8) {
    const uint64_t m = n - i < 8 ? n - i : 8;
    const uint64_t x = ld8_be(a + i, m), y = be_chunk(b + i, m);
    if (x != y) return x < y ? -1 : 1;
  }
  return al < bl ? -1 : (al > bl ? 1 : 0);
}

// Standard-alphabet value of a byte, -1 if outside it.
__device__ __forceinline__ int b64v(uint32_t c) {
  int v = -1;
  v = (c - 'A' < 26u) ? (int)(c - 'A') : v;
  v = (c - 'a' < 26u) ? (int)(c - 'a') + 26 : v;
  v = (c - '0' < 10u) ? (int)(c - '0') + 52 : v;
  v = c == '+' ? 62 : v;
  v = c == '/' ? 63 : v;
  return v;
}

// base64 0.21.7 STANDARD (canonical padding, zero trailing bits): decoded
// length of p[0..len) (table data), or -1 if STANDARD.decode would fail.
__device__ __forceinline__ int64_t b64_len(const uint8_t* p, uint64_t len) {
  if (len & 3) return -1;
  if (!len) return 0;
  const uint32_t pad = p[len - 1] == '=' ? (p[len - 2] == '=' ? 2 : 1) : 0;
  const uint64_t body = len - pad;
  int last = 0;
  for (uint64_t i = 0; i < body; i += 8) {
    const uint64_t w = ld8(p + i);
    int bad = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const int v = i + j < body ? b64v((uint32_t)(w >> (8 * j)) & 0xFF) : 0;
      bad |= v;  // negative iff some v < 0
      if (i + j == body - 1) last = v;
    }
    if (bad < 0) return -1;
  }
  if (pad == 2 && (last & 0x0F)) return -1;
  if (pad == 1 && (last & 0x03)) return -1;
  return (int64_t)(len / 4 * 3 - pad);
}

// ---- line index ----

// The 16 bytes of a thread's slice and the byte before it ('\n' before the
// file: the first byte can start a line).
__device__ __forceinline__ void load_slice(const uint8_t* data, uint64_t len, uint64_t base,
                                           uint8_t b[16], uint32_t& prev) {
  if (base + 16 <= len) {
    const uint4 v = *reinterpret_cast<const uint4*>(data + base);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) b[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) b[i] = base + i < len ? data[base + i] : (uint8_t)'\n';
  }
  prev = base ? data[base - 1] : (uint32_t)'\n';
}

__global__ __launch_bounds__(kNT) void k_line_count(const uint8_t* __restrict__ data, uint64_t len,
                                                    uint64_t* __restrict__ cnt) {
  const uint64_t base = (uint64_t)blockIdx.x * kLineChunk + threadIdx.x * 16;
  uint32_t c = 0;
  if (base < len) {
    uint8_t b[16];
    uint32_t prev;
    load_slice(data, len, base, b, prev);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      c += (b[i] != '\n') & (prev == '\n');
      prev = b[i];
    }
  }
  uint64_t total;
  block_scan<kNT>(c, &total);
  if (threadIdx.x == 0) cnt[blockIdx.x] = total;
}

__global__ __launch_bounds__(kNT) void k_line_emit(const uint8_t* __restrict__ data, uint64_t len,
                                                   const uint64_t* __restrict__ bbase,
                                                   uint64_t* __restrict__ start,
                                                   uint64_t* __restrict__ end) {
  const uint64_t base = (uint64_t)blockIdx.x * kLineChunk + threadIdx.x * 16;
  uint8_t b[16];
  uint32_t prev = '\n', c = 0;
  if (base < len) {
    load_slice(data, len, base, b, prev);
    uint32_t p = prev;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      c += (b[i] != '\n') & (p == '\n');
      p = b[i];
    }
  }
  uint64_t total;
  uint64_t idx = bbase[blockIdx.x] + block_scan<kNT>(c, &total);
  if (base >= len) return;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint64_t pos = base + i;
    if (pos < len) {
      if (b[i] != '\n' && prev == '\n') start[idx++] = pos;
      else if (b[i] == '\n' && prev != '\n') end[idx - 1] = pos;  // idx >= 1 here
    }
    prev = b[i];
  }
}

__global__ __launch_bounds__(kNT) void k_line_finish(const uint8_t* __restrict__ data, uint64_t len,
                                                     uint64_t nlines,
                                                     const uint64_t* __restrict__ start,
                                                     const uint64_t* __restrict__ end,
                                                     LineRec* __restrict__ rec, uint32_t* __restrict__ llen,
                                                     uint32_t* err) {
  const uint64_t l = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  if (l >= nlines) return;
  const uint64_t s = start[l];
  const uint64_t e = end[l] == ~0ull ? len : end[l];
  const uint64_t n = e - s;
  if (n >= kNoSep) {
    atomicOr(err, 1u);
    return;
  }
  uint32_t k = kNoSep;
  for (uint32_t i = 0; i < (uint32_t)n; i += 8) {  // first TAB, 8 bytes per step
    const uint64_t w = ld8(data + s + i);
    uint32_t hit = 8;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j)
      if (hit == 8 && i + j < n && ((w >> (8 * j)) & 0xFF) == '\t') hit = j;
    if (hit < 8) {
      k = i + hit;
      break;
    }
  }
  LineRec r;
  r.start = s;
  r.pfx2 = 0;
  r.klen = k;
  r.vdl = kBadValue;
  r.pfx0 = 0;
  rec[l] = r;
  llen[l] = (uint32_t)n;
}

__global__ __launch_bounds__(kNT) void k_line_keys(const uint8_t* __restrict__ data, uint64_t nlines,
                                                   LineRec* __restrict__ rec, const uint32_t* __restrict__ llen,
                                                   uint64_t* __restrict__ pfx,
                                                   uint64_t* __restrict__ fence, uint32_t* ok) {
  const uint64_t l = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  const bool live = l < nlines;
  LineRec r = live ? rec[l] : LineRec{};
  bool good = !live || r.klen != kNoSep;
  const uint8_t* p = data + r.start;
  uint64_t v = 0;
  if (live && good) {
    v = ld8_be(p, r.klen < 8 ? r.klen : 8);
    r.pfx2 = r.klen > 8 ? ld8_be(p + 8, r.klen - 8 < 8 ? r.klen - 8 : 8) : 0;
    const int64_t d = b64_len(p + r.klen + 1, llen[l] - r.klen - 1);
    r.vdl = d < 0 ? kBadValue : (uint32_t)d;
  }
  if (live) {
    pfx[l] = v;
    fence_put(fence, nlines, l, v);
    if (good && l > 0) {
      const LineRec q = rec[l - 1];  // start/klen only: written by k_line_finish
      good = q.klen != kNoSep && bytes_cmp(data + q.start, q.klen, p, r.klen) < 0;
    }
    // pfx2, vdl and pfx0 go to their own words so the neighbour read above
    // (start / klen) stays race-free
    rec[l].pfx2 = r.pfx2;
    rec[l].vdl = r.vdl;
    rec[l].pfx0 = v;
  }
  // one atomic per block, none once the flag is down
  if (__syncthreads_or(!good) && threadIdx.x == 0 && *(volatile uint32_t*)ok) atomicAnd(ok, 0u);
}

// In-place exclusive scan of the nt tile sums a producer kernel left (one
// block: a few thousand values), *total_out = their sum. The consumer kernel
// then reads its block's base in one load; see launch_tile_scan.
__global__ __launch_bounds__(1024) void k_tile_scan(uint64_t* __restrict__ tsum, uint64_t nt,
                                                    uint64_t* __restrict__ total_out) {
  // 4 consecutive values per thread: 4096 tiles (1M keys at 256 per tile) in
  // one round of loads, one block scan and one round of stores
  constexpr uint64_t kPer = 4, kChunk = 1024 * kPer;
  uint64_t carry = 0;
  for (uint64_t c0 = 0; c0 < nt; c0 += kChunk) {
    const uint64_t i0 = c0 + threadIdx.x * kPer;
    uint64_t v[kPer], sum = 0;
#pragma unroll
    for (uint64_t j = 0; j < kPer; ++j) {
      v[j] = i0 + j < nt ? tsum[i0 + j] : 0;
      sum += v[j];
    }
    uint64_t total;
    uint64_t p = carry + block_scan<1024>(sum, &total);
#pragma unroll
    for (uint64_t j = 0; j < kPer; ++j) {
      if (i0 + j < nt) tsum[i0 + j] = p;
      p += v[j];
    }
    carry += total;
  }
  if (threadIdx.x == 0) *total_out = carry;
}

// ---- SsTable::load's rebuild from the data file (src/sstable.rs:109-120) ----

// Rust's str::from_utf8 acceptance (Unicode well-formed sequences: no
// overlongs, no surrogates, nothing above U+10FFFF).
__device__ __forceinline__ bool utf8_valid(const uint8_t* p, uint64_t n) {
  uint64_t i = 0;
  while (i < n) {
    const uint32_t c = p[i];
    if (c < 0x80) {
      ++i;
      continue;
    }
    uint32_t len, lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) len = 2;
    else if (c == 0xE0) { len = 3; lo = 0xA0; }
    else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) len = 3;
    else if (c == 0xED) { len = 3; hi = 0x9F; }
    else if (c == 0xF0) { len = 4; lo = 0x90; }
    else if (c >= 0xF1 && c <= 0xF3) len = 4;
    else if (c == 0xF4) { len = 4; hi = 0x8F; }
    else return false;
    if (n - i < len) return false;
    if (p[i + 1] < lo || p[i + 1] > hi) return false;
    for (uint32_t k = 2; k < len; ++k)
      if (p[i + k] < 0x80 || p[i + k] > 0xBF) return false;
    i += len;
  }
  return true;
}

// Per line: has[l] = 1 when the line has a TAB (its key is inserted), klen[l]
// = the key's bytes (0 otherwise); *bad = the first line whose key is not
// UTF-8 (the reference's load returns Err there).
__global__ __launch_bounds__(kNT) void k_rebuild_mark(const uint8_t* __restrict__ data,
                                                      const LineRec* __restrict__ rec, uint64_t nlines,
                                                      uint64_t* __restrict__ has, uint64_t* __restrict__ klen,
                                                      unsigned long long* __restrict__ bad) {
  const uint64_t l = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  if (l >= nlines) return;
  const LineRec r = rec[l];
  const bool tab = r.klen != kNoSep;
  has[l] = tab ? 1 : 0;
  klen[l] = tab ? r.klen : 0;
  if (tab && !utf8_valid(data + r.start, r.klen)) atomicMin(bad, (unsigned long long)l);
}

// The TAB lines' keys packed into one ragged batch in file order: key i =
// out[off[i] .. off[i+1]) is the key of line lmap[i].
__global__ __launch_bounds__(kNT) void k_rebuild_gather(const uint8_t* __restrict__ data,
                                                        const LineRec* __restrict__ rec, uint64_t nlines,
                                                        const uint64_t* __restrict__ has_scan,
                                                        const uint64_t* __restrict__ len_scan,
                                                        uint8_t* __restrict__ out, uint64_t* __restrict__ off,
                                                        uint64_t* __restrict__ lmap) {
  const uint64_t l = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  if (l >= nlines) return;
  if (l == nlines - 1) off[has_scan[nlines]] = len_scan[nlines];
  const LineRec r = rec[l];
  if (r.klen == kNoSep) return;
  const uint64_t i = has_scan[l], o = len_scan[l];
  off[i] = o;
  lmap[i] = l;
  const uint8_t* src = data + r.start;
  for (uint32_t j = 0; j < r.klen; ++j) out[o + j] = src[j];
}

// ---- exclusive scan of uint64: one rocPRIM look-back scan over n + 1 items
// (the last reads as 0, so out[n] = total) ----

// ---- search ----

// A query key with its first 16 bytes as big-endian words.
struct Query {
  const uint8_t* p;
  uint64_t len, w0, w1;
};

template <int KEYK>
__device__ __forceinline__ Query make_query(const KeySrc& ks, uint64_t k) {
  Query q;
  key_span<KEYK>(ks, k, q.p, q.len);
  if constexpr (KEYK == KEY_FIXED16) {
    const uint4 v = reinterpret_cast<const uint4*>(ks.bytes)[k];
    q.w0 = (uint64_t)__builtin_bswap32(v.x) << 32 | __builtin_bswap32(v.y);
    q.w1 = (uint64_t)__builtin_bswap32(v.z) << 32 | __builtin_bswap32(v.w);
  } else {
    q.w0 = be_chunk(q.p, q.len < 8 ? q.len : 8);
    q.w1 = q.len > 8 ? be_chunk(q.p + 8, q.len - 8 < 8 ? q.len - 8 : 8) : 0;
  }
  return q;
}

// Line key (pfx already known equal to q.w0) against the query. Keys of at
// most 16 bytes compare from the index alone: zero-padded 16-byte forms
// first, then length — the same order as Rust's str order for such keys.
__device__ __forceinline__ int rec_cmp(const TableView& t, const LineRec& r, const Query& q) {
  if (r.klen <= 16 && q.len <= 16) {
    if (r.pfx2 != q.w1) return r.pfx2 < q.w1 ? -1 : 1;
    return r.klen < q.len ? -1 : (r.klen > q.len ? 1 : 0);
  }
  return line_cmp(t.data + r.start, r.klen, q.p, q.len);
}

// Index loads as global (not flat) loads: every index array is device memory,
// and a flat load also holds the LDS counter, so the LDS-resident views and
// the search's loads would wait on each other.
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) u64x2* g64x2;
static_assert(sizeof(LineRec) == 32 && offsetof(LineRec, pfx2) == 8 && offsetof(LineRec, klen) == 16 &&
                  offsetof(LineRec, vdl) == 20 && offsetof(LineRec, pfx0) == 24,
              "grec reads LineRec as two 16-byte words");
__device__ __forceinline__ LineRec grec(const LineRec* r, uint64_t i) {
  const g64x2 p = (g64x2)(r + i);
  const u64x2 lo = p[0], hi = p[1];
  LineRec o;
  o.start = lo.x;
  o.pfx2 = lo.y;
  o.klen = (uint32_t)hi.x;
  o.vdl = (uint32_t)(hi.x >> 32);
  o.pfx0 = hi.y;
  return o;
}
__device__ __forceinline__ uint64_t g64(const uint64_t* p, uint64_t i) {
  return ((const __attribute__((address_space(1))) uint64_t*)p)[i];
}

// SsTable::binary_search (src/sstable.rs:161-179), same mid sequence.
__device__ __forceinline__ int64_t search_exact(const TableView& t, const Query& q, LineRec& hit) {
  uint64_t lo = 0, hi = t.nlines();
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    const LineRec r = grec(t.rec, mid);
    if (r.klen == kNoSep) break;
    const int c = line_cmp(t.data + r.start, r.klen, q.p, q.len);
    if (c < 0)
      lo = mid + 1;
    else if (c > 0)
      hi = mid;
    else {
      hit = r;
      return (int64_t)mid;
    }
  }
  return -1;
}

// First index in [lo, hi) with a[i] >= x, or hi (a non-decreasing).
__device__ __forceinline__ uint64_t lower_bound_u64(const uint64_t* a, uint64_t lo, uint64_t hi, uint64_t x) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (g64(a, mid) < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// Line l's key against the query, in a well-formed file: its record (which
// holds the prefix) in one load, r receives it.
__device__ __forceinline__ int line_vs_query(const TableView& t, uint64_t l, const Query& q, LineRec& r) {
  r = grec(t.rec, l);
  if (r.pfx0 != q.w0) return r.pfx0 < q.w0 ? -1 : 1;
  return rec_cmp(t, r, q);
}

// The lines from b on that share the query's prefix, by a galloping search
// with record compares (b: the prefix's lower bound, < nlines).
// Line b (the prefix's lower bound, its prefix equal to the query's) with
// its record r already loaded: the record compare, then the lines after b
// that share the prefix by a galloping search.
__device__ __forceinline__ int64_t resolve_rec(const TableView& t, const Query& q, uint64_t b, LineRec r,
                                               LineRec& hit) {
  int c = rec_cmp(t, r, q);
  if (c == 0) {
    hit = r;
    return (int64_t)b;
  }
  if (c > 0) return -1;
  // every line before lo is below the query; gallop to a line above it
  uint64_t lo = b + 1, hi = t.nlines(), step = 1;
  while (lo < t.nlines()) {
    const uint64_t p = lo + step - 1 < t.nlines() ? lo + step - 1 : t.nlines() - 1;
    c = line_vs_query(t, p, q, r);
    if (c == 0) {
      hit = r;
      return (int64_t)p;
    }
    if (c > 0) {
      hi = p;
      break;
    }
    lo = p + 1;
    step <<= 1;
  }
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    c = line_vs_query(t, mid, q, r);
    if (c == 0) {
      hit = r;
      return (int64_t)mid;
    }
    if (c < 0)
      lo = mid + 1;
    else
      hi = mid;
  }
  return -1;
}

__device__ __forceinline__ int64_t resolve_from(const TableView& t, const Query& q, uint64_t b, LineRec& hit) {
  // line b's record holds its prefix: one load (the record is needed
  // whenever the prefix matches, i.e. for every key that is present)
  const LineRec r = grec(t.rec, b);
  if (r.pfx0 != q.w0) return -1;  // pfx0 > q.w0: b is the prefix's lower bound
  return resolve_rec(t, q, b, r, hit);
}

// Level j's array (0: pfx).
__device__ __forceinline__ const uint64_t* level_array(const TableView& t, uint32_t j) {
  return j ? t.fence + level_offset(t.nlines(), j) : t.pfx;
}

// The range of level j-1 that holds the lower bound, from level j's answer i
// (E_j[i-1] < x <= E_j[i], E_j[i] = E_{j-1}[16 i]): at most 16 entries.
__device__ __forceinline__ void level_down(const TableView& t, uint32_t j, uint64_t i, uint64_t& lo, uint64_t& hi) {
  const uint64_t cnt = level_count(t.nlines(), j - 1);
  lo = i ? ((i - 1) << kFanBits) + 1 : 0;
  hi = (i << kFanBits) < cnt ? (i << kFanBits) : cnt;
}

constexpr uint32_t kWin = 8;     // buckets of up to this many lines: one round of prefix loads
constexpr uint32_t kRecWin = 2;  // ... of up to this many: the records alone (32 B each, prefix inside)

// The key buckets' answer (sstable.hpp, TableView::bkt): kBktFound (hit
// holds the line's record, the line index unknown), -1 (absent, proven by a
// complete bucket), or kBktGoOn (the directory search decides).
constexpr int64_t kBktFound = INT64_MAX;
constexpr int64_t kBktGoOn = -2;
// The bucket's first 16 bytes (its count and slot 0's prefix) for key word
// w0: what bucket_probe reads first.
__device__ __forceinline__ u64x2 bucket_head(const TableView& t, uint64_t w0) {
  return *(g64x2)(t.bkt + bkt_index(w0, t.bkbits()) * kBktWords);
}

// bucket_probe with its first load (bucket_head) already made.
__device__ __forceinline__ int64_t bucket_probe_from(const TableView& t, const Query& q, LineRec& hit, u64x2 a) {
  const uint64_t* b = t.bkt + bkt_index(q.w0, t.bkbits()) * kBktWords;
  // the count and slot 0 first (at one line per bucket on average, most keys
  // are in slot 0), the next pairs only when needed: fewer registers live
  const uint64_t cnt = a.x + 1;  // all-ones: empty
  uint32_t c = 0;
  if (cnt == 0 || a.y != q.w0) {
    if (cnt <= 1) return -1;
    const u64x2 c23 = *(g64x2)(b + 2);
    c = (c23.x == q.w0) ? 1u : (cnt > 2 && c23.y == q.w0) ? 2u : 4u;
    if (c == 4u) {
      if (cnt <= 3) return -1;
      if (g64(b, 4) != q.w0) return cnt == 4 ? -1 : kBktGoOn;
      c = 3u;
    }
  }
  const u64x2 tl = *(g64x2)(b + 6 + 2 * c);
  LineRec r;
  r.start = tl.y & ((1ull << 40) - 1);
  r.pfx2 = tl.x;
  r.klen = (uint32_t)(tl.y >> 40) & 0xFFFu;
  if (r.klen == 0xFFFu) return kBktGoOn;  // a slot left unwritten (its bucket also holds a line left out)
  r.vdl = (uint32_t)(tl.y >> 52);
  r.pfx0 = q.w0;
  const int cmp = rec_cmp(t, r, q);
  if (cmp == 0) {
    hit = r;
    return kBktFound;
  }
  return kBktGoOn;  // another line with this prefix may be the one
}

__device__ __forceinline__ int64_t bucket_probe(const TableView& t, const Query& q, LineRec& hit) {
  return bucket_probe_from(t, q, hit, bucket_head(t, q.w0));
}

// Where x's descent starts: level j and the run [lo, hi) of at most 16
// entries holding its lower bound (returns false), or true when x is absent
// outright: its bucket is empty. dm: the table's DirMap (LDS-staged by the read path).
// Lines before dir[B] have smaller buckets (so smaller prefixes) and lines
// from dir[B+1] on larger ones, so on every level the entries sampled from
// [dir[B], dir[B+1]] bracket x's lower bound.
__device__ __forceinline__ bool dir_start(const TableView& t, const DirMap* dm, uint64_t x, uint32_t& j,
                                          uint64_t& lo, uint64_t& hi) {
  j = t.nlev();
  lo = 0;
  hi = level_count(t.nlines(), j);
  if (!t.dir) return false;
  const uint64_t bk = dir_bucket(*dm, x);
  // dir[B] and dir[B + 1] as one 8-byte load (one L2 request, not two: the
  // search is bound by the requests a CU keeps in flight)
  const u32x2 ae = *(const __attribute__((address_space(1))) u32x2*)(t.dir + bk);
  const uint64_t a = ae.x, e = ae.y;
  if (a == e) return true;
  for (uint32_t l = 0; l < t.nlev(); ++l) {
    const uint64_t l0 = a >> (kFanBits * l);
    const uint64_t c = level_count(t.nlines(), l);
    uint64_t l1 = (e + (1ull << (kFanBits * l)) - 1) >> (kFanBits * l);
    l1 = l1 < c ? l1 : c;
    if (l1 - l0 <= kFanout) {
      j = l;
      lo = l0;
      hi = l1;
      return false;
    }
  }
  return false;  // the top level (at most 16 entries)
}

// Well-formed files (keys strictly increasing, so any correct search returns
// the reference's line): the lower bound of the key's 8-byte prefix down the
// fence levels (one run of at most 16 entries, one 128-B line, per level),
// then the lines sharing that prefix by a galloping search with record
// compares: O(log run) for keys that share long prefixes ('user0000...'), one
// record compare when the prefix is unique.
__device__ __forceinline__ int64_t search_fast(const TableView& t, const Query& q, LineRec& hit,
                                               const DirMap* dm) {
  if (t.bkt) {
    const int64_t b = bucket_probe(t, q, hit);
    if (b != kBktGoOn) return b;
  }
  uint32_t j;
  uint64_t lo, hi;
  // an empty bucket: absent
  if (dir_start(t, dm, q.w0, j, lo, hi)) return -1;
  if (j == 0 && hi - lo <= kRecWin) {
    // a bucket of at most kRecWin lines: its records hold the prefixes, so
    // the records are all that is read (one round of independent loads: one
    // or two 128-B lines where the prefixes and then the matching record
    // took two); the matching one is already in registers
    LineRec rr[kRecWin];
#pragma unroll
    for (uint32_t k = 0; k < kRecWin; ++k)
      if (lo + k < hi) rr[k] = grec(t.rec, lo + k);
    uint32_t c = 0;
#pragma unroll
    for (uint32_t k = 0; k < kRecWin; ++k) c += (lo + k < hi && rr[k].pfx0 < q.w0) ? 1u : 0u;
    if (lo + c == hi) return -1;  // every line below the key: the next one is in a larger bucket
    LineRec r = rr[0];
#pragma unroll
    for (uint32_t k = 1; k < kRecWin; ++k)
      if (k == c) r = rr[k];
    if (r.pfx0 != q.w0) return -1;
    return resolve_rec(t, q, lo + c, r, hit);
  }
  if (j == 0 && hi - lo <= kWin) {
    // a larger bucket (or the whole table): its prefixes from the dense
    // prefix array in one round of independent loads (64 B for 8 lines),
    // then the matching record
    uint64_t v[kWin];
    // in pairs: two neighbouring prefixes as one 16-byte load where both
    // are in the bucket (one L2 request per pair, not per prefix)

#pragma unroll
    for (uint32_t k = 0; k < kWin; k += 2) {
      if (lo + k + 1 < hi) {
        const u64x2 pr = *(g64x2)(t.pfx + lo + k);
        v[k] = pr.x;
        v[k + 1] = pr.y;
      } else {
        v[k] = lo + k < hi ? g64(t.pfx, lo + k) : ~0ull;
        v[k + 1] = ~0ull;
      }
    }
    uint32_t c = 0;
#pragma unroll
    for (uint32_t k = 0; k < kWin; ++k) c += (lo + k < hi && v[k] < q.w0) ? 1u : 0u;
    // every line below the key: the next one is in a larger bucket
    if (lo + c == hi) return -1;
    uint64_t p0 = v[0];
#pragma unroll
    for (uint32_t k = 1; k < kWin; ++k) p0 = k == c ? v[k] : p0;
    if (p0 != q.w0) return -1;
    return resolve_rec(t, q, lo + c, grec(t.rec, lo + c), hit);
  }
  for (;; --j) {
    const uint64_t i = lower_bound_u64(level_array(t, j), lo, hi, q.w0);
    if (!j) {
      if (i >= t.nlines()) return -1;
      return resolve_from(t, q, i, hit);
    }
    level_down(t, j, i, lo, hi);
  }
}

// dm: the table's DirMap (LDS or global); used only when t.dir is set.
__device__ __forceinline__ int64_t search(const TableView& t, const Query& q, LineRec& hit, const DirMap* dm) {
  return t.fast() ? search_fast(t, q, hit, dm) : search_exact(t, q, hit);
}

// dir from the sorted prefixes, one lane per line (dir_fill). Block 0 also
// stores the map (the table's device copy).
__global__ __launch_bounds__(kNT) void k_table_dir(const uint64_t* __restrict__ pfx, uint64_t nl, DirMap dm,
                                                   uint32_t* __restrict__ dir, DirMap* dmap_out) {
  __shared__ DirMap sdm;
  if (threadIdx.x == 0) {
    sdm = dm;
    if (blockIdx.x == 0) *dmap_out = dm;
  }
  __syncthreads();
  const uint64_t p = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  const bool live = p < nl;
  const uint64_t w = live ? pfx[p] : 0;
  const uint64_t b = live ? dir_bucket(sdm, w) : 0;
  uint64_t bp = __shfl_up(b, 1, 64);
  if (live && (threadIdx.x & 63u) == 0 && p > 0) bp = dir_bucket(sdm, pfx[p - 1]);
  dir_fill(dir, sdm.nbuckets, nl, p, live, b, bp);
}

__global__ __launch_bounds__(kNT) void k_pfx_masks(const uint64_t* __restrict__ pfx, uint64_t nl,
                                                   uint64_t* __restrict__ mask) {
  sample_pfx_masks(nl, [&](uint64_t q) { return pfx[q]; }, mask);
}

// The key buckets (sstable.hpp) of a fast table, one lane per line: the
// bucket's count word hands out slots (1 per stored line, 16 per line left
// out, so a bucket holding one is never taken as complete).
__global__ __launch_bounds__(kNT) void k_table_buckets(const LineRec* __restrict__ rec, uint64_t nl,
                                                       uint64_t* __restrict__ bkt, uint32_t bits) {
  const uint64_t l = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  if (l >= nl) return;
  const LineRec r = grec(rec, l);
  const bool keep = r.klen < 4095u && r.vdl <= 4095u && r.start < (1ull << 40);  // klen 0xFFF: unwritten slot
  uint64_t* b = bkt + bkt_index(r.pfx0, bits) * kBktWords;
  const uint64_t s = atomicAdd(reinterpret_cast<unsigned long long*>(b), keep ? 1ull : 16ull) + 1;
  if (keep && s < kBktSlots) {
    b[1 + s] = r.pfx0;
    b[6 + 2 * s] = r.pfx2;
    b[7 + 2 * s] = r.start | ((uint64_t)r.klen << 40) | ((uint64_t)r.vdl << 52);
  }
}

// The buckets' summary words (sstable.hpp bkt_fp), one lane per bucket,
// after k_table_buckets.
__global__ __launch_bounds__(kNT) void k_table_bucket_fp(uint64_t* __restrict__ bkt, uint32_t bits) {
  const uint64_t nbk = 1ull << bits;
  const uint64_t i = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  if (i >= nbk) return;
  const uint64_t* b = bkt + i * kBktWords;
  const uint64_t cnt = b[0] + 1;  // all-ones: empty
  uint64_t f = cnt <= kBktSlots ? cnt : 15u;
  if (f != 15u)
    for (uint32_t s = 0; s < (uint32_t)cnt; ++s) f |= (uint64_t)bkt_fp(b[1 + s]) << (4 + 15 * s);
  bkt[nbk * kBktWords + i] = f;
}

// A block's views of the first min(nt, 64) tables into LDS. Barrier inside.
// The first min(nt, 64) tables' views, staged once per block into LDS: loaded
// into registers first (issued with the key and gate loads, so their round
// trip overlaps those), then stored after the gate. Barrier in store_views.
constexpr uint32_t kViewDw = sizeof(TableView) / 4;
constexpr uint32_t kViewPer = (64 * kViewDw + kNT - 1) / kNT;
static_assert(sizeof(TableView) % 4 == 0, "dword copy");
struct ViewRegs {
  uint32_t w[kViewPer];
};
__device__ __forceinline__ ViewRegs load_views(const TableView* tv, uint32_t nt) {
  ViewRegs v;
  const uint32_t nd = (nt < 64 ? nt : 64) * kViewDw;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(tv);
#pragma unroll
  for (uint32_t i = 0; i < kViewPer; ++i) {
    const uint32_t d = threadIdx.x + i * kNT;
    v.w[i] = d < nd ? src[d] : 0u;
  }
  return v;
}
__device__ __forceinline__ void store_views(const ViewRegs& v, uint32_t nt, TableView* stv) {
  const uint32_t nd = (nt < 64 ? nt : 64) * kViewDw;
  uint32_t* dst = reinterpret_cast<uint32_t*>(stv);
#pragma unroll
  for (uint32_t i = 0; i < kViewPer; ++i) {
    const uint32_t d = threadIdx.x + i * kNT;
    if (d < nd) dst[d] = v.w[i];
  }
  __syncthreads();
}

// The first min(nt, 64) tables' DirMaps (their views already in LDS) into
// LDS, 16 B per thread and step; barrier at the end. The search computes
// its bucket from these words (sstable.hpp dir_bucket) without a memory
// round trip.
constexpr uint32_t kMapWords = sizeof(DirMap) / 16;
__device__ __forceinline__ void stage_maps(const TableView* stv, uint32_t nt, DirMap* sdm) {
  const uint32_t nm = (nt < 64 ? nt : 64) * kMapWords;
  for (uint32_t i = threadIdx.x; i < nm; i += kNT) {
    const uint32_t t = i / kMapWords, k = i - t * kMapWords;
    const DirMap* g = stv[t].dmap;
    if (g) reinterpret_cast<uint4*>(sdm + t)[k] = reinterpret_cast<const uint4*>(g)[k];
  }
  __syncthreads();
}

template <int KEYK>
__global__ __launch_bounds__(kNT) void k_table_search(TableView t, KeySrc ks, uint64_t n,
                                                      int64_t* __restrict__ line) {
  const uint64_t k = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  if (k >= n) return;
  const Query q = make_query<KEYK>(ks, k);
  LineRec r;
  line[k] = search(t, q, r, t.dmap);
}

// One group of up to 64 tables (t0 .. t0 + 63): every candidate in cand,
// newest first, until a table answers Ok(Some). Returns whether one did.
// LDS_VIEWS (every table among the first 64): the search reads its table's
// view fields from LDS where it uses them instead of copying the 56-byte view
// into registers (88 -> 80 VGPRs: 6 waves per SIMD instead of 5).
template <bool LDS_VIEWS = false>
__device__ __forceinline__ bool resolve_group(const TableView* stv, const TableView* __restrict__ tv,
                                              const DirMap* sdm, uint32_t t0, uint64_t cand, const Query& q,
                                              int32_t& w, uint64_t& src, uint64_t& d) {
  while (cand) {
    const uint32_t t = t0 + (uint32_t)__builtin_ctzll(cand);
    cand &= cand - 1;
    auto try_table = [&](const TableView& v) {
      LineRec r;
      if (search(v, q, r, t < 64 ? &sdm[t] : v.dmap) < 0) return false;  // Ok(None)
      if (r.vdl == kBadValue) return false;   // Err(..) is skipped by `if let Ok(Some(v))`
      w = (int32_t)t;
      src = (uint64_t)(uintptr_t)(v.data + r.start + r.klen + 1);
      d = r.vdl;
      return true;
    };
    if constexpr (LDS_VIEWS) {
      if (try_table(stv[t])) return true;
    } else {
      const TableView v = t < 64 ? stv[t] : tv[t];
      if (try_table(v)) return true;
    }
  }
  return false;
}

// Database::get's walk for one key (src/lib.rs:129-134): tables in groups
// of 64, newest first (tables.iter().rev()). Each lane holds its candidate
// tables of the group as a bit mask (cand0 for the first 64; past them, from
// the hit rows), then every lane searches its OWN next candidate in the same
// iteration, so lanes whose keys live in different tables search concurrently
// instead of the wave stepping through the tables one by one. w / src / d:
// the first table whose SsTable::get returns Ok(Some), the value's base64
// bytes and their decoded length.
template <bool LDS_VIEWS>
__device__ __forceinline__ void resolve_key(const TableView* stv, const TableView* __restrict__ tv,
                                            const DirMap* sdm, uint32_t nt, uint64_t cand0,
                                            const uint64_t* __restrict__ hits,
                                            const uint32_t* __restrict__ rows, uint64_t hwords, uint64_t k,
                                            const Query& q, int32_t& w, uint64_t& src, uint64_t& d) {
  for (uint32_t t0 = 0; t0 < nt; t0 += 64) {
    const uint32_t gn = nt - t0 < 64 ? nt - t0 : 64;
    uint64_t cand = gn == 64 ? ~0ull : ((1ull << gn) - 1);
    if (t0 == 0) {
      cand = cand0;
    } else if (hits) {  // tables past the first 64: one broadcast load per table
      cand = 0;
      for (uint32_t i = 0; i < gn; ++i) {
        const uint64_t row = rows ? rows[t0 + i] : t0 + i;
        cand |= ((hits[row * hwords + (k >> 6)] >> (k & 63)) & 1) << i;  // the gate
      }
    }
    if (resolve_group<LDS_VIEWS>(stv, tv, sdm, t0, cand, q, w, src, d)) return;
  }
}

// LDS_VIEWS: nt <= 64 (every view staged in LDS; see resolve_group).
template <int KEYK, bool LDS_VIEWS>
__global__ __launch_bounds__(kNT, 6) void k_get_many(const TableView* __restrict__ tv, uint32_t nt,
                                                  const uint64_t* __restrict__ hits,
                                                  const uint32_t* __restrict__ rows,
                                                  uint64_t hwords, KeySrc ks, uint64_t n,
                                                  int32_t* __restrict__ which,
                                                  uint64_t* __restrict__ vsrc,
                                                  uint64_t* __restrict__ dlen,
                                                  uint64_t* __restrict__ tsum) {
  const uint64_t k = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  // The gate for the first 64 tables, with every lane of the wave active: a
  // wave's 64 keys share one hit word per table row, so lane i loads row i's
  // word (one load instruction for the wave, not one per table) and every
  // lane takes its bit of each row from lane i by a uniform shuffle.
  const ViewRegs vr = load_views(tv, nt);
  const uint32_t gn0 = nt < 64 ? nt : 64;
  uint64_t cand0 = gn0 == 64 ? ~0ull : ((1ull << gn0) - 1);
  // the key's loads go out with the gate's (independent of it)
  const Query q = make_query<KEYK>(ks, k < n ? k : 0);
  if (hits) {
    const uint64_t wi = ((uint64_t)blockIdx.x * kNT + (threadIdx.x & ~63u)) >> 6;
    uint64_t hw = 0;
    if (lane < gn0 && wi < hwords) hw = hits[(uint64_t)(rows ? rows[lane] : lane) * hwords + wi];
    cand0 = 0;
    for (uint32_t i = 0; i < gn0; ++i) cand0 |= ((__shfl(hw, (int)i, 64) >> lane) & 1ull) << i;
  }
  // the first 64 tables' views, staged once per block: each lane's search
  // reads its table's view from LDS instead of a divergent global gather
  __shared__ TableView stv[64];
  __shared__ DirMap sdm[64];
  store_views(vr, nt, stv);
  stage_maps(stv, nt, sdm);
  uint64_t d = 0;
  if (k < n) {
    int32_t w = -1;
    uint64_t src = 0;
    if constexpr (LDS_VIEWS)
      (void)resolve_group<true>(stv, tv, sdm, 0, cand0, q, w, src, d);  // one group
    else
      resolve_key<false>(stv, tv, sdm, nt, cand0, hits, rows, hwords, k, q, w, src, d);
    which[k] = w;
    vsrc[k] = src;
    dlen[k] = d;
  }
  // this block's value bytes, for k_b64_decode's offsets
  uint64_t total;
  (void)block_scan<kNT>(d, &total);
  if (threadIdx.x == 0) tsum[blockIdx.x] = total;
}

// Database::get in one launch (src/lib.rs:129-134 with SsTable::get's gate,
// src/sstable.rs:138): k_get_many with the gate computed per key from the
// FilterSet (set_key_mask: set[a] & set[b] over every slot, the zone check
// for gated slots) instead of read from hit rows, so no rows are written or
// read and the set's random reads overlap the searches' in one kernel. Table
// t is slot slots[t] (slots NULL: slot t); nt <= W.
template <int KEYK, int MODE, int W>
__global__ __launch_bounds__(kNT, 6) void k_set_get_many(const void* __restrict__ set, ModP mp, ZoneView zv,
                                                      const TableView* __restrict__ tv, uint32_t nt,
                                                      const uint32_t* __restrict__ slots, KeySrc ks, uint64_t n,
                                                      int32_t* __restrict__ which, uint64_t* __restrict__ vsrc,
                                                      uint64_t* __restrict__ dlen, uint64_t* __restrict__ tsum) {
  const uint64_t k = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  const ViewRegs vr = load_views(tv, nt);
  __shared__ BoundPrefix zp[2 * W];
  __shared__ uint32_t sslot[64];
  __shared__ TableView stv[64];
  __shared__ DirMap sdm[64];
  stage_zone_prefixes<KEYK, W>(zv, zp, kNT);
  if (slots && threadIdx.x < nt) sslot[threadIdx.x] = slots[threadIdx.x];
  // the key's loads go out before the barrier (after it, the compiler kept
  // the whole search's state live across the gate: 256 VGPRs, 1 wave/SIMD)
  const Query q = make_query<KEYK>(ks, k < n ? k : 0);
  store_views(vr, nt, stv);  // barrier: views, slots and zone prefixes staged
  const auto mask = set_key_mask<KEYK, MODE, W, true, false>(set, nullptr, ks, k, k < n, mp, zv, zp);
  uint64_t cand0 = 0;
  if (slots) {
    for (uint32_t i = 0; i < nt; ++i) cand0 |= (((uint64_t)mask >> sslot[i]) & 1ull) << i;
  } else {
    cand0 = (uint64_t)mask & (nt == 64 ? ~0ull : ((1ull << nt) - 1));
  }
  stage_maps(stv, nt, sdm);
  uint64_t d = 0;
  if (k < n) {
    int32_t w = -1;
    uint64_t src = 0;
    (void)resolve_group<true>(stv, tv, sdm, 0, cand0, q, w, src, d);  // nt <= 64: one group
    which[k] = w;
    vsrc[k] = src;
    dlen[k] = d;
  }
  uint64_t total;
  (void)block_scan<kNT>(d, &total);
  if (threadIdx.x == 0) tsum[blockIdx.x] = total;
}

// The wide walk's screen (wideset.hpp WideScreen): bit (B, h, slot) is clear
// only when the table in that slot has a complete key bucket B none of whose
// stored fingerprints falls in bin h (fp & (H - 1)). One thread per (table,
// bucket); bits are ORed in (tables share screen words). Tables whose
// buckets the screen cannot speak for (none yet, not well-formed, another
// bucket count) set every bin: they always pass.
__global__ __launch_bounds__(kNT) void k_wide_screen(const TableView* __restrict__ tv, const uint32_t* __restrict__ slots,
                                                     uint32_t nt, uint32_t R, uint32_t bits, uint32_t hbits,
                                                     uint64_t* __restrict__ scr) {
  const uint64_t nb = 1ull << bits, H = 1ull << hbits;
  const uint64_t idx = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  if (idx >= nb * nt) return;
  const uint32_t i = (uint32_t)(idx >> bits);
  const uint64_t B = idx & (nb - 1);
  const uint32_t slot = slots ? slots[i] : i;
  const TableView v = tv[i];
  unsigned long long* row = reinterpret_cast<unsigned long long*>(scr) + B * H * R + (slot >> 6);
  const unsigned long long bit = 1ull << (slot & 63u);
  if (v.bkt && v.fast() && v.bkbits() == bits) {
    const uint64_t sw = v.bkt[nb * kBktWords + B];
    const uint32_t nst = (uint32_t)(sw & 15u);
    if (nst <= kBktSlots) {  // the bins of the stored fingerprints
      for (uint32_t s = 0; s < nst; ++s) atomicOr(row + ((sw >> (4 + 15 * s)) & (H - 1)) * R, bit);
      return;
    }
  }
  for (uint64_t h = 0; h < H; ++h) atomicOr(row + h * R, bit);  // no proof: every bin
}

// Database::get in one launch over a wide set (wideset.hpp): k_set_get_many
// for more than 64 tables. Per key: rows a and b of the set (h1 % m, h2 % m,
// src/bloom.rs:26-37); then the tables in groups of 64, newest first
// (tables.iter().rev(), src/lib.rs:130): the group's candidate bits are a
// 64-bit window of row a AND the same window of row b, the latter read only
// when the former is non-zero (src/bloom.rs:50), reordered to table order
// (groups[g].kind); then the candidates newest first: each one's bucket
// summary word, the zone gate for gated tables (src/sstable.rs:138), the
// search, and the first Ok(Some) ends the walk. The group's views and maps
// are staged in LDS.
// The wide walk's summary words loaded together: 4 / 8 / 16 at once measured
// 671-679 / 792-809 / 816-820 M gets/s against 517-519 one at a time (300
// tables of m = 1024); 16 doubles the scratch spill (36 -> 72 B per lane).
// With the screen (round 5) the batch no longer matters: 8 / 4 / 2 at once
// measured 2.145 / 2.140 / 2.139 G gets/s, the same VGPRs (experiment builds).
#if defined(CB_EXPERIMENTS) && defined(CB_WIDE_SCREEN_BATCH)
constexpr uint32_t kScreen = CB_WIDE_SCREEN_BATCH;
#else
constexpr uint32_t kScreen = 8;
#endif
// (Round 4, before the screen: five waves per SIMD at its natural 96 VGPRs;
// forcing six, 80 VGPRs with 112 B of scratch per lane, measured 606-617
// against 782-804 M gets/s.)
// Four waves per SIMD, 109 VGPRs and no spill (round 5, with the screen):
// 1.81-1.84 against 1.63 G gets/s for five waves at 96 VGPRs and 56 B of
// spill per lane (experiment r05_wide4, HISTORY.md, alternating on one box).
// The walk's workgroup: kWideNT keys (two 256-key tiles of the value scan);
// a group's views and maps are staged once per workgroup, so 512 keys per
// workgroup halve the staging's L2 requests per lookup against 256.
#if defined(CB_EXPERIMENTS) && defined(CB_WIDE_THREADS)
constexpr uint32_t kWideNT = CB_WIDE_THREADS;
#else
constexpr uint32_t kWideNT = 512;
#endif
static_assert(kWideNT % kNT == 0 && kWideNT / kNT <= 4, "up to four value tiles per workgroup");
template <int KEYK, int MODE>
__global__ __launch_bounds__(kWideNT, 4) void k_wide_get_many(const uint64_t* __restrict__ set, uint32_t R, ModP mp,
                                                       WideZone z, const TableView* __restrict__ tv, uint32_t nt,
                                                       const WideGroup* __restrict__ groups,
                                                       const uint32_t* __restrict__ slots, KeySrc ks, uint64_t n,
                                                       int32_t* __restrict__ which, uint64_t* __restrict__ vsrc,
                                                       uint64_t* __restrict__ dlen, uint64_t* __restrict__ tsum,
                                                       WideScreen ws, const DirMap* __restrict__ maps) {
  const uint64_t k = (uint64_t)blockIdx.x * kWideNT + threadIdx.x;
  const bool live = k < n;
  const Query q = make_query<KEYK>(ks, live ? k : 0);
  uint64_t pa = 0, pb = 0;
  if (live) key_positions<KEYK, MODE>(ks, k, mp, pa, pb);
  const uint64_t* ra = set + pa * R;
  const uint64_t* rb = set + pb * R;
  // the screen row of this key's bucket and fingerprint bin: one R-word row
  // says, for every slot at once, whether the summary word could pass
  const uint64_t* rs = ws.scr ? ws.scr + ((bkt_index(q.w0, ws.bits) << ws.hbits) +
                                          (bkt_fp(q.w0) & ((1u << ws.hbits) - 1u))) * R
                              : nullptr;
  const uint32_t kw[4] = {(uint32_t)(q.w0 >> 32), (uint32_t)q.w0, (uint32_t)(q.w1 >> 32), (uint32_t)q.w1};
  // The block walks the groups together: each group's 64 views and DirMaps
  // are staged in LDS once for the block (every search then reads its
  // table's view and map from LDS, not 56 + 320 B from global memory per
  // search), and the walk ends when no lane of the block is still looking.
  // The maps come from the table list's contiguous copy (maps, round 6) in
  // the same pass as the views, one barrier per group; without it each map
  // is found through its view (a second pass after the views' barrier).
  __shared__ TableView stv[64];
  __shared__ DirMap sdm[64];
  __shared__ WideGroup sg[kWideMax / 64];
  const uint32_t ng = (nt + 63) / 64;
  for (uint32_t i = threadIdx.x; i < ng; i += kWideNT) sg[i] = groups[i];
  __syncthreads();
  int32_t w = -1;
  uint64_t src = 0, d = 0;
  bool active = live;
  for (uint32_t g = 0; g < ng; ++g) {
    if (!__syncthreads_or(active)) break;  // (also: the previous group's stage is consumed)
    const uint32_t t0 = 64 * g, gn = nt - t0 < 64 ? nt - t0 : 64;
    if (maps) {
      const uint32_t* vs = reinterpret_cast<const uint32_t*>(tv + t0);
      uint32_t* vd = reinterpret_cast<uint32_t*>(stv);
      for (uint32_t i = threadIdx.x; i < gn * kViewDw; i += kWideNT) vd[i] = vs[i];
      const uint4* ms = reinterpret_cast<const uint4*>(maps + t0);
      uint4* md = reinterpret_cast<uint4*>(sdm);
      for (uint32_t i = threadIdx.x; i < gn * kMapWords; i += kWideNT) md[i] = ms[i];
      __syncthreads();
    } else {
      const uint32_t* vs = reinterpret_cast<const uint32_t*>(tv + t0);
      uint32_t* vd = reinterpret_cast<uint32_t*>(stv);
      for (uint32_t i = threadIdx.x; i < gn * kViewDw; i += kWideNT) vd[i] = vs[i];
      __syncthreads();
      for (uint32_t i = threadIdx.x; i < gn * kMapWords; i += kWideNT) {
        const uint32_t t = i / kMapWords, j = i - t * kMapWords;
        const DirMap* gm = stv[t].dmap;
        if (gm) reinterpret_cast<uint4*>(sdm + t)[j] = reinterpret_cast<const uint4*>(gm)[j];
      }
      __syncthreads();
    }
    if (!active) continue;
    const WideGroup gd = sg[g];
    const uint64_t gmask = gd.gn >= 64 ? ~0ull : ((1ull << gd.gn) - 1);
    // The group's row windows one after another, each only when it can
    // matter: row b where row a's window has bits (src/bloom.rs:50's &&),
    // the screen where both do. Loading the three together, with the next
    // group's in flight during this group's walk, measured slower (round 6:
    // 93.9-94.2 against 92.1-92.3 us one lane, 3.07 against 3.29 G gets/s
    // on three lanes) and cost ~2 more L2 requests per lookup: a lane found
    // in this group had already loaded the next group's three windows.
    uint64_t ca = 0, cb = 0, cs = ~0ull;
    if (gd.kind != 2) {
      ca = wide_window(ra, R, gd.lo) & gmask;
      cb = ca ? wide_window(rb, R, gd.lo) : 0ull;
      cs = (ca & cb) && rs ? wide_window(rs, R, gd.lo) : ~0ull;
    }
    uint64_t cand = 0;
    if (gd.kind == 2) {  // scattered slots: one bit per table
      for (uint32_t i = 0; i < gd.gn; ++i) {
        const uint32_t s = slots[t0 + i];
        if ((ra[s >> 6] >> (s & 63)) & 1ull) cand |= ((rb[s >> 6] >> (s & 63)) & 1ull) << i;
      }
    } else {
      const uint64_t a = ca & gmask;
      cand = a ? (a & cb) : 0ull;  // src/bloom.rs:50's &&
      cand &= cs;                  // the screen (slot order, like the rows; all ones without one)
      if (gd.kind == 1 && cand) cand = __builtin_bitreverse64(cand) >> (64 - gd.gn);  // bit gn-1-i -> i
    }
    if (gd.kind == 2 && cand && rs) {
      uint64_t sc = 0;
      for (uint32_t i = 0; i < gd.gn; ++i) {
        const uint32_t s = slots[t0 + i];
        sc |= ((rs[s >> 6] >> (s & 63)) & 1ull) << i;
      }
      cand &= sc;
    }
    // the candidates newest first, the group's views and maps from LDS. At
    // the product's m = 1024 most candidates are false positives (~3/4 of
    // the tables pass the Bloom gate); each is settled by its key bucket's
    // 8-byte summary word (sstable.hpp bkt_fp), which stays in the L2s,
    // before any bucket line is read (a complete bucket without the key's
    // fingerprint: Ok(None)). Loading the words of 2 or 4 candidates at once
    // measured the same (profiles/wide_summary_r04.json).
    // The zone gate (src/sstable.rs:138) is checked after the summary word:
    // both only answer Ok(None), so their order leaves the walk's result as
    // it is, and the summary word settles nearly every candidate first.
    const uint32_t kfp = bkt_fp(q.w0);
    while (cand) {
      // screen the next kScreen candidates by their summary words, the
      // loads in flight together (one L2 round trip per kScreen candidates,
      // not per candidate); ~0: no summary word, no proof
      uint64_t taken = 0, keep = 0;
      {
        uint32_t ii[kScreen];
        uint64_t sw[kScreen];
        uint64_t c = cand;
#pragma unroll
        for (uint32_t j = 0; j < kScreen; ++j) {
          ii[j] = c ? (uint32_t)__builtin_ctzll(c) : 64u;
          c &= c - 1;
        }
#pragma unroll
        for (uint32_t j = 0; j < kScreen; ++j) {
          sw[j] = ~0ull;
          if (ii[j] < 64u) {
            const TableView& v = stv[ii[j]];
            if (v.bkt && v.fast()) {
              const uint32_t bits = v.bkbits();
              sw[j] = g64(v.bkt, (1ull << bits) * kBktWords + bkt_index(q.w0, bits));
            }
          }
        }
#pragma unroll
        for (uint32_t j = 0; j < kScreen; ++j) {
          if (ii[j] >= 64u) continue;
          taken |= 1ull << ii[j];
          const uint32_t nst = (uint32_t)(sw[j] & 15u);
          bool pass = nst > kBktSlots;  // not complete: the search decides
#pragma unroll
          for (uint32_t s = 0; s < kBktSlots; ++s)
            pass |= s < nst && (uint32_t)((sw[j] >> (4 + 15 * s)) & 0x7FFFu) == kfp;
          if (pass) keep |= 1ull << ii[j];  // else Ok(None)
        }
      }
      cand &= ~taken;
      bool found = false;
      while (keep) {  // the survivors, newest first
        const uint32_t i = (uint32_t)__builtin_ctzll(keep);
        keep &= keep - 1;
        if (z.any) {
          const uint32_t s = gd.kind == 2 ? slots[t0 + i] : gd.kind == 1 ? gd.lo + gd.gn - 1 - i : gd.lo + i;
          if (!wide_zone_ok<KEYK>(z, s, kw, q.p, q.len)) continue;  // Ok(None)
        }
        const TableView& v = stv[i];
        LineRec r;
        if (search(v, q, r, &sdm[i]) < 0) continue;  // Ok(None)
        if (r.vdl == kBadValue) continue;             // Err(..) is skipped by `if let Ok(Some(v))`
        w = (int32_t)(t0 + i);
        src = (uint64_t)(uintptr_t)(v.data + r.start + r.klen + 1);
        d = r.vdl;
        found = true;
        break;
      }
      if (found) {
        active = false;
        break;
      }
    }
  }
  if (live) {
    which[k] = w;
    vsrc[k] = src;
    dlen[k] = d;
  }
  // one value-byte sum per 256-key tile (get_tiles): the workgroup's tiles
  // from the prefixes at their bounds
  uint64_t total;
  const uint64_t pre = block_scan<kWideNT>(d, &total);
  if constexpr (kWideNT == kNT) {
    if (threadIdx.x == 0) tsum[blockIdx.x] = total;
  } else {
    constexpr uint32_t T = kWideNT / kNT;
    __shared__ uint64_t bnd[T + 1];
    if (threadIdx.x % kNT == 0) bnd[threadIdx.x / kNT] = pre;
    if (threadIdx.x == 0) bnd[T] = total;
    __syncthreads();
    const uint64_t t0 = (uint64_t)T * blockIdx.x;
    if (threadIdx.x < T && (t0 + threadIdx.x) * kNT < n) tsum[t0 + threadIdx.x] = bnd[threadIdx.x + 1] - bnd[threadIdx.x];
  }
}

// ---- base64 decode of the found values ----

// Decode 4 base64 chars (canonical, validated at index time) to 3 bytes.
__device__ __forceinline__ uint32_t b64_quad(const uint8_t c[4]) {
  return (uint32_t)(b64v(c[0]) & 63) << 18 | (uint32_t)(b64v(c[1]) & 63) << 12 |
         (uint32_t)(b64v(c[2]) & 63) << 6 | (uint32_t)(b64v(c[3]) & 63);
}

// dl bytes decoded from src (4*ceil(dl/3) canonical chars), written through
// put(j, byte).
template <class Put>
__device__ __forceinline__ void b64_decode_into(const uint8_t* src, uint64_t dl, Put put) {
  const uint64_t len = (dl + 2) / 3 * 4;
  uint64_t j = 0;
  for (uint64_t q = 0; q < len; q += 8) {  // two quads per step
    const uint64_t x = ld8(src + q);
    uint8_t c[8];
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) c[i] = (uint8_t)(x >> (8 * i));
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
      const uint32_t w = b64_quad(c + 4 * h);
      if (j < dl) put(j++, (uint8_t)(w >> 16));
      if (j < dl) put(j++, (uint8_t)(w >> 8));
      if (j < dl) put(j++, (uint8_t)w);
    }
  }
}

// Values of up to 18 bytes (24 chars): the dwords their chars span, loaded
// unconditionally (indices clamped to the last one, so every load stays inside
// the span) so the caller can issue them before other work.
struct SmallB64 {
  uint32_t x[7];
  uint32_t sh;
};
constexpr uint64_t kSmallB64Bytes = 18;

__device__ __forceinline__ void b64_small_load(const uint8_t* src, uint64_t dl, SmallB64& v) {
  const uint64_t len = (dl + 2) / 3 * 4;
  const uintptr_t a = (uintptr_t)src;
  v.sh = (uint32_t)(a & 3);
#ifndef CB_B64_DWORD_LOADS
  // three 16-B loads of the aligned 48 B holding the chars (each clamped to
  // the last 16 B the chars reach, so no load leaves their span), then the 7
  // dwords from dword (a & 15) / 4 on: 3 load instructions per value instead
  // of 7 (the loads' random lines are the kernel's cost)
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) u32x4* gq;
  const gq q = (gq)(a & ~(uintptr_t)15);
  const uint32_t lastq = ((uint32_t)(a & 15) + (uint32_t)len - 1) >> 4;
  const u32x4 q0 = q[0], q1 = q[lastq < 1 ? lastq : 1], q2 = q[lastq < 2 ? lastq : 2];
  const uint32_t d[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
  const uint32_t o = (uint32_t)(a & 12) >> 2;
#pragma unroll
  for (uint32_t i = 0; i < 7; ++i)
    v.x[i] = o == 0 ? d[i] : o == 1 ? d[i + 1] : o == 2 ? d[i + 2] : d[i + 3];
#else
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t last = (v.sh + (uint32_t)len + 3) / 4 - 1;
#pragma unroll
  for (uint32_t i = 0; i < 7; ++i) v.x[i] = w[i < last ? i : last];
#endif
}

// dl <= 18 bytes decoded from the loaded dwords (realigned: y = one quad).
template <class Put>
__device__ __forceinline__ void b64_small_decode(const SmallB64& v, uint64_t dl, Put put) {
  uint64_t j = 0;
#pragma unroll
  for (uint32_t i = 0; i < 6; ++i) {
    const uint32_t y = __builtin_amdgcn_alignbyte(v.x[i + 1], v.x[i], v.sh);
    const uint8_t c[4] = {(uint8_t)y, (uint8_t)(y >> 8), (uint8_t)(y >> 16), (uint8_t)(y >> 24)};
    const uint32_t q = b64_quad(c);
    if (j < dl) put(j++, (uint8_t)(q >> 16));
    if (j < dl) put(j++, (uint8_t)(q >> 8));
    if (j < dl) put(j++, (uint8_t)q);
  }
}

constexpr uint32_t kDecodeLds = 16384;  // staged output bytes per block

// Value offsets: the block's base is the scanned value-byte tile sum (tsum:
// k_get_many, then k_tile_scan, which also wrote voff[n] = the total), plus
// the scan of its own lengths; voff[k] is written here. out ==
// nullptr, or a total above cap: offsets only. Otherwise the block's values
// are one contiguous output range; when it fits in LDS, lanes decode into LDS
// and the block writes the range with aligned dword stores, else lanes write
// their bytes directly.
#ifdef CB_EXPERIMENTS
__constant__ int g_b64_x;
#endif
// (Two adjacent keys per thread, so all of a 1M-key batch's value loads are
// in flight in one round, measured slower: read path 14.3 against 14.8-14.9 G
// gets/s, wide fan-out 1.97-2.00 against 2.04-2.06; experiment r05_b64kpt, HISTORY.md.)
// RAW (grids of at most kRawTiles blocks): tsum holds the producer's
// unscanned tile sums, and every block sums the ones before it (and all of
// them, for the total; block 0 stores it as voff[n]) from one round of loads
// issued with its other loads, in place of a k_tile_scan launch between the
// two kernels.
constexpr uint32_t kRawPer = 4, kRawTiles = kNT * kRawPer;
static_assert(kNT == kDecodeTile && (uint64_t)kRawTiles * kNT == 262144, "decode_raw_max()");
template <bool RAW>
__global__ __launch_bounds__(kNT) void k_b64_decode(const uint64_t* __restrict__ vsrc,
                                                    const uint64_t* __restrict__ dlen,
                                                    const uint64_t* __restrict__ tsum, uint64_t n,
                                                    uint64_t* __restrict__ voff,
                                                    uint8_t* __restrict__ out, uint64_t cap) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[kDecodeLds + 4];  // +4: the last dword pair
  const uint64_t b0 = (uint64_t)blockIdx.x * kNT;
  const uint64_t k = b0 + threadIdx.x;
  // Every independent load first (lengths, sources, the block's base, the
  // total), then small values' chars, so one memory wait covers each round
  // and the block scan runs while the chars arrive.
  const uint64_t dl = k < n ? dlen[k] : 0;
  const uint8_t* src = (const uint8_t*)(uintptr_t)(k < n ? vsrc[k] : 0);
  uint64_t base = 0, vn = 0, ts[kRawPer];
  if constexpr (RAW) {
#pragma unroll
    for (uint32_t j = 0; j < kRawPer; ++j) {
      const uint32_t i = threadIdx.x * kRawPer + j;
      ts[j] = i < gridDim.x ? tsum[i] : 0;
    }
  } else {
    base = tsum[blockIdx.x];  // k_tile_scan: the tiles before
    vn = voff[n];             // k_tile_scan's total
  }
  SmallB64 sv;
  const bool small = dl && dl <= kSmallB64Bytes;
  // (RAW: the total is not known yet, so the chars load whenever there is an
  // output; a total above cap then leaves them unused)
  const bool want = out && (RAW || vn <= cap);
#ifdef CB_EXPERIMENTS
  // (timing-only A/B, wrong bytes: CB_B64_X bit 0 skips the value loads)
  if (want && small && !(g_b64_x & 1)) b64_small_load(src, dl, sv);
  if (g_b64_x & 1) sv = SmallB64{{0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u}, 0};
#else
  if (want && small) b64_small_load(src, dl, sv);
#endif
  uint64_t total, pre;
  if constexpr (RAW) {
    uint64_t before = 0, all = 0;
#pragma unroll
    for (uint32_t j = 0; j < kRawPer; ++j) {
      all += ts[j];
      before += threadIdx.x * kRawPer + j < blockIdx.x ? ts[j] : 0;
    }
    pre = block_scan_sum2<kNT>(dl, before, all, &total, &base, &vn);
    if (blockIdx.x == 0 && threadIdx.x == 0) voff[n] = vn;
  } else {
    pre = block_scan<kNT>(dl, &total);
  }
  const bool write = out && vn <= cap;  // uniform
  const uint64_t o = base + pre;
  if (k < n) voff[k] = o;
  if (!write) return;
  if (total > kDecodeLds) {  // uniform: large values, direct byte stores
    if (small) b64_small_decode(sv, dl, [&](uint64_t j, uint8_t v) { out[o + j] = v; });
    else if (dl) b64_decode_into(src, dl, [&](uint64_t j, uint8_t v) { out[o + j] = v; });
    return;
  }
  if (small) b64_small_decode(sv, dl, [&](uint64_t j, uint8_t v) { stage[o - base + j] = v; });
  else if (dl) b64_decode_into(src, dl, [&](uint64_t j, uint8_t v) { stage[o - base + j] = v; });
  __syncthreads();
  // out[base .. base+total): bytes before the first 4-aligned address, then
  // aligned dwords, then the tail
  uint8_t* g = out + base;
  const uint64_t mis = (4 - ((uintptr_t)g & 3)) & 3;
  const uint64_t head = mis < total ? mis : total;
  if (threadIdx.x < head) g[threadIdx.x] = stage[threadIdx.x];
  const uint64_t body = (total - head) / 4;
  uint32_t* gw = reinterpret_cast<uint32_t*>(g + head);
  for (uint64_t i = threadIdx.x; i < body; i += kNT) {
    const uint32_t p = (uint32_t)(head + 4 * i);  // two aligned LDS dwords, realigned
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(stage) + (p >> 2);
    gw[i] = __builtin_amdgcn_alignbyte(sw[1], sw[0], p & 3);
  }
  const uint64_t tail0 = head + 4 * body;
  if (tail0 + threadIdx.x < total) g[tail0 + threadIdx.x] = stage[tail0 + threadIdx.x];
}

inline uint32_t blocks_for(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }

}  // namespace

hipError_t launch_line_count(const uint8_t* data, uint64_t len, uint64_t* cnt, hipStream_t s) {
  if (!len) return hipSuccess;
  ProfScope ps("k_line_count", s);
  hipLaunchKernelGGL(k_line_count, dim3((uint32_t)line_blocks(len)), dim3(kNT), 0, s, data, len,
                     cnt);
  return hipGetLastError();
}

hipError_t launch_line_emit(const uint8_t* data, uint64_t len, const uint64_t* base,
                            uint64_t* start, uint64_t* end, hipStream_t s) {
  if (!len) return hipSuccess;
  ProfScope ps("k_line_emit", s);
  hipLaunchKernelGGL(k_line_emit, dim3((uint32_t)line_blocks(len)), dim3(kNT), 0, s, data, len,
                     base, start, end);
  return hipGetLastError();
}

hipError_t launch_line_finish(const uint8_t* data, uint64_t len, uint64_t nlines,
                              const uint64_t* start, const uint64_t* end, LineRec* rec,
                              uint32_t* llen, uint32_t* err, hipStream_t s) {
  if (!nlines) return hipSuccess;
  ProfScope ps("k_line_finish", s);
  hipLaunchKernelGGL(k_line_finish, dim3(blocks_for(nlines, kNT)), dim3(kNT), 0, s, data, len,
                     nlines, start, end, rec, llen, err);
  return hipGetLastError();
}

hipError_t launch_line_keys(const uint8_t* data, uint64_t nlines, LineRec* rec, const uint32_t* llen,
                            uint64_t* pfx, uint64_t* fence, uint32_t* ok, hipStream_t s) {
  if (!nlines) return hipSuccess;
  ProfScope ps("k_line_keys", s);
  hipLaunchKernelGGL(k_line_keys, dim3(blocks_for(nlines, kNT)), dim3(kNT), 0, s, data, nlines,
                     rec, llen, pfx, fence, ok);
  return hipGetLastError();
}

hipError_t launch_rebuild_mark(const uint8_t* data, const LineRec* rec, uint64_t nlines, uint64_t* has,
                               uint64_t* klen, uint64_t* bad, hipStream_t s) {
  if (!nlines) return hipSuccess;
  ProfScope ps("k_rebuild_mark", s);
  hipLaunchKernelGGL(k_rebuild_mark, dim3(blocks_for(nlines, kNT)), dim3(kNT), 0, s, data, rec, nlines, has,
                     klen, reinterpret_cast<unsigned long long*>(bad));
  return hipGetLastError();
}

hipError_t launch_rebuild_gather(const uint8_t* data, const LineRec* rec, uint64_t nlines,
                                 const uint64_t* has_scan, const uint64_t* len_scan, uint8_t* out,
                                 uint64_t* off, uint64_t* lmap, hipStream_t s) {
  if (!nlines) return hipSuccess;
  ProfScope ps("k_rebuild_gather", s);
  hipLaunchKernelGGL(k_rebuild_gather, dim3(blocks_for(nlines, kNT)), dim3(kNT), 0, s, data, rec, nlines,
                     has_scan, len_scan, out, off, lmap);
  return hipGetLastError();
}

// Exclusive scan of n uint64 (out[n] = total) in three launches: each block
// of 4096 values reduces to one partial, k_tile_scan scans the partials in
// place (and writes the total to out[n]), and each block rescans its values
// from its partial. 16 B of traffic per value; used by the line index
// (per-4-KiB-block line counts) and SsTable::load's rebuild (per-line flags
// and key lengths).
constexpr uint64_t kScanPer = 4, kScanChunk = 1024 * kScanPer;

__global__ __launch_bounds__(1024) void k_scan_reduce(const uint64_t* __restrict__ in, uint64_t n,
                                                      uint64_t* __restrict__ part) {
  const uint64_t i0 = (uint64_t)blockIdx.x * kScanChunk + threadIdx.x * kScanPer;
  uint64_t sum = 0;
#pragma unroll
  for (uint64_t j = 0; j < kScanPer; ++j) sum += i0 + j < n ? in[i0 + j] : 0;
  uint64_t total;
  (void)block_scan<1024>(sum, &total);
  if (threadIdx.x == 0) part[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void k_scan_apply(const uint64_t* __restrict__ in, uint64_t n,
                                                     const uint64_t* __restrict__ part,
                                                     uint64_t* __restrict__ out) {
  const uint64_t i0 = (uint64_t)blockIdx.x * kScanChunk + threadIdx.x * kScanPer;
  uint64_t v[kScanPer], sum = 0;
#pragma unroll
  for (uint64_t j = 0; j < kScanPer; ++j) {
    v[j] = i0 + j < n ? in[i0 + j] : 0;
    sum += v[j];
  }
  const uint64_t base = part[blockIdx.x];
  uint64_t total;
  uint64_t p = base + block_scan<1024>(sum, &total);
#pragma unroll
  for (uint64_t j = 0; j < kScanPer; ++j) {
    if (i0 + j < n) out[i0 + j] = p;
    p += v[j];
  }
}

uint64_t scan_tmp_words(uint64_t n) { return (n + kScanChunk - 1) / kScanChunk + 1; }

hipError_t launch_scan_u64(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* tmp,
                           hipStream_t s) {
  if (!n) return hipMemsetAsync(out, 0, 8, s);
  const uint64_t nb = (n + kScanChunk - 1) / kScanChunk;
  {
    ProfScope ps("k_scan_reduce", s);
    hipLaunchKernelGGL(k_scan_reduce, dim3((uint32_t)nb), dim3(1024), 0, s, in, n, tmp);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = launch_tile_scan(tmp, nb, out + n, s);
  if (e != hipSuccess) return e;
  ProfScope ps("k_scan_apply", s);
  hipLaunchKernelGGL(k_scan_apply, dim3((uint32_t)nb), dim3(1024), 0, s, in, n, tmp, out);
  return hipGetLastError();
}

hipError_t launch_table_search(int keyk, const TableView& t, const KeySrc& ks, uint64_t n,
                               int64_t* line, hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("k_table_search", s);
  const dim3 g(blocks_for(n, kNT));
  switch (keyk) {
    case KEY_FIXED16: hipLaunchKernelGGL(k_table_search<KEY_FIXED16>, g, dim3(kNT), 0, s, t, ks, n, line); break;
    case KEY_FIXED: hipLaunchKernelGGL(k_table_search<KEY_FIXED>, g, dim3(kNT), 0, s, t, ks, n, line); break;
    case KEY_VAR: hipLaunchKernelGGL(k_table_search<KEY_VAR>, g, dim3(kNT), 0, s, t, ks, n, line); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_table_buckets(const LineRec* rec, uint64_t nlines, uint64_t* bkt, uint32_t bits,
                                hipStream_t s) {
  if (!nlines) return hipSuccess;
  ProfScope ps("k_table_buckets", s);
  hipLaunchKernelGGL(k_table_buckets, dim3(blocks_for(nlines, kNT)), dim3(kNT), 0, s, rec, nlines, bkt, bits);
  hipLaunchKernelGGL(k_table_bucket_fp, dim3(blocks_for(1ull << bits, kNT)), dim3(kNT), 0, s, bkt, bits);
  return hipGetLastError();
}

hipError_t launch_table_dir(const uint64_t* pfx, uint64_t nlines, const DirMap& dm, uint32_t* dir,
                            DirMap* dmap_out, hipStream_t s) {
  if (!nlines || !dir || !dmap_out) return hipErrorInvalidValue;
  ProfScope ps("k_table_dir", s);
  hipLaunchKernelGGL(k_table_dir, dim3(blocks_for(nlines, kNT)), dim3(kNT), 0, s, pfx, nlines, dm, dir, dmap_out);
  return hipGetLastError();
}

hipError_t launch_pfx_masks(const uint64_t* pfx, uint64_t nlines, uint64_t* mask, hipStream_t s) {
  if (!nlines) return hipSuccess;
  ProfScope ps("k_pfx_masks", s);
  hipLaunchKernelGGL(k_pfx_masks, dim3(kSampleBlocks), dim3(kNT), 0, s, pfx, nlines, mask);
  return hipGetLastError();
}

hipError_t launch_get_many(int keyk, const TableView* tv, uint32_t nt, const uint64_t* hits,
                           const uint32_t* rows, uint64_t hwords, const KeySrc& ks, uint64_t n,
                           int32_t* which, uint64_t* vsrc, uint64_t* dlen, uint64_t* tsum,
                           hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("k_get_many", s);
  const dim3 g(blocks_for(n, kNT));
#define GM_LAUNCH(K)                                                                                              \
  if (nt <= 64)                                                                                                   \
    hipLaunchKernelGGL((k_get_many<K, true>), g, dim3(kNT), 0, s, tv, nt, hits, rows, hwords, ks, n, which, vsrc, \
                       dlen, tsum);                                                                               \
  else                                                                                                            \
    hipLaunchKernelGGL((k_get_many<K, false>), g, dim3(kNT), 0, s, tv, nt, hits, rows, hwords, ks, n, which,      \
                       vsrc, dlen, tsum)
  switch (keyk) {
    case KEY_FIXED16: GM_LAUNCH(KEY_FIXED16); break;
    case KEY_FIXED: GM_LAUNCH(KEY_FIXED); break;
    case KEY_VAR: GM_LAUNCH(KEY_VAR); break;
    default: return hipErrorInvalidValue;
  }
#undef GM_LAUNCH
  return hipGetLastError();
}

template <int KK, int MM, int WW>
static void set_get_many(const void* set, const ModP& mp, const ZoneView& zv, const TableView* tv, uint32_t nt,
                         const uint32_t* slots, const KeySrc& ks, uint64_t n, int32_t* which, uint64_t* vsrc,
                         uint64_t* dlen, uint64_t* tsum, hipStream_t s) {
  // Measured and not kept (one lane, us per 1M keys): forcing 6 or 7 waves
  // per SIMD (80 / 72 VGPRs with spills) 112-115 / 131 against 108-110 at the
  // natural 90 VGPRs and 5 waves; set[b] read without the short-circuit
  // 111-113; the first two records of each bucket loaded with its prefixes
  // 107-109; gathering and decoding values of <= 18 bytes here (so
  // k_b64_decode reads them coalesced: 27 -> 14 us) 132, the value load being
  // one more dependent step at the end of every found key's chain;
  // compacting the searches (the gate for 2 or 3 keys per lane, the keys
  // with a candidate queued in LDS, then one queue entry per lane, so search
  // waves run full) 243-249: the wave count, not lane occupancy, bounds it.
  hipLaunchKernelGGL((k_set_get_many<KK, MM, WW>), dim3(blocks_for(n, kNT)), dim3(kNT), 0, s, set, mp, zv, tv, nt,
                     slots, ks, n, which, vsrc, dlen, tsum);
}

hipError_t launch_set_get_many(int keyk, int mode, uint32_t width, const void* set, const ModP& mp,
                               const ZoneView* zones, const TableView* tv, uint32_t nt, const uint32_t* slots,
                               const KeySrc& ks, uint64_t n, int32_t* which, uint64_t* vsrc, uint64_t* dlen,
                               uint64_t* tsum, hipStream_t s) {
  if (!n) return hipSuccess;
  if (nt > width || (width != 32 && width != 64)) return hipErrorInvalidValue;
  const ZoneView zv = zones ? *zones : ZoneView{nullptr, nullptr, nullptr, 0};
  ProfScope ps("k_set_get_many", s);
  CB_SET_DISPATCH(keyk, mode, width,
                  (set_get_many<KK, MM, WW>(set, mp, zv, tv, nt, slots, ks, n, which, vsrc, dlen, tsum, s)));
  return hipGetLastError();
}

hipError_t launch_wide_screen(const TableView* tv, const uint32_t* slots, uint32_t nt, uint32_t R, uint32_t bits,
                              uint32_t hbits, uint64_t* scr, hipStream_t s) {
  if (!nt || bits > 24 || hbits > 8) return hipErrorInvalidValue;
  ProfScope ps("k_wide_screen", s);
  const hipError_t e = hipMemsetAsync(scr, 0, wide_screen_bytes(R, bits, hbits), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_wide_screen, dim3(blocks_for(((uint64_t)nt) << bits, kNT)), dim3(kNT), 0, s, tv, slots, nt, R,
                     bits, hbits, scr);
  return hipGetLastError();
}

// The tables' DirMaps copied into one contiguous array (a table without a
// directory: zeros), so the walk stages a group's maps with plain loads in
// the same pass as its views (k_wide_get_many). One lane per 16 B.
__global__ __launch_bounds__(kNT) void k_gather_maps(const TableView* __restrict__ tv, uint32_t nt,
                                                     DirMap* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  if (i >= (uint64_t)nt * kMapWords) return;
  const uint32_t t = (uint32_t)(i / kMapWords), j = (uint32_t)(i - (uint64_t)t * kMapWords);
  const DirMap* g = tv[t].dmap;
  reinterpret_cast<uint4*>(out + t)[j] = g ? reinterpret_cast<const uint4*>(g)[j] : make_uint4(0, 0, 0, 0);
}

hipError_t launch_gather_maps(const TableView* tv, uint32_t nt, DirMap* out, hipStream_t s) {
  if (!nt) return hipSuccess;
  hipLaunchKernelGGL(k_gather_maps, dim3(blocks_for((uint64_t)nt * kMapWords, kNT)), dim3(kNT), 0, s, tv, nt, out);
  return hipGetLastError();
}

hipError_t launch_wide_get_many(int keyk, int mode, uint32_t R, const uint64_t* set, const ModP& mp,
                                const WideZone* zones, const TableView* tv, uint32_t nt, const WideGroup* groups,
                                const uint32_t* slots, const KeySrc& ks, uint64_t n, int32_t* which,
                                uint64_t* vsrc, uint64_t* dlen, uint64_t* tsum, hipStream_t s,
                                const WideScreen* screen, const DirMap* maps) {
  if (!n) return hipSuccess;
  if (!nt || nt > 64 * R || R > kWideMax / 64) return hipErrorInvalidValue;
  const WideZone z = zones ? *zones : WideZone{nullptr, nullptr, nullptr, nullptr, 0};
  const WideScreen sc = screen ? *screen : WideScreen{nullptr, 0, 0, 0};
  const dim3 g(blocks_for(n, kWideNT));
  ProfScope ps("k_wide_get_many", s);
#define WG(KK, MM)                                                                                                 \
  hipLaunchKernelGGL((k_wide_get_many<KK, MM>), g, dim3(kWideNT), 0, s, set, R, mp, z, tv, nt, groups, slots, ks, n, \
                     which, vsrc, dlen, tsum, sc, maps)
  switch (keyk * 3 + mode) {
    case 0: WG(KEY_FIXED16, MOD_POW2_32); break;
    case 1: WG(KEY_FIXED16, MOD_POW2_64); break;
    case 2: WG(KEY_FIXED16, MOD_GENERIC); break;
    case 3: WG(KEY_FIXED, MOD_POW2_32); break;
    case 4: WG(KEY_FIXED, MOD_POW2_64); break;
    case 5: WG(KEY_FIXED, MOD_GENERIC); break;
    case 6: WG(KEY_VAR, MOD_POW2_32); break;
    case 7: WG(KEY_VAR, MOD_POW2_64); break;
    case 8: WG(KEY_VAR, MOD_GENERIC); break;
    default: return hipErrorInvalidValue;
  }
#undef WG
  return hipGetLastError();
}

hipError_t launch_tile_scan(uint64_t* tsum, uint64_t nt, uint64_t* total_out, hipStream_t s) {
  ProfScope ps("k_tile_scan", s);
  hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(1024), 0, s, tsum, nt, total_out);
  return hipGetLastError();
}

hipError_t launch_b64_decode(const uint64_t* vsrc, const uint64_t* dlen, const uint64_t* tsum,
                             uint64_t n, uint64_t* voff, uint8_t* out, uint64_t cap, hipStream_t s, bool raw) {
#ifdef CB_EXPERIMENTS
  static const int env_x = [] {
    const int x = getenv("CB_B64_X") ? atoi(getenv("CB_B64_X")) : 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_b64_x), &x, sizeof(x));
    return x;
  }();
  (void)env_x;
#endif
  if (!n) return hipSuccess;
  const uint32_t nb = blocks_for(n, kNT);
  if (raw && nb > kRawTiles) return hipErrorInvalidValue;
  ProfScope ps("k_b64_decode", s);
  if (raw)
    hipLaunchKernelGGL(k_b64_decode<true>, dim3(nb), dim3(kNT), 0, s, vsrc, dlen, tsum, n, voff, out, cap);
  else
    hipLaunchKernelGGL(k_b64_decode<false>, dim3(nb), dim3(kNT), 0, s, vsrc, dlen, tsum, n, voff, out, cap);
  return hipGetLastError();
}

}  // namespace cb
