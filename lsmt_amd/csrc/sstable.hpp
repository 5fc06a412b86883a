// sstable.hpp — SSTable data files resident in HBM and the batched read-path
// resolution after the Bloom/zone gate.
//
// A data file is SsTable::create's output (/root/reference/src/sstable.rs:
// 57-72): lines `key \t base64(value) \n` sorted by key. SsTable::get
// (src/sstable.rs:133-153) splits it on '\n', drops empty lines, binary-
// searches the lines (161-179) and base64-decodes the hit (148). Database::get
// (src/lib.rs:128-134) asks the tables newest-first and keeps the first
// Ok(Some). Here one lane resolves one key across all its candidate tables.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hash.hpp"
#include "zone.hpp"

namespace cb {

constexpr uint32_t kNoSep = 0xFFFFFFFFu;  // line without a TAB: ends a search

// The prefix index of a well-formed table is a fan-out-16 tree kept as
// levels of sampled prefixes: level 0 is pfx itself, level j >= 1 holds
// pfx[l] for every l that is a multiple of 16^j, up to the first level of at
// most 16 entries. A lookup reads one run of at most 16 consecutive entries
// (one 128-B line) per level. Levels 1..L are stored one after another in
// the fence array.
constexpr uint32_t kFanBits = 4;
constexpr uint32_t kFanout = 1u << kFanBits;
__host__ __device__ inline uint64_t level_count(uint64_t nl, uint32_t j) {
  return (nl + (1ull << (kFanBits * j)) - 1) >> (kFanBits * j);
}
// L: the top level (0 when the table has at most 16 lines)
__host__ __device__ inline uint32_t fence_levels(uint64_t nl) {
  uint32_t L = 0;
  while (level_count(nl, L) > kFanout) ++L;
  return L;
}
// offset of level j >= 1 in the fence array
__host__ __device__ inline uint64_t level_offset(uint64_t nl, uint32_t j) {
  uint64_t o = 0;
  for (uint32_t i = 1; i < j; ++i) o += level_count(nl, i);
  return o;
}
__host__ __device__ inline uint64_t fence_words(uint64_t nl) { return level_offset(nl, fence_levels(nl) + 1); }
// level j >= 1 entry of line l (a multiple of 16^j): fence[level_offset(nl, j) + (l >> 4j)]
__device__ __forceinline__ void fence_put(uint64_t* fence, uint64_t nl, uint64_t l, uint64_t v) {
  const uint32_t L = fence_levels(nl);
  uint64_t off = 0;
  for (uint32_t j = 1; j <= L; ++j) {
    if (l & ((1ull << (kFanBits * j)) - 1)) break;
    fence[off + (l >> (kFanBits * j))] = v;
    off += level_count(nl, j);
  }
}
// Directory of a well-formed table, on a byte-rank radix of the 8-byte
// prefix (an order-preserving compression of the key alphabet). For each
// byte position j a DirMap records byte values the table's prefixes hold
// (mask: from a sample of the lines); a prefix's digit j is the rank of its
// byte among them, the bucket the mixed-radix number of its first npos
// digits (the last one coarsened by `shift`), sized to ~2 lines per bucket.
// dir[B] = the first line whose bucket is >= B (dir[nbuckets] = nlines). A
// lookup computes its bucket from a few LDS words, then reads dir[B],
// dir[B+1]: a bucket of at most 8 lines is searched with one round of prefix
// loads, a larger one starts the fence descent at the lowest level where it
// spans at most 16 entries. A plain bit radix leaves text keys in a few huge
// buckets (16-hex-char keys: 512 occupied buckets of ~1000 lines at 512K
// lines, whatever the bit count); the ranks spread them over every bucket.
//
// The bucket must only be monotone (x < y => bucket(x) <= bucket(y)) for
// any prefix, sampled byte values or not: then lines before dir[B] are below
// every key of bucket B and lines from dir[B+1] on above it, so a key's lower
// bound lies in its bucket's window. A byte v missing from the mask at
// position j takes the rank of the next larger value and forces the later
// digits to 0 (v sorts before every prefix of that digit); a byte above the
// largest value takes the last digit and forces the later digits to their
// maximum. The sample therefore only shapes the buckets' sizes, never the
// answers. Tables of fewer than 16 lines have none.
constexpr uint32_t kDirPos = 8;  // byte positions of the 8-byte prefix
constexpr uint32_t kDirSample = 8192;  // lines sampled (evenly spaced) for the masks
struct DirMap {
  uint64_t mask[kDirPos][4];  // byte values at position j: bit v & 63 of word v >> 6
  uint32_t pre[kDirPos];      // byte w of pre[j] = popcount(mask[j][0 .. w)), w < 4
  uint16_t radix[kDirPos];    // digit j's radix (1 past npos)
  uint32_t npos;              // positions whose digits name the bucket
  uint32_t shift;             // position npos-1's digit is its rank >> shift
  uint64_t nbuckets;          // product of the radices: dir has nbuckets + 1 entries
};
static_assert(sizeof(DirMap) == 320, "DirMap is staged into LDS as 20 x 16 B");

// Directory size for nl lines: ~2 lines per bucket, at most 2^24 buckets.
__host__ __device__ inline uint64_t dir_target(uint64_t nl) {
  if (nl < 16 || nl >= (1ull << 32)) return 0;
  return nl / 2 < (1ull << 24) ? nl / 2 : (1ull << 24);
}
inline uint64_t dir_words(uint64_t nl) {  // uint32 words (an upper bound of nbuckets + 1)
  const uint64_t t = dir_target(nl);
  return t ? t + 1 : 0;
}

// The bucket of prefix w (monotone in w; see above).
__host__ __device__ inline uint64_t dir_bucket(const DirMap& d, uint64_t w) {
  uint64_t b = 0;
  int force = 0;  // 0: exact digits; -1: later digits 0; +1: later digits at their maximum
  for (uint32_t j = 0; j < d.npos; ++j) {
    const uint32_t R = d.radix[j];
    uint32_t r;
    if (force) {
      r = force < 0 ? 0u : R - 1;
    } else {
      const uint32_t c = (uint32_t)(w >> (56 - 8 * j)) & 255u;
      const uint64_t m = d.mask[j][c >> 6];
      const uint32_t cnt = ((d.pre[j] >> 24) & 255u) + (uint32_t)__builtin_popcountll(d.mask[j][3]);
      r = ((d.pre[j] >> (8 * (c >> 6))) & 255u) + (uint32_t)__builtin_popcountll(m & ((1ull << (c & 63)) - 1));
      if (!((m >> (c & 63)) & 1ull)) {
        if (r >= cnt) {  // above every sampled value: the last digit, later digits at their maximum
          r = cnt - 1;
          force = 1;
        } else {  // before the next sampled value: its digit, later digits 0
          force = -1;
        }
      }
      if (j + 1 == d.npos) r >>= d.shift;
    }
    b = b * R + r;
  }
  return b;
}

// The DirMap of a table whose sampled prefixes hold the byte values `mask`,
// for nl lines: ~target buckets (default dir_target(nl)) (host, or one device thread).
__host__ __device__ inline DirMap make_dirmap(const uint64_t (&mask)[kDirPos][4], uint64_t nl, uint64_t target = ~0ull) {
  DirMap d{};
  if (target == ~0ull) target = dir_target(nl);
  uint64_t D = 1;
  for (uint32_t j = 0; j < kDirPos; ++j) {
    uint32_t pre = 0, acc = 0;
    for (uint32_t w = 0; w < 4; ++w) {
      d.mask[j][w] = mask[j][w];
      pre |= acc << (8 * w);
      acc += (uint32_t)__builtin_popcountll(mask[j][w]);
    }
    d.pre[j] = pre;
    d.radix[j] = 1;
  }
  for (uint32_t j = 0; j < kDirPos && target; ++j) {
    uint64_t c = 0;
    for (uint32_t w = 0; w < 4; ++w) c += (uint64_t)__builtin_popcountll(mask[j][w]);
    if (!c) break;
    if (D * c <= target) {
      D *= c;
      d.radix[j] = (uint16_t)c;
      d.npos = j + 1;
      continue;
    }
    uint32_t sh = 0;
    while (D * (((c - 1) >> sh) + 1) > target) ++sh;
    const uint64_t r = ((c - 1) >> sh) + 1;
    if (r > 1) {
      D *= r;
      d.radix[j] = (uint16_t)r;
      d.npos = j + 1;
      d.shift = sh;
    }
    break;
  }
  d.nbuckets = D;
  return d;
}

// mask[kDirPos][4] |= the byte values of the prefixes pfx_of(i) of
// kDirSample evenly spaced items i of [0, n) (all of them when n is
// smaller), over the first kSampleBlocks 256-thread blocks of a launch (the
// caller zeroes mask; other blocks return at once). Each lane loads its
// kSamplePer items together, marks their bytes in an LDS byte table, then
// wave v ballots values 64v..64v+63 of each position: one mask word per
// ballot, ORed into global memory by lane 0 (8 blocks x 32 atomics).
constexpr uint32_t kSampleBlocks = 8, kSamplePer = 4;
static_assert(kSampleBlocks * 256 * kSamplePer == kDirSample, "sample size");
template <class PfxOf>
__device__ __forceinline__ void sample_pfx_masks(uint64_t n, PfxOf pfx_of, uint64_t* mask) {
  if (blockIdx.x >= kSampleBlocks) return;
  __shared__ uint64_t seen64[kDirPos * 256 / 8];
  uint8_t* seen = reinterpret_cast<uint8_t*>(seen64);
  seen64[threadIdx.x] = 0;  // 256 threads x 8 B = the whole table
  const uint64_t S = n < kDirSample ? n : kDirSample;
  uint64_t w[kSamplePer];
#pragma unroll
  for (uint32_t k = 0; k < kSamplePer; ++k) {  // every load in flight together
    const uint64_t sidx = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * kSamplePer + k;
    w[k] = sidx < S ? pfx_of(S == n ? sidx : sidx * n / S) : 0;
  }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kSamplePer; ++k) {
    const uint64_t sidx = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * kSamplePer + k;
    if (sidx < S) {
#pragma unroll
      for (uint32_t j = 0; j < kDirPos; ++j) seen[j * 256 + ((w[k] >> (56 - 8 * j)) & 255u)] = 1;
    }
  }
  __syncthreads();
  const uint32_t v = threadIdx.x, wv = v >> 6;
#pragma unroll
  for (uint32_t j = 0; j < kDirPos; ++j) {
    const uint64_t m = __ballot(seen[j * 256 + v] != 0);
    if ((v & 63u) == 0 && m) atomicOr((unsigned long long*)(mask + j * 4 + wv), (unsigned long long)m);
  }
}

// Wave-cooperative fill: every lane holds a range dir[s, s + c) to set to v.
// The wave walks the non-empty ranges one by one, all 64 lanes storing each,
// so one long range (a wide gap between two lines' buckets) costs its length
// / 64 stores per lane instead of one lane's serial loop. Whole wave.
__device__ __forceinline__ void wave_fill(uint32_t* dir, uint64_t s, uint64_t c, uint32_t v) {
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t m = __ballot(c != 0);
  while (m) {
    const int L = __builtin_ctzll(m);
    m &= m - 1;
    const uint64_t ls = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)s, L) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(s >> 32), L) << 32;
    const uint64_t lc = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)c, L) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(c >> 32), L) << 32;
    const uint32_t lv = (uint32_t)__builtin_amdgcn_readlane((int)v, L);
    uint32_t* d = dir + ls;
    uint64_t j = lane;
    for (; j + 192 < lc; j += 256) {  // 4 contiguous 256-B stores per round
      d[j] = lv;
      d[j + 64] = lv;
      d[j + 128] = lv;
      d[j + 192] = lv;
    }
    for (; j < lc; j += 64) d[j] = lv;
  }
}

// The directory entries line p of nl owns, given its bucket b and the
// previous line's bp: dir[B] = p for B in (bp, b] ([0, b] for line 0), and
// dir[B] = nl for B in (b, nb] after the last line. Short ranges (~2 lines
// per bucket: the common case) each lane stores itself, long ones go to
// wave_fill. Whole wave; only live lanes own entries.
__device__ __forceinline__ void dir_fill(uint32_t* dir, uint64_t nb, uint64_t nl, uint64_t p, bool live,
                                         uint64_t b, uint64_t bp) {
  uint64_t s0 = 0, c0 = 0, s1 = 0, c1 = 0;
  if (live) {
    s0 = p ? bp + 1 : 0;
    c0 = b + 1 >= s0 ? b + 1 - s0 : 0;  // (prefixes are sorted: never negative)
    if (p == nl - 1) {
      s1 = b + 1;
      c1 = nb + 1 - s1;
    }
  }
  if (c0 && c0 <= 8) {
    for (uint32_t k = 0; k < (uint32_t)c0; ++k) dir[s0 + k] = (uint32_t)p;
    c0 = 0;
  }
  if (c1 && c1 <= 8) {
    for (uint32_t k = 0; k < (uint32_t)c1; ++k) dir[s1 + k] = (uint32_t)nl;
    c1 = 0;
  }
  wave_fill(dir, s0, c0, (uint32_t)p);
  wave_fill(dir, s1, c1, (uint32_t)nl);
}

constexpr uint32_t kBadValue = 0xFFFFFFFFu;  // value that STANDARD.decode rejects

// Per-line index record (32 B, one load). vdl is computed once at index
// time: the decoded length of the line's value, or kBadValue when base64
// 0.21.7 STANDARD.decode would fail (or the line has no TAB) — so the read
// path never re-validates a value. pfx0 / pfx2 (the key's first 16 bytes)
// let keys of <= 16 bytes be compared from the record alone, so a search
// that lands on a directory bucket reads the bucket's records and nothing
// else (round 4: the prefix array is no longer read next to the record).
// The line's length, needed only while indexing and by cb_table_lines, is
// kept apart (llen[], 4 B per line).
struct alignas(16) LineRec {
  uint64_t start;  // line start offset in the file
  uint64_t pfx2;   // key bytes 8..15, big-endian, zero-padded
  uint32_t klen;   // bytes before the first TAB, or kNoSep
  uint32_t vdl;    // decoded value length, or kBadValue
  uint64_t pfx0;   // key bytes 0..7, big-endian, zero-padded (= pfx[line])
};

// One data file and its line index. When the file is well-formed — every
// line has a TAB and the keys are strictly increasing, as SsTable::create
// writes it — any correct search returns what the reference's binary search
// returns, so `fast` files are searched through pfx (each key's first 8
// bytes, big-endian, zero-padded: monotone in the key order) and the fence
// levels above it (fence_levels), so a lookup reads one run of at most 16
// entries per level, then the record. Other files replay the exact
// (lo+hi)/2 trajectory.
struct TableView {
  const uint8_t* data;    // the file, with 16 bytes of readable slack
  const LineRec* rec;     // nlines
  const uint64_t* pfx;    // nlines
  const uint64_t* fence;  // fence_words(nlines): levels 1..nlev
  const uint32_t* dir;    // dmap->nbuckets + 1 entries (nullptr: none)
  const DirMap* dmap;     // the directory's map (device; staged into LDS by the read path)
  const uint64_t* bkt;    // the key buckets (below; nullptr: none — the read path builds them)
  uint32_t nl_lo;         // nlines, low 32 bits
  uint32_t meta;          // nlines >> 32 (8 bits) | nlev << 8 | fast << 16 | bkbits << 24
  // 64 B: the read kernels stage 64 views per block through registers and LDS
  __host__ __device__ uint64_t nlines() const { return ((uint64_t)(meta & 255u) << 32) | nl_lo; }
  __host__ __device__ uint32_t nlev() const { return (meta >> 8) & 255u; }
  __host__ __device__ bool fast() const { return (meta >> 16) & 1u; }
  __host__ __device__ uint32_t bkbits() const { return meta >> 24; }
};
static_assert(sizeof(TableView) == 64, "TableView is 64 B");
__host__ __device__ inline TableView make_view(const uint8_t* data, const LineRec* rec, const uint64_t* pfx,
                                               const uint64_t* fence, uint64_t nlines, uint32_t nlev, bool fast,
                                               const uint32_t* dir, const DirMap* dmap) {
  return TableView{data, rec, pfx, fence, dir, dmap, nullptr, (uint32_t)nlines,
                   (uint32_t)((nlines >> 32) & 255u) | (nlev << 8) | ((fast ? 1u : 0u) << 16)};
}
inline void view_set_buckets(TableView& v, const uint64_t* bkt, uint32_t bits) {
  v.bkt = bkt;
  v.meta = (v.meta & 0x00FFFFFFu) | (bits << 24);
}

// Key buckets of a well-formed table (the read path's first probe, built on
// a table's first get_many): 2^bkbits buckets of 128 B, a line's bucket
// picked by a multiplicative hash of its 8-byte prefix, 2^bkbits >= nlines
// (at most one line per bucket on average). Words of bucket b:
//   [0]      count - 1 (all-ones: empty): 1 per stored line, 16 per line left out
//   [1..4]   the prefix (pfx0) of slots 0..3
//   [6+2s]   slot s's pfx2
//   [7+2s]   slot s's start | klen << 40 | vdl << 52
// A bucket stores its first four lines, in no particular order; a line with
// a key of 4095 bytes or more (klen 0xFFF marks an unwritten slot), an undecodable value or one decoding to more
// than 4095 bytes, or a start at or past 2^40, is left out (and makes its
// bucket's count say so). A lookup reads words 0..3 (the count and three
// prefixes, two 16-byte loads of one line), word 4 only when the count passes
// 3, then the matching slot's pair: one 128-B line where the directory and
// the record took two or three. A count of at most 4 with no matching prefix
// is a proof of absence; anything else it cannot settle (a bucket past four
// lines, a prefix shared by another key) goes on to the directory search.
constexpr uint32_t kBktWords = 16;
constexpr uint32_t kBktSlots = 4;
__host__ __device__ inline uint32_t bkt_bits(uint64_t nlines) {
  uint32_t b = 1;
  while (b < 40 && (1ull << b) < nlines) ++b;
  return b;
}
__host__ __device__ inline uint64_t bkt_index(uint64_t pfx0, uint32_t bits) {
  return (pfx0 * 0x9E3779B97F4A7C15ull) >> (64 - bits);
}
// After the buckets, one 8-byte summary word per bucket (the wide read path
// settles its many false-positive candidates from these alone: 8 B per
// bucket stay in the L2s where the 128-B buckets would be fetched from the
// Infinity Cache): bits 0-3 the stored count, 0-4, or 15 when the bucket is
// not complete (more than four lines, or a line left out); bits 4 + 15 s ..
// 18 + 15 s slot s's 15-bit fingerprint of its prefix (bkt_fp). A complete
// bucket none of whose fingerprints matches the key's proves absence.
__host__ __device__ inline uint32_t bkt_fp(uint64_t pfx0) {
  return (uint32_t)((pfx0 * 0xC2B2AE3D27D4EB4Full) >> 49);
}
__host__ __device__ inline uint64_t bkt_bytes(uint32_t bits) {
  return ((uint64_t)1 << bits) * (kBktWords * 8 + 8);
}
// Buckets of a fast table from its records, then their summary words; bkt
// (bkt_bytes(bits)) must be all-ones first (the caller's memset).
hipError_t launch_table_buckets(const LineRec* rec, uint64_t nlines, uint64_t* bkt, uint32_t bits,
                                hipStream_t s);

// ---- line index build: count -> scan -> emit -> finish ----
constexpr uint32_t kLineChunk = 4096;  // bytes per block (256 threads x 16 B)
inline uint64_t line_blocks(uint64_t len) { return (len + kLineChunk - 1) / kLineChunk; }
// cnt[b] = non-empty line starts in chunk b
hipError_t launch_line_count(const uint8_t* data, uint64_t len, uint64_t* cnt, hipStream_t s);
// start[base[b] + j] = j-th line start of chunk b; end[l] = its '\n' (ends of
// the last line at EOF stay ~0: finish fills them with len)
hipError_t launch_line_emit(const uint8_t* data, uint64_t len, const uint64_t* base,
                            uint64_t* start, uint64_t* end, hipStream_t s);
// rec[l].start/klen/llen; *err |= 1 if a line is 4 GiB or longer
hipError_t launch_line_finish(const uint8_t* data, uint64_t len, uint64_t nlines,
                              const uint64_t* start, const uint64_t* end, LineRec* rec,
                              uint32_t* llen, uint32_t* err, hipStream_t s);
// pfx, rec[l].pfx0 / pfx2 / vdl, fence[j] = pfx[64 j], and the well-formed
// check: *ok &= (every line has a TAB and key[l-1] < key[l]).
hipError_t launch_line_keys(const uint8_t* data, uint64_t nlines, LineRec* rec, const uint32_t* llen,
                            uint64_t* pfx, uint64_t* fence, uint32_t* ok, hipStream_t s);

// dir[0 .. dm.nbuckets] of a table whose pfx is sorted, one lane per line
// (dir_fill; built for every table, used only when the table is
// well-formed); block 0 also stores dm at dmap_out (the table's device copy).
hipError_t launch_table_dir(const uint64_t* pfx, uint64_t nlines, const DirMap& dm, uint32_t* dir,
                            DirMap* dmap_out, hipStream_t s);
// mask[kDirPos][4] |= the byte values of kDirSample evenly spaced prefixes
// (sample_pfx_masks; kSampleBlocks blocks; the caller zeroes mask).
hipError_t launch_pfx_masks(const uint64_t* pfx, uint64_t nlines, uint64_t* mask, hipStream_t s);

// Exclusive scan of n uint64 (out[n] = total). tmp: scan_tmp_words(n) words.
uint64_t scan_tmp_words(uint64_t n);
hipError_t launch_scan_u64(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* tmp,
                           hipStream_t s);

// ---- SsTable::load's rebuild (src/sstable.rs:109-120) ----
// has[l] = line l has a TAB, klen[l] = its key length (0 without a TAB);
// *bad = min(*bad, first line whose key is not UTF-8).
hipError_t launch_rebuild_mark(const uint8_t* data, const LineRec* rec, uint64_t nlines, uint64_t* has,
                               uint64_t* klen, uint64_t* bad, hipStream_t s);
// From the exclusive scans of has / klen (n + 1 entries each): the TAB lines'
// keys as a ragged batch out/off (has_scan[n] keys, off has_scan[n] + 1
// entries) and lmap[i] = the line of key i.
hipError_t launch_rebuild_gather(const uint8_t* data, const LineRec* rec, uint64_t nlines,
                                 const uint64_t* has_scan, const uint64_t* len_scan, uint8_t* out,
                                 uint64_t* off, uint64_t* lmap, hipStream_t s);

// ---- resolution ----
// line[k] = SsTable::binary_search(key k) over one table, or -1.
hipError_t launch_table_search(int keyk, const TableView& t, const KeySrc& ks, uint64_t n,
                               int64_t* line, hipStream_t s);
// Database::get's walk over tv[0..nt) (tv[0] newest). Table t is asked only
// where hits (nullable, [rows][hwords]) has bit k of row rows[t] (rows
// nullable = identity). which[k] = first t whose line decodes as base64,
// else -1; vsrc[k] the device address of that value's base64 bytes; dlen[k]
// the decoded length (0 if none); tsum[b] = the sum of dlen over key tile b
// (kDecodeTile keys, get_tiles(n) entries).
constexpr uint32_t kDecodeTile = 256;
inline uint64_t get_tiles(uint64_t n) { return (n + kDecodeTile - 1) / kDecodeTile; }
// Database::get in one launch: the FilterSet gate (set_key_mask over the
// set of `width` slots, zones nullable) computed per key, then the same walk
// and outputs as launch_get_many; table t is slot slots[t] (nullptr: slot t),
// nt <= width.
hipError_t launch_set_get_many(int keyk, int mode, uint32_t width, const void* set, const ModP& mp,
                               const ZoneView* zones, const TableView* tv, uint32_t nt, const uint32_t* slots,
                               const KeySrc& ks, uint64_t n, int32_t* which, uint64_t* vsrc, uint64_t* dlen,
                               uint64_t* tsum, hipStream_t s);
// Database::get in one launch over a WIDE set (wideset.hpp: more than 64
// slots, R = W/64 words per row): the groups of 64 tables (newest first)
// take their candidate bits from windows of rows a and b (groups[g], the
// slot mapping of tables 64 g ..; slots[t] for kind 2), the zone gate from
// zones (nullable), then the same walk and outputs as launch_get_many.
struct WideZone;
struct WideGroup;
// The wide walk's screen: for a set whose tables share one bucket count
// (2^bits), row (B << hbits) + h (R words, slot-major like the set's rows)
// has slot s's bit clear only when that table's key bucket B is complete and
// holds no fingerprint (bkt_fp) in bin h = fp & (2^hbits - 1): a key whose
// bucket is B and whose fingerprint falls in bin h is then absent from that
// table (Ok(None)) without its summary word being read. scr == nullptr: none.
struct WideScreen {
  const uint64_t* scr;
  uint32_t bits, hbits, pad;
};
__host__ __device__ inline uint64_t wide_screen_bytes(uint32_t R, uint32_t bits, uint32_t hbits) {
  return ((uint64_t)1 << (bits + hbits)) * R * 8;
}
// Builds the screen of tables tv[0..nt) in slots slots[i] (nullptr: slot i)
// into scr (wide_screen_bytes), on stream s after their buckets.
hipError_t launch_wide_screen(const TableView* tv, const uint32_t* slots, uint32_t nt, uint32_t R, uint32_t bits,
                              uint32_t hbits, uint64_t* scr, hipStream_t s);
hipError_t launch_wide_get_many(int keyk, int mode, uint32_t R, const uint64_t* set, const ModP& mp,
                                const WideZone* zones, const TableView* tv, uint32_t nt, const WideGroup* groups,
                                const uint32_t* slots, const KeySrc& ks, uint64_t n, int32_t* which,
                                uint64_t* vsrc, uint64_t* dlen, uint64_t* tsum, hipStream_t s,
                                const WideScreen* screen = nullptr, const DirMap* maps = nullptr);
// The tables' DirMaps (tv[i].dmap, zeros where none) into out[0..nt): the
// contiguous copy the wide walk stages with its views (maps above).
hipError_t launch_gather_maps(const TableView* tv, uint32_t nt, DirMap* out, hipStream_t s);
hipError_t launch_get_many(int keyk, const TableView* tv, uint32_t nt, const uint64_t* hits,
                           const uint32_t* rows, uint64_t hwords, const KeySrc& ks, uint64_t n,
                           int32_t* which, uint64_t* vsrc, uint64_t* dlen, uint64_t* tsum,
                           hipStream_t s);
// Tile sums -> their exclusive scan in place; *total_out = the sum (one
// single-block kernel; producers leave one sum per tile, consumers read their
// block's base in one load, so no full-length scan pass).
hipError_t launch_tile_scan(uint64_t* tsum, uint64_t nt, uint64_t* total_out, hipStream_t s);
// voff[0..n) = exclusive scan of dlen from the scanned tsum (voff[n] is the
// total launch_tile_scan wrote), and the decoded values into out + voff[k];
// values are written only when out != nullptr and the total fits in cap.
// raw: tsum is the producer's unscanned tile sums (left as they are) and the
// kernel scans them itself, voff[n] included: no launch_tile_scan first.
// Batches of at most decode_raw_max() keys.
hipError_t launch_b64_decode(const uint64_t* vsrc, const uint64_t* dlen, const uint64_t* tsum,
                             uint64_t n, uint64_t* voff, uint8_t* out, uint64_t cap, hipStream_t s,
                             bool raw = false);
inline uint64_t decode_raw_max() { return (uint64_t)kDecodeTile * 1024; }

}  // namespace cb
