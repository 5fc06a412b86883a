// zone.hpp — device restatement of ZoneMap (/root/reference/src/zonemap.rs)
// and the per-table gate of SsTable::get (src/sstable.rs:138):
//
//   if !zone_map.contains(key) || !bloom.may_contain(key) { return None }
//
// ZoneMap keeps the lexicographically smallest and largest key a table holds
// (update, zonemap.rs:21-32; Rust's `str` order = byte-wise, a proper prefix
// sorts first). contains(key) is min <= key <= max, and true when either
// bound is missing (zonemap.rs:37-42).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hash.hpp"

namespace cb {

// A bound's first 16 bytes as 4 big-endian words (zero-padded) + its length:
// enough to order any 16-byte key against it exactly. 32 B, two loads.
struct alignas(32) BoundPrefix {
  uint32_t w[4];
  uint32_t len;
  uint32_t pad[3];
};

// Per-slot bounds of a FilterSet, resident in HBM (a few KB, L2-resident
// during a probe). hdr[4*s .. 4*s+3] = (lo_off, lo_len, hi_off, hi_len) into
// blob; pre[2*s + j] = prefix of slot s's lower (j = 0) / upper (j = 1)
// bound, precomputed on the host. `gated` has bit s set iff slot s has both
// bounds: only those slots can reject a key (a half-open zone map accepts
// everything).
struct ZoneView {
  const uint32_t* hdr;
  const BoundPrefix* pre;
  const uint8_t* blob;
  uint64_t gated;
};

// Up to 8 bytes p[0..m) as a big-endian word (zero-padded). The loads are
// independent, so they issue back to back: one memory latency per 8 bytes
// instead of one per byte.
__device__ __forceinline__ uint64_t be_chunk(const uint8_t* p, uint64_t m) {
  uint64_t v = 0;
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j)
    if (j < m) v |= (uint64_t)p[j] << (56 - 8 * j);
  return v;
}

// Rust `Ord for str`: byte-wise, then length. Returns <0, 0, >0. Compares 8
// bytes per step as big-endian words.
__device__ __forceinline__ int bytes_cmp(const uint8_t* a, uint64_t al, const uint8_t* b,
                                         uint64_t bl) {
  const uint64_t n = al < bl ? al : bl;
  for (uint64_t i = 0; i < n; i += 8) {
    const uint64_t m = n - i < 8 ? n - i : 8;
    const uint64_t x = be_chunk(a + i, m), y = be_chunk(b + i, m);
    if (x != y) return x < y ? -1 : 1;
  }
  return al < bl ? -1 : (al > bl ? 1 : 0);
}

// Byte span of key k in a key batch.
template <int KEYK>
__device__ __forceinline__ void key_span(const KeySrc& ks, uint64_t k, const uint8_t*& p,
                                         uint64_t& len) {
  if constexpr (KEYK == KEY_FIXED16) {
    p = ks.bytes + k * 16;
    len = 16;
  } else if constexpr (KEYK == KEY_FIXED) {
    p = ks.bytes + k * ks.key_len;
    len = ks.key_len;
  } else {
    const uint64_t o0 = ks.offsets[k];
    p = ks.bytes + o0;
    len = ks.offsets[k + 1] - o0;
  }
}

// ZoneMap::contains for slot s (whose bit is set in zv.gated).
__device__ __forceinline__ bool zone_contains(const ZoneView& zv, uint32_t s, const uint8_t* key,
                                              uint64_t len) {
  const uint4 h = reinterpret_cast<const uint4*>(zv.hdr)[s];
  return bytes_cmp(key, len, zv.blob + h.x, h.y) >= 0 &&
         bytes_cmp(key, len, zv.blob + h.z, h.w) <= 0;
}

// Byte-swap to big-endian so an unsigned word compare is a lexicographic
// compare of 4 bytes.
__device__ __forceinline__ uint32_t be32(uint32_t x) { return __builtin_bswap32(x); }

// Rust str order of a 16-byte key (big-endian words kw) against a bound.
__device__ __forceinline__ int cmp16(const uint32_t kw[4], const BoundPrefix& b) {
  // b is read field by field (LDS-staged in the gated set probe)
  const uint32_t n = b.len < 16 ? b.len : 16;
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) {
    if (4 * i >= n) break;
    const uint32_t nb = n - 4 * i;  // bytes of this word inside the bound
    const uint32_t m = nb >= 4 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (8 * nb));
    const uint32_t x = kw[i] & m, y = b.w[i];
    if (x != y) return x < y ? -1 : 1;
  }
  // the first min(16, len) bytes agree: the shorter string sorts first
  return b.len > 16 ? -1 : (b.len < 16 ? 1 : 0);
}

// Lexicographic min / max index of a key batch (the ZoneMap::update loop of
// SsTable::create, src/sstable.rs:62-65, over a whole batch). idx[0] = index
// of the first smallest key, idx[1] = index of the first largest key (ties
// keep the earliest, as `key < min` / `key > max` do). idx is device memory;
// tmp holds 2 * 1024 uint64 partials.
hipError_t launch_zone_bounds(int keyk, const KeySrc& ks, uint64_t n, uint64_t* tmp,
                              uint64_t* idx, hipStream_t s);

}  // namespace cb
