// wideset.hpp — wide bit-sliced filter sets: more than 64 SSTable filters of
// one small m in one set (the reference's real shape: every table's filter
// is m = 1024, src/sstable.rs:44,59, and a flush every 1024 inserts,
// src/lib.rs:72,105, so Database::get walks an unbounded number of them,
// src/lib.rs:129-134).
//
// Layout: position-major rows of R = W/64 uint64 words. Row p holds bit p of
// every slot: word j bit i = slot 64 j + i. At the product's m = 1024 and W =
// 1024 the whole set is 128 KiB (1024 rows of 128 B), L2-resident; one key's
// answer for 64 slots is word j of row a AND word j of row b
// (BloomFilter::may_contain for each of them, src/bloom.rs:48-51), and row b
// is read only where row a's word is non-zero (the reference's `&&`).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hash.hpp"
#include "zone.hpp"

namespace cb {

constexpr uint32_t kWideMax = 4096;  // slots of a wide set, at most (R <= 64 words per row)

// Per-slot zone bounds of a wide set (the ZoneView of a 32/64-slot set with
// the gated mask as an R-word bit array): hdr[4 s ..] = (lo_off, lo_len,
// hi_off, hi_len) into blob, pre[2 s + j] = the bounds' 16-byte prefixes,
// gbits word j bit i = slot 64 j + i has both bounds. any = 0: no slot
// gated (the gate is skipped).
struct WideZone {
  const uint32_t* hdr;
  const BoundPrefix* pre;
  const uint8_t* blob;
  const uint64_t* gbits;
  uint32_t any;
};

// How a group of up to 64 tables (newest first, t0 .. t0 + gn - 1) maps to
// the set's slots, so the kernel can take the group's candidate bits from a
// window of the rows instead of one bit per table:
//   kind 0: slot(t0 + i) = lo + i          (ascending)
//   kind 1: slot(t0 + i) = lo + gn - 1 - i (descending: the LSM's age order,
//           slot = position in Vec<SsTable>, walked with .rev())
//   kind 2: any other mapping, one bit read per table (slots[t0 + i]).
struct WideGroup {
  uint32_t kind, lo, gn, pad;
};

// slots 0..nf-1 := the packed filters fw[0..nf-1] (device array of nf word
// pointers, all of size m); slots nf..W-1 zero.
hipError_t launch_wide_build(const uint32_t* const* fw, uint32_t nf, uint64_t m, uint32_t R, uint64_t* set,
                             hipStream_t s);
// slot |= filter (slot known all-zero: sparse, O(set bits)).
hipError_t launch_wide_or_slot(const uint32_t* words, uint64_t m, uint32_t slot, uint32_t R, uint64_t* set,
                               hipStream_t s);
// slot := filter (words == nullptr clears it): every row.
hipError_t launch_wide_put_slot(const uint32_t* words, uint64_t m, uint32_t slot, uint32_t R, uint64_t* set,
                                hipStream_t s);
// hits[slot][ceil(n/64)] for slots 0..used-1 (cb_set_probe_* on a wide set);
// zones (nullable): the SsTable::get zone gate.
hipError_t launch_wide_probe(int keyk, int mode, uint32_t R, const uint64_t* set, uint32_t used, const KeySrc& ks,
                             uint64_t n, const ModP& mp, const WideZone* zones, uint64_t* hits, uint64_t hwords,
                             hipStream_t s);

// ---- device helpers shared with the fused read path (sstable.hip) ----

// Bits [lo, lo + 64) of a row (R words), zero past the row.
// A window across two words takes them in one 16-byte load (rows are 8-byte
// aligned; gfx950 loads them unaligned): two loads of one line issued back to
// back are two L2 requests, the L1 does not merge them (round 6).
__device__ __forceinline__ uint64_t wide_window(const uint64_t* __restrict__ row, uint32_t R, uint32_t lo) {
  const uint32_t j = lo >> 6, sh = lo & 63u;
  if (!sh) return j < R ? row[j] : 0ull;
  if (j + 1 < R) {
    typedef uint64_t u64x2a __attribute__((ext_vector_type(2), aligned(8)));
    const u64x2a v = *(const __attribute__((address_space(1))) u64x2a*)(row + j);
    return (v.x >> sh) | (v.y << (64 - sh));
  }
  return j < R ? row[j] >> sh : 0ull;
}

// ZoneMap::contains for slot s of a wide set (src/zonemap.rs:37-42): true
// when the slot is not gated. kw: a 16-byte key's big-endian words (KEY_FIXED16),
// else the key's bytes.
template <int KEYK>
__device__ __forceinline__ bool wide_zone_ok(const WideZone& z, uint32_t s, const uint32_t kw[4],
                                             const uint8_t* kp, uint64_t kl) {
  if (!((z.gbits[s >> 6] >> (s & 63)) & 1ull)) return true;
  if constexpr (KEYK == KEY_FIXED16) {
    return cmp16(kw, z.pre[2 * s]) >= 0 && cmp16(kw, z.pre[2 * s + 1]) <= 0;
  } else {
    const uint4 h = reinterpret_cast<const uint4*>(z.hdr)[s];
    return bytes_cmp(kp, kl, z.blob + h.x, h.y) >= 0 && bytes_cmp(kp, kl, z.blob + h.z, h.w) <= 0;
  }
}

}  // namespace cb
