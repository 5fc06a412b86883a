// setmask.hpp — one key's FilterSet answer (device code shared by the
// FilterSet probe, filterset.hip, and the fused read path, sstable.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "hash.hpp"
#include "zone.hpp"

namespace cb {

typedef const __attribute__((address_space(1))) uint32_t* gsp32;

// One key's answer for every slot: bit s of the result = slot s's
// may_contain (and, for gated slots, its ZoneMap::contains). SC = the
// reference's `&&` short-circuit (src/bloom.rs:50): set[b] is read only when
// set[a] != 0 (fewer bytes, but b waits for a).
//
// Zone gate (SsTable::get, src/sstable.rs:138): when zv.gated != 0 each
// surviving candidate slot s of a gated slot is re-checked with
// ZoneMap::contains and dropped if the key is outside [min, max]. The
// reference tests the zone first; the conjunction is the same either way and
// testing it only for Bloom candidates costs ~0.5 compare pairs per key
// instead of one per (key, table). zp: the bounds' 16-byte prefixes staged in
// LDS (16-byte keys only).
// ZP_SYNC: the block barrier that publishes zp is taken here, after the
// key's loads have issued (callers where every thread calls this exactly once).
template <int KEYK, int MODE, int W, bool SC, bool ZP_SYNC>
__device__ __forceinline__ typename std::conditional<W == 32, uint32_t, uint64_t>::type set_key_mask(
    const void* __restrict__ set, const uint32_t* __restrict__ any, const KeySrc& ks, uint64_t k,
    bool ok, const ModP& mp, const ZoneView& zv, const BoundPrefix* zp) {
  typedef typename std::conditional<W == 32, uint32_t, uint64_t>::type word_t;
  typedef const __attribute__((address_space(1))) word_t* gptr;
  const gptr sp = (gptr)set;
  uint64_t pa = 0, pb = 0;
  uint4 kv = make_uint4(0, 0, 0, 0);  // KEY_FIXED16: the key, kept for the zone gate
  if (ok) {
    if constexpr (KEYK == KEY_FIXED16) {
      kv = reinterpret_cast<const uint4*>(ks.bytes)[k];
      key_positions_u4<MODE>(kv, mp, pa, pb);
    } else {
      key_positions<KEYK, MODE>(ks, k, mp, pa, pb);
    }
  }
  // Union pre-test: any[p] = (set[p] != 0) is the Bloom filter of every
  // slot's keys (m bits, L2/MALL-resident). A key whose a or b bit is clear
  // there is absent from every slot and skips both set reads.
  if (any) {
    const gsp32 ap = (gsp32)any;
    const uint32_t ua = ok ? ap[pa >> 5] : 0u;
    const uint32_t ub = ok ? ap[pb >> 5] : 0u;
    ok = ok && ((ua >> (pa & 31)) & (ub >> (pb & 31)) & 1u);
  }
  const word_t va = ok ? sp[pa] : (word_t)0;
  word_t vb;
  if constexpr (!SC)
    vb = ok ? sp[pb] : (word_t)0;
  else
    vb = va ? sp[pb] : (word_t)0;
  word_t mask = va & vb;
  if (zv.gated) {  // uniform: only gated launches pay for the zone check
    if constexpr (ZP_SYNC && KEYK == KEY_FIXED16) __syncthreads();  // zp staged
    word_t c = mask & (word_t)zv.gated;
    if constexpr (KEYK == KEY_FIXED16) {
      // 16-byte keys: the key (still in registers from the hash) compared as
      // 4 big-endian words against the bounds' host-computed prefixes.
      if (c) {
        const uint32_t kw[4] = {be32(kv.x), be32(kv.y), be32(kv.z), be32(kv.w)};
        while (c) {
          const uint32_t s = (uint32_t)__builtin_ctzll((uint64_t)c);
          c &= c - 1;
          if (cmp16(kw, zp[2 * s]) < 0 || cmp16(kw, zp[2 * s + 1]) > 0)
            mask &= ~((word_t)1 << s);
        }
      }
    } else if (c) {
      const uint8_t* kp;
      uint64_t kl;
      key_span<KEYK>(ks, k, kp, kl);
      while (c) {
        const uint32_t s = (uint32_t)__builtin_ctzll((uint64_t)c);
        c &= c - 1;
        if (!zone_contains(zv, s, kp, kl)) mask &= ~((word_t)1 << s);
      }
    }
  }
  return mask;
}

// The gated slots' bound prefixes into LDS (16-byte keys; set_key_mask's zp).
template <int KEYK, int W>
__device__ __forceinline__ void stage_zone_prefixes(const ZoneView& zv, BoundPrefix* zp, uint32_t nthreads) {
  if constexpr (KEYK == KEY_FIXED16) {
    if (zv.gated) {  // uniform
      const uint32_t* src = reinterpret_cast<const uint32_t*>(zv.pre);
      uint32_t* dst = reinterpret_cast<uint32_t*>(zp);
      for (uint32_t i = threadIdx.x; i < 2 * W * sizeof(BoundPrefix) / 4; i += nthreads) dst[i] = src[i];
    }
  }
}

// Every (key kind, hash mode, set width) instantiation, by runtime values.
#define CB_SET_DISPATCH(keyk, mode, width, CALL)                                              \
  switch (((keyk) * 3 + (mode)) * 2 + ((width) == 64)) {                                     \
    case 0: { constexpr int KK = KEY_FIXED16, MM = MOD_POW2_32, WW = 32; CALL; } break;     \
    case 1: { constexpr int KK = KEY_FIXED16, MM = MOD_POW2_32, WW = 64; CALL; } break;     \
    case 2: { constexpr int KK = KEY_FIXED16, MM = MOD_POW2_64, WW = 32; CALL; } break;     \
    case 3: { constexpr int KK = KEY_FIXED16, MM = MOD_POW2_64, WW = 64; CALL; } break;     \
    case 4: { constexpr int KK = KEY_FIXED16, MM = MOD_GENERIC, WW = 32; CALL; } break;     \
    case 5: { constexpr int KK = KEY_FIXED16, MM = MOD_GENERIC, WW = 64; CALL; } break;     \
    case 6: { constexpr int KK = KEY_FIXED, MM = MOD_POW2_32, WW = 32; CALL; } break;       \
    case 7: { constexpr int KK = KEY_FIXED, MM = MOD_POW2_32, WW = 64; CALL; } break;       \
    case 8: { constexpr int KK = KEY_FIXED, MM = MOD_POW2_64, WW = 32; CALL; } break;       \
    case 9: { constexpr int KK = KEY_FIXED, MM = MOD_POW2_64, WW = 64; CALL; } break;       \
    case 10: { constexpr int KK = KEY_FIXED, MM = MOD_GENERIC, WW = 32; CALL; } break;      \
    case 11: { constexpr int KK = KEY_FIXED, MM = MOD_GENERIC, WW = 64; CALL; } break;      \
    case 12: { constexpr int KK = KEY_VAR, MM = MOD_POW2_32, WW = 32; CALL; } break;        \
    case 13: { constexpr int KK = KEY_VAR, MM = MOD_POW2_32, WW = 64; CALL; } break;        \
    case 14: { constexpr int KK = KEY_VAR, MM = MOD_POW2_64, WW = 32; CALL; } break;        \
    case 15: { constexpr int KK = KEY_VAR, MM = MOD_POW2_64, WW = 64; CALL; } break;        \
    case 16: { constexpr int KK = KEY_VAR, MM = MOD_GENERIC, WW = 32; CALL; } break;        \
    case 17: { constexpr int KK = KEY_VAR, MM = MOD_GENERIC, WW = 64; CALL; } break;        \
    default: return hipErrorInvalidValue;                                                   \
  }

}  // namespace cb
