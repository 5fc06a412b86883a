// hash.hpp — device-side restatement of BloomFilter::hashes
// (/root/reference/src/bloom.rs:26-37) for gfx950.
//
//   h1 = fold(h*33 + byte) from 5381, h2 = fold(h*31 + byte) from 0, both
//   u64 wrapping; index = h % m.
//
// Three exact arithmetic modes, chosen per filter size on the host:
//   MOD_POW2_32 : m = 2^k <= 2^32. Wrapping x33/x31 only carries upward, so
//                 the low 32 bits of the u64 state depend only on the low 32
//                 bits of the previous state: a 32-bit state is exact and
//                 h % m == h & (m-1). (SURVEY.md §7 hard part 1.)
//   MOD_POW2_64 : m = 2^k > 2^32: 64-bit state, mask.
//   MOD_GENERIC : any other m: 64-bit state and an exact 64-bit remainder via
//                 q = umulhi(h, floor((2^64-1)/m)), r = h - q*m, one
//                 correction (the estimate is q or q-1).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cb {

enum : int { MOD_POW2_32 = 0, MOD_POW2_64 = 1, MOD_GENERIC = 2 };
enum : int { KEY_FIXED16 = 0, KEY_FIXED = 1, KEY_VAR = 2 };

struct ModP {
  uint64_t m;
  uint64_t mask;   // m - 1 (power-of-two modes)
  uint64_t magic;  // floor((2^64 - 1) / m) (generic mode)
};

struct KeySrc {
  const uint8_t* bytes;
  const uint64_t* offsets;  // KEY_VAR only: n + 1 entries
  uint32_t key_len;         // KEY_FIXED / KEY_FIXED16
};

struct H32 {
  uint32_t h1 = 5381u, h2 = 0u;
  __device__ __forceinline__ void step(uint32_t b) {
    h1 = (h1 << 5) + h1 + b;  // x33 + b
    h2 = (h2 << 5) - h2 + b;  // x31 + b
  }
  __device__ __forceinline__ void word(uint32_t w) {
    step(w & 0xFFu);
    step((w >> 8) & 0xFFu);
    step((w >> 16) & 0xFFu);
    step(w >> 24);
  }
};

struct H64 {
  uint64_t h1 = 5381u, h2 = 0u;
  __device__ __forceinline__ void step(uint32_t b) {
    h1 = (h1 << 5) + h1 + b;
    h2 = (h2 << 5) - h2 + b;
  }
  __device__ __forceinline__ void word(uint32_t w) {
    step(w & 0xFFu);
    step((w >> 8) & 0xFFu);
    step((w >> 16) & 0xFFu);
    step(w >> 24);
  }
};

// 16-byte keys, 32-bit state, without the byte loop. Unrolled, the fold is
//   h = seed*M^16 + sum_i b_i * M^(15-i)   (mod 2^32),  M = 33 or 31.
// Splitting each coefficient c_i = M^(15-i) into its four bytes c_i[p] gives
//   sum_i b_i c_i = sum_p 2^(8p) * sum_i b_i c_i[p],
// and each inner sum over a key word's four bytes is one v_dot4_u32_u8 (u8 x
// u8 products accumulated in u32; a plane's total is < 16 * 255^2, so it never
// wraps). 16 dot4 + 4 adds per hash instead of 16 multiply-add steps plus byte
// extraction. Exact mod 2^32, hence exact for MOD_POW2_32 (see the header).
namespace dot16 {
constexpr uint32_t powm(uint32_t mul, int e) {
  uint32_t r = 1;
  for (int i = 0; i < e; ++i) r *= mul;
  return r;
}
// K(mul, w, p): byte j = byte p of mul^(15 - (4w + j))
constexpr uint32_t K(uint32_t mul, int w, int p) {
  uint32_t k = 0;
  for (int j = 0; j < 4; ++j) k |= ((powm(mul, 15 - (4 * w + j)) >> (8 * p)) & 0xFFu) << (8 * j);
  return k;
}
// The seed term rides in plane 0's accumulator (the dot4 wraps mod 2^32,
// clamp off) and the planes combine by shift-adds: three v_lshl_add_u32.
template <uint32_t MUL, uint32_t SEED>
__device__ __forceinline__ uint32_t fold(const uint4& v) {
  constexpr uint32_t H0 = SEED * powm(MUL, 16);
  uint32_t acc[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    uint32_t a = __builtin_amdgcn_udot4(v.x, K(MUL, 0, p), p == 0 ? H0 : 0u, false);
    a = __builtin_amdgcn_udot4(v.y, K(MUL, 1, p), a, false);
    a = __builtin_amdgcn_udot4(v.z, K(MUL, 2, p), a, false);
    acc[p] = __builtin_amdgcn_udot4(v.w, K(MUL, 3, p), a, false);
  }
  return acc[0] + (acc[1] << 8) + (acc[2] << 16) + (acc[3] << 24);
}
}  // namespace dot16

__device__ __forceinline__ void hash16_u32(const uint4& v, uint32_t& h1, uint32_t& h2) {
  h1 = dot16::fold<33u, 5381u>(v);  // src/bloom.rs:29-31
  h2 = dot16::fold<31u, 0u>(v);     // src/bloom.rs:32-34
}

template <class H>
__device__ __forceinline__ void hash_range(const uint8_t* p, uint64_t len, H& h) {
  uint64_t i = 0;
  while (i < len && (reinterpret_cast<uintptr_t>(p + i) & 3u)) h.step(p[i++]);
  for (; i + 4 <= len; i += 4) h.word(*reinterpret_cast<const uint32_t*>(p + i));
  while (i < len) h.step(p[i++]);
}

template <int KEYK, class H>
__device__ __forceinline__ void hash_key(const KeySrc& ks, uint64_t k, H& h) {
  if constexpr (KEYK == KEY_FIXED16) {
    // 16-byte keys, 16-byte-aligned base: one dwordx4 load per lane, and
    // consecutive lanes read consecutive keys (fully coalesced).
    const uint4 v = reinterpret_cast<const uint4*>(ks.bytes)[k];
    h.word(v.x);
    h.word(v.y);
    h.word(v.z);
    h.word(v.w);
  } else if constexpr (KEYK == KEY_FIXED) {
    hash_range(ks.bytes + k * ks.key_len, ks.key_len, h);
  } else {
    const uint64_t o0 = ks.offsets[k], o1 = ks.offsets[k + 1];
    hash_range(ks.bytes + o0, o1 - o0, h);
  }
}

__device__ __forceinline__ uint64_t fastmod(uint64_t h, const ModP& mp) {
  uint64_t q = __umul64hi(h, mp.magic);
  uint64_t r = h - q * mp.m;
  return r >= mp.m ? r - mp.m : r;
}

// Positions (a, b) = (h1 % m, h2 % m) of key k.
template <int KEYK, int MODE>
__device__ __forceinline__ void key_positions(const KeySrc& ks, uint64_t k, const ModP& mp,
                                              uint64_t& a, uint64_t& b) {
  if constexpr (MODE == MOD_POW2_32 && KEYK == KEY_FIXED16) {
    uint32_t h1, h2;
    hash16_u32(reinterpret_cast<const uint4*>(ks.bytes)[k], h1, h2);
    const uint32_t mask = static_cast<uint32_t>(mp.mask);
    a = h1 & mask;
    b = h2 & mask;
  } else if constexpr (MODE == MOD_POW2_32) {
    // ragged or unaligned batches: a key that happens to be 16 bytes on a
    // 4-byte boundary still takes the dot4 fold (same hash, fewer ops)
    const uint8_t* p;
    uint64_t len;
    if constexpr (KEYK == KEY_FIXED) {
      p = ks.bytes + k * ks.key_len;
      len = ks.key_len;
    } else {
      const uint64_t o0 = ks.offsets[k];
      p = ks.bytes + o0;
      len = ks.offsets[k + 1] - o0;
    }
    uint32_t h1, h2;
    if (len == 16 && !(reinterpret_cast<uintptr_t>(p) & 3u)) {
      const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
      hash16_u32(make_uint4(w[0], w[1], w[2], w[3]), h1, h2);
    } else {
      H32 h;
      hash_range(p, len, h);
      h1 = h.h1;
      h2 = h.h2;
    }
    const uint32_t mask = static_cast<uint32_t>(mp.mask);
    a = h1 & mask;
    b = h2 & mask;
  } else {
    H64 h;
    hash_key<KEYK>(ks, k, h);
    if constexpr (MODE == MOD_POW2_64) {
      a = h.h1 & mp.mask;
      b = h.h2 & mp.mask;
    } else {
      a = fastmod(h.h1, mp);
      b = fastmod(h.h2, mp);
    }
  }
}

// Positions of a 16-byte key already in registers (KEY_FIXED16 callers that
// need the key bytes again afterwards, e.g. the zone gate).
template <int MODE>
__device__ __forceinline__ void key_positions_u4(const uint4& v, const ModP& mp, uint64_t& a,
                                                 uint64_t& b) {
  if constexpr (MODE == MOD_POW2_32) {
    uint32_t h1, h2;
    hash16_u32(v, h1, h2);
    const uint32_t mask = static_cast<uint32_t>(mp.mask);
    a = h1 & mask;
    b = h2 & mask;
  } else {
    H64 h;
    h.word(v.x);
    h.word(v.y);
    h.word(v.z);
    h.word(v.w);
    if constexpr (MODE == MOD_POW2_64) {
      a = h.h1 & mp.mask;
      b = h.h2 & mp.mask;
    } else {
      a = fastmod(h.h1, mp);
      b = fastmod(h.h2, mp);
    }
  }
}

inline ModP make_modp(uint64_t m, int* mode) {
  ModP mp{m, 0, 0};
  const bool pow2 = m && !(m & (m - 1));
  if (pow2) {
    mp.mask = m - 1;
    *mode = m <= (1ull << 32) ? MOD_POW2_32 : MOD_POW2_64;
  } else {
    mp.magic = ~0ull / m;  // == floor(2^64 / m) because m is not a power of two
    *mode = MOD_GENERIC;
  }
  return mp;
}

}  // namespace cb
