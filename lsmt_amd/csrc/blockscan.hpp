// blockscan.hpp — block-wide scans shared by the flush and read-path kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cb {

// Inclusive wave64 scan in DPP moves (no LDS crossbar): row_shr 1/2/4/8 scan
// each row of 16 lanes, row_bcast:15 adds row 0's total to row 1 and row 2's
// to row 3, row_bcast:31 adds rows 0-1's total to rows 2-3. A lane whose
// source is outside its row, or whose row the row mask leaves out, takes the
// `old` operand, 0. Six VALU ops against six ds_bpermute round trips.
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

// Exclusive scan of arr[0..len4) in LDS by wave 0 alone (the other waves wait
// at the caller's next barrier): one barrier fewer than block_exclusive_scan
// and no cross-wave partials. len4 is a multiple of 4 and arr 16-B aligned and
// zero past the counts, so each lane takes whole quads: one ds_read_b128
// round, the wave scan, one ds_write_b128 round (a word at a time the scan
// took ~1 us of k_build_part's 7.7 at 257 tiles). Over the zero padding the
// exclusive prefix is the total, so arr[len] receives it for any len < len4.
__device__ __forceinline__ void wave0_exclusive_scan4(uint32_t* arr, uint32_t len4) {
  if (threadIdx.x >= 64) return;
  const uint32_t lane = threadIdx.x, q = len4 / 4;
  const uint32_t per = (q + 63) / 64;
  const uint32_t beg = min(lane * per, q), end = min(beg + per, q);
  uint4* a4 = reinterpret_cast<uint4*>(arr);
  uint32_t sum = 0;
  for (uint32_t i = beg; i < end; ++i) {
    const uint4 v = a4[i];
    sum += v.x + v.y + v.z + v.w;
  }
  uint32_t run = wave_inclusive_scan(sum) - sum;
  for (uint32_t i = beg; i < end; ++i) {
    const uint4 v = a4[i];
    uint4 o;
    o.x = run;
    o.y = o.x + v.x;
    o.z = o.y + v.y;
    o.w = o.z + v.z;
    run = o.w + v.w;
    a4[i] = o;
  }
}

// Block-wide exclusive scan of one uint64 per thread (NT threads). Returns the
// thread's prefix; *total = block sum. Contains barriers: call uniformly.
template <int NT>
__device__ __forceinline__ uint64_t block_scan(uint64_t v, uint64_t* total) {
  static_assert(NT % 64 == 0 && NT <= 4096, "block size");
  constexpr int NW = NT / 64;
  __shared__ uint64_t ws[NW];
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned long long x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long y = __shfl_up(x, d, 64);
    if ((int)lane >= d) x += y;
  }
  if (lane == 63) ws[wid] = x;
  __syncthreads();
  if (wid == 0) {
    unsigned long long w = lane < NW ? ws[lane] : 0ull;
#pragma unroll
    for (int d = 1; d < NW; d <<= 1) {
      const unsigned long long y = __shfl_up(w, d, 64);
      if ((int)lane >= d) w += y;
    }
    if (lane < NW) ws[lane] = w;
  }
  __syncthreads();
  const uint64_t pre = wid ? ws[wid - 1] : 0;
  *total = ws[NW - 1];
  __syncthreads();  // ws is reused by the next call
  return pre + (uint64_t)x - v;
}

// block_scan of v plus the block sums of a and b, in one LDS round and two
// barriers (three block_scan calls take six): the decode's own scan of the
// lengths with its sums of the tile sums before it and of all of them.
template <int NT>
__device__ __forceinline__ uint64_t block_scan_sum2(uint64_t v, uint64_t a, uint64_t b, uint64_t* total,
                                                    uint64_t* sa, uint64_t* sb) {
  static_assert(NT % 64 == 0 && NT <= 4096, "block size");
  constexpr int NW = NT / 64;
  __shared__ uint64_t ws[3][NW];
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned long long x = v, p = a, q = b;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long y = __shfl_up(x, d, 64);
    if ((int)lane >= d) x += y;
    p += __shfl_xor(p, d, 64);
    q += __shfl_xor(q, d, 64);
  }
  if (lane == 63) ws[0][wid] = x;
  if (lane == 0) {
    ws[1][wid] = p;
    ws[2][wid] = q;
  }
  __syncthreads();
  uint64_t pre = 0, t = 0, s1 = 0, s2 = 0;
#pragma unroll
  for (uint32_t w = 0; w < (uint32_t)NW; ++w) {
    const uint64_t c = ws[0][w];
    pre += w < wid ? c : 0;
    t += c;
    s1 += ws[1][w];
    s2 += ws[2][w];
  }
  *total = t;
  *sa = s1;
  *sb = s2;
  __syncthreads();  // ws is reused by the next call
  return pre + (uint64_t)x - v;
}

}  // namespace cb
