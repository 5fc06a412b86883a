// exchange.hpp — sparse hit-bitmap exchange for the multi-GPU probe (see
// exchange.hip; C ABI: cb_hits_compress / cb_hits_expand, and comm.cpp's
// cb_hits_allgather which runs both around an RCCL all-gather).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cb {

constexpr uint32_t kMaxRanks = 64;
struct RankRows {
  uint64_t row_off[kMaxRanks];  // first global row of each rank's slice
};

// Compress: one block (and one directory entry) per kCompressWords words.
constexpr uint64_t kCompressWords = 2048;
// rows*words*64 must stay below 2^32 (positions are u32).
constexpr uint64_t kMaxCompressWords = (1ull << 26) - 1;

inline uint64_t pack_blocks(uint64_t nw) { return (nw + kCompressWords - 1) / kCompressWords; }
// Pack size in uint32 for nw words of hit rows and cap positions:
// {count, 0, positions[cap], dir[2 * pack_blocks(nw)]}. Packs that are
// all-gathered use the largest shard's nw on every rank.
inline uint64_t pack_words(uint64_t nw, uint64_t cap) { return 2 + cap + 2 * pack_blocks(nw); }

// Per-stream compress claim words (device, 2 uint64 zeroed once when allocated;
// launches that share them must be stream-ordered) and the host-side parity.
struct CompressState {
  uint32_t* ctl = nullptr;
  uint32_t parity = 0;
};

struct ExpandPlan {
  uint64_t row_off[kMaxRanks + 1];  // first global row of each rank; [nranks] = total rows
  uint64_t blk_off[kMaxRanks];      // first expand block of each rank
};

// pack (pack_words(rows*words, cap) uint32) := {count, 0, positions,
// directory}; one launch, no inter-block waiting. count may exceed cap: the
// pack is then incomplete and must not be expanded.
hipError_t launch_hits_compress(const uint64_t* hits, uint64_t rows, uint64_t words,
                                uint32_t* pack, uint64_t cap, CompressState& st, hipStream_t s);
// full := every rank's positions (packs from launch_hits_compress,
// all-gathered with stride pack_words(max shard words, cap)) as the dense
// map; a rank with count > cap contributes zeros and clears *ok (if ok !=
// nullptr). row_off must start at 0 and be non-decreasing.
hipError_t launch_hits_expand(const uint32_t* packs, uint32_t nranks, uint64_t cap,
                              const RankRows& rr, uint64_t words, uint64_t total_rows,
                              uint64_t* full, uint32_t* ok, hipStream_t s);

// The expand for packs written by the set probe itself (filterset.hpp
// PackSink: one directory entry per probe block of kBlockWords words of
// every row): one workgroup per (rank, probe block) rebuilds that block's
// rows x kBlockWords words in LDS and writes each row's segment once.
// nblk = probe blocks per rank (the same on every rank); rows of a rank <= 64.
hipError_t launch_hits_expand_blocks(const uint32_t* packs, uint32_t nranks, uint64_t cap, uint64_t stride,
                                     const RankRows& rr, uint64_t hwords, uint64_t total_rows, uint32_t nblk,
                                     uint32_t block_words, uint64_t* full, uint32_t* ok, hipStream_t s);

}  // namespace cb
