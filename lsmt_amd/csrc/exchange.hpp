// exchange.hpp — sparse hit-bitmap exchange for the multi-GPU probe (see
// exchange.hip; C ABI: cb_hits_compress / cb_hits_expand).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cb {

constexpr uint32_t kMaxRanks = 64;
struct RankRows {
  uint64_t row_off[kMaxRanks];  // first global row of each rank's slice
};

constexpr uint32_t kMaxCompressBlocks = 256;

// pack: uint32[2 + cap] = {count, 0, positions ascending}; requires
// rows*words*64 <= 2^32. sums: kMaxCompressBlocks words of device scratch.
hipError_t launch_hits_compress(const uint64_t* hits, uint64_t rows, uint64_t words,
                                uint32_t* pack, uint64_t cap, uint32_t* sums, hipStream_t s);
// full := every rank's positions (packs from launch_hits_compress, all-gathered)
// as the dense map; a rank with count > cap contributes nothing and clears *ok
// (if ok != nullptr).
hipError_t launch_hits_expand(const uint32_t* packs, uint32_t nranks, uint64_t cap,
                              const RankRows& rr, uint64_t words, uint64_t total_rows,
                              uint64_t* full, uint32_t* ok, hipStream_t s);

}  // namespace cb
