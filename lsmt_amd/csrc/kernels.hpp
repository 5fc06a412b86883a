// kernels.hpp — host-side launchers for the gfx950 Bloom kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hash.hpp"

namespace cb {

constexpr uint32_t kMaxFiltersPerLaunch = 64;  // filter pointers carried in kernargs
constexpr uint32_t kFiltersPerGroup = 32;      // one uint32 result mask per key
constexpr uint32_t kMaxTiles = 4096;           // LDS histogram bound in the partition pass
constexpr uint32_t kMaxTileBits = 19;          // build: 64 KiB LDS tiles at most
constexpr uint32_t kMaxBuildBlocks = 4096;     // partition blocks per build launch (host chunks keys)
constexpr uint32_t kMinTileBits = 12;          // build: 512 B tiles at least
constexpr uint32_t kMinProbeTileBits = 16;     // probe kernel instantiations: 2^16..2^18
constexpr uint32_t kMaxProbeTileBits = 18;
// Filter allocations are padded to whole tiles of the largest tile size a pass
// may use, so no tiled pass reads or writes past the allocation.
constexpr uint64_t kTileAlignBits = 1ull << kMaxTileBits;
constexpr uint64_t kSmallAlignBits = 1ull << kMinProbeTileBits;

struct FilterPtrs {
  const uint32_t* w[kMaxFiltersPerLaunch];
  uint32_t row[kMaxFiltersPerLaunch];  // hits row for filter i of this launch
};

// A batch of filters (same m) built together: one partition launch and one
// tile launch for all of them (blockIdx.y = filter). C4's concurrent flushes.
constexpr uint32_t kMaxBuildBatch = 64;
struct BuildBatch {
  KeySrc ks[kMaxBuildBatch];
  uint64_t n[kMaxBuildBatch];
  uint32_t* words[kMaxBuildBatch];
  uint64_t fresh;  // bit i: filter i is known all-zero
};
static_assert(sizeof(BuildBatch) <= 3072, "a launch's arguments stay within the 4 KiB kernarg limit");

// Geometry of one tiled pass (build or probe) over filters of m bits.
struct TilePlan {
  uint32_t tb;    // log2(tile bits)
  uint32_t T;     // number of tiles = ceil(m / 2^tb)
  uint32_t kpt;   // keys per thread in the partition pass
  uint32_t C;     // keys per partition block = threads * kpt
  uint32_t nblk;  // partition blocks = ceil(n / C)
  uint32_t sub;   // build only: 0, or log2 of the 2^16-bit sub-tiles per tile (16-bit entries)
};

// nb: filters built together in one launch pair (insert_fixed_many batches).
TilePlan plan_build(uint64_t m, uint64_t n, uint32_t nb = 1);
TilePlan plan_probe(uint64_t m, uint64_t n);
bool plan_ok(const TilePlan& p);  // tile count fits the partition histogram

// Workspace bytes a tiled pass needs.
size_t build_seg_bytes(const TilePlan& p);
size_t build_ent_bytes(const TilePlan& p);
size_t probe_seg_bytes(const TilePlan& p);
size_t probe_ent_bytes(const TilePlan& p);
size_t probe_lkey_bytes(const TilePlan& p);

hipError_t launch_insert_direct(int keyk, int mode, uint32_t* words, const KeySrc& ks, uint64_t n,
                                const ModP& mp, hipStream_t s);
// Filters of m <= kInsertLdsMaxBits: the batch ORed into an LDS copy per
// block. store_all (a fresh filter, n <= kInsertLdsOneBlock): one block writes
// all nw_alloc words, so no fill is needed first; otherwise the words must be
// initialised and each block ORs its non-zero words in.
constexpr uint64_t kInsertLdsMaxBits = 1ull << 19;
constexpr uint64_t kInsertLdsOneBlock = 8192;
hipError_t launch_insert_lds(int keyk, int mode, uint32_t* words, uint64_t m, uint64_t nw_alloc, const KeySrc& ks,
                             uint64_t n, const ModP& mp, bool store_all, hipStream_t s);
hipError_t launch_probe_direct(int keyk, int mode, const FilterPtrs& fp, uint32_t nf,
                               const KeySrc& ks, uint64_t n, const ModP& mp, uint64_t* hits,
                               uint64_t hwords, hipStream_t s);

// seg / ent hold nb consecutive per-filter regions of build_seg_bytes /
// build_ent_bytes each (p planned for the largest n of the batch).
hipError_t launch_build_batch(int keyk, int mode, const BuildBatch& bb, uint32_t nb,
                              const ModP& mp, const TilePlan& p, uint32_t* seg, uint32_t* ent,
                              hipStream_t s);
hipError_t launch_build_tiled(int keyk, int mode, uint32_t* words, bool fresh, const KeySrc& ks,
                              uint64_t n, const ModP& mp, const TilePlan& p, uint32_t* seg,
                              uint32_t* ent, hipStream_t s);
// Probe = partition the key batch once per filter size (K1), then per launch
// of <= 64 filters: tile pass (K2) into masks (ceil(nf/32) * n uint32) and the
// ballot transpose into hits (K3).
hipError_t launch_probe_partition(int keyk, int mode, const KeySrc& ks, uint64_t n,
                                  const ModP& mp, const TilePlan& p, uint32_t* seg, uint2* ent,
                                  uint16_t* lkey, hipStream_t s);
hipError_t launch_probe_tiles(const FilterPtrs& fp, uint32_t nf, uint64_t n, const TilePlan& p,
                              const uint32_t* seg, const uint2* ent, const uint16_t* lkey,
                              uint32_t* masks, uint64_t* hits, uint64_t hwords, hipStream_t s);
hipError_t launch_mask_tail(uint32_t* words, uint64_t m, hipStream_t s);

hipError_t launch_export_bools(const uint32_t* words, uint64_t m, uint8_t* out, hipStream_t s);
hipError_t launch_import_bools(uint32_t* words, uint64_t m, const uint8_t* in, hipStream_t s);

}  // namespace cb
