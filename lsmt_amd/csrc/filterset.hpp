// filterset.hpp — launchers for bit-sliced filter sets (filterset.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"
#include "zone.hpp"

namespace cb {

// slots 0..nf-1 := the packed filters fp.w[0..nf-1] (all of size m); other slots zero.
// Every update also maintains any[m/32] (packed): bit p = (set[p] != 0), the
// union filter the probe tests first.
hipError_t launch_set_build(const FilterPtrs& fp, uint32_t nf, uint64_t m, uint32_t width,
                            void* set, uint32_t* any, hipStream_t s);
// slot |= packed filter words (slot known all-zero: sparse update).
hipError_t launch_set_or_slot(const uint32_t* words, uint64_t m, uint32_t slot, uint32_t width,
                              void* set, uint32_t* any, hipStream_t s);
// slot := packed filter words (words == nullptr clears the slot): full pass.
hipError_t launch_set_put_slot(const uint32_t* words, uint64_t m, uint32_t slot, uint32_t width,
                               void* set, uint32_t* any, hipStream_t s);
// The probe block: kSetWords hit words (64 keys each) of every slot.
constexpr uint32_t kSetWords = 16;
inline uint64_t set_probe_blocks(uint64_t n) { return ((n + 63) / 64 + kSetWords - 1) / kSetWords; }

// Optional sparse output of the probe for the multi-GPU exchange (the
// compress step fused into the probe): pack = {count, 0, positions[cap],
// dir[2 * set_probe_blocks(n)]}, position = slot * hwords * 64 + key, and
// dir[2b], dir[2b+1] = first slot and number of probe block b's positions
// (kSetWords words of every slot). ctl: the stream's claim words
// (CompressState), par: this launch's parity.
struct PackSink {
  uint32_t* pack;
  uint64_t cap;
  unsigned long long* ctl;
  uint32_t par;
};

// hits[slot][ceil(n/64)] for slots 0..used-1. zones (nullable): the
// SsTable::get zone gate, applied to the slots in zones->gated. sink
// (nullable): also write the hit positions as a pack (the block form only).
hipError_t launch_set_probe(int keyk, int mode, uint32_t width, const void* set,
                            const uint32_t* any, uint32_t used, const KeySrc& ks, uint64_t n,
                            const ModP& mp, const ZoneView* zones, uint64_t* hits,
                            uint64_t hwords, hipStream_t s, const PackSink* sink = nullptr);

// Dense batches (densefs.hip): the same hits from a region-partitioned probe
// that streams the set through LDS once. set_probe_dense_ok: the shapes it
// takes (32- or 64-slot sets, m <= 2^32 with at most 4096 regions of 64 KiB)
// and whether the batch is dense enough to pay (n >= 2 keys per 128-B line
// of the set). scratch: dense_scratch_bytes of device memory (the entries
// and the run table; reusable once the launch pair has run). No zone gate
// and no exchange pack: callers keep k_set_probe for those.
bool set_probe_dense_ok(uint32_t width, uint64_t m, uint64_t n);
bool set_dense_shape_ok(uint32_t width, uint64_t m);  // the shape alone (forced mode)
uint32_t dense_regions(uint32_t width, uint64_t m);
uint64_t dense_scratch_bytes(uint32_t width, uint64_t m, uint64_t n);
hipError_t launch_set_probe_dense(int keyk, int mode, uint32_t width, const void* set, uint32_t used,
                                  const KeySrc& ks, uint64_t n, const ModP& mp, uint64_t* hits, uint64_t hwords,
                                  void* scratch, hipStream_t s);

}  // namespace cb
