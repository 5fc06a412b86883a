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
// hits[slot][ceil(n/64)] for slots 0..used-1. zones (nullable): the
// SsTable::get zone gate, applied to the slots in zones->gated.
hipError_t launch_set_probe(int keyk, int mode, uint32_t width, const void* set,
                            const uint32_t* any, uint32_t used, const KeySrc& ks, uint64_t n,
                            const ModP& mp, const ZoneView* zones, uint64_t* hits,
                            uint64_t hwords, hipStream_t s);

}  // namespace cb
