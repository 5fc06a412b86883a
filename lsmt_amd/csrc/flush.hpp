// flush.hpp — SsTable::create's data file on the device (flush.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "sstable.hpp"

namespace cb {

// Sort record of one entry: the key's first 16 bytes as big-endian words
// (zero-padded), its length (clamped) and the entry's input index.
struct SortKey {
  uint64_t w0, w1;
  uint32_t len, idx;
};

// out[i] = the sort record of key i.
hipError_t launch_sort_keys(const uint8_t* kb, const uint64_t* ko, uint64_t n, SortKey* out,
                            hipStream_t s);
// *ok &= (keys already in non-decreasing order)
hipError_t launch_sorted_check(const uint8_t* kb, const uint64_t* ko, uint64_t n, uint32_t* ok,
                               hipStream_t s);
// Stable sort of the records by key (rocPRIM merge sort). tmp == nullptr:
// only writes the scratch size to tmp_bytes.
hipError_t entry_sort(void* tmp, size_t& tmp_bytes, const SortKey* in, SortKey* out, uint64_t n,
                      const uint8_t* kb, const uint64_t* ko, hipStream_t s);
// lens[p] = byte length of the p-th output line (order == nullptr: input order)
hipError_t launch_line_lens(const SortKey* order, const uint64_t* ko, const uint64_t* vo, uint64_t n,
                            uint64_t* lens, hipStream_t s);
// The lines into out at loff[p], and 16 zero bytes of slack after the last.
hipError_t launch_format(const SortKey* order, const uint8_t* kb, const uint64_t* ko,
                         const uint8_t* vb, const uint64_t* vo, const uint64_t* loff, uint64_t n,
                         uint8_t* out, hipStream_t s);
// The created file's line index without re-reading it (sstable.hpp layout):
// entry p is line p, so rec / pfx / fence follow from the entry itself. Valid
// only when no key holds '\n' or '\t' (a key byte the reference's line split
// or TAB search would see): flags[1] |= 1 otherwise, and the caller re-indexes
// the file. flags[2] &= (keys strictly increasing: the well-formed check).
hipError_t launch_format_index(const SortKey* order, const uint8_t* kb, const uint64_t* ko,
                               const uint64_t* vo, const uint64_t* loff, uint64_t n,
                               LineRec* rec, uint64_t* pfx, uint64_t* fence, uint32_t* flags,
                               hipStream_t s);

}  // namespace cb
