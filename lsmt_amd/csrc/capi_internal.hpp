// capi_internal.hpp — what the C ABI's translation units share (capi.cpp:
// filters, probes, sets, codec, exchange; capi_sstable.cpp: SSTable files,
// the read path and SsTable::create): the handle structs, error reporting,
// device buffers, the block pool, per-stream workspaces and key staging.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "cassbloom.h"
#include "exchange.hpp"
#include "filterset.hpp"
#include "flush.hpp"
#include "kernels.hpp"
#include "sstable.hpp"
#include "wideset.hpp"
#include "zone.hpp"

// An event recorded after a device write to one or more filters (a batched
// build shares one among all its filters: one hipEventRecord per call, not
// per filter).
struct WriteMark {
  hipEvent_t ev = nullptr;
  ~WriteMark() {
    if (ev) (void)hipEventDestroy(ev);
  }
};

struct cb_filter {
  uint64_t m = 0;
  int device = 0;
  uint32_t* words = nullptr;  // device, nwords_alloc words
  uint64_t nwords_alloc = 0;
  size_t words_cap = 0;  // pool block size
  bool known_zero = true;  // logically all-zero (lets the tiled build skip the read)
  // cb_filter_clear is lazy: the memset is issued by the next operation that
  // needs the words, and skipped by a fresh tiled build (which writes every
  // tile). Exchanged atomically so concurrent readers issue it once.
  std::atomic<bool> needs_zero{false};
  // Pool blocks are reused, so the padding words past ceil(m/32) are cleared
  // once (lazily, on the caller's stream) by paths that skip the full fill.
  std::atomic<bool> needs_pad_zero{false};
  int mode = 0;
  cb::ModP mp{};
  // Host mirror of the packed words for single-key may_contain (DESIGN §2,
  // SURVEY §7 hard part 8): a per-key GPU round trip costs ~10 us, a host
  // probe of the mirror two word loads. Every write to `words` bumps `gen`
  // and records `wmark` on its stream; the first cb_may_contain after a write
  // waits for that event and copies ceil(m/32) words back once (128 B at the
  // product's m = 1024), later ones read the mirror.
  std::atomic<uint64_t> gen{1};       // bumped by every write to words
  std::atomic<uint64_t> host_gen{0};  // the gen `host` holds
  std::mutex host_mu;                 // one refresh at a time
  std::mutex zero_mu;                 // the lazy clear's issue vs. a refresh (capi.cpp ensure_zeroed)
  std::vector<uint32_t> host;         // ceil(m/32) words
  // recorded after the last device write made with the mirror on
  // (atomic_load / atomic_store). Writes from several streams are ordered by
  // their exclusive writer (the reference's `&mut self` insert), so the last
  // mark covers them all.
  std::shared_ptr<WriteMark> wmark;
  // a write was made with the mirror off (nothing recorded, no stream handle
  // kept: VERDICT r5): the refresh waits for every stream the library knows
  // on the device, by events (capi.cpp wait_known_streams)
  std::atomic<bool> unmarked{false};
  // -1 auto (m <= kMirrorAutoBits), 0 off, 1 on; read by concurrent `&self`
  // callers (cb_may_contain, probes) while cb_filter_host_mirror may write it
  std::atomic<int> mirror{-1};
};

// auto mirror up to 2 MiB of host words: past that, the first per-key call
// after every build copies megabytes, and each write would pay an event
// record only for it (SSTable filters are m = 1024, src/sstable.rs:44)
constexpr uint64_t kMirrorAutoBits = 1ull << 24;

inline bool mirror_on(const cb_filter* f) {
  const int mode = f->mirror.load(std::memory_order_relaxed);
  return mode == 1 || (mode == -1 && f->m <= kMirrorAutoBits);
}

struct cb_filterset {
  uint64_t m = 0;
  int device = 0;
  uint32_t width = 32;
  void* words = nullptr;  // device, m (rounded up to 32) words of width bits
  uint32_t* any = nullptr;  // device, ceil(m/32) words: bit p = (words[p] != 0)
  size_t words_cap = 0, any_cap = 0;  // their pool blocks
  uint32_t used = 0;      // 1 + highest assigned slot
  std::vector<uint64_t> dirty;  // word j bit i: slot 64 j + i may hold set bits
  int mode = 0;
  cb::ModP mp{};
  // width > 64: a wide set (wideset.hpp), rows of R = width / 64 uint64 words;
  // wfw is a device array of filter word pointers (cb_set_assign_all's build)
  uint32_t R = 0;
  void* wfw = nullptr;
  size_t wfw_cap = 0;
  // Per-slot ZoneMap (src/zonemap.rs): host copy, and the device table the
  // gated probe reads (cb::ZoneView: 64 x 16-B headers, then the bytes).
  std::vector<std::string> zlo, zhi;
  std::vector<uint8_t> zhas_lo, zhas_hi;
  void* zdev = nullptr;
  size_t zcap = 0;
  uint64_t zgated = 0;         // slots with both bounds (sets of <= 64 slots: the kernels' mask)
  std::vector<uint64_t> zg;    // the same for every width: word j bit i = slot 64 j + i
  bool zany = false;           // any slot gated
  // Readers of the device zone table: one event per stream, recorded after
  // every launch that reads it (gated probes, the fused read path). A zone
  // update waits for these events — the streams' last readers — instead of
  // the whole device, then rewrites the table (capi.cpp upload_zones).
  mutable std::mutex zmu;
  mutable std::map<hipStream_t, hipEvent_t> zread;
  std::vector<void*> zretired;  // outgrown tables, freed by cb_set_destroy
};

// The device zone table of a set (capi.cpp upload_zones): 64 cb::ZoneView
// headers, then the bounds' 16-byte prefixes, then the bound bytes.
constexpr size_t cb_zone_hdr_bytes = 64 * 16;
constexpr size_t cb_zone_pre_bytes = 64 * 2 * sizeof(cb::BoundPrefix);
constexpr size_t cb_zone_blob_off = cb_zone_hdr_bytes + cb_zone_pre_bytes;
inline cb::ZoneView set_zone_view(const cb_filterset* set) {
  const uint8_t* z = (const uint8_t*)set->zdev;
  return cb::ZoneView{(const uint32_t*)z, (const cb::BoundPrefix*)(z + cb_zone_hdr_bytes), z + cb_zone_blob_off,
                      set->zgated};
}
// A wide set's zone table: W 16-B headers, 2 W bound prefixes, the R-word
// gated bit array, then the bound bytes.
inline bool set_is_wide(const cb_filterset* set) { return set->width > 64; }
inline size_t wide_zone_hdr_bytes(uint32_t w) { return (size_t)w * 16; }
inline size_t wide_zone_pre_bytes(uint32_t w) { return (size_t)w * 2 * sizeof(cb::BoundPrefix); }
inline size_t wide_zone_blob_off(uint32_t w) {
  return wide_zone_hdr_bytes(w) + wide_zone_pre_bytes(w) + (size_t)(w / 64) * 8;
}
inline cb::WideZone wide_zone_view(const cb_filterset* set) {
  const uint8_t* z = (const uint8_t*)set->zdev;
  const uint32_t w = set->width;
  return cb::WideZone{(const uint32_t*)z, (const cb::BoundPrefix*)(z + wide_zone_hdr_bytes(w)),
                      z + wide_zone_blob_off(w),
                      (const uint64_t*)(z + wide_zone_hdr_bytes(w) + wide_zone_pre_bytes(w)), set->zany ? 1u : 0u};
}

// What a table made by cb_sstable_create still owes the host until its
// enqueued work has run (capi_sstable.cpp finalize_table): the event after
// the result copy, the pinned result block, and what a fallback sort needs
// (the batch: the caller's device buffers, or the table's own staged copy).
// Owns the staged block and the result slot of an enqueued SsTable::create;
// the destructor returns both (capi_sstable.cpp), so an error return from the
// enqueue leaks neither. Destroy it only once its work can no longer run
// (finalised, or the stream synchronised).
struct TablePending {
  ~TablePending();
  int device = 0;
  hipEvent_t ev = nullptr;
  cb::CreateResult* hres = nullptr;  // pinned, from the result pool
  hipStream_t stream = nullptr;      // the creation stream (the fallback runs on it)
  const uint8_t *dk = nullptr, *dv = nullptr;
  const uint64_t *dko = nullptr, *dvo = nullptr;
  uint64_t n = 0, cap_bytes = 0;
  bool binned = false;                // the bin sort was enqueued (its merge-sort fallback after it)
  void* staged = nullptr;             // host inputs staged into this pool block
  size_t staged_cap = 0;
};

// An SSTable data file resident in HBM with its line index (sstable.hpp).
// A process-unique table id (never reused, unlike a freed table's addresses):
// caches keyed by the tables they were built from compare these.
inline uint64_t next_table_uid() {
  static std::atomic<uint64_t> next{1};
  return next.fetch_add(1, std::memory_order_relaxed);
}

struct cb_table {
  uint64_t uid = next_table_uid();
  int device = 0;
  uint64_t len = 0, nlines = 0;
  uint8_t* data = nullptr;      // the file + 16 bytes of slack
  size_t data_cap = 0, rec_cap = 0;  // pool block sizes
  cb::LineRec* rec = nullptr;   // per-line index record
  uint64_t* pfx = nullptr;      // per-line 8-byte key prefix
  uint64_t* fence = nullptr;    // the fence levels above pfx (sstable.hpp)
  uint32_t* dir = nullptr;      // the byte-rank directory (sstable.hpp; nullptr under 16 lines)
  uint32_t* llen = nullptr;     // per-line length without the '\n' (cb_table_lines; in the index allocation)
  cb::DirMap* dmap = nullptr;   // its map (device, in the index allocation)
  bool fast = false;  // well-formed: TAB on every line, keys strictly increasing
  bool has_zone = false;   // made by cb_sstable_create with n >= 1
  std::string zmin, zmax;  // its ZoneMap bounds (first / last key of the file)
  // cb_sstable_create only enqueues: until `ready`, len / fast / zone /
  // (rarely) the index are still on their way. Every accessor finalises the
  // table first (waits for its work, reads the results once); ferr keeps a
  // deferred error (the batch exceeded the byte bounds it was sized from).
  std::unique_ptr<TablePending> pend;
  uint64_t zidx[2] = {~0ull, ~0ull};  // input indices of the zone's min / max key
  std::atomic<bool> ready{true};
  std::mutex fin_mu;
  int ferr = 0;
  std::string ferr_msg;
  // The read path's key buckets (sstable.hpp), built by the table's first
  // get_many on that call's stream (capi_sstable.cpp table_buckets); every
  // later read enqueues a wait on bkt_ev until it has been seen complete.
  uint64_t* bkt = nullptr;
  size_t bkt_cap = 0;
  uint32_t bkbits = 0;
  hipEvent_t bkt_ev = nullptr;
  std::atomic<int> bkt_state{0};  // 0 none yet, 1 enqueued, 2 complete, -1 never (not fast / no memory)
  std::mutex bkt_mu;
  cb::TableView view() const {
    return cb::make_view(data, rec, pfx, fence, nlines, cb::fence_levels(nlines), fast, dmap ? dir : nullptr, dmap);
  }
};

namespace cbx {

using cb::FilterPtrs;
using cb::KeySrc;
using cb::ModP;
using cb::TilePlan;

extern thread_local std::string g_err;  // cb_last_error
extern thread_local int g_last_path;    // cb_last_path

int fail(int code, const char* what);
int hip_fail(hipError_t e, const char* where);

#define HIP_TRY(expr)                                       \
  do {                                                      \
    hipError_t _e = (expr);                                 \
    if (_e != hipSuccess) return ::cbx::hip_fail(_e, #expr); \
  } while (0)

// Device buffer that grows on demand. Growth synchronises the owning stream
// first, so a buffer still read by queued work is never freed under it.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t reserve(size_t bytes, hipStream_t s) {
    if (bytes <= cap) return hipSuccess;
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 16);
    want = (want + 4095) & ~size_t(4095);
    e = hipMalloc(&p, want);
    if (e != hipSuccess) return e;
    cap = want;
    return hipSuccess;
  }
};

// Device block pool for table, filter and set storage (capi.cpp). *cap
// receives the block's size (pass it back to pool_release). Release is
// stream-ordered: the block is retired behind an event on every stream the
// library knows on that device and reused only once they have all completed;
// the host never waits.
hipError_t pool_alloc(int device, size_t bytes, void** p, size_t* cap);
void pool_release(int device, void* p, size_t cap);

struct Workspace {
  std::mutex mu;
  DevBuf keys, offsets, hits, seg, ent, masks, bools, lkey, zone;
  DevBuf t_views, t_rows, t_which, t_line, t_dlen, t_voff, t_scan, t_vals;
  // what t_views / t_rows hold (a call with the same tables and rows uploads nothing)
  std::vector<uint8_t> t_views_host;
  std::vector<uint32_t> t_rows_host;
  DevBuf t_groups;                          // a wide set's table groups (cb::WideGroup)
  DevBuf t_maps;                            // the tables' DirMaps, contiguous (the wide walk stages them)
  std::vector<uint64_t> t_maps_sig;         // what t_maps was gathered from (table uids and map pointers)
  DevBuf w_scr;                             // the wide walk's screen (sstable.hpp WideScreen)
  std::vector<uint64_t> w_scr_sig;          // what it was built from (table uids, slots, buckets)
  uint32_t w_scr_bits = 0, w_scr_hbits = 0;
  std::vector<uint8_t> t_groups_host;
  DevBuf i_cnt, i_base, i_tmp, i_end, i_err, i_start;                 // line indexing
  DevBuf f_vb, f_vo, f_sk, f_sk2, f_sort, f_tsum, f_flag, f_vsp;  // SsTable::create
  DevBuf x_ctl;                   // cb_hits_compress: slot / finish counters (zeroed once)
  DevBuf dense;                   // the dense set probe's entries and run table (densefs.hip)
  std::vector<std::shared_ptr<WriteMark>> marks;  // write marks, reused once no filter holds them
  cb::CompressState xst;
  cb::CreateResult* hres = nullptr;  // pinned host mirror of f_flag (SsTable::create)
  uint64_t* htot = nullptr;          // pinned, kHostScratch B: get_many's value byte total; index_table's read-backs
  hipEvent_t ev = nullptr;           // marks hres's first copy in the stream
};

constexpr size_t kHostScratch = 16 + sizeof(uint64_t) * cb::kDirPos * 4;  // Workspace::htot bytes

Workspace& workspace(int device, hipStream_t s);
// Registers s as a stream the library has enqueued on for `device` (its
// workspace, created empty if need be): pool_release retires blocks behind
// every registered stream. Every entry point that enqueues work touching a
// pool block on the caller's stream goes through workspace() or this.
void note_stream(int device, hipStream_t s);
// Host wait for the work queued so far on every stream the library has
// enqueued on for `device` (an event per stream; a device-wide sync only
// when one of them is no longer a valid handle or is hipStreamPerThread).
int wait_known_streams(int device);
// Frees what a workspace holds (cb_stream_release, once its stream is idle).
void workspace_free(Workspace& ws);

// The stream's compress state, its counters allocated and zeroed on first
// use (ws.mu held by the caller).
int compress_state(Workspace& ws, hipStream_t s, cb::CompressState** out);

// The FilterSet probe of a device-resident fixed-length key batch into
// device hits, optionally (sink_pack != nullptr) also writing the exchange
// pack (filterset.hpp PackSink; the stream's compress state supplies the
// claim words). Used by cb_set_probe_pack_fixed and the comm layer.
int set_probe_device(const cb_filterset* set, const uint8_t* keys, uint32_t key_len, uint64_t n, bool gated,
                     uint64_t* hits, uint32_t* sink_pack, uint64_t cap, hipStream_t s);

// A launch that reads set's device zone table was enqueued on s (capi.cpp).
int note_zone_read(const cb_filterset* set, hipStream_t s);

// Device-accessible memory (hipMalloc, managed) is used in place; anything
// else (pageable or pinned host memory) is staged by the library.
bool is_device_ptr(const void* p);

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

struct StagedKeys {
  KeySrc ks{};
  int keyk = cb::KEY_FIXED;
  bool staged = false;
};

int stage_fixed(Workspace& ws, const uint8_t* keys, uint32_t key_len, uint64_t n, hipStream_t s,
                StagedKeys& out);
int stage_var(Workspace& ws, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
              hipStream_t s, StagedKeys& out);
// A batched insert with the stream's workspace already locked by the caller.
int insert_locked(Workspace& ws, cb_filter* f, const uint8_t* keys, const uint64_t* offsets,
                  uint32_t key_len, uint64_t n, hipStream_t s);
// A table from cb_sstable_create: wait for its enqueued work and take its
// results (once; thread-safe). Returns the table's deferred error, if any.
// Every entry point that reads a table calls it first (capi_sstable.cpp).
int finalize_table(cb_table* t);
// Host bytes into an output buffer that may be host or device memory.
int put_bytes(uint8_t* dst, const void* src, size_t n);
// A write to f's words was enqueued on s (build, import): the host mirror is
// stale from here, and its refresh waits for this point of s.
int mark_written(cb_filter* f, hipStream_t s);
// One write mark recorded on s for filters fs[0..nf) (ws.mu held).
int mark_written_many(Workspace& ws, cb_filter* const* fs, uint32_t nf, hipStream_t s);

// Device output: used in place when device-resident, else a workspace buffer
// copied back at the end.
template <class T>
int out_buf(DevBuf& b, T* user, size_t count, hipStream_t s, T** dev) {
  if (is_device_ptr(user)) {
    *dev = user;
    return CB_OK;
  }
  HIP_TRY(b.reserve(count * sizeof(T) + 8, s));
  *dev = (T*)b.p;
  return CB_OK;
}

}  // namespace cbx
