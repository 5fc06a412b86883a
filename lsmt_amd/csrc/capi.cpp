// capi.cpp — the extern "C" boundary (include/cassbloom.h) over the gfx950
// kernels: filter handles in HBM, per-stream workspaces, host buffer staging,
// path selection, filter sets, the BloomProto / TableMeta (prost) codec and
// the multi-GPU hit exchange. The SSTable entry points are in
// capi_sstable.cpp; what both share is in capi_internal.hpp.
//
// Reference: /root/reference/src/bloom.rs (BloomFilter / BloomProto) and its
// callers src/sstable.rs:59-65,96-119,138 and src/lib.rs:129-134.
#include "capi_internal.hpp"

namespace cbx {

thread_local std::string g_err;
thread_local int g_last_path = 0;

int fail(int code, const char* what) {
  g_err = what;
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  g_err = std::string(where) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
  return CB_EHIP;
}

// Device block pool for table, filter and set storage. hipMalloc of tens of
// MB costs ~0.1 ms, which dominates a 1M-entry flush; released blocks are
// kept per device (up to kPoolCap bytes) and handed to the next request they
// fit (large blocks are rounded to 2 MiB; a block is reused for requests of
// at least half its size).
//
// Release is stream-ordered (round 6; VERDICT r5: a Drop used to run
// hipDeviceSynchronize, stalling every stream of a concurrent server, e.g.
// readers under sstables.read(), /root/reference/src/lib.rs:21,129). The
// library does not know which streams last used a block, but every stream it
// has enqueued work on has a workspace (workspace() registers it). A release
// records one unfenced event on each of them and retires the block; the pool
// hands it out again only once all those events have completed, as seen by
// the host (hipEventQuery), so no queued kernel can still be using it. The
// host never waits, and no stream waits on another.
//
// Small blocks (round 6) come from slabs. A table of the reference's own
// shape (1024 lines, src/lib.rs:72,105) needs ~44 KB of file, ~60 KB of index
// and 128 KB of key buckets, and its m = 1024 filter 8 KB; rounded to 2 MiB
// blocks, 300 such tables spread over ~1.8 GB of address space, and the wide
// read walk missed the per-CU translation cache (UTCL1) on 8 % of its
// requests, its value decode on 58 % (rocprofv3 TCP_UTCL1_TRANSLATION_MISS,
// tools/gpu/tlb_pmc.sh). Requests of at most kSmallMax are rounded to a power
// of two (at least 4 KiB) and carved, aligned to their size, from 64 MiB
// slabs, so those tables sit in a few tens of MB; released small blocks go
// to a free list per size (behind the same stream-ordered retirement), and
// slabs are kept for the process's life.
constexpr size_t kPoolGrain = 2u << 20;
constexpr size_t kPoolCap = size_t(16) << 30;
constexpr size_t kSmallMax = 1u << 20, kSmallMin = 4096;
constexpr size_t kSlabBytes = 64u << 20;

struct Retired {
  void* p = nullptr;
  size_t cap = 0;
  std::vector<hipEvent_t> evs;  // one per stream known at the release
};

struct Slab {
  uint8_t* base = nullptr;
  size_t used = 0;
};

struct BlockPool {
  std::mutex mu;
  std::map<int, std::multimap<size_t, void*>> free;
  std::map<int, size_t> cached;               // bytes in free + retired (large blocks)
  std::map<int, std::vector<Retired>> retired;  // released, their streams' events still pending
  std::vector<hipEvent_t> spare;              // completed retire events, for reuse
  std::map<std::pair<int, size_t>, std::vector<void*>> small_free;  // (device, block size)
  std::map<int, Slab> slab;                   // the slab small blocks are carved from
};
BlockPool g_pool;

// Experiment builds: CB_POOL_SLAB=0 gives small requests their own 2 MiB
// blocks again (the A/B); CB_POOL_CONTIG=1 allocates slabs and large blocks
// physically contiguous (hipDeviceMallocContiguous).
bool small_blocks_on() {
#ifdef CB_EXPERIMENTS
  static const bool off = getenv("CB_POOL_SLAB") && getenv("CB_POOL_SLAB")[0] == '0';
  return !off;
#else
  return true;
#endif
}

hipError_t device_malloc(void** p, size_t bytes) {
#ifdef CB_EXPERIMENTS
  static const bool contig = getenv("CB_POOL_CONTIG") && getenv("CB_POOL_CONTIG")[0] == '1';
  if (contig) return hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous);
#endif
  return hipMalloc(p, bytes);
}

size_t small_size(size_t bytes) {
  size_t z = kSmallMin;
  while (z < bytes) z <<= 1;
  return z;
}

std::mutex g_ws_mu;
std::map<std::pair<int, void*>, std::unique_ptr<Workspace>> g_ws;

size_t pool_round(size_t bytes) { return (std::max<size_t>(bytes, 1) + kPoolGrain - 1) / kPoolGrain * kPoolGrain; }

namespace {

// Retired blocks of `device` whose events have all completed go to the free
// list (g_pool.mu held). wait: block on the events first (allocation failure).
void reap(int device, bool wait) {
  auto& rl = g_pool.retired[device];
  auto& fl = g_pool.free[device];
  for (size_t i = 0; i < rl.size();) {
    Retired& r = rl[i];
    bool done = true;
    for (hipEvent_t e : r.evs) {
      const hipError_t q = wait ? hipEventSynchronize(e) : hipEventQuery(e);
      if (q == hipErrorNotReady) {
        done = false;
        break;
      }
      if (q != hipSuccess) (void)hipGetLastError();  // an error ends the wait as completion would
    }
    if (!done) {
      ++i;
      continue;
    }
    for (hipEvent_t e : r.evs) g_pool.spare.push_back(e);
    if (r.cap <= kSmallMax)
      g_pool.small_free[{device, r.cap}].push_back(r.p);
    else
      fl.emplace(r.cap, r.p);
    rl[i] = std::move(rl.back());
    rl.pop_back();
  }
}

}  // namespace

// *cap receives the block's size (pass it back to pool_release).
hipError_t pool_alloc(int device, size_t bytes, void** p, size_t* cap) {
  if (bytes <= kSmallMax && small_blocks_on()) {
    const size_t z = small_size(bytes);
    std::lock_guard<std::mutex> lk(g_pool.mu);
    if (!g_pool.retired[device].empty()) reap(device, false);
    auto& fl = g_pool.small_free[{device, z}];
    if (!fl.empty()) {
      *p = fl.back();
      fl.pop_back();
      *cap = z;
      return hipSuccess;
    }
    Slab& sb = g_pool.slab[device];
    size_t off = (sb.used + z - 1) & ~(z - 1);
    if (!sb.base || off + z > kSlabBytes) {  // a new slab (the old one's tail stays unused)
      void* base = nullptr;
      hipError_t e = device_malloc(&base, kSlabBytes);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        // out of memory: as for large blocks, let the retired blocks' work
        // finish, release every cached large block and retry once (on this
        // rare path the pool's lock is held across the frees)
        reap(device, true);
        for (auto& b : g_pool.free[device]) (void)hipFree(b.second);
        g_pool.free[device].clear();
        g_pool.cached[device] = 0;
        if (!fl.empty()) {  // a block of this size came back from the retired list
          *p = fl.back();
          fl.pop_back();
          *cap = z;
          return hipSuccess;
        }
        e = device_malloc(&base, kSlabBytes);
        if (e != hipSuccess) {
          (void)hipGetLastError();
          return e;
        }
      }
      sb.base = (uint8_t*)base;
      off = 0;
    }
    *p = sb.base + off;
    sb.used = off + z;
    *cap = z;
    return hipSuccess;
  }
  const size_t want = pool_round(bytes);
  {
    std::lock_guard<std::mutex> lk(g_pool.mu);
    if (!g_pool.retired[device].empty()) reap(device, false);
    auto& fl = g_pool.free[device];
    auto it = fl.lower_bound(want);
    if (it != fl.end() && it->first <= 2 * want) {
      *p = it->second;
      *cap = it->first;
      g_pool.cached[device] -= it->first;
      fl.erase(it);
      return hipSuccess;
    }
  }
  hipError_t e = device_malloc(p, want);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    // out of memory: let the retired blocks' work finish, release every
    // cached block and retry once
    std::multimap<size_t, void*> drop;
    {
      std::lock_guard<std::mutex> lk(g_pool.mu);
      reap(device, true);
      drop.swap(g_pool.free[device]);
      g_pool.cached[device] = 0;
    }
    for (auto& b : drop) (void)hipFree(b.second);
    e = device_malloc(p, want);
    if (e != hipSuccess) return e;
  }
  *cap = want;
  return hipSuccess;
}

void pool_release(int device, void* p, size_t cap) {
  if (!p) return;
  // the streams that may still have work on the block: every stream the
  // library has enqueued on for this device
  std::vector<hipStream_t> streams;
  {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    for (auto& kv : g_ws)
      if (kv.first.first == device) streams.push_back((hipStream_t)kv.first.second);
  }
  Retired r;
  r.p = p;
  r.cap = cap;
  const bool small = cap <= kSmallMax;  // a slab block (large blocks are whole multiples of 2 MiB)
  bool sync = false;
  {
    std::lock_guard<std::mutex> lk(g_pool.mu);
    if (!small && g_pool.cached[device] + cap > kPoolCap) {
      sync = true;  // the pool is full: hipFree below, which waits as it always has
    } else {
      for (hipStream_t s : streams) {
        // hipStreamPerThread names a different stream on each thread: an
        // event here would not cover another thread's work
        if (s == hipStreamPerThread) {
          sync = true;
          break;
        }
        hipEvent_t ev = nullptr;
        if (!g_pool.spare.empty()) {
          ev = g_pool.spare.back();
          g_pool.spare.pop_back();
        } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) {
          (void)hipGetLastError();
          sync = true;
          break;
        }
        r.evs.push_back(ev);
        if (hipEventRecord(ev, s) != hipSuccess) {
          // a stream destroyed without cb_stream_release: its handle is no
          // longer valid, so fall back to what hipFree implies
          (void)hipGetLastError();
          sync = true;
          break;
        }
      }
      if (!sync) {
        if (!small) g_pool.cached[device] += cap;
        g_pool.retired[device].push_back(std::move(r));
        return;
      }
      for (hipEvent_t e : r.evs) g_pool.spare.push_back(e);
      r.evs.clear();
    }
  }
  (void)hipDeviceSynchronize();  // what hipFree implies
  {
    std::lock_guard<std::mutex> lk(g_pool.mu);
    if (small) {  // slab memory is never freed: back to its size's list
      g_pool.small_free[{device, cap}].push_back(p);
      return;
    }
    if (g_pool.cached[device] + cap <= kPoolCap) {
      g_pool.free[device].emplace(cap, p);
      g_pool.cached[device] += cap;
      return;
    }
  }
  (void)hipFree(p);
}

int wait_known_streams(int device) {
  std::vector<hipStream_t> streams;
  {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    for (auto& kv : g_ws)
      if (kv.first.first == device) streams.push_back((hipStream_t)kv.first.second);
  }
  bool device_sync = false;
  std::vector<hipEvent_t> evs;
  for (hipStream_t s : streams) {
    hipEvent_t ev = nullptr;
    // fenced (system-scope release): the host copies right after the wait
    if (s == hipStreamPerThread || hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      device_sync = true;
      break;
    }
    evs.push_back(ev);
    if (hipEventRecord(ev, s) != hipSuccess) {  // a stream destroyed without cb_stream_release
      (void)hipGetLastError();
      device_sync = true;
      break;
    }
  }
  hipError_t e = hipSuccess;
  if (device_sync) {
    e = hipDeviceSynchronize();
  } else {
    for (hipEvent_t ev : evs)
      if (e == hipSuccess) e = hipEventSynchronize(ev);
  }
  for (hipEvent_t ev : evs) (void)hipEventDestroy(ev);
  if (e != hipSuccess) return hip_fail(e, "waiting for the library's streams");
  return CB_OK;
}

Workspace& workspace(int device, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  auto& slot = g_ws[{device, (void*)s}];
  if (!slot) slot.reset(new Workspace());
  return *slot;
}

void note_stream(int device, hipStream_t s) { (void)workspace(device, s); }

// Everything a workspace holds (cb_stream_release; its stream is idle).
void workspace_free(Workspace& ws) {
  for (DevBuf* b : {&ws.keys, &ws.offsets, &ws.hits, &ws.seg, &ws.ent, &ws.masks, &ws.bools, &ws.lkey, &ws.zone,
                    &ws.t_views, &ws.t_rows, &ws.t_which, &ws.t_line, &ws.t_dlen, &ws.t_voff, &ws.t_scan,
                    &ws.t_vals, &ws.t_groups, &ws.t_maps, &ws.w_scr, &ws.i_cnt, &ws.i_base, &ws.i_tmp, &ws.i_end, &ws.i_err,
                    &ws.i_start, &ws.f_vb, &ws.f_vo, &ws.f_sk, &ws.f_sk2, &ws.f_sort, &ws.f_tsum, &ws.f_flag,
                    &ws.f_vsp, &ws.x_ctl, &ws.dense}) {
    if (b->p) (void)hipFree(b->p);
    b->p = nullptr;
    b->cap = 0;
  }
  if (ws.hres) (void)hipHostFree(ws.hres);
  if (ws.htot) (void)hipHostFree(ws.htot);
  if (ws.ev) (void)hipEventDestroy(ws.ev);
  ws.hres = nullptr;
  ws.htot = nullptr;
  ws.ev = nullptr;
}

int compress_state(Workspace& ws, hipStream_t s, cb::CompressState** out) {
  if (!ws.x_ctl.p) {
    HIP_TRY(ws.x_ctl.reserve(4 * sizeof(uint32_t), s));
    HIP_TRY(hipMemsetAsync(ws.x_ctl.p, 0, 4 * sizeof(uint32_t), s));
    ws.xst = cb::CompressState{};
    ws.xst.ctl = (uint32_t*)ws.x_ctl.p;
  }
  *out = &ws.xst;
  return CB_OK;
}

bool is_device_ptr(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t attr;
  hipError_t e = hipPointerGetAttributes(&attr, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

// Host bytes into an output buffer that may be host or device memory.
int put_bytes(uint8_t* dst, const void* src, size_t n) {
  if (!n) return CB_OK;
  if (is_device_ptr(dst)) {
    HIP_TRY(hipMemcpy(dst, src, n, hipMemcpyHostToDevice));
  } else {
    memcpy(dst, src, n);
  }
  return CB_OK;
}

}  // namespace cbx

using namespace cbx;

namespace {

int g_path_override = 0;  // 0 auto, 1 direct, 2 tiled

constexpr int PATH_DIRECT = 1, PATH_TILED = 2;

uint64_t alloc_words_for(uint64_t m) {
  // Pad to whole 2^18-bit tiles (the largest LDS tile) so tiled passes never
  // read or write past the allocation; small filters pad to one 2^16-bit
  // tile (the smallest probe tile).
  const uint64_t align = m >= cb::kSmallAlignBits ? cb::kTileAlignBits : cb::kSmallAlignBits;
  const uint64_t bits = std::max<uint64_t>((m + align - 1) / align * align, align);
  return bits / 32;
}

hipError_t ensure_pad_zeroed(const cb_filter* cf, hipStream_t s) {
  cb_filter* f = const_cast<cb_filter*>(cf);
  const uint64_t nw = (f->m + 31) / 32;
  if (f->needs_pad_zero.exchange(false) && f->nwords_alloc > nw)
    return hipMemsetAsync(f->words + nw, 0, (f->nwords_alloc - nw) * 4, s);
  return hipSuccess;
}

// A new write mark (recorded with the system-scope release: the mirror's
// refresh copies right after waiting on it).
hipError_t make_mark(std::shared_ptr<WriteMark>* out) {
  auto m = std::make_shared<WriteMark>();
  const hipError_t e = hipEventCreateWithFlags(&m->ev, hipEventDisableTiming);
  if (e != hipSuccess) return e;
  *out = std::move(m);
  return hipSuccess;
}

// Record f's write mark on s: its own mark again when no one else holds it
// (no batch shares it, no mirror refresh is waiting on it), else a new one.
// With the mirror off nothing is recorded (an event per write cost the C2
// one-lane build 1 us of device time, round 6): the write is only flagged,
// and the refresh that meets the flag waits for every stream the library
// knows (wait_known_streams), never for a stored stream handle.
hipError_t record_own_mark(cb_filter* f, hipStream_t s) {
  if (!mirror_on(f)) {
    f->unmarked.store(true, std::memory_order_release);
    return hipSuccess;
  }
  std::shared_ptr<WriteMark> m = std::atomic_load(&f->wmark);
  if (!m || m.use_count() > 2) {  // (2: f's reference and this copy)
    const hipError_t e = make_mark(&m);
    if (e != hipSuccess) return e;
  }
  const hipError_t e = hipEventRecord(m->ev, s);
  if (e == hipSuccess) std::atomic_store(&f->wmark, m);
  return e;
}

// The pending lazy clear, issued on s by whichever operation needs the words
// first (readers may race: zero_mu makes the exchange, the memset and the
// event that orders the host mirror's refresh after it one step).
hipError_t ensure_zeroed(const cb_filter* cf, hipStream_t s) {
  cb_filter* f = const_cast<cb_filter*>(cf);
  note_stream(f->device, s);  // (pool_release retires the words behind every stream that touched them)
  if (!f->needs_zero.load()) return hipSuccess;
  std::lock_guard<std::mutex> lk(f->zero_mu);
  if (f->needs_zero.exchange(false)) {
    f->needs_pad_zero.store(false);
    hipError_t e = hipMemsetAsync(f->words, 0, f->nwords_alloc * 4, s);
    if (e == hipSuccess) e = record_own_mark(f, s);
    return e;
  }
  return hipSuccess;
}

// Every tiled pass reads/writes whole tiles [0, T * 2^tb): refuse to launch
// one the allocation does not cover (a safety net over alloc_words_for).
bool covers(const cb_filter* f, const TilePlan& p) {
  return cb::plan_ok(p) && ((uint64_t)p.T << p.tb) <= f->nwords_alloc * 32;
}

// Largest m a tiled pass covers: kMaxTiles tiles of the largest tile size.
bool build_tiled_ok(uint64_t m) { return m >= 1 && m <= (uint64_t)cb::kMaxTiles << cb::kMaxTileBits; }
bool probe_tiled_ok(uint64_t m) {
  return m >= 1 && m <= (uint64_t)cb::kMaxTiles << cb::kMaxProbeTileBits;
}

int choose_build_path(uint64_t m, uint64_t n) {
  if (g_path_override == PATH_DIRECT || !build_tiled_ok(m)) return PATH_DIRECT;
  if (g_path_override == PATH_TILED) return PATH_TILED;
  return (m >= (1ull << 20) && n >= (1ull << 15)) ? PATH_TILED : PATH_DIRECT;
}

int choose_probe_path(uint64_t m, uint64_t n, uint32_t nf) {
  if (g_path_override == PATH_DIRECT || !probe_tiled_ok(m)) return PATH_DIRECT;
  if (g_path_override == PATH_TILED) return PATH_TILED;
  (void)nf;
  return (m >= (1ull << 20) && n >= (1ull << 16)) ? PATH_TILED : PATH_DIRECT;
}

// Keys as the kernels see them (device pointers), staging host keys.
}  // namespace

namespace cbx {

int stage_fixed(Workspace& ws, const uint8_t* keys, uint32_t key_len, uint64_t n, hipStream_t s,
                StagedKeys& out) {
  const uint64_t bytes = (uint64_t)key_len * n;
  const uint8_t* dk = keys;
  if (bytes && !is_device_ptr(keys)) {
    HIP_TRY(ws.keys.reserve(bytes, s));
    HIP_TRY(hipMemcpyAsync(ws.keys.p, keys, bytes, hipMemcpyHostToDevice, s));
    dk = (const uint8_t*)ws.keys.p;
    out.staged = true;
  }
  out.ks.bytes = dk;
  out.ks.offsets = nullptr;
  out.ks.key_len = key_len;
  out.keyk = (key_len == 16 && !((uintptr_t)dk & 15)) ? cb::KEY_FIXED16 : cb::KEY_FIXED;
  return CB_OK;
}

int stage_var(Workspace& ws, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
              hipStream_t s, StagedKeys& out) {
  // offsets are validated on the host when they live there; device offsets
  // are the caller's contract (non-decreasing, n+1 entries).
  const uint64_t* doff = offsets;
  const uint8_t* db = bytes;
  uint64_t total = 0;
  if (!is_device_ptr(offsets)) {
    for (uint64_t i = 0; i < n; ++i)
      if (offsets[i + 1] < offsets[i]) return fail(CB_EINVAL, "offsets must be non-decreasing");
    total = offsets[n];
    HIP_TRY(ws.offsets.reserve((n + 1) * 8, s));
    HIP_TRY(hipMemcpyAsync(ws.offsets.p, offsets, (n + 1) * 8, hipMemcpyHostToDevice, s));
    doff = (const uint64_t*)ws.offsets.p;
    out.staged = true;
  } else if (!is_device_ptr(bytes) && bytes) {
    HIP_TRY(hipMemcpyAsync(&total, offsets + n, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  }
  if (bytes && total && !is_device_ptr(bytes)) {
    HIP_TRY(ws.keys.reserve(total, s));
    HIP_TRY(hipMemcpyAsync(ws.keys.p, bytes, total, hipMemcpyHostToDevice, s));
    db = (const uint8_t*)ws.keys.p;
    out.staged = true;
  }
  out.ks.bytes = db;
  out.ks.offsets = doff;
  out.ks.key_len = 0;
  out.keyk = cb::KEY_VAR;
  return CB_OK;
}

// insert_impl with the stream's workspace already locked by the caller.
int insert_locked(Workspace& ws, cb_filter* f, const uint8_t* keys, const uint64_t* offsets,
                  uint32_t key_len, uint64_t n, hipStream_t s) {
  StagedKeys sk;
  int rc = offsets ? stage_var(ws, keys, offsets, n, s, sk)
                   : stage_fixed(ws, keys, key_len, n, s, sk);
  if (rc) return rc;

  const int path = choose_build_path(f->m, n);
  g_last_path = path;
  if (path == PATH_DIRECT && f->m <= cb::kInsertLdsMaxBits) {
    // small filters (the product's m = 1024): the batch ORed in LDS; a fresh
    // filter built by one block is written whole, without a fill first
    const bool store_all = f->known_zero && n <= cb::kInsertLdsOneBlock;
    if (store_all) {
      std::lock_guard<std::mutex> lk(f->zero_mu);
      f->needs_zero.store(false);
      f->needs_pad_zero.store(false);
    } else {
      HIP_TRY(ensure_zeroed(f, s));
    }
    HIP_TRY(cb::launch_insert_lds(sk.keyk, f->mode, f->words, f->m, f->nwords_alloc, sk.ks, n, f->mp, store_all, s));
  } else if (path == PATH_DIRECT) {
    HIP_TRY(ensure_zeroed(f, s));
    HIP_TRY(cb::launch_insert_direct(sk.keyk, f->mode, f->words, sk.ks, n, f->mp, s));
  } else {
    // a fresh tiled build writes every tile of [0, T * 2^tb): the words past
    // it are padding that no insert ever sets, so a pending clear is moot.
    if (f->known_zero) {
      if (f->needs_zero.exchange(false)) f->needs_pad_zero.store(true);
      HIP_TRY(ensure_pad_zeroed(f, s));  // tiles past ceil(m/32) may not all be rewritten
    } else {
      HIP_TRY(ensure_zeroed(f, s));
    }
    // chunks of at most 4096 partition blocks of the largest block size
    const uint64_t chunk = 4096ull * 256 * 16;
    for (uint64_t k0 = 0; k0 < n; k0 += chunk) {
      const uint64_t nk = std::min(chunk, n - k0);
      KeySrc ks = sk.ks;
      if (sk.keyk == cb::KEY_VAR)
        ks.offsets += k0;
      else
        ks.bytes += k0 * key_len;
      const int keyk = (sk.keyk == cb::KEY_FIXED16 && ((uintptr_t)ks.bytes & 15)) ? cb::KEY_FIXED
                                                                                   : sk.keyk;
      const TilePlan p = cb::plan_build(f->m, nk);
      if (!covers(f, p)) return fail(CB_EINVAL, "internal: build tile plan exceeds the filter allocation");
      HIP_TRY(ws.seg.reserve(cb::build_seg_bytes(p), s));
      HIP_TRY(ws.ent.reserve(cb::build_ent_bytes(p), s));
      HIP_TRY(cb::launch_build_tiled(keyk, f->mode, f->words, f->known_zero, ks, nk, f->mp, p,
                                     (uint32_t*)ws.seg.p, (uint32_t*)ws.ent.p, s));
      f->known_zero = false;
    }
  }
  f->known_zero = false;
  int mrc = mark_written(f, s);
  if (mrc) return mrc;
  if (sk.staged) HIP_TRY(hipStreamSynchronize(s));
  return CB_OK;
}

int mark_written(cb_filter* f, hipStream_t s) {
  HIP_TRY(record_own_mark(f, s));
  f->gen.fetch_add(1, std::memory_order_acq_rel);
  return CB_OK;
}

int mark_written_many(Workspace& ws, cb_filter* const* fs, uint32_t nf, hipStream_t s) {
  if (!nf) return CB_OK;
  bool any_on = false;
  for (uint32_t i = 0; i < nf; ++i) any_on |= mirror_on(fs[i]);
  if (!any_on) {  // no mirror to order: flagged only (see record_own_mark)
    for (uint32_t i = 0; i < nf; ++i) {
      fs[i]->unmarked.store(true, std::memory_order_release);
      fs[i]->gen.fetch_add(1, std::memory_order_acq_rel);
    }
    return CB_OK;
  }
  std::shared_ptr<WriteMark> m;
  for (auto& c : ws.marks)
    if (c.use_count() == 1) {  // only the pool holds it: no filter, no waiting refresh
      m = c;
      break;
    }
  if (!m) {
    HIP_TRY(make_mark(&m));
    ws.marks.push_back(m);
  }
  HIP_TRY(hipEventRecord(m->ev, s));
  for (uint32_t i = 0; i < nf; ++i) {
    std::atomic_store(&fs[i]->wmark, m);
    fs[i]->gen.fetch_add(1, std::memory_order_acq_rel);
  }
  return CB_OK;
}

}  // namespace cbx

namespace {

int insert_impl(cb_filter* f, const uint8_t* keys, const uint64_t* offsets, uint32_t key_len,
                uint64_t n, hipStream_t s) {
  if (!f) return fail(CB_EINVAL, "null filter");
  if (n == 0) return CB_OK;  // no hashes() call in the reference: no panic
  if (f->m == 0) return fail(CB_EZEROM, "attempt to calculate the remainder with a divisor of zero");
  if (offsets == nullptr && keys == nullptr && key_len) return fail(CB_EINVAL, "null keys");
  DeviceGuard dg(f->device);
  Workspace& ws = workspace(f->device, s);
  std::lock_guard<std::mutex> lk(ws.mu);
  return insert_locked(ws, f, keys, offsets, key_len, n, s);
}

int probe_impl(const cb_filter* const* filters, uint32_t nf, const uint8_t* keys,
               const uint64_t* offsets, uint32_t key_len, uint64_t n, uint64_t* hits,
               hipStream_t s) {
  if (nf == 0 || n == 0) return CB_OK;
  if (!filters || !hits) return fail(CB_EINVAL, "null filters or hits");
  for (uint32_t i = 0; i < nf; ++i) {
    if (!filters[i]) return fail(CB_EINVAL, "null filter");
    if (filters[i]->device != filters[0]->device)
      return fail(CB_EINVAL, "all filters of one probe must live on one device");
    if (filters[i]->m == 0)
      return fail(CB_EZEROM, "attempt to calculate the remainder with a divisor of zero");
  }
  for (uint32_t i = 0; i < nf; ++i) HIP_TRY(ensure_zeroed(filters[i], s));
  if (offsets == nullptr && keys == nullptr && key_len) return fail(CB_EINVAL, "null keys");
  const int dev = filters[0]->device;
  DeviceGuard dg(dev);
  Workspace& ws = workspace(dev, s);
  std::lock_guard<std::mutex> lk(ws.mu);
  StagedKeys sk;
  int rc = offsets ? stage_var(ws, keys, offsets, n, s, sk)
                   : stage_fixed(ws, keys, key_len, n, s, sk);
  if (rc) return rc;

  const uint64_t hwords = (n + 63) / 64;
  uint64_t* dhits = hits;
  const bool host_hits = !is_device_ptr(hits);
  if (host_hits) {
    HIP_TRY(ws.hits.reserve((size_t)nf * hwords * 8, s));
    dhits = (uint64_t*)ws.hits.p;
  }

  // Group filters by m (positions depend only on m), preserving hit rows.
  std::map<uint64_t, std::vector<uint32_t>> groups;
  for (uint32_t i = 0; i < nf; ++i) groups[filters[i]->m].push_back(i);

  int last_path = PATH_DIRECT;
  for (auto& kv : groups) {
    const uint64_t m = kv.first;
    const std::vector<uint32_t>& idx = kv.second;
    const cb_filter* f0 = filters[idx[0]];
    const int path = choose_probe_path(m, n, (uint32_t)idx.size());
    last_path = path;
    if (path == PATH_DIRECT) {
      for (size_t g0 = 0; g0 < idx.size(); g0 += cb::kMaxFiltersPerLaunch) {
        FilterPtrs fp{};
        const uint32_t cnt = (uint32_t)std::min<size_t>(cb::kMaxFiltersPerLaunch, idx.size() - g0);
        for (uint32_t j = 0; j < cnt; ++j) {
          fp.w[j] = filters[idx[g0 + j]]->words;
          fp.row[j] = idx[g0 + j];
        }
        HIP_TRY(cb::launch_probe_direct(sk.keyk, f0->mode, fp, cnt, sk.ks, n, f0->mp, dhits,
                                        hwords, s));
      }
    } else {
      const uint64_t chunk = 4096ull * 256 * 8;  // keys per partition pass (multiple of 64)
      for (uint64_t k0 = 0; k0 < n; k0 += chunk) {
        const uint64_t nk = std::min(chunk, n - k0);
        KeySrc ks = sk.ks;
        if (sk.keyk == cb::KEY_VAR)
          ks.offsets += k0;
        else
          ks.bytes += k0 * key_len;
        const int keyk = (sk.keyk == cb::KEY_FIXED16 && ((uintptr_t)ks.bytes & 15))
                             ? cb::KEY_FIXED
                             : sk.keyk;
        const TilePlan p = cb::plan_probe(m, nk);
        for (uint32_t i : idx)
          if (!covers(filters[i], p))
            return fail(CB_EINVAL, "internal: probe tile plan exceeds the filter allocation");
        HIP_TRY(ws.seg.reserve(cb::probe_seg_bytes(p), s));
        HIP_TRY(ws.ent.reserve(cb::probe_ent_bytes(p), s));
        HIP_TRY(ws.masks.reserve((size_t)2 * nk * 4, s));
        HIP_TRY(ws.lkey.reserve(cb::probe_lkey_bytes(p), s));
        HIP_TRY(cb::launch_probe_partition(keyk, f0->mode, ks, nk, f0->mp, p, (uint32_t*)ws.seg.p,
                                           (uint2*)ws.ent.p, (uint16_t*)ws.lkey.p, s));
        for (size_t g0 = 0; g0 < idx.size(); g0 += cb::kMaxFiltersPerLaunch) {
          FilterPtrs fp{};
          const uint32_t cnt =
              (uint32_t)std::min<size_t>(cb::kMaxFiltersPerLaunch, idx.size() - g0);
          for (uint32_t j = 0; j < cnt; ++j) {
            fp.w[j] = filters[idx[g0 + j]]->words;
            fp.row[j] = idx[g0 + j];
          }
          HIP_TRY(cb::launch_probe_tiles(fp, cnt, nk, p, (const uint32_t*)ws.seg.p,
                                         (const uint2*)ws.ent.p, (const uint16_t*)ws.lkey.p,
                                         (uint32_t*)ws.masks.p, dhits + k0 / 64, hwords, s));
        }
      }
    }
  }
  g_last_path = last_path;
  if (host_hits) {
    HIP_TRY(hipMemcpyAsync(hits, dhits, (size_t)nf * hwords * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  } else if (sk.staged) {
    HIP_TRY(hipStreamSynchronize(s));
  }
  return CB_OK;
}

bool is_pinned_host(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t attr;
  hipError_t e = hipPointerGetAttributes(&attr, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeHost;
}

// Pinned host keys in, pinned host hits out (the query layer's buffers,
// SURVEY.md §8d end-to-end leg): the probe kernel itself loads the keys over
// PCIe and stores the hit rows over PCIe (zero-copy; pinned memory is mapped
// into the device's address space), so the two PCIe directions overlap each
// other and the HBM gathers inside ONE launch. Measured on this stack
// (tools/ubench_pcie.hip): chunked pipelines across copy streams cost more
// per cross-stream event than they overlap (4 chunks, 3 streams: 0.87 ms vs
// 0.50 ms on one stream), while kernel loads from pinned memory run at
// 43-46 GB/s and kernel stores to it at 53 GB/s, the copy engines' rates.
int set_probe_zero_copy(const cb_filterset* set, const uint8_t* keys, uint32_t key_len, uint64_t n,
                        uint64_t* hits, hipStream_t s, const cb::ZoneView* zv) {
  void *dk = nullptr, *dh = nullptr;
  HIP_TRY(hipHostGetDevicePointer(&dk, const_cast<uint8_t*>(keys), 0));
  HIP_TRY(hipHostGetDevicePointer(&dh, hits, 0));
  const int keyk = (key_len == 16 && !((uintptr_t)dk & 15)) ? cb::KEY_FIXED16 : cb::KEY_FIXED;
  cb::KeySrc ks{(const uint8_t*)dk, nullptr, key_len};
  if (set_is_wide(set)) {
    const cb::WideZone wz = wide_zone_view(set);
    HIP_TRY(cb::launch_wide_probe(keyk, set->mode, set->R, (const uint64_t*)set->words, set->used, ks, n, set->mp,
                                  zv ? &wz : nullptr, (uint64_t*)dh, (n + 63) / 64, s));
  } else {
    HIP_TRY(cb::launch_set_probe(keyk, set->mode, set->width, set->words, set->any, set->used, ks, n,
                                 set->mp, zv, (uint64_t*)dh, (n + 63) / 64, s));
  }
  HIP_TRY(hipStreamSynchronize(s));  // the table is no longer read: no reader event needed
  return CB_OK;
}

// The dense set probe (densefs.hip) for this batch? cb_set_dense: 0 auto (by
// density), 1 whenever the shape allows it, -1 never. Never with the zone gate
// or a fused exchange pack.
std::atomic<int> g_set_dense{0};

bool use_dense(const cb_filterset* set, uint64_t n, bool gated, bool pack) {
  const int mode = g_set_dense.load(std::memory_order_relaxed);
  if (mode < 0 || gated || pack || set_is_wide(set)) return false;
  if (mode > 0) return cb::set_dense_shape_ok(set->width, set->m);
  return cb::set_probe_dense_ok(set->width, set->m, n);
}

int dense_probe(Workspace& ws, const cb_filterset* set, int keyk, const cb::KeySrc& ks, uint64_t n,
                uint64_t* hits, uint64_t hwords, hipStream_t s) {
  HIP_TRY(ws.dense.reserve(cb::dense_scratch_bytes(set->width, set->m, n), s));
  HIP_TRY(cb::launch_set_probe_dense(keyk, set->mode, set->width, set->words, set->used, ks, n, set->mp, hits, hwords,
                                     ws.dense.p, s));
  g_last_path = 6;
  return CB_OK;
}

int set_probe_impl(const cb_filterset* set, const uint8_t* keys, const uint64_t* offsets,
                   uint32_t key_len, uint64_t n, uint64_t* hits, hipStream_t s, bool gated) {
  if (!set) return fail(CB_EINVAL, "null set");
  if (n == 0 || set->used == 0) return CB_OK;
  if (!hits) return fail(CB_EINVAL, "null hits");
  if (offsets == nullptr && keys == nullptr && key_len) return fail(CB_EINVAL, "null keys");
  DeviceGuard dg(set->device);
  Workspace& ws = workspace(set->device, s);
  std::lock_guard<std::mutex> lk(ws.mu);
  const cb::ZoneView zv = set_zone_view(set);
  if (!offsets && key_len && is_pinned_host(keys) && is_pinned_host(hits)) {
    g_last_path = 4;
    return set_probe_zero_copy(set, keys, key_len, n, hits, s, (gated && set->zany) ? &zv : nullptr);
  }
  StagedKeys sk;
  int rc = offsets ? stage_var(ws, keys, offsets, n, s, sk)
                   : stage_fixed(ws, keys, key_len, n, s, sk);
  if (rc) return rc;
  const uint64_t hwords = (n + 63) / 64;
  uint64_t* dhits = hits;
  const bool host_hits = !is_device_ptr(hits);
  if (host_hits) {
    HIP_TRY(ws.hits.reserve((size_t)set->used * hwords * 8, s));
    dhits = (uint64_t*)ws.hits.p;
  }
  const bool dense = use_dense(set, n, gated && set->zany, false);
  if (set_is_wide(set)) {
    const cb::WideZone wz = wide_zone_view(set);
    HIP_TRY(cb::launch_wide_probe(sk.keyk, set->mode, set->R, (const uint64_t*)set->words, set->used, sk.ks, n,
                                  set->mp, (gated && set->zany) ? &wz : nullptr, dhits, hwords, s));
  } else if (dense) {
    if ((rc = dense_probe(ws, set, sk.keyk, sk.ks, n, dhits, hwords, s))) return rc;
  } else {
    HIP_TRY(cb::launch_set_probe(sk.keyk, set->mode, set->width, set->words, set->any, set->used,
                                 sk.ks, n, set->mp, (gated && set->zany) ? &zv : nullptr, dhits,
                                 hwords, s));
  }
  if (gated && set->zany) {
    int zr = note_zone_read(set, s);
    if (zr) return zr;
  }
  if (!dense) g_last_path = 3;
  if (host_hits) {
    HIP_TRY(hipMemcpyAsync(hits, dhits, (size_t)set->used * hwords * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  } else if (sk.staged) {
    HIP_TRY(hipStreamSynchronize(s));
  }
  return CB_OK;
}

}  // namespace

namespace cbx {

int set_probe_device(const cb_filterset* set, const uint8_t* keys, uint32_t key_len, uint64_t n, bool gated,
                     uint64_t* hits, uint32_t* sink_pack, uint64_t cap, hipStream_t s) {
  if (!set) return fail(CB_EINVAL, "null set");
  if (!n || !set->used) {
    if (sink_pack) {  // no rows or no keys: an empty pack (count 0, every directory entry empty)
      DeviceGuard dg(set->device);
      HIP_TRY(hipMemsetAsync(sink_pack, 0, 8, s));
      if (n) HIP_TRY(hipMemsetAsync(sink_pack + 2 + cap, 0, 8 * cb::set_probe_blocks(n), s));
    }
    return CB_OK;
  }
  if (!hits || (!keys && key_len)) return fail(CB_EINVAL, "null argument");
  if (!is_device_ptr(hits) || (key_len && !is_device_ptr(keys)) || (sink_pack && !is_device_ptr(sink_pack)))
    return fail(CB_EINVAL, "keys, hits and pack must be device memory");
  const uint64_t hwords = (n + 63) / 64;
  if (sink_pack && set_is_wide(set))
    return fail(CB_EINVAL, "the fused probe + pack takes sets of at most 64 slots");
  if (sink_pack && (uint64_t)set->used * hwords * 64 >= (1ull << 32))
    return fail(CB_EINVAL, "used * ceil(n/64) * 64 must be below 2^32 (u32 positions and counts)");
  DeviceGuard dg(set->device);
  Workspace& ws = workspace(set->device, s);
  std::lock_guard<std::mutex> lk(ws.mu);
  const cb::ZoneView zv = set_zone_view(set);
  const int keyk = (key_len == 16 && !((uintptr_t)keys & 15)) ? cb::KEY_FIXED16 : cb::KEY_FIXED;
  const cb::KeySrc ks{keys, nullptr, key_len};
  cb::PackSink sink{};
  cb::CompressState* st = nullptr;
  if (sink_pack) {
    int rc = compress_state(ws, s, &st);
    if (rc) return rc;
    sink = cb::PackSink{sink_pack, cap, reinterpret_cast<unsigned long long*>(st->ctl), st->parity};
  }
  hipError_t e;
  if (use_dense(set, n, gated && set->zany, sink_pack != nullptr)) {
    return dense_probe(ws, set, keyk, ks, n, hits, hwords, s);
  } else if (set_is_wide(set)) {
    const cb::WideZone wz = wide_zone_view(set);
    e = cb::launch_wide_probe(keyk, set->mode, set->R, (const uint64_t*)set->words, set->used, ks, n, set->mp,
                              (gated && set->zany) ? &wz : nullptr, hits, hwords, s);
  } else {
    e = cb::launch_set_probe(keyk, set->mode, set->width, set->words, set->any, set->used, ks, n, set->mp,
                             (gated && set->zany) ? &zv : nullptr, hits, hwords, s, sink_pack ? &sink : nullptr);
  }
  if (e != hipSuccess) {
    // the kernel may still have been queued (an earlier sticky error): clear
    // both claim words behind it, so the next launch never reuses a dirty one
    if (st) (void)hipMemsetAsync(st->ctl, 0, 16, s);
    return hip_fail(e, "launch_set_probe");
  }
  if (st) st->parity ^= 1u;  // the launch cleared the other claim word for the next one
  g_last_path = 3;
  if (gated && set->zany) return note_zone_read(set, s);
  return CB_OK;
}

int note_zone_read(const cb_filterset* set, hipStream_t s) {
  std::lock_guard<std::mutex> lk(set->zmu);
  hipEvent_t& ev = set->zread[s];
  // The event only tells the host that the readers of the zone table are done
  // (they never write it), so it needs no system-scope release: without the
  // cache write-back an event costs the stream little GPU time.
  if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventDisableSystemFence));
  HIP_TRY(hipEventRecord(ev, s));
  return CB_OK;
}

}  // namespace cbx

namespace {

// Rebuild and upload the set's zone table (cb::ZoneView layout). Called on
// zone updates, which happen once per table flush: the upload is ordered on
// stream s and waited for, so the host staging vector can be reused.
int upload_zones(cb_filterset* set, hipStream_t s) {
  // layout: 32/64-slot sets cb::ZoneView (64 headers, 128 prefixes, blob);
  // wide sets cb::WideZone (W headers, 2 W prefixes, the gated bits, blob)
  const bool wide = set_is_wide(set);
  const uint32_t nslot = wide ? set->width : 64;
  const size_t hdr_bytes = wide ? wide_zone_hdr_bytes(nslot) : cb_zone_hdr_bytes;
  const size_t pre_bytes = wide ? wide_zone_pre_bytes(nslot) : cb_zone_pre_bytes;
  const size_t blob_off = wide ? wide_zone_blob_off(nslot) : cb_zone_blob_off;
  std::vector<uint32_t> hdr((size_t)nslot * 4, 0u);
  std::vector<cb::BoundPrefix> pre((size_t)nslot * 2);
  std::memset(pre.data(), 0, pre.size() * sizeof(cb::BoundPrefix));
  std::vector<uint8_t> blob;
  set->zg.assign(std::max<uint32_t>(1, set->width / 64), 0ull);
  set->zany = false;
  for (uint32_t i = 0; i < set->width; ++i) {
    if (!(set->zhas_lo[i] && set->zhas_hi[i])) continue;
    set->zg[i >> 6] |= 1ull << (i & 63);
    set->zany = true;
    hdr[4 * i + 0] = (uint32_t)blob.size();
    hdr[4 * i + 1] = (uint32_t)set->zlo[i].size();
    blob.insert(blob.end(), set->zlo[i].begin(), set->zlo[i].end());
    hdr[4 * i + 2] = (uint32_t)blob.size();
    hdr[4 * i + 3] = (uint32_t)set->zhi[i].size();
    blob.insert(blob.end(), set->zhi[i].begin(), set->zhi[i].end());
    // big-endian 16-byte prefixes of both bounds (cb::cmp16's operands)
    for (int j = 0; j < 2; ++j) {
      const std::string& bnd = j ? set->zhi[i] : set->zlo[i];
      cb::BoundPrefix& p = pre[2 * i + j];
      for (size_t k = 0; k < bnd.size() && k < 16; ++k)
        p.w[k >> 2] |= (uint32_t)(uint8_t)bnd[k] << (24 - 8 * (k & 3));
      p.len = (uint32_t)bnd.size();
    }
  }
  set->zgated = wide ? 0 : set->zg[0];
  std::vector<uint8_t> tab(blob_off + blob.size());
  memcpy(tab.data(), hdr.data(), hdr_bytes);
  memcpy(tab.data() + hdr_bytes, pre.data(), pre_bytes);
  if (wide) memcpy(tab.data() + hdr_bytes + pre_bytes, set->zg.data(), set->zg.size() * 8);
  if (!blob.empty()) memcpy(tab.data() + blob_off, blob.data(), blob.size());
  if (!set->zany) return CB_OK;
  // A gated probe or fused read queued on another stream may still read the
  // old table: wait for every stream's last reader (their events), not the
  // whole device, before overwriting it. An outgrown table is retired, not
  // freed (hipFree would synchronise the device), until cb_set_destroy.
  {
    std::lock_guard<std::mutex> lk(set->zmu);
    for (auto& kv : set->zread) HIP_TRY(hipEventSynchronize(kv.second));
  }
  if (tab.size() > set->zcap) {
    if (set->zdev) set->zretired.push_back(set->zdev);
    set->zdev = nullptr;
    set->zcap = 0;
    const size_t want = (tab.size() * 2 + 4095) & ~size_t(4095);
    if (hipMalloc(&set->zdev, want) != hipSuccess) {
      (void)hipGetLastError();
      set->zgated = 0;
      set->zany = false;
      return fail(CB_ENOMEM, "hipMalloc failed for zone table");
    }
    set->zcap = want;
  }
  HIP_TRY(hipMemcpyAsync(set->zdev, tab.data(), tab.size(), hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  return CB_OK;
}

// A slot that receives another table's filter starts with no zone map
// (accept-all), so a stale zone can never hide a key. Headers of ungated
// slots are never read, so no upload is needed.
bool reset_zone(cb_filterset* set, uint32_t slot) {
  const bool was = (slot >> 6) < set->zg.size() && ((set->zg[slot >> 6] >> (slot & 63)) & 1ull);
  set->zlo[slot].clear();
  set->zhi[slot].clear();
  set->zhas_lo[slot] = set->zhas_hi[slot] = 0;
  if (slot < 64) set->zgated &= ~(1ull << slot);
  if ((slot >> 6) < set->zg.size()) set->zg[slot >> 6] &= ~(1ull << (slot & 63));
  bool any = false;
  for (uint64_t w : set->zg) any |= w != 0;
  set->zany = any;
  return was;
}

// After zone resets: a wide set's kernels read the gated bits from its device
// table (a 32/64-slot set passes them by value), so a reset slot that was
// gated needs a new table before the next gated launch.
int zones_after_reset(cb_filterset* set, bool changed, hipStream_t s) {
  if (!changed || !set_is_wide(set)) return CB_OK;
  return upload_zones(set, s);
}

bool slot_dirty(const cb_filterset* set, uint32_t slot) { return (set->dirty[slot >> 6] >> (slot & 63)) & 1ull; }

// Bytes of key i of a staged batch (device-resident) into out.
int fetch_key(const StagedKeys& sk, uint64_t i, std::string& out, hipStream_t s) {
  uint64_t o[2];
  if (sk.keyk == cb::KEY_VAR) {
    HIP_TRY(hipMemcpyAsync(o, sk.ks.offsets + i, 16, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  } else {
    o[0] = i * sk.ks.key_len;
    o[1] = o[0] + sk.ks.key_len;
  }
  out.assign((size_t)(o[1] - o[0]), '\0');
  if (o[1] > o[0]) {
    HIP_TRY(hipMemcpyAsync(&out[0], sk.ks.bytes + o[0], (size_t)(o[1] - o[0]),
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  }
  return CB_OK;
}

int zone_bounds_impl(int device, const uint8_t* keys, const uint64_t* offsets, uint32_t key_len,
                     uint64_t n, hipStream_t s, uint64_t* min_idx, uint64_t* max_idx,
                     std::string* lo, std::string* hi) {
  if (min_idx) *min_idx = ~0ull;
  if (max_idx) *max_idx = ~0ull;
  if (n == 0) return CB_OK;
  if (offsets == nullptr && keys == nullptr && key_len) return fail(CB_EINVAL, "null keys");
  int rc = cb_init(device);
  if (rc) return rc;
  DeviceGuard dg(device);
  Workspace& ws = workspace(device, s);
  std::lock_guard<std::mutex> lk(ws.mu);
  StagedKeys sk;
  rc = offsets ? stage_var(ws, keys, offsets, n, s, sk) : stage_fixed(ws, keys, key_len, n, s, sk);
  if (rc) return rc;
  HIP_TRY(ws.zone.reserve((2 * 1024 + 2) * 8, s));
  uint64_t* dtmp = (uint64_t*)ws.zone.p;
  uint64_t* didx = dtmp + 2 * 1024;
  HIP_TRY(cb::launch_zone_bounds(sk.keyk, sk.ks, n, dtmp, didx, s));
  uint64_t idx[2];
  HIP_TRY(hipMemcpyAsync(idx, didx, 16, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (min_idx) *min_idx = idx[0];
  if (max_idx) *max_idx = idx[1];
  if (lo && (rc = fetch_key(sk, idx[0], *lo, s))) return rc;
  if (hi && (rc = fetch_key(sk, idx[1], *hi, s))) return rc;
  return CB_OK;
}

// ---- prost codec helpers (product side; see DESIGN.md "Persistence") ----

uint64_t varint_len(uint64_t v) {
  uint64_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}

bool get_varint(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
  uint64_t r = 0;
  for (int i = 0; i < 10; ++i) {
    if (p >= end) return false;
    const uint8_t b = *p++;
    if (i == 9 && b > 1) return false;  // prost: overflowing varint
    r |= (uint64_t)(b & 0x7F) << (7 * i);
    if (!(b & 0x80)) {
      v = r;
      return true;
    }
  }
  return false;
}

bool skip_field(const uint8_t*& p, const uint8_t* end, uint32_t wt, uint64_t field, int depth);

bool skip_group(const uint8_t*& p, const uint8_t* end, uint64_t field, int depth) {
  if (depth > 100) return false;
  for (;;) {
    uint64_t key;
    if (!get_varint(p, end, key) || key > 0xFFFFFFFFull) return false;
    const uint32_t wt = (uint32_t)(key & 7);
    const uint64_t fn = key >> 3;
    if (fn == 0) return false;
    if (wt == 4) return fn == field;
    if (!skip_field(p, end, wt, fn, depth + 1)) return false;
  }
}

bool skip_field(const uint8_t*& p, const uint8_t* end, uint32_t wt, uint64_t field, int depth) {
  uint64_t v;
  switch (wt) {
    case 0: return get_varint(p, end, v);
    case 1:
      if (end - p < 8) return false;
      p += 8;
      return true;
    case 2:
      if (!get_varint(p, end, v) || v > (uint64_t)(end - p)) return false;
      p += v;
      return true;
    case 3: return skip_group(p, end, field, depth);
    case 5:
      if (end - p < 4) return false;
      p += 4;
      return true;
    default: return false;
  }
}

// 0x0A varint(m): the BloomProto header written before m 0/1 bytes.
size_t put_bloom_header(uint8_t* p, uint64_t m) {
  size_t n = 0;
  p[n++] = 0x0A;  // field 1 (bits), wire type 2 (packed)
  while (m >= 0x80) {
    p[n++] = (uint8_t)(m | 0x80);
    m >>= 7;
  }
  p[n++] = (uint8_t)m;
  return n;
}

size_t put_varint_buf(uint8_t* p, uint64_t v) {
  size_t n = 0;
  while (v >= 0x80) {
    p[n++] = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  p[n++] = (uint8_t)v;
  return n;
}

// Rust's str::from_utf8 acceptance (prost rejects a `string` field that is
// not well-formed UTF-8). Classifies each lead byte by its range and checks
// the tightened second-byte window that rules out overlongs, surrogates and
// code points above U+10FFFF.
bool utf8_ok(const uint8_t* p, uint64_t n) {
  const uint8_t* end = p + n;
  while (p < end) {
    const uint8_t c = *p;
    if (c < 0x80) {
      ++p;
      continue;
    }
    int need;
    uint8_t lo = 0x80, hi = 0xBF;
    switch (c >> 4) {
      case 0xC:
      case 0xD:
        if (c < 0xC2) return false;
        need = 1;
        break;
      case 0xE:
        need = 2;
        if (c == 0xE0) lo = 0xA0;
        if (c == 0xED) hi = 0x9F;
        break;
      case 0xF:
        if (c > 0xF4) return false;
        need = 3;
        if (c == 0xF0) lo = 0x90;
        if (c == 0xF4) hi = 0x8F;
        break;
      default:
        return false;  // stray continuation byte
    }
    if (end - p <= need) return false;
    if (p[1] < lo || p[1] > hi) return false;
    for (int k = 2; k <= need; ++k)
      if ((p[k] & 0xC0) != 0x80) return false;
    p += need + 1;
  }
  return true;
}

// One pass over a TableMeta message: the spans of every `bloom` (field 1)
// occurrence, and the last `min` / `max` of every `zone_map` (field 2)
// occurrence — prost's merge of a repeated singular message field is the
// decode of the concatenated payloads, so bloom spans are concatenated and
// zone strings are last-wins.
struct MetaScan {
  std::vector<std::pair<const uint8_t*, uint64_t>> bloom;
  bool has_zone = false, has_min = false, has_max = false;
  const uint8_t *min = nullptr, *max = nullptr;
  uint64_t min_len = 0, max_len = 0;
};

int scan_zone(const uint8_t* p, const uint8_t* end, MetaScan& ms) {
  while (p < end) {
    uint64_t key, l;
    if (!get_varint(p, end, key) || key > 0xFFFFFFFFull)
      return fail(CB_EDECODE, "ZoneMapProto decode: invalid key");
    const uint32_t wt = (uint32_t)(key & 7);
    const uint64_t fn = key >> 3;
    if (fn == 0) return fail(CB_EDECODE, "ZoneMapProto decode: invalid tag value 0");
    if (fn == 1 || fn == 2) {
      if (wt != 2) return fail(CB_EDECODE, "ZoneMapProto decode: invalid wire type");
      if (!get_varint(p, end, l) || l > (uint64_t)(end - p))
        return fail(CB_EDECODE, "ZoneMapProto decode: bad length");
      if (!utf8_ok(p, l)) return fail(CB_EDECODE, "ZoneMapProto decode: invalid string value: data is not UTF-8 encoded");
      if (fn == 1) {
        ms.min = p;
        ms.min_len = l;
        ms.has_min = true;
      } else {
        ms.max = p;
        ms.max_len = l;
        ms.has_max = true;
      }
      p += l;
    } else if (!skip_field(p, end, wt, fn, 0)) {
      return fail(CB_EDECODE, "ZoneMapProto decode: malformed unknown field");
    }
  }
  return CB_OK;
}

int scan_meta(const uint8_t* in, uint64_t len, MetaScan& ms) {
  const uint8_t* p = in;
  const uint8_t* end = in + len;
  while (p < end) {
    uint64_t key, l;
    if (!get_varint(p, end, key) || key > 0xFFFFFFFFull)
      return fail(CB_EDECODE, "TableMeta decode: invalid key");
    const uint32_t wt = (uint32_t)(key & 7);
    const uint64_t fn = key >> 3;
    if (fn == 0) return fail(CB_EDECODE, "TableMeta decode: invalid tag value 0");
    if (fn == 1 || fn == 2) {
      if (wt != 2) return fail(CB_EDECODE, "TableMeta decode: invalid wire type");
      if (!get_varint(p, end, l) || l > (uint64_t)(end - p))
        return fail(CB_EDECODE, "TableMeta decode: bad length");
      if (fn == 1) {
        ms.bloom.emplace_back(p, l);
      } else {
        ms.has_zone = true;
        int rc = scan_zone(p, p + l, ms);
        if (rc) return rc;
      }
      p += l;
    } else if (!skip_field(p, end, wt, fn, 0)) {
      return fail(CB_EDECODE, "TableMeta decode: malformed unknown field");
    }
  }
  return CB_OK;
}

}  // namespace

extern "C" {

const char* cb_last_error(void) { return g_err.c_str(); }
const char* cb_version(void) { return "cassbloom 0.1.0 (gfx950)"; }
int cb_set_path(int path) {
  if (path < 0 || path > 2) return fail(CB_EINVAL, "path must be 0, 1 or 2");
  g_path_override = path;
  return CB_OK;
}
int cb_last_path(void) { return g_last_path; }
int cb_set_dense(int mode) {
  if (mode < -1 || mode > 1) return fail(CB_EINVAL, "mode must be -1, 0 or 1");
  g_set_dense.store(mode, std::memory_order_relaxed);
  return CB_OK;
}

int cb_device_count(int* out) {
  if (!out) return fail(CB_EINVAL, "null out");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *out = 0;
    return fail(CB_ENODEV, "no HIP device");
  }
  *out = n;
  return CB_OK;
}

int cb_init(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    (void)hipGetLastError();
    return fail(CB_ENODEV, "no HIP device");
  }
  if (device < 0 || device >= n) return fail(CB_ENODEV, "device index out of range");
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(CB_ENODEV, "device is not gfx950 (MI355X); this library carries gfx950 code only");
  // No hipSetDevice here: the calling thread's current device is left as it
  // was (entry points that work on `device` switch under a DeviceGuard, which
  // restores the caller's device on return).
  return CB_OK;
}

int cb_stream_synchronize(void* stream) {
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return CB_OK;
}

int cb_stream_release(void* stream) {
  std::vector<std::pair<int, std::unique_ptr<Workspace>>> mine;
  {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    for (auto it = g_ws.begin(); it != g_ws.end();) {
      if (it->first.second == stream) {
        mine.emplace_back(it->first.first, std::move(it->second));
        it = g_ws.erase(it);
      } else {
        ++it;
      }
    }
  }
  if (mine.empty()) return CB_OK;
  // its queued work may still use the workspace's buffers (and, from here
  // on, releases record no event on it)
  int rc = CB_OK;
  const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
  if (e != hipSuccess) rc = hip_fail(e, "cb_stream_release: hipStreamSynchronize");
  for (auto& w : mine) {
    DeviceGuard dg(w.first);
    std::lock_guard<std::mutex> wl(w.second->mu);  // a call still inside it finishes first
    workspace_free(*w.second);
  }
  return rc;
}

int cb_hits_compress(const uint64_t* hits, uint64_t rows, uint64_t words, uint32_t* pack,
                     uint64_t cap, void* stream) {
  if (!pack || (rows * words && !hits)) return fail(CB_EINVAL, "null argument");
  if (rows && words && (words > cb::kMaxCompressWords || rows * words > cb::kMaxCompressWords))
    return fail(CB_EINVAL, "rows * words * 64 must be below 2^32");
  hipStream_t s = (hipStream_t)stream;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  Workspace& ws = workspace(dev, s);
  std::lock_guard<std::mutex> lk(ws.mu);
  cb::CompressState* st = nullptr;
  int rc = compress_state(ws, s, &st);
  if (rc) return rc;
  HIP_TRY(cb::launch_hits_compress(hits, rows, words, pack, cap, *st, s));
  return CB_OK;
}

int cb_hits_expand(const uint32_t* packs, uint32_t nranks, uint64_t cap, const uint64_t* row_off,
                   uint64_t words, uint64_t total_rows, uint64_t* full, uint32_t* ok, void* stream) {
  if (!full || (nranks && (!packs || !row_off))) return fail(CB_EINVAL, "null argument");
  if (nranks > cb::kMaxRanks) return fail(CB_EINVAL, "more than 64 ranks");
  cb::RankRows rr{};
  for (uint32_t r = 0; r < nranks; ++r) {
    rr.row_off[r] = row_off[r];
    const uint64_t end = r + 1 < nranks ? row_off[r + 1] : total_rows;
    if ((r == 0 && row_off[0] != 0) || end < row_off[r] || end > total_rows)
      return fail(CB_EINVAL, "row_off must start at 0 and be non-decreasing up to total_rows");
    if ((end - row_off[r]) * words > cb::kMaxCompressWords)
      return fail(CB_EINVAL, "a rank's rows * words * 64 must be below 2^32");
  }
  HIP_TRY(cb::launch_hits_expand(packs, nranks, cap, rr, words, total_rows, full, ok, (hipStream_t)stream));
  return CB_OK;
}

int cb_hits_pack_words(uint64_t rows, uint64_t words, uint64_t cap, uint64_t* out) {
  if (!out) return fail(CB_EINVAL, "null out");
  *out = cb::pack_words(rows * words, cap);
  return CB_OK;
}

int cb_set_pack_words(uint64_t n, uint64_t cap, uint64_t* out) {
  if (!out) return fail(CB_EINVAL, "null out");
  *out = 2 + cap + 2 * cb::set_probe_blocks(n);
  return CB_OK;
}

int cb_set_probe_pack_fixed(const cb_filterset* set, const uint8_t* keys, uint32_t key_len, uint64_t n, int gated,
                            uint64_t* hits, uint32_t* pack, uint64_t cap, void* stream) {
  if (!pack) return fail(CB_EINVAL, "null pack");
  return set_probe_device(set, keys, key_len, n, gated != 0, hits, pack, cap, (hipStream_t)stream);
}

int cb_hits_expand_set(const uint32_t* packs, uint32_t nranks, uint64_t cap, const uint64_t* row_off, uint64_t n,
                       uint64_t total_rows, uint64_t* full, uint32_t* ok, void* stream) {
  if (!full || (nranks && (!packs || !row_off))) return fail(CB_EINVAL, "null argument");
  if (!nranks || nranks > cb::kMaxRanks) return fail(CB_EINVAL, "need 1..64 ranks");
  cb::RankRows rr{};
  for (uint32_t r = 0; r < nranks; ++r) rr.row_off[r] = row_off[r];
  const uint64_t nblk = cb::set_probe_blocks(n);
  const uint64_t stride = 2 + cap + 2 * nblk;
  hipError_t e = cb::launch_hits_expand_blocks(packs, nranks, cap, stride, rr, (n + 63) / 64, total_rows,
                                               (uint32_t)nblk, cb::kSetWords, full, ok, (hipStream_t)stream);
  if (e == hipErrorInvalidValue)
    return fail(CB_EINVAL, "row_off must start at 0 and grow to total_rows with at most 64 rows per rank");
  HIP_TRY(e);
  return CB_OK;
}

int cb_host_alloc(uint64_t bytes, void** out) {
  if (!out) return fail(CB_EINVAL, "null out");
  *out = nullptr;
  if (!bytes) return CB_OK;
  HIP_TRY(hipHostMalloc(out, bytes, hipHostMallocDefault));
  return CB_OK;
}

int cb_host_free(void* p) {
  if (p) HIP_TRY(hipHostFree(p));
  return CB_OK;
}

int cb_filter_create(uint64_t m_bits, int device, cb_filter** out) {
  if (!out) return fail(CB_EINVAL, "null out");
  *out = nullptr;
  int rc = cb_init(device);
  if (rc) return rc;
  DeviceGuard dg(device);
  std::unique_ptr<cb_filter> f(new cb_filter());
  f->m = m_bits;
  f->device = device;
  f->nwords_alloc = alloc_words_for(m_bits);
  if (m_bits) f->mp = cb::make_modp(m_bits, &f->mode);
  if (pool_alloc(device, f->nwords_alloc * 4, (void**)&f->words, &f->words_cap) != hipSuccess)
    return fail(CB_ENOMEM, "device allocation failed for filter words");
  // zero-filled lazily by the first operation that reads the words; a fresh
  // tiled build writes every tile and skips the fill (see ensure_zeroed)
  f->needs_zero.store(true);
  f->known_zero = true;
  *out = f.release();
  return CB_OK;
}

int cb_filter_destroy(cb_filter* f) {
  if (!f) return CB_OK;
  {
    DeviceGuard dg(f->device);
    pool_release(f->device, f->words, f->words_cap);
    std::atomic_store(&f->wmark, std::shared_ptr<WriteMark>());
  }
  delete f;
  return CB_OK;
}

int cb_filter_bits(const cb_filter* f, uint64_t* m_out) {
  if (!f || !m_out) return fail(CB_EINVAL, "null argument");
  *m_out = f->m;
  return CB_OK;
}

int cb_filter_device(const cb_filter* f, int* device_out) {
  if (!f || !device_out) return fail(CB_EINVAL, "null argument");
  *device_out = f->device;
  return CB_OK;
}

int cb_filter_words(const cb_filter* f, const uint32_t** words_out, uint64_t* nwords_out) {
  if (!f || !words_out || !nwords_out) return fail(CB_EINVAL, "null argument");
  if (f->needs_zero.load()) {
    DeviceGuard dg(f->device);
    HIP_TRY(ensure_zeroed(f, nullptr));
    HIP_TRY(hipStreamSynchronize(nullptr));
  }
  *words_out = f->words;
  *nwords_out = f->nwords_alloc;
  return CB_OK;
}

int cb_filter_clear(cb_filter* f, void* stream) {
  if (!f) return fail(CB_EINVAL, "null filter");
  (void)stream;
  f->known_zero = true;
  f->needs_zero.store(true);
  f->gen.fetch_add(1, std::memory_order_acq_rel);  // the mirror refresh sees needs_zero: all-zero words
  return CB_OK;
}

int cb_filter_host_mirror(cb_filter* f, int mode) {
  if (!f) return fail(CB_EINVAL, "null filter");
  if (mode < -1 || mode > 1) return fail(CB_EINVAL, "mode must be -1 (auto), 0 (off) or 1 (on)");
  f->mirror.store(mode, std::memory_order_relaxed);
  return CB_OK;
}

int cb_filter_host_mirror_info(const cb_filter* f, int* on, int* current) {
  if (!f) return fail(CB_EINVAL, "null filter");
  if (on) *on = mirror_on(f);
  if (current)
    *current = f->host_gen.load(std::memory_order_acquire) == f->gen.load(std::memory_order_acquire);
  return CB_OK;
}

int cb_filter_insert_fixed(cb_filter* f, const uint8_t* keys, uint32_t key_len, uint64_t n,
                           void* stream) {
  return insert_impl(f, keys, nullptr, key_len, n, (hipStream_t)stream);
}

int cb_filter_insert_var(cb_filter* f, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                         void* stream) {
  if (!offsets) return fail(CB_EINVAL, "null offsets");
  return insert_impl(f, bytes, offsets, 0, n, (hipStream_t)stream);
}

int cb_probe_fixed(const cb_filter* const* filters, uint32_t nf, const uint8_t* keys,
                   uint32_t key_len, uint64_t n, uint64_t* hits, void* stream) {
  return probe_impl(filters, nf, keys, nullptr, key_len, n, hits, (hipStream_t)stream);
}

int cb_probe_var(const cb_filter* const* filters, uint32_t nf, const uint8_t* bytes,
                 const uint64_t* offsets, uint64_t n, uint64_t* hits, void* stream) {
  if (!offsets) return fail(CB_EINVAL, "null offsets");
  return probe_impl(filters, nf, bytes, offsets, 0, n, hits, (hipStream_t)stream);
}

namespace {

// Refresh the host mirror if a write happened since it was taken: wait for
// the last write's event (on its own stream: no device-wide sync), then copy
// the words back once. Readers race only on the flag (acquire/release).
//
// A write made while the mirror was off recorded nothing (record_own_mark):
// the refresh that meets it waits for every stream the library has enqueued
// on for the device (wait_known_streams), by events, so a destroyed stream's
// handle never matters and streams the library never saw (the
// caller's other work) are not waited for.
int refresh_mirror(const cb_filter* cf) {
  cb_filter* f = const_cast<cb_filter*>(cf);
  const uint64_t g = f->gen.load(std::memory_order_acquire);
  if (f->host_gen.load(std::memory_order_acquire) == g) return CB_OK;
  std::lock_guard<std::mutex> lk(f->host_mu);
  const uint64_t g2 = f->gen.load(std::memory_order_acquire);
  if (f->host_gen.load(std::memory_order_acquire) == g2) return CB_OK;
  const uint64_t nw = (f->m + 31) / 32;
  f->host.resize(nw);
  {
    std::lock_guard<std::mutex> zl(f->zero_mu);  // a racing reader's lazy clear is issued and recorded, or not yet
    if (f->needs_zero.load()) {  // cleared, nothing on the device yet: all zero
      std::fill(f->host.begin(), f->host.end(), 0u);
    } else {
      DeviceGuard dg(f->device);
      // the last write's mark (every write to one filter is ordered by its
      // exclusive writer, so it covers them all): an event, not a stream, so
      // a stream destroyed since, or its handle reused, changes nothing
      if (f->unmarked.exchange(false, std::memory_order_acq_rel)) {
        int rc = wait_known_streams(f->device);
        if (rc) return rc;
      }
      const std::shared_ptr<WriteMark> m = std::atomic_load(&f->wmark);
      if (m) HIP_TRY(hipEventSynchronize(m->ev));
      HIP_TRY(hipMemcpy(f->host.data(), f->words, nw * 4, hipMemcpyDeviceToHost));
    }
  }
  f->host_gen.store(g2, std::memory_order_release);
  return CB_OK;
}

// BloomFilter::hashes + may_contain (src/bloom.rs:26-37,48-51) on the mirror:
// u64 wrapping x33 / x31 folds, h % m, and bit b read only when bit a is set.
int mirror_contains(const cb_filter* f, const uint8_t* key, uint64_t len) {
  uint64_t h1 = 5381, h2 = 0;
  for (uint64_t i = 0; i < len; ++i) {
    h1 = (h1 << 5) + h1 + key[i];
    h2 = h2 * 31 + key[i];
  }
  const uint64_t a = h1 % f->m, b = h2 % f->m;
  const uint32_t* w = f->host.data();
  return ((w[a >> 5] >> (a & 31)) & 1u) && ((w[b >> 5] >> (b & 31)) & 1u);
}

}  // namespace

int cb_may_contain(const cb_filter* f, const uint8_t* key, uint64_t len, int* out) {
  if (!f || !out || (!key && len)) return fail(CB_EINVAL, "null argument");
  if (f->m == 0) return fail(CB_EZEROM, "attempt to calculate the remainder with a divisor of zero");
  if (mirror_on(f)) {
    int rc = refresh_mirror(f);
    if (rc) return rc;
    *out = mirror_contains(f, key, len);
    g_last_path = 5;
    return CB_OK;
  }
  uint64_t offs[2] = {0, len};
  uint64_t hit = 0;
  const cb_filter* fs[1] = {f};
  int rc = probe_impl(fs, 1, key ? key : (const uint8_t*)"", offs, 0, 1, &hit, nullptr);
  if (rc) return rc;
  *out = (int)(hit & 1);
  return CB_OK;
}

int cb_filter_export_bools(const cb_filter* f, uint8_t* out, void* stream) {
  if (!f) return fail(CB_EINVAL, "null filter");
  if (f->m == 0) return CB_OK;
  if (!out) return fail(CB_EINVAL, "null out");
  hipStream_t s = (hipStream_t)stream;
  DeviceGuard dg(f->device);
  note_stream(f->device, s);
  HIP_TRY(ensure_zeroed(f, s));
  if (is_device_ptr(out)) {
    HIP_TRY(cb::launch_export_bools(f->words, f->m, out, s));
    return CB_OK;
  }
  Workspace& ws = workspace(f->device, s);
  std::lock_guard<std::mutex> lk(ws.mu);
  HIP_TRY(ws.bools.reserve(f->m, s));
  HIP_TRY(cb::launch_export_bools(f->words, f->m, (uint8_t*)ws.bools.p, s));
  HIP_TRY(hipMemcpyAsync(out, ws.bools.p, f->m, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return CB_OK;
}

int cb_filter_import_bools(cb_filter* f, const uint8_t* in, uint64_t m, void* stream) {
  if (!f) return fail(CB_EINVAL, "null filter");
  if (m != f->m) return fail(CB_EINVAL, "bool array length differs from the filter's m");
  if (m == 0) return CB_OK;
  if (!in) return fail(CB_EINVAL, "null input");
  hipStream_t s = (hipStream_t)stream;
  DeviceGuard dg(f->device);
  note_stream(f->device, s);
  if (is_device_ptr(in)) {
    HIP_TRY(cb::launch_import_bools(f->words, m, in, s));
  } else {
    Workspace& ws = workspace(f->device, s);
    std::lock_guard<std::mutex> lk(ws.mu);
    HIP_TRY(ws.bools.reserve(m, s));
    HIP_TRY(hipMemcpyAsync(ws.bools.p, in, m, hipMemcpyHostToDevice, s));
    HIP_TRY(cb::launch_import_bools(f->words, m, (const uint8_t*)ws.bools.p, s));
    HIP_TRY(hipStreamSynchronize(s));
  }
  if (f->needs_zero.exchange(false)) f->needs_pad_zero.store(true);
  HIP_TRY(ensure_pad_zeroed(f, s));  // every word < ceil(m/32) was rewritten
  f->known_zero = false;
  return mark_written(f, s);
}

int cb_filter_export_packed(const cb_filter* f, uint32_t* out, void* stream) {
  if (!f) return fail(CB_EINVAL, "null filter");
  const uint64_t nw = (f->m + 31) / 32;
  if (!nw) return CB_OK;
  if (!out) return fail(CB_EINVAL, "null out");
  hipStream_t s = (hipStream_t)stream;
  DeviceGuard dg(f->device);
  note_stream(f->device, s);
  HIP_TRY(ensure_zeroed(f, s));
  const bool dev = is_device_ptr(out);
  HIP_TRY(hipMemcpyAsync(out, f->words, nw * 4, dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                         s));
  if (!dev) HIP_TRY(hipStreamSynchronize(s));
  return CB_OK;
}

int cb_filter_import_packed(cb_filter* f, const uint32_t* in, uint64_t nwords, void* stream) {
  if (!f) return fail(CB_EINVAL, "null filter");
  const uint64_t nw = (f->m + 31) / 32;
  if (nwords != nw) return fail(CB_EINVAL, "word count differs from ceil(m/32)");
  if (!nw) return CB_OK;
  if (!in) return fail(CB_EINVAL, "null input");
  hipStream_t s = (hipStream_t)stream;
  DeviceGuard dg(f->device);
  note_stream(f->device, s);
  const bool dev = is_device_ptr(in);
  HIP_TRY(hipMemcpyAsync(f->words, in, nw * 4, dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                         s));
  HIP_TRY(cb::launch_mask_tail(f->words, f->m, s));
  if (f->needs_zero.exchange(false)) f->needs_pad_zero.store(true);
  HIP_TRY(ensure_pad_zeroed(f, s));
  if (!dev) HIP_TRY(hipStreamSynchronize(s));
  f->known_zero = false;
  return mark_written(f, s);
}

int cb_filter_to_bytes(const cb_filter* f, uint8_t* out, uint64_t cap, uint64_t* len_out) {
  if (!f || !len_out) return fail(CB_EINVAL, "null argument");
  // prost: proto3 repeated scalars are packed; an empty field is omitted.
  const uint64_t total = f->m ? 1 + varint_len(f->m) + f->m : 0;
  *len_out = total;
  if (!out || cap < total || !total) return CB_OK;
  uint8_t hdr[11];
  const size_t hl = put_bloom_header(hdr, f->m);
  int rc = put_bytes(out, hdr, hl);
  if (rc) return rc;
  return cb_filter_export_bools(f, out + hl, nullptr);
}

int cb_filter_from_bytes(const uint8_t* in, uint64_t len, int device, cb_filter** out) {
  if (!out || (!in && len)) return fail(CB_EINVAL, "null argument");
  *out = nullptr;
  const uint8_t* p = in;
  const uint8_t* end = in + len;
  // Fast path: exactly one packed field-1 run of single-byte 0/1 varints (what
  // to_bytes writes) is imported straight from the input buffer.
  std::vector<uint8_t> bits;
  const uint8_t* direct = nullptr;
  uint64_t direct_len = 0;
  int runs = 0;
  while (p < end) {
    uint64_t key;
    if (!get_varint(p, end, key) || key > 0xFFFFFFFFull)
      return fail(CB_EDECODE, "BloomProto decode: invalid key");
    const uint32_t wt = (uint32_t)(key & 7);
    const uint64_t fn = key >> 3;
    if (fn == 0) return fail(CB_EDECODE, "BloomProto decode: invalid tag value 0");
    if (fn == 1 && wt == 2) {
      uint64_t l;
      if (!get_varint(p, end, l) || l > (uint64_t)(end - p))
        return fail(CB_EDECODE, "BloomProto decode: bad length");
      const uint8_t* lim = p + l;
      bool simple = true;
      for (const uint8_t* q = p; q < lim; ++q)
        if (*q > 1) {
          simple = false;
          break;
        }
      if (simple && runs == 0 && bits.empty()) {
        direct = p;
        direct_len = l;
        p = lim;
        ++runs;
        continue;
      }
      if (direct) {
        bits.assign(direct, direct + direct_len);
        direct = nullptr;
      }
      while (p < lim) {
        uint64_t v;
        if (!get_varint(p, lim, v)) return fail(CB_EDECODE, "BloomProto decode: bad varint");
        bits.push_back(v != 0);
      }
      ++runs;
    } else if (fn == 1 && wt == 0) {
      uint64_t v;
      if (!get_varint(p, end, v)) return fail(CB_EDECODE, "BloomProto decode: bad varint");
      if (direct) {
        bits.assign(direct, direct + direct_len);
        direct = nullptr;
      }
      bits.push_back(v != 0);
      ++runs;
    } else if (fn == 1) {
      return fail(CB_EDECODE, "BloomProto decode: invalid wire type for field 1");
    } else if (!skip_field(p, end, wt, fn, 0)) {
      return fail(CB_EDECODE, "BloomProto decode: malformed unknown field");
    }
  }
  const uint8_t* src = direct ? direct : bits.data();
  const uint64_t m = direct ? direct_len : bits.size();
  cb_filter* f = nullptr;
  int rc = cb_filter_create(m, device, &f);
  if (rc) return rc;
  if (m) {
    rc = cb_filter_import_bools(f, src, m, nullptr);
    if (rc) {
      cb_filter_destroy(f);
      return rc;
    }
  }
  *out = f;
  return CB_OK;
}


// ---- TableMeta, the SSTable `.meta` file (src/sstable.rs:31-37) ----

int cb_meta_encode(const cb_filter* bloom, const cb_zone_bounds* zone, uint8_t* out, uint64_t cap,
                   uint64_t* len_out) {
  if (!len_out) return fail(CB_EINVAL, "null len_out");
  if (zone && ((zone->has_min && zone->min_len && !zone->min) ||
               (zone->has_max && zone->max_len && !zone->max)))
    return fail(CB_EINVAL, "null zone bound");
  if (zone && ((zone->has_min && !utf8_ok(zone->min, zone->min_len)) ||
               (zone->has_max && !utf8_ok(zone->max, zone->max_len))))
    return fail(CB_EINVAL, "zone bound is not UTF-8 (ZoneMapProto strings are Rust Strings)");
  const uint64_t bl = bloom && bloom->m ? 1 + varint_len(bloom->m) + bloom->m : 0;
  uint64_t zl = 0, total = 0;
  if (bloom) total += 1 + varint_len(bl) + bl;
  if (zone) {
    if (zone->has_min) zl += 1 + varint_len(zone->min_len) + zone->min_len;
    if (zone->has_max) zl += 1 + varint_len(zone->max_len) + zone->max_len;
    total += 1 + varint_len(zl) + zl;
  }
  *len_out = total;
  if (!out || cap < total) return CB_OK;
  // [0x0A len(bloom) [0x0A varint(m) m x 0/1]] [0x12 len(zone) [0x0A min] [0x12 max]]
  uint8_t hdr[32];
  uint64_t pos = 0;
  int rc;
  if (bloom) {
    size_t h = 0;
    hdr[h++] = 0x0A;
    h += put_varint_buf(hdr + h, bl);
    if (bloom->m) h += put_bloom_header(hdr + h, bloom->m);
    if ((rc = put_bytes(out, hdr, h))) return rc;
    pos = h;
    if (bloom->m) {
      if ((rc = cb_filter_export_bools(bloom, out + pos, nullptr))) return rc;
      pos += bloom->m;
    }
  }
  if (zone) {
    std::vector<uint8_t> z;
    z.reserve(zl + 11);
    uint8_t v[11];
    z.push_back(0x12);
    z.insert(z.end(), v, v + put_varint_buf(v, zl));
    if (zone->has_min) {
      z.push_back(0x0A);
      z.insert(z.end(), v, v + put_varint_buf(v, zone->min_len));
      z.insert(z.end(), zone->min, zone->min + zone->min_len);
    }
    if (zone->has_max) {
      z.push_back(0x12);
      z.insert(z.end(), v, v + put_varint_buf(v, zone->max_len));
      z.insert(z.end(), zone->max, zone->max + zone->max_len);
    }
    if ((rc = put_bytes(out + pos, z.data(), z.size()))) return rc;
  }
  return CB_OK;
}

int cb_meta_decode(const uint8_t* in, uint64_t len, int device, cb_filter** bloom_out,
                   cb_meta_info* info) {
  if (!bloom_out || !info || (!in && len)) return fail(CB_EINVAL, "null argument");
  *bloom_out = nullptr;
  memset(info, 0, sizeof(*info));
  MetaScan ms;
  int rc = scan_meta(in, len, ms);
  if (rc) return rc;
  cb_filter* f = nullptr;
  if (ms.bloom.empty()) {
    // SsTable::load: meta.bloom.map(from_proto).unwrap_or_else(|| BloomFilter::new(1024))
    rc = cb_filter_create(1024, device, &f);
  } else if (ms.bloom.size() == 1) {
    rc = cb_filter_from_bytes(ms.bloom[0].first, ms.bloom[0].second, device, &f);
  } else {
    std::vector<uint8_t> cat;
    for (auto& sp : ms.bloom) cat.insert(cat.end(), sp.first, sp.first + sp.second);
    rc = cb_filter_from_bytes(cat.data(), cat.size(), device, &f);
  }
  if (rc) return rc == CB_EDECODE ? fail(CB_EDECODE, (std::string("TableMeta decode: ") + g_err).c_str()) : rc;
  *bloom_out = f;
  info->has_bloom = !ms.bloom.empty();
  info->has_zone = ms.has_zone;
  info->zone.min = ms.min;
  info->zone.min_len = ms.min_len;
  info->zone.has_min = ms.has_min;
  info->zone.max = ms.max;
  info->zone.max_len = ms.max_len;
  info->zone.has_max = ms.has_max;
  return CB_OK;
}

int cb_set_load_meta(cb_filterset* set, uint32_t slot, const uint8_t* in, uint64_t len, void* stream) {
  if (!set) return fail(CB_EINVAL, "null set");
  if (slot >= set->width) return fail(CB_EINVAL, "slot out of range");
  cb_filter* f = nullptr;
  cb_meta_info info;
  int rc = cb_meta_decode(in, len, set->device, &f, &info);
  if (rc) return rc;
  if (f->m != set->m) {
    cb_filter_destroy(f);
    return fail(CB_EINVAL, "the table's filter size differs from the set's m");
  }
  rc = cb_set_assign(set, slot, f, stream);
  if (!rc) {
    const cb_zone_bounds& z = info.zone;
    rc = cb_set_zone(set, slot, z.min, z.min_len, z.has_min, z.max, z.max_len, z.has_max, stream);
  }
  // the assign is stream-ordered: wait before the temporary filter goes away
  if (!rc) rc = cb_stream_synchronize(stream);
  cb_filter_destroy(f);
  return rc;
}

// ---- bit-sliced filter sets ----

int cb_set_create(uint64_t m_bits, uint32_t width, int device, cb_filterset** out) {
  if (!out) return fail(CB_EINVAL, "null out");
  *out = nullptr;
  if (!(width == 32 || width == 64 || (width % 64 == 0 && width <= cb::kWideMax)))
    return fail(CB_EINVAL, "set width must be 32, 64 or a multiple of 64 up to 4096");
  if (m_bits == 0) return fail(CB_EZEROM, "attempt to calculate the remainder with a divisor of zero");
  int rc = cb_init(device);
  if (rc) return rc;
  DeviceGuard dg(device);
  std::unique_ptr<cb_filterset> set(new cb_filterset());
  set->m = m_bits;
  set->device = device;
  set->width = width;
  set->mp = cb::make_modp(m_bits, &set->mode);
  set->zlo.assign(width, std::string());
  set->zhi.assign(width, std::string());
  set->zhas_lo.assign(width, 0);
  set->zhas_hi.assign(width, 0);
  set->dirty.assign(std::max<uint32_t>(1, width / 64), 0ull);
  set->zg.assign(std::max<uint32_t>(1, width / 64), 0ull);
  set->R = width > 64 ? width / 64 : 0;
  const size_t bytes = width > 64 ? (size_t)m_bits * (width / 8) : (size_t)((m_bits + 31) / 32 * 32) * (width / 8);
  if (pool_alloc(device, bytes, &set->words, &set->words_cap) != hipSuccess) {
    set->words = nullptr;
    return fail(CB_ENOMEM, "device allocation failed for filter set words");
  }
  HIP_TRY(hipMemsetAsync(set->words, 0, bytes, nullptr));
  if (width > 64) {  // wide sets keep no union words (the pre-test is a 32/64-slot experiment)
    HIP_TRY(hipStreamSynchronize(nullptr));
    *out = set.release();
    return CB_OK;
  }
  const size_t any_bytes = (size_t)((m_bits + 31) / 32) * 4;
  if (pool_alloc(device, any_bytes, (void**)&set->any, &set->any_cap) != hipSuccess) {
    set->any = nullptr;
    pool_release(device, set->words, set->words_cap);
    return fail(CB_ENOMEM, "device allocation failed for filter set union words");
  }
  HIP_TRY(hipMemsetAsync(set->any, 0, any_bytes, nullptr));
  HIP_TRY(hipStreamSynchronize(nullptr));
  *out = set.release();
  return CB_OK;
}

int cb_set_destroy(cb_filterset* set) {
  if (!set) return CB_OK;
  {
    DeviceGuard dg(set->device);
    pool_release(set->device, set->words, set->words_cap);  // (stream-ordered: no device sync)
    pool_release(set->device, set->any, set->any_cap);
    if (set->zdev) (void)hipFree(set->zdev);
    if (set->wfw) (void)hipFree(set->wfw);
    for (void* z : set->zretired) (void)hipFree(z);
    for (auto& kv : set->zread) (void)hipEventDestroy(kv.second);
  }
  delete set;
  return CB_OK;
}

int cb_set_info(const cb_filterset* set, uint64_t* m_out, uint32_t* width_out, uint32_t* used_out) {
  if (!set) return fail(CB_EINVAL, "null set");
  if (m_out) *m_out = set->m;
  if (width_out) *width_out = set->width;
  if (used_out) *used_out = set->used;
  return CB_OK;
}

int cb_set_assign(cb_filterset* set, uint32_t slot, const cb_filter* f, void* stream) {
  if (!set || !f) return fail(CB_EINVAL, "null argument");
  if (slot >= set->width) return fail(CB_EINVAL, "slot out of range");
  if (f->m != set->m) return fail(CB_EINVAL, "filter size differs from the set's m");
  if (f->device != set->device) return fail(CB_EINVAL, "filter and set live on different devices");
  hipStream_t s = (hipStream_t)stream;
  DeviceGuard dg(set->device);
  HIP_TRY(ensure_zeroed(f, s));
  if (set_is_wide(set)) {
    uint64_t* w = (uint64_t*)set->words;
    if (slot_dirty(set, slot))
      HIP_TRY(cb::launch_wide_put_slot(f->words, set->m, slot, set->R, w, s));
    else
      HIP_TRY(cb::launch_wide_or_slot(f->words, set->m, slot, set->R, w, s));
  } else if (slot_dirty(set, slot)) {
    HIP_TRY(cb::launch_set_put_slot(f->words, set->m, slot, set->width, set->words, set->any, s));
  } else {
    HIP_TRY(cb::launch_set_or_slot(f->words, set->m, slot, set->width, set->words, set->any, s));
  }
  set->dirty[slot >> 6] |= 1ull << (slot & 63);
  set->used = std::max(set->used, slot + 1);
  return zones_after_reset(set, reset_zone(set, slot), s);
}

int cb_set_assign_all(cb_filterset* set, const cb_filter* const* filters, uint32_t nf, void* stream) {
  if (!set) return fail(CB_EINVAL, "null set");
  if (nf > set->width) return fail(CB_EINVAL, "more filters than set slots");
  if (nf && !filters) return fail(CB_EINVAL, "null filters");
  hipStream_t s = (hipStream_t)stream;
  DeviceGuard dg(set->device);
  FilterPtrs fp{};
  std::vector<const uint32_t*> ptrs(nf);
  for (uint32_t i = 0; i < nf; ++i) {
    const cb_filter* f = filters[i];
    if (!f) return fail(CB_EINVAL, "null filter");
    if (f->m != set->m) return fail(CB_EINVAL, "filter size differs from the set's m");
    if (f->device != set->device) return fail(CB_EINVAL, "filter and set live on different devices");
    HIP_TRY(ensure_zeroed(f, s));
    ptrs[i] = f->words;
    if (i < 64) {
      fp.w[i] = f->words;
      fp.row[i] = i;
    }
  }
  if (set_is_wide(set)) {
    // the filters' word pointers in device memory for the one-launch build
    const size_t pb = std::max<size_t>(8, (size_t)nf * sizeof(void*));
    if (pb > set->wfw_cap) {
      HIP_TRY(hipStreamSynchronize(s));  // an earlier build may still read the old array
      if (set->wfw) HIP_TRY(hipFree(set->wfw));
      set->wfw = nullptr;
      set->wfw_cap = 0;
      HIP_TRY(hipMalloc(&set->wfw, pb));
      set->wfw_cap = pb;
    }
    if (nf) HIP_TRY(hipMemcpyAsync(set->wfw, ptrs.data(), (size_t)nf * sizeof(void*), hipMemcpyHostToDevice, s));
    HIP_TRY(cb::launch_wide_build((const uint32_t* const*)set->wfw, nf, set->m, set->R, (uint64_t*)set->words, s));
    HIP_TRY(hipStreamSynchronize(s));  // the pageable pointer array is copied, and wfw is reused
  } else {
    HIP_TRY(cb::launch_set_build(fp, nf, set->m, set->width, set->words, set->any, s));
  }
  set->used = nf;
  for (size_t j = 0; j < set->dirty.size(); ++j) {
    const uint32_t lo = (uint32_t)j * 64;
    set->dirty[j] = nf >= lo + 64 ? ~0ull : (nf > lo ? ((1ull << (nf - lo)) - 1) : 0ull);
  }
  bool changed = false;
  for (uint32_t i = 0; i < set->width; ++i) changed |= reset_zone(set, i);
  return zones_after_reset(set, changed, s);
}

int cb_set_clear_slot(cb_filterset* set, uint32_t slot, void* stream) {
  if (!set) return fail(CB_EINVAL, "null set");
  if (slot >= set->width) return fail(CB_EINVAL, "slot out of range");
  DeviceGuard dg(set->device);
  note_stream(set->device, (hipStream_t)stream);
  int rc = zones_after_reset(set, reset_zone(set, slot), (hipStream_t)stream);
  if (rc || !slot_dirty(set, slot)) return rc;
  if (set_is_wide(set))
    HIP_TRY(cb::launch_wide_put_slot(nullptr, set->m, slot, set->R, (uint64_t*)set->words, (hipStream_t)stream));
  else
    HIP_TRY(cb::launch_set_put_slot(nullptr, set->m, slot, set->width, set->words, set->any,
                                    (hipStream_t)stream));
  set->dirty[slot >> 6] &= ~(1ull << (slot & 63));
  return CB_OK;
}

int cb_set_probe_fixed(const cb_filterset* set, const uint8_t* keys, uint32_t key_len, uint64_t n,
                       uint64_t* hits, void* stream) {
  return set_probe_impl(set, keys, nullptr, key_len, n, hits, (hipStream_t)stream, false);
}

int cb_set_probe_var(const cb_filterset* set, const uint8_t* bytes, const uint64_t* offsets,
                     uint64_t n, uint64_t* hits, void* stream) {
  if (!offsets) return fail(CB_EINVAL, "null offsets");
  return set_probe_impl(set, bytes, offsets, 0, n, hits, (hipStream_t)stream, false);
}

// ---- zone maps (src/zonemap.rs) and the SsTable::get gate ----

int cb_set_zone(cb_filterset* set, uint32_t slot, const uint8_t* min, uint64_t min_len,
                int has_min, const uint8_t* max, uint64_t max_len, int has_max, void* stream) {
  if (!set) return fail(CB_EINVAL, "null set");
  if (slot >= set->width) return fail(CB_EINVAL, "slot out of range");
  if ((has_min && min_len && !min) || (has_max && max_len && !max))
    return fail(CB_EINVAL, "null zone bound");
  if ((has_min && min_len > 0xFFFFFFFFull) || (has_max && max_len > 0xFFFFFFFFull))
    return fail(CB_EINVAL, "zone bound longer than 4 GiB");
  DeviceGuard dg(set->device);
  set->zlo[slot].assign(has_min ? (const char*)min : "", has_min ? (size_t)min_len : 0);
  set->zhi[slot].assign(has_max ? (const char*)max : "", has_max ? (size_t)max_len : 0);
  set->zhas_lo[slot] = has_min ? 1 : 0;
  set->zhas_hi[slot] = has_max ? 1 : 0;
  return upload_zones(set, (hipStream_t)stream);
}

int cb_set_zone_get(const cb_filterset* set, uint32_t slot, uint8_t* min, uint64_t min_cap,
                    uint64_t* min_len, int* has_min, uint8_t* max, uint64_t max_cap,
                    uint64_t* max_len, int* has_max) {
  if (!set) return fail(CB_EINVAL, "null set");
  if (slot >= set->width) return fail(CB_EINVAL, "slot out of range");
  const std::string &lo = set->zlo[slot], &hi = set->zhi[slot];
  if (has_min) *has_min = set->zhas_lo[slot];
  if (has_max) *has_max = set->zhas_hi[slot];
  if (min_len) *min_len = lo.size();
  if (max_len) *max_len = hi.size();
  if (min && min_cap >= lo.size() && !lo.empty()) memcpy(min, lo.data(), lo.size());
  if (max && max_cap >= hi.size() && !hi.empty()) memcpy(max, hi.data(), hi.size());
  return CB_OK;
}

int cb_set_zone_from_keys_fixed(cb_filterset* set, uint32_t slot, const uint8_t* keys,
                                uint32_t key_len, uint64_t n, void* stream) {
  if (!set) return fail(CB_EINVAL, "null set");
  if (slot >= set->width) return fail(CB_EINVAL, "slot out of range");
  std::string lo, hi;
  int rc = zone_bounds_impl(set->device, keys, nullptr, key_len, n, (hipStream_t)stream, nullptr,
                            nullptr, &lo, &hi);
  if (rc || n == 0) return rc;  // no keys: ZoneMap::update never ran, zone unchanged
  // ZoneMap::update over the batch, merged with the slot's current bounds.
  DeviceGuard dg(set->device);
  auto less = [](const std::string& a, const std::string& b) {
    return std::lexicographical_compare(a.begin(), a.end(), b.begin(), b.end(),
                                        [](char x, char y) { return (uint8_t)x < (uint8_t)y; });
  };
  if (!set->zhas_lo[slot] || less(lo, set->zlo[slot])) set->zlo[slot] = lo;
  if (!set->zhas_hi[slot] || less(set->zhi[slot], hi)) set->zhi[slot] = hi;
  set->zhas_lo[slot] = set->zhas_hi[slot] = 1;
  return upload_zones(set, (hipStream_t)stream);
}

int cb_set_zone_from_keys_var(cb_filterset* set, uint32_t slot, const uint8_t* bytes,
                              const uint64_t* offsets, uint64_t n, void* stream) {
  if (!set) return fail(CB_EINVAL, "null set");
  if (slot >= set->width) return fail(CB_EINVAL, "slot out of range");
  if (!offsets) return fail(CB_EINVAL, "null offsets");
  std::string lo, hi;
  int rc = zone_bounds_impl(set->device, bytes, offsets, 0, n, (hipStream_t)stream, nullptr,
                            nullptr, &lo, &hi);
  if (rc || n == 0) return rc;
  DeviceGuard dg(set->device);
  auto less = [](const std::string& a, const std::string& b) {
    return std::lexicographical_compare(a.begin(), a.end(), b.begin(), b.end(),
                                        [](char x, char y) { return (uint8_t)x < (uint8_t)y; });
  };
  if (!set->zhas_lo[slot] || less(lo, set->zlo[slot])) set->zlo[slot] = lo;
  if (!set->zhas_hi[slot] || less(set->zhi[slot], hi)) set->zhi[slot] = hi;
  set->zhas_lo[slot] = set->zhas_hi[slot] = 1;
  return upload_zones(set, (hipStream_t)stream);
}

int cb_zone_bounds_fixed(const uint8_t* keys, uint32_t key_len, uint64_t n, int device,
                         uint64_t* min_idx, uint64_t* max_idx, void* stream) {
  return zone_bounds_impl(device, keys, nullptr, key_len, n, (hipStream_t)stream, min_idx,
                          max_idx, nullptr, nullptr);
}

int cb_zone_bounds_var(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, int device,
                       uint64_t* min_idx, uint64_t* max_idx, void* stream) {
  if (!offsets) return fail(CB_EINVAL, "null offsets");
  return zone_bounds_impl(device, bytes, offsets, 0, n, (hipStream_t)stream, min_idx, max_idx,
                          nullptr, nullptr);
}

int cb_set_probe_gated_fixed(const cb_filterset* set, const uint8_t* keys, uint32_t key_len,
                             uint64_t n, uint64_t* hits, void* stream) {
  return set_probe_impl(set, keys, nullptr, key_len, n, hits, (hipStream_t)stream, true);
}

int cb_set_probe_gated_var(const cb_filterset* set, const uint8_t* bytes, const uint64_t* offsets,
                           uint64_t n, uint64_t* hits, void* stream) {
  if (!offsets) return fail(CB_EINVAL, "null offsets");
  return set_probe_impl(set, bytes, offsets, 0, n, hits, (hipStream_t)stream, true);
}


int cb_filter_insert_fixed_many(cb_filter* const* filters, uint32_t nf, const uint8_t* const* keys,
                                uint32_t key_len, const uint64_t* n, void* stream) {
  if (nf == 0) return CB_OK;
  if (!filters || !keys || !n) return fail(CB_EINVAL, "null argument");
  hipStream_t s = (hipStream_t)stream;
  const cb_filter* f0 = filters[0];
  if (!f0) return fail(CB_EINVAL, "null filter");
  uint64_t nmax = 0;
  for (uint32_t i = 0; i < nf; ++i) {
    const cb_filter* f = filters[i];
    if (!f) return fail(CB_EINVAL, "null filter");
    if (f->m != f0->m || f->device != f0->device)
      return fail(CB_EINVAL, "batched builds need filters of one size on one device");
    if (n[i] && f->m == 0) return fail(CB_EZEROM, "attempt to calculate the remainder with a divisor of zero");
    if (n[i] && key_len && !keys[i]) return fail(CB_EINVAL, "null keys");
    nmax = std::max(nmax, n[i]);
  }
  if (nmax == 0) return CB_OK;
  const uint64_t chunk_limit = 4096ull * 256 * 16;
  if (choose_build_path(f0->m, nmax) != PATH_TILED || nmax > chunk_limit) {
    for (uint32_t i = 0; i < nf; ++i) {  // per-filter builds (direct path or huge batches)
      int rc = insert_impl(filters[i], keys[i], nullptr, key_len, n[i], s);
      if (rc) return rc;
    }
    return CB_OK;
  }
  DeviceGuard dg(f0->device);
  Workspace& ws = workspace(f0->device, s);
  std::lock_guard<std::mutex> lk(ws.mu);
  // Stage host key arrays into one workspace buffer (16-byte aligned slices).
  std::vector<const uint8_t*> dkeys(nf);
  std::vector<uint64_t> stage_off(nf, 0);
  uint64_t stage_bytes = 0;
  for (uint32_t i = 0; i < nf; ++i) {
    dkeys[i] = keys[i];
    if (n[i] && key_len && !is_device_ptr(keys[i])) {
      stage_off[i] = stage_bytes;
      stage_bytes += ((uint64_t)key_len * n[i] + 15) & ~15ull;
      dkeys[i] = nullptr;
    }
  }
  bool staged = false;
  if (stage_bytes) {
    HIP_TRY(ws.keys.reserve(stage_bytes, s));
    for (uint32_t i = 0; i < nf; ++i)
      if (!dkeys[i]) {
        HIP_TRY(hipMemcpyAsync((uint8_t*)ws.keys.p + stage_off[i], keys[i], (uint64_t)key_len * n[i],
                               hipMemcpyHostToDevice, s));
        dkeys[i] = (const uint8_t*)ws.keys.p + stage_off[i];
      }
    staged = true;
  }
#ifdef CB_EXPERIMENTS
  static const uint32_t batch_env = [] {  // filters per launch pair (tuning)
    const char* v = getenv("CB_BUILD_BATCH");
    const int b = v && *v ? atoi(v) : 0;
    return b >= 1 && b <= (int)cb::kMaxBuildBatch ? (uint32_t)b : cb::kMaxBuildBatch;
  }();
  const uint32_t kBatch = batch_env;
#else
  const uint32_t kBatch = cb::kMaxBuildBatch;
#endif
  const TilePlan p = cb::plan_build(f0->m, nmax, std::min<uint32_t>(nf, kBatch));
  for (uint32_t i = 0; i < nf; ++i)
    if (!covers(filters[i], p)) return fail(CB_EINVAL, "internal: build tile plan exceeds the filter allocation");
  bool all16 = key_len == 16;
  for (uint32_t i = 0; i < nf; ++i) all16 = all16 && !((uintptr_t)dkeys[i] & 15);
  const int keyk = all16 ? cb::KEY_FIXED16 : cb::KEY_FIXED;
  for (uint32_t b0 = 0; b0 < nf; b0 += kBatch) {
    const uint32_t nb = std::min<uint32_t>(kBatch, nf - b0);
    cb::BuildBatch bb{};
    for (uint32_t j = 0; j < nb; ++j) {
      cb_filter* f = filters[b0 + j];
      if (f->known_zero) {
        if (f->needs_zero.exchange(false)) f->needs_pad_zero.store(true);
        HIP_TRY(ensure_pad_zeroed(f, s));
      } else {
        HIP_TRY(ensure_zeroed(f, s));
      }
      bb.ks[j].bytes = dkeys[b0 + j];
      bb.ks[j].offsets = nullptr;
      bb.ks[j].key_len = key_len;
      bb.n[j] = n[b0 + j];
      bb.words[j] = f->words;
      bb.fresh |= (f->known_zero ? 1ull : 0ull) << j;
    }
    HIP_TRY(ws.seg.reserve(cb::build_seg_bytes(p) * nb, s));
    HIP_TRY(ws.ent.reserve(cb::build_ent_bytes(p) * nb, s));
    HIP_TRY(cb::launch_build_batch(keyk, f0->mode, bb, nb, f0->mp, p, (uint32_t*)ws.seg.p,
                                   (uint32_t*)ws.ent.p, s));
    for (uint32_t j = 0; j < nb; ++j)
      if (n[b0 + j]) filters[b0 + j]->known_zero = false;
    if (int rc = mark_written_many(ws, filters + b0, nb, s)) return rc;  // one event for the batch
  }
  g_last_path = PATH_TILED;
  if (staged) HIP_TRY(hipStreamSynchronize(s));
  return CB_OK;
}

}  // extern "C"
