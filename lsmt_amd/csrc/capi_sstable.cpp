// capi_sstable.cpp — the C ABI for SSTable data files in HBM (SURVEY.md §8f
// rows 3 and 4): indexing an existing file (cb_table_create), SsTable::create
// on the device (cb_sstable_create), the batched binary search and
// Database::get's newest-first walk (cb_get_many_*).
//
// Reference: /root/reference/src/sstable.rs:51-179, src/lib.rs:125-136.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <cstring>

#include "capi_internal.hpp"

using namespace cbx;

namespace {

bool g_table_exact = false;  // cb_table_force_exact: index files for the exact-trajectory search only
std::atomic<uint64_t> g_bucket_limit{1ull << 30};  // cb_table_bucket_limit

// The most bytes a table's key buckets may take on this device now: the
// process-wide limit, and a quarter of the free device memory (the buckets
// are kept for the table's lifetime and must not starve later flushes).
uint64_t bucket_budget(int device) {
  const uint64_t lim = g_bucket_limit.load(std::memory_order_relaxed);
  if (!lim) return 0;
  size_t free_b = 0, total_b = 0;
  DeviceGuard dg(device);
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return std::min<uint64_t>(lim, free_b / 4);
}

int table_search_impl(const cb_table* t, const uint8_t* keys, const uint64_t* offsets,
                      uint32_t key_len, uint64_t n, int64_t* line_out, hipStream_t s) {
  if (!t || !line_out) return fail(CB_EINVAL, "null argument");
  if (int rc = finalize_table(const_cast<cb_table*>(t))) return rc;
  if (n == 0) return CB_OK;
  if (offsets == nullptr && keys == nullptr && key_len) return fail(CB_EINVAL, "null keys");
  DeviceGuard dg(t->device);
  Workspace& ws = workspace(t->device, s);
  std::lock_guard<std::mutex> lk(ws.mu);
  StagedKeys sk;
  int rc = offsets ? stage_var(ws, keys, offsets, n, s, sk) : stage_fixed(ws, keys, key_len, n, s, sk);
  if (rc) return rc;
  int64_t* dl;
  if ((rc = out_buf(ws.t_line, line_out, n, s, &dl))) return rc;
  HIP_TRY(cb::launch_table_search(sk.keyk, t->view(), sk.ks, n, dl, s));
  if (dl != line_out) {
    HIP_TRY(hipMemcpyAsync(line_out, dl, n * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  } else if (sk.staged) {
    HIP_TRY(hipStreamSynchronize(s));
  }
  return CB_OK;
}

bool buckets_enabled() {
#ifdef CB_EXPERIMENTS
  static const bool off = getenv("CB_NO_BUCKETS") && getenv("CB_NO_BUCKETS")[0] == '1';
  return !off;
#else
  return true;
#endif
}

// The key buckets (sstable.hpp) for a read on stream s: the first read of a
// well-formed table enqueues their build on s and records bkt_ev after it.
// Until that event is seen complete, every read (on any stream, the building
// one included) enqueues a wait on it before using the buckets: the host never
// blocks, and no reader relies on stream-handle identity (the same handle can
// name another stream: hipStreamPerThread from two threads, or a destroyed
// stream's handle reused). A table whose bucket memory cannot be had is simply
// read without them. v receives bkt / bkbits.
int table_buckets(cb_table* t, hipStream_t s, cb::TableView* v) {
  int st = t->bkt_state.load(std::memory_order_acquire);
  if (st < 0 || (st == 0 && (!t->fast || !t->nlines || !buckets_enabled()))) return CB_OK;
  if (st == 1 || st == 0) {
    std::lock_guard<std::mutex> lk(t->bkt_mu);
    st = t->bkt_state.load(std::memory_order_relaxed);
    if (st == 0) {
      const uint32_t bits = cb::bkt_bits(t->nlines);
      const size_t bytes = (size_t)cb::bkt_bytes(bits);  // the buckets and their summary words
      if (bytes > bucket_budget(t->device) ||
          pool_alloc(t->device, bytes, (void**)&t->bkt, &t->bkt_cap) != hipSuccess) {
        t->bkt = nullptr;
        (void)hipGetLastError();
        t->bkt_state.store(-1, std::memory_order_release);
        return CB_OK;
      }
      t->bkbits = bits;
      // a failure past the allocation leaves the table without buckets for good
      // (the block is freed with the table) and reports the error once
      t->bkt_state.store(-1, std::memory_order_relaxed);
      HIP_TRY(hipMemsetAsync(t->bkt, 0xFF, bytes, s));
      HIP_TRY(cb::launch_table_buckets(t->rec, t->nlines, t->bkt, bits, s));
      HIP_TRY(hipEventCreateWithFlags(&t->bkt_ev, hipEventDisableTiming | hipEventDisableSystemFence));
      HIP_TRY(hipEventRecord(t->bkt_ev, s));
      t->bkt_state.store(st = 1, std::memory_order_release);
      // (s itself is ordered after the build: no wait needed on this call)
    } else if (st == 1) {
      if (hipEventQuery(t->bkt_ev) == hipSuccess) {
        t->bkt_state.store(st = 2, std::memory_order_release);
      } else {
        HIP_TRY(hipStreamWaitEvent(s, t->bkt_ev, 0));
      }
    }
  }
  if (st >= 1) cb::view_set_buckets(*v, t->bkt, t->bkbits);
  return CB_OK;
}

// The wide walk's screen for these tables in these slots (sstable.hpp
// WideScreen): built on s after their buckets, and kept in the stream's
// workspace until the tables, their slots or their buckets change (compared
// by the tables' process-unique ids). Only when the tables share one bucket
// count and the screen stays small; otherwise the walk runs without it.
// The most fingerprint bins (up to 256) whose screen fits kScreenMaxBytes.
// 300 tables of 1024 lines: 64 bins (a 2.6 MB screen) 1.91-1.92 G gets/s
// against 1.84-1.87 for 32 and 1.76-1.77 for 16; then 256 bins (10.5 MB)
// 1.92-1.99 against 1.89-1.92 for 64 and 1.90-1.96 for 128
// (experiments r05_wide5 and r05_wide6, HISTORY.md; alternating on one box).
constexpr uint32_t kScreenHbits = 8;
constexpr uint64_t kScreenMaxBytes = 16ull << 20;
int wide_screen(Workspace& ws, const cb_table* const* tables, const std::vector<cb::TableView>& views,
                const std::vector<uint32_t>& rows, uint32_t R, const cb::TableView* dviews, const uint32_t* drows,
                hipStream_t s, cb::WideScreen* out) {
  const uint32_t nt = (uint32_t)views.size();
  uint32_t hbits = kScreenHbits;
#ifdef CB_EXPERIMENTS
  static const bool off = getenv("CB_NO_SCREEN") && getenv("CB_NO_SCREEN")[0] == '1';  // the A/B
  if (off) return CB_OK;
  static const int env_h = getenv("CB_SCREEN_HBITS") ? atoi(getenv("CB_SCREEN_HBITS")) : -1;
  if (env_h >= 0 && env_h <= 8) hbits = (uint32_t)env_h;
#endif
  uint32_t bits = 0;
  for (const auto& v : views)
    if (v.bkt && v.fast()) {
      bits = v.bkbits();
      break;
    }
  while (hbits > 4 && bits && cb::wide_screen_bytes(R, bits, hbits) > kScreenMaxBytes) --hbits;
  if (!bits || cb::wide_screen_bytes(R, bits, hbits) > kScreenMaxBytes) return CB_OK;
  std::vector<uint64_t> sig;
  sig.reserve(4 + 4 * (size_t)nt);
  sig.push_back(nt);
  sig.push_back(R);
  sig.push_back(bits);
  sig.push_back(hbits);
  for (uint32_t i = 0; i < nt; ++i) {
    sig.push_back(tables[i]->uid);
    sig.push_back(rows.empty() ? i : rows[i]);
    sig.push_back((uint64_t)(uintptr_t)views[i].bkt);
    sig.push_back(views[i].meta);
  }
  if (sig != ws.w_scr_sig) {
    HIP_TRY(ws.w_scr.reserve(cb::wide_screen_bytes(R, bits, hbits), s));
    HIP_TRY(cb::launch_wide_screen(dviews, rows.empty() ? nullptr : drows, nt, R, bits, hbits,
                                   (uint64_t*)ws.w_scr.p, s));
    ws.w_scr_sig.swap(sig);
  }
  *out = cb::WideScreen{(const uint64_t*)ws.w_scr.p, bits, hbits, 0};
  return CB_OK;
}

// set != NULL: the fused form (cb_set_get_many_*): the gate comes from the
// FilterSet inside the search kernel, hit_rows are the tables' slots and
// hits is unused.
int get_many_impl(const cb_table* const* tables, uint32_t nt, const uint64_t* hits,
                  const uint32_t* hit_rows, const uint8_t* keys, const uint64_t* offsets,
                  uint32_t key_len, uint64_t n, int32_t* which, uint64_t* val_off, uint8_t* vals,
                  uint64_t cap, uint64_t* total, hipStream_t s, const cb_filterset* set = nullptr) {
  if (!which || !val_off || (nt && !tables)) return fail(CB_EINVAL, "null argument");
  if (set) {
    if (nt > set->width) return fail(CB_EINVAL, "more tables than the set's slots");
    if (hit_rows)
      for (uint32_t i = 0; i < nt; ++i)
        if (hit_rows[i] >= set->width) return fail(CB_EINVAL, "slot out of range");
    hits = nullptr;
  }
  // total == NULL: enqueue only (every buffer on the device; val_off[n] = the total)
  const bool async = total == nullptr;
  if (async && (!is_device_ptr(which) || !is_device_ptr(val_off) || (vals && !is_device_ptr(vals)) ||
                (hits && !is_device_ptr(hits)) || (n && keys && !is_device_ptr(keys)) ||
                (offsets && !is_device_ptr(offsets))))
    return fail(CB_EINVAL, "total may be NULL only when keys, hits and outputs are device memory");
  if (total) *total = 0;
  if (n == 0) {
    const uint64_t z = 0;
    if (async) {
      HIP_TRY(hipMemsetAsync(val_off, 0, 8, s));
      return CB_OK;
    }
    return put_bytes((uint8_t*)val_off, &z, 8);
  }
  if (offsets == nullptr && keys == nullptr && key_len) return fail(CB_EINVAL, "null keys");
  if (nt == 0) return fail(CB_EINVAL, "no tables");
  const int dev = tables[0] ? tables[0]->device : 0;
  std::vector<cb::TableView> views(nt);
  uint64_t nrows = nt;
  for (uint32_t i = 0; i < nt; ++i) {
    if (!tables[i]) return fail(CB_EINVAL, "null table");
    if (tables[i]->device != dev) return fail(CB_EINVAL, "tables live on different devices");
    if (int rc = finalize_table(const_cast<cb_table*>(tables[i]))) return rc;
    views[i] = tables[i]->view();
  }
  if (set && set->device != dev) return fail(CB_EINVAL, "set and tables live on different devices");
  std::vector<uint32_t> rows;
  if ((hits || set) && hit_rows) {
    rows.assign(hit_rows, hit_rows + nt);
    nrows = 0;
    for (uint32_t r : rows) nrows = std::max<uint64_t>(nrows, (uint64_t)r + 1);
  }
  DeviceGuard dg(dev);
  for (uint32_t i = 0; i < nt; ++i)
    if (int rc = table_buckets(const_cast<cb_table*>(tables[i]), s, &views[i])) return rc;
  Workspace& ws = workspace(dev, s);
  std::lock_guard<std::mutex> lk(ws.mu);
  StagedKeys sk;
  int rc = offsets ? stage_var(ws, keys, offsets, n, s, sk) : stage_fixed(ws, keys, key_len, n, s, sk);
  if (rc) return rc;
  const uint64_t hwords = (n + 63) / 64;
  const uint64_t* dhits = hits;
  if (hits && !is_device_ptr(hits)) {
    HIP_TRY(ws.hits.reserve(nrows * hwords * 8, s));
    HIP_TRY(hipMemcpyAsync(ws.hits.p, hits, nrows * hwords * 8, hipMemcpyHostToDevice, s));
    dhits = (const uint64_t*)ws.hits.p;
  }
  // views and rows: uploaded only when they differ from what the workspace
  // holds (stream-ordered, so earlier launches have read the old ones)
  const size_t vbytes = nt * sizeof(cb::TableView);
  const uint8_t* vb = (const uint8_t*)views.data();
  if (ws.t_views_host.size() != vbytes || memcmp(ws.t_views_host.data(), vb, vbytes)) {
    HIP_TRY(ws.t_views.reserve(vbytes, s));
    HIP_TRY(hipMemcpyAsync(ws.t_views.p, vb, vbytes, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));  // the source is pageable
    ws.t_views_host.assign(vb, vb + vbytes);
  }
  const uint32_t* drows = nullptr;
  if (!rows.empty()) {
    if (ws.t_rows_host != rows) {
      HIP_TRY(ws.t_rows.reserve(nt * 4, s));
      HIP_TRY(hipMemcpyAsync(ws.t_rows.p, rows.data(), nt * 4, hipMemcpyHostToDevice, s));
      HIP_TRY(hipStreamSynchronize(s));
      ws.t_rows_host = rows;
    }
    drows = (const uint32_t*)ws.t_rows.p;
  }
  int32_t* dwhich;
  uint64_t* dvoff;
  if ((rc = out_buf(ws.t_which, which, n, s, &dwhich))) return rc;
  if ((rc = out_buf(ws.t_voff, val_off, n + 1, s, &dvoff))) return rc;
  HIP_TRY(ws.t_line.reserve(n * 8, s));
  HIP_TRY(ws.t_dlen.reserve(n * 8, s));
  HIP_TRY(ws.t_scan.reserve(cb::get_tiles(n) * 8, s));
  const cb::TableView* dviews = (const cb::TableView*)ws.t_views.p;
  const uint64_t* vsrc = (const uint64_t*)ws.t_line.p;
  const uint64_t* dlen = (const uint64_t*)ws.t_dlen.p;
  uint64_t* tsum = (uint64_t*)ws.t_scan.p;
  if (set && set_is_wide(set)) {
    // the groups of 64 tables (newest first) and how each maps to slots:
    // ascending or descending runs take their candidate bits from one window
    // of the rows (wideset.hpp WideGroup), anything else one bit per table
    const uint32_t ng = (nt + 63) / 64;
    std::vector<cb::WideGroup> groups(ng);
    bool need_slots = false;
    for (uint32_t g = 0; g < ng; ++g) {
      const uint32_t t0 = 64 * g, gn = std::min<uint32_t>(64, nt - t0);
      auto slot = [&](uint32_t i) { return rows.empty() ? t0 + i : rows[t0 + i]; };
      bool asc = true, desc = true;
      for (uint32_t i = 1; i < gn; ++i) {
        asc = asc && slot(i) == slot(0) + i;
        desc = desc && slot(i) + i == slot(0);
      }
      cb::WideGroup& gd = groups[g];
      gd.gn = gn;
      if (asc) {
        gd.kind = 0;
        gd.lo = slot(0);
      } else if (desc) {
        gd.kind = 1;
        gd.lo = slot(gn - 1);
      } else {
        gd.kind = 2;
        gd.lo = 0;
        need_slots = true;
      }
    }
    const uint8_t* gb = (const uint8_t*)groups.data();
    const size_t gbytes = ng * sizeof(cb::WideGroup);
    if (ws.t_groups_host.size() != gbytes || memcmp(ws.t_groups_host.data(), gb, gbytes)) {
      HIP_TRY(ws.t_groups.reserve(gbytes, s));
      HIP_TRY(hipMemcpyAsync(ws.t_groups.p, gb, gbytes, hipMemcpyHostToDevice, s));
      HIP_TRY(hipStreamSynchronize(s));  // the source is pageable
      ws.t_groups_host.assign(gb, gb + gbytes);
    }
    const cb::WideZone wz = wide_zone_view(set);
    cb::WideScreen scr{nullptr, 0, 0, 0};
    if ((rc = wide_screen(ws, tables, views, rows, set->R, dviews, drows, s, &scr))) return rc;
    // the tables' DirMaps in one contiguous array (gathered on the device
    // when the table list changes: the walk stages a group's maps in the same
    // pass as its views)
    std::vector<uint64_t> msig;
    msig.reserve(2 * (size_t)nt);
    for (uint32_t i = 0; i < nt; ++i) {
      msig.push_back(tables[i]->uid);
      msig.push_back((uint64_t)(uintptr_t)views[i].dmap);
    }
    if (msig != ws.t_maps_sig) {
      HIP_TRY(ws.t_maps.reserve((size_t)nt * sizeof(cb::DirMap), s));
      HIP_TRY(cb::launch_gather_maps(dviews, nt, (cb::DirMap*)ws.t_maps.p, s));
      ws.t_maps_sig.swap(msig);
    }
    const cb::DirMap* dmaps = (const cb::DirMap*)ws.t_maps.p;
#ifdef CB_EXPERIMENTS
    // the A/B: maps found through the views (the round-5 staging)
    static const bool no_maps = getenv("CB_WIDE_MAPS") && getenv("CB_WIDE_MAPS")[0] == '0';
    if (no_maps) dmaps = nullptr;
#endif
    HIP_TRY(cb::launch_wide_get_many(sk.keyk, set->mode, set->R, (const uint64_t*)set->words, set->mp,
                                     set->zany ? &wz : nullptr, dviews, nt, (const cb::WideGroup*)ws.t_groups.p,
                                     need_slots ? drows : nullptr, sk.ks, n, dwhich, (uint64_t*)ws.t_line.p,
                                     (uint64_t*)ws.t_dlen.p, tsum, s, scr.scr ? &scr : nullptr, dmaps));
    if (set->zany && (rc = note_zone_read(set, s))) return rc;
  } else if (set) {
    const cb::ZoneView zv = set_zone_view(set);
    HIP_TRY(cb::launch_set_get_many(sk.keyk, set->mode, set->width, set->words, set->mp,
                                    set->zany ? &zv : nullptr, dviews, nt, drows, sk.ks, n, dwhich,
                                    (uint64_t*)ws.t_line.p, (uint64_t*)ws.t_dlen.p, tsum, s));
    if (set->zany && (rc = note_zone_read(set, s))) return rc;
  } else {
    HIP_TRY(cb::launch_get_many(sk.keyk, dviews, nt, dhits, drows, hwords, sk.ks, n, dwhich,
                                (uint64_t*)ws.t_line.p, (uint64_t*)ws.t_dlen.p, tsum, s));
  }
  // batches of up to 256K keys: the decode scans the tile sums itself (one
  // launch fewer per batch); larger ones: the one-block scan between
  bool raw = n && n <= cb::decode_raw_max();  // (n = 0: the scan kernel writes voff[0] = 0)
#ifdef CB_EXPERIMENTS
  static const bool no_raw = getenv("CB_DECODE_RAW") && getenv("CB_DECODE_RAW")[0] == '0';
  if (no_raw) raw = false;
#endif
  if (!raw) HIP_TRY(cb::launch_tile_scan(tsum, cb::get_tiles(n), dvoff + n, s));
  if (!ws.htot) HIP_TRY(hipHostMalloc((void**)&ws.htot, kHostScratch, hipHostMallocDefault));
  if (async) {
    HIP_TRY(cb::launch_b64_decode(vsrc, dlen, tsum, n, dvoff, vals, vals ? cap : 0, s, raw));
    return CB_OK;
  }
  if (vals && is_device_ptr(vals)) {
    // device values: offsets and values in one pass (the kernel skips the
    // value writes when the total exceeds cap): one host round trip
    HIP_TRY(cb::launch_b64_decode(vsrc, dlen, tsum, n, dvoff, vals, cap, s, raw));
    HIP_TRY(hipMemcpyAsync(ws.htot, dvoff + n, 8, hipMemcpyDeviceToHost, s));
  } else {
    HIP_TRY(cb::launch_b64_decode(vsrc, dlen, tsum, n, dvoff, nullptr, 0, s, raw));  // offsets only
    HIP_TRY(hipMemcpyAsync(ws.htot, dvoff + n, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const uint64_t tot = *ws.htot;
    if (vals && cap >= tot && tot) {
      uint8_t* dvals;
      if ((rc = out_buf(ws.t_vals, vals, tot, s, &dvals))) return rc;
      HIP_TRY(cb::launch_b64_decode(vsrc, dlen, tsum, n, dvoff, dvals, tot, s, raw));
      HIP_TRY(hipMemcpyAsync(vals, dvals, tot, hipMemcpyDeviceToHost, s));
    }
  }
  if (dwhich != which) HIP_TRY(hipMemcpyAsync(which, dwhich, n * 4, hipMemcpyDeviceToHost, s));
  if (dvoff != val_off) HIP_TRY(hipMemcpyAsync(val_off, dvoff, (n + 1) * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  *total = *ws.htot;
  return CB_OK;
}

// The index of nl lines is one allocation: rec | pfx | fence | dir | dmap | llen.
size_t dir_bytes(uint64_t nl) { return cb::dir_words(nl) ? ((cb::dir_words(nl) * 4 + 15) & ~15ull) : 0; }
size_t index_bytes(uint64_t nl) {
  return nl * sizeof(cb::LineRec) + nl * 8 + cb::fence_words(nl) * 8 + 8 + dir_bytes(nl) +
         (cb::dir_words(nl) ? sizeof(cb::DirMap) : 0) + nl * 4;
}
void carve_index(cb_table* t) {
  const uint64_t nl = t->nlines;
  t->pfx = (uint64_t*)(t->rec + nl);
  t->fence = t->pfx + nl;
  // 16-B aligned: the read path copies the map into LDS in 16-B words
  uint8_t* d = (uint8_t*)(((uintptr_t)(t->fence + cb::fence_words(nl)) + 15) & ~(uintptr_t)15);
  t->dir = cb::dir_words(nl) ? (uint32_t*)d : nullptr;
  t->dmap = nullptr;  // set once the directory is written (make_dirmap needs every prefix)
  t->llen = (uint32_t*)(d + (t->dir ? dir_bytes(nl) + sizeof(cb::DirMap) : 0));
}
cb::DirMap* dmap_slot(const cb_table* t) {
  return t->dir ? (cb::DirMap*)((uint8_t*)t->dir + dir_bytes(t->nlines)) : nullptr;
}

// Line index of t->data[0..t->len) (count -> scan -> emit -> finish -> keys).
// Temporaries come from the stream's workspace (taken here: callers must not
// hold its lock); the index itself is one allocation: rec | pfx | fence.
int index_table(cb_table* t, hipStream_t s) {
  const uint64_t len = t->len;
  if (!len) return CB_OK;
  Workspace& ws = workspace(t->device, s);
  std::lock_guard<std::mutex> lk(ws.mu);
  const uint64_t nb = cb::line_blocks(len);
  HIP_TRY(ws.i_cnt.reserve(nb * 8, s));
  HIP_TRY(ws.i_base.reserve((nb + 1) * 8, s));
  HIP_TRY(ws.i_tmp.reserve(cb::scan_tmp_words(nb) * 8, s));
  HIP_TRY(ws.i_err.reserve(16 + sizeof(uint64_t) * cb::kDirPos * 4, s));  // error words, then the prefix byte masks
  uint64_t* cnt = (uint64_t*)ws.i_cnt.p;
  uint64_t* base = (uint64_t*)ws.i_base.p;
  uint32_t* err = (uint32_t*)ws.i_err.p;
  HIP_TRY(cb::launch_line_count(t->data, len, cnt, s));
  HIP_TRY(cb::launch_scan_u64(cnt, base, nb, (uint64_t*)ws.i_tmp.p, s));
  HIP_TRY(hipMemcpyAsync(&t->nlines, base + nb, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (!t->nlines) return CB_OK;
  const uint64_t nl = t->nlines;
  const size_t bytes = index_bytes(nl);
  if (pool_alloc(t->device, bytes, (void**)&t->rec, &t->rec_cap) != hipSuccess) {
    t->rec = nullptr;
    return fail(CB_ENOMEM, "device allocation failed for an SSTable index");
  }
  carve_index(t);
  HIP_TRY(ws.i_start.reserve(nl * 8, s));
  HIP_TRY(ws.i_end.reserve(nl * 8, s));
  uint64_t* start = (uint64_t*)ws.i_start.p;
  uint64_t* end = (uint64_t*)ws.i_end.p;
  HIP_TRY(hipMemsetAsync(end, 0xFF, nl * 8, s));
  HIP_TRY(hipMemsetAsync(err, 0, 4, s));
  const uint32_t one = 1;
  HIP_TRY(hipMemcpyAsync(err + 1, &one, 4, hipMemcpyHostToDevice, s));
  HIP_TRY(cb::launch_line_emit(t->data, len, base, start, end, s));
  HIP_TRY(cb::launch_line_finish(t->data, len, nl, start, end, t->rec, t->llen, err, s));
  // prefix + fence index, value validity and the well-formed check (sstable.hpp)
  HIP_TRY(cb::launch_line_keys(t->data, nl, t->rec, t->llen, t->pfx, t->fence, err + 1, s));
  // the byte values of every prefix position (the directory's map)
  uint64_t* dmask = (uint64_t*)(err + 4);
  if (t->dir) {
    HIP_TRY(hipMemsetAsync(dmask, 0, sizeof(uint64_t) * cb::kDirPos * 4, s));
    HIP_TRY(cb::launch_pfx_masks(t->pfx, nl, dmask, s));
  }
  // the error words and the masks in one pinned copy, one wait
  if (!ws.htot) HIP_TRY(hipHostMalloc((void**)&ws.htot, kHostScratch, hipHostMallocDefault));
  HIP_TRY(hipMemcpyAsync(ws.htot, err, 16 + (t->dir ? sizeof(uint64_t) * cb::kDirPos * 4 : 0),
                         hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  uint32_t e[2];
  memcpy(e, ws.htot, 8);
  if (e[0]) return fail(CB_EINVAL, "an SSTable line is 4 GiB or longer");
  t->fast = e[1] != 0 && !g_table_exact;
  if (t->dir && e[1]) {  // well-formed (sorted prefixes): the directory applies
    uint64_t m[cb::kDirPos][4];
    memcpy(m, ws.htot + 2, sizeof m);
    const cb::DirMap dm = cb::make_dirmap(m, nl);
    t->dmap = dmap_slot(t);
    HIP_TRY(cb::launch_table_dir(t->pfx, nl, dm, t->dir, t->dmap, s));
  }
  return CB_OK;
}

// ---- SsTable::create: enqueue now, finalise on first use ----
//
// cb_sstable_create only enqueues its kernels (sortedness check, Bloom
// build, the sort the device picks, tile scan, format) and one copy of the
// CreateResult into a pinned block, followed by an event; nothing waits. The
// host-side results (file length, zone bounds, the well-formed flag) are read
// when the table is first used (finalize_table). One case needs the host
// there: a key holding '\n' or '\t' (the file is re-indexed the way
// SsTable::get splits it). A batch the bin sort cannot place (one bin, or a
// bin larger than an LDS tile) is sorted again on the device, by the merge
// sort enqueued after it that runs only then. Until a table is finalised its inputs must stay valid (host
// inputs are staged into a block the table owns).

// Pinned result blocks and their events, reused across tables.
struct ResultSlot {
  cb::CreateResult* h = nullptr;
  hipEvent_t ev = nullptr;
};
std::mutex g_res_mu;
std::vector<ResultSlot> g_res_free;

int result_slot(ResultSlot* out) {
  {
    std::lock_guard<std::mutex> lk(g_res_mu);
    if (!g_res_free.empty()) {
      *out = g_res_free.back();
      g_res_free.pop_back();
      return CB_OK;
    }
  }
  ResultSlot r;
  HIP_TRY(hipHostMalloc((void**)&r.h, sizeof(cb::CreateResult), hipHostMallocDefault));
  // host-waited after a copy into pinned memory: the default (system-scope) release
  HIP_TRY(hipEventCreateWithFlags(&r.ev, hipEventDisableTiming));
  *out = r;
  return CB_OK;
}

void result_release(cb::CreateResult* h, hipEvent_t ev) {
  if (!h) return;
  std::lock_guard<std::mutex> lk(g_res_mu);
  g_res_free.push_back(ResultSlot{h, ev});
}

}  // namespace

TablePending::~TablePending() {
  if (staged) pool_release(device, staged, staged_cap);
  result_release(hres, ev);
}

namespace {

// Bin-sort group target: ~n / 1536 records (six 1024-record group sorts per
// CU on 256 CUs, one wave), at least 640, at most 1536 (2048-record sorts).
uint32_t bin_group_target(uint64_t n) {
#ifdef CB_EXPERIMENTS
  static const int env = [] {
    const char* v = getenv("CB_BIN_T");  // group size target (tuning); 0 disables the bin sort
    return v && *v ? atoi(v) : -1;
  }();
  if (env >= 0) return (uint32_t)env;
#endif
  return (uint32_t)std::min<uint64_t>(1536, std::max<uint64_t>(640, (n + 1535) / 1536));
}

// The format pass and everything after the sort, on s (ws.mu held).
int enqueue_format(cb_table* t, Workspace& ws, const TablePending& p, cb::CreateResult* dr, hipStream_t s) {
  const uint64_t n = p.n;
  uint64_t* tsum = (uint64_t*)ws.f_tsum.p;
  const bool inline_scan = cb::format_tiles(n) <= cb::kFormatInlineTiles;  // small flushes: no scan launch
  if (!inline_scan) HIP_TRY(cb::launch_tile_scan(tsum, cb::format_tiles(n), &dr->len, s));
  HIP_TRY(cb::launch_format((const cb::SortKey*)ws.f_sk2.p, p.dk, p.dko, p.dv, p.dvo, tsum, n, t->data, t->rec,
                            t->pfx, t->fence, t->llen, dr, p.cap_bytes, s, (const ulonglong2*)ws.f_vsp.p, t->dir,
                            t->dir ? dmap_slot(t) : nullptr, inline_scan));
  return CB_OK;
}

int sstable_enqueue(const uint8_t* keys, const uint64_t* key_off, uint64_t kbytes, const uint8_t* vals,
                    const uint64_t* val_off, uint64_t vbytes, uint64_t n, uint64_t m_bits, int device, hipStream_t s,
                    cb_table** table_out, cb_filter** bloom_out) {
  *table_out = nullptr;
  if (bloom_out) *bloom_out = nullptr;
  if (n >= 0xFFFFFFFFull) return fail(CB_EINVAL, "too many entries for one table");
  int rc = cb_init(device);
  if (rc) return rc;
  if (bloom_out && n && m_bits == 0)  // BloomFilter::insert's `% 0` (src/bloom.rs:36)
    return fail(CB_EZEROM, "attempt to calculate the remainder with a divisor of zero");
  if ((kbytes && !keys) || (vbytes && !vals)) return fail(CB_EINVAL, "null bytes");
  DeviceGuard dg(device);
  std::unique_ptr<cb_table, int (*)(cb_table*)> t(new cb_table(), cb_table_destroy);
  std::unique_ptr<cb_filter, int (*)(cb_filter*)> f(nullptr, cb_filter_destroy);
  t->device = device;
  std::unique_ptr<TablePending> pend(new TablePending());
  TablePending& p = *pend;
  p.device = device;
  p.n = n;
  p.stream = s;
  // an error return past this point may leave work enqueued that reads the
  // staged block or writes the result slot: finish the stream before `pend`
  // hands them back (declared after pend, so it runs first)
  // (armed only at the first enqueue: a refusal before it — bad offsets,
  // bounds, a failed allocation — returns without blocking on the caller's
  // stream)
  struct SyncOnError {
    hipStream_t s;
    bool ok = true;
    ~SyncOnError() {
      if (!ok) (void)hipStreamSynchronize(s);
    }
  } on_error{s};
  // Host inputs go into one block the table owns (the work reads them after
  // this call returns, and a fallback sort at finalisation reads them again);
  // device inputs are used in place.
  const bool ko_h = !is_device_ptr(key_off), vo_h = !is_device_ptr(val_off);
  const bool kb_h = kbytes && !is_device_ptr(keys), vb_h = vbytes && !is_device_ptr(vals);
  if (ko_h)
    for (uint64_t i = 0; i < n; ++i)
      if (key_off[i + 1] < key_off[i]) return fail(CB_EINVAL, "offsets must be non-decreasing");
  if (vo_h)
    for (uint64_t i = 0; i < n; ++i)
      if (val_off[i + 1] < val_off[i]) return fail(CB_EINVAL, "offsets must be non-decreasing");
  if ((kb_h && !ko_h) || (vb_h && !vo_h)) {
    // host bytes with device offsets: they are staged into exactly kbytes /
    // vbytes, so offsets past those would send every kernel past the staged
    // block. Check the totals before anything is enqueued (one read-back).
    uint64_t tot[2] = {0, 0};
    if (kb_h && !ko_h) HIP_TRY(hipMemcpyAsync(&tot[0], key_off + n, 8, hipMemcpyDeviceToHost, s));
    if (vb_h && !vo_h) HIP_TRY(hipMemcpyAsync(&tot[1], val_off + n, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (tot[0] > kbytes) return fail(CB_EINVAL, "key bytes exceed key_bytes");
    if (tot[1] > vbytes) return fail(CB_EINVAL, "value bytes exceed val_bytes");
  }
  auto up16 = [](uint64_t x) { return (x + 15) & ~15ull; };
  const uint64_t offb = up16((n + 1) * 8);
  const uint64_t stage = (ko_h ? offb : 0) + (vo_h ? offb : 0) + (kb_h ? up16(kbytes) : 0) + (vb_h ? up16(vbytes) : 0);
  if (stage) {
    if (pool_alloc(device, stage, &p.staged, &p.staged_cap) != hipSuccess) {
      p.staged = nullptr;
      return fail(CB_ENOMEM, "device allocation failed for a staged flush batch");
    }
    on_error.ok = false;  // the staging copies are the first enqueued work
    uint8_t* at = (uint8_t*)p.staged;
    auto put = [&](const void* src, uint64_t bytes) -> uint8_t* {
      uint8_t* d = at;
      at += up16(bytes);
      return d;
    };
    if (ko_h) {
      uint8_t* d = put(key_off, (n + 1) * 8);
      HIP_TRY(hipMemcpyAsync(d, key_off, (n + 1) * 8, hipMemcpyHostToDevice, s));
      key_off = (const uint64_t*)d;
    }
    if (vo_h) {
      uint8_t* d = put(val_off, (n + 1) * 8);
      HIP_TRY(hipMemcpyAsync(d, val_off, (n + 1) * 8, hipMemcpyHostToDevice, s));
      val_off = (const uint64_t*)d;
    }
    if (kb_h) {
      uint8_t* d = put(keys, kbytes);
      HIP_TRY(hipMemcpyAsync(d, keys, kbytes, hipMemcpyHostToDevice, s));
      keys = d;
    }
    if (vb_h) {
      uint8_t* d = put(vals, vbytes);
      HIP_TRY(hipMemcpyAsync(d, vals, vbytes, hipMemcpyHostToDevice, s));
      vals = d;
    }
  }
  p.dk = keys;
  p.dko = key_off;
  p.dv = vals;
  p.dvo = val_off;
  // the file's buffer: sum(k + 2 + 4 ceil(v / 3)) <= K + 2n + (4V + 8n) / 3,
  // plus slack; its length comes back with the results
  p.cap_bytes = kbytes + 2 * n + (4 * vbytes + 8 * n) / 3 + 1 + 16;
  if (pool_alloc(device, p.cap_bytes, (void**)&t->data, &t->data_cap) != hipSuccess) {
    t->data = nullptr;
    return fail(CB_ENOMEM, "device allocation failed for an SSTable buffer");
  }
  if (!n) {  // an empty file: nothing to sort, index or bound
    on_error.ok = false;
    HIP_TRY(hipMemsetAsync(t->data, 0, 16, s));
    if (bloom_out) {
      cb_filter* fp = nullptr;
      if ((rc = cb_filter_create(m_bits, device, &fp))) return rc;
      *bloom_out = fp;
    }
    t->pend = std::move(pend);  // (no result block: the staged block is released with the table)
    HIP_TRY(hipStreamSynchronize(s));
    on_error.ok = true;
    *table_out = t.release();
    return CB_OK;
  }
  t->nlines = n;
  if (pool_alloc(device, index_bytes(n), (void**)&t->rec, &t->rec_cap) != hipSuccess) {
    t->rec = nullptr;
    return fail(CB_ENOMEM, "device allocation failed for an SSTable index");
  }
  carve_index(t.get());
  ResultSlot slot;
  if ((rc = result_slot(&slot))) return rc;
  p.hres = slot.h;
  p.ev = slot.ev;
  on_error.ok = false;  // from here on every step enqueues
  Workspace& ws = workspace(device, s);
  std::unique_lock<std::mutex> lk(ws.mu);
  HIP_TRY(ws.f_flag.reserve(sizeof(cb::CreateResult), s));
  HIP_TRY(ws.f_tsum.reserve(cb::format_tiles(n) * 8, s));
  HIP_TRY(ws.f_sk2.reserve(n * sizeof(cb::SortKey), s));
  HIP_TRY(ws.f_vsp.reserve(n * sizeof(ulonglong2), s));
  cb::CreateResult* dr = (cb::CreateResult*)ws.f_flag.p;
  uint64_t* tsum = (uint64_t*)ws.f_tsum.p;
  HIP_TRY(hipMemsetAsync(dr, 0, cb::kCreateHead, s));
  HIP_TRY(cb::launch_sorted_check(p.dk, p.dko, p.dvo, n, dr, tsum, kbytes, vbytes, s));
  // the Bloom build needs neither the order nor the totals (OR is order-free)
  if (bloom_out) {
    cb_filter* fp = nullptr;
    if ((rc = cb_filter_create(m_bits, device, &fp))) return rc;
    f.reset(fp);
    if ((rc = insert_locked(ws, fp, p.dk, p.dko, 0, n, s))) return rc;
  }
  // the stable sort by key, enqueued before anyone knows whether the batch
  // needs one: every sort launch returns at once for a sorted batch (memtable
  // flushes arrive sorted). Bin sort for 4096 < n <= 2^24 (its fallback, at
  // finalisation, is the merge sort); the merge sort otherwise.
  const uint32_t T = bin_group_target(n);
  p.binned = T && T <= cb::bin_sort_max_group() && n > 4096 && n <= (1ull << 24);
  const uint64_t tmp = p.binned ? cb::bin_sort_tmp_bytes(n, T) : cb::entry_sort_tmp_bytes(n);
  HIP_TRY(ws.f_sort.reserve(tmp, s));
  if (p.binned) {
    HIP_TRY(cb::launch_bin_sort(p.dk, p.dko, n, T, (cb::SortKey*)ws.f_sk2.p, ws.f_sort.p, s, p.dvo,
                                (ulonglong2*)ws.f_vsp.p, tsum, dr));
    // its fallback, on the device and on this stream: the merge sort, whose
    // launches return at once unless the bin sort set flags[3] (one bin, or a
    // bin larger than an LDS tile: keys sharing a long prefix); it rewrites
    // the records, value spans and tile sums whole
    HIP_TRY(cb::launch_entry_sort(nullptr, (cb::SortKey*)ws.f_sk2.p, (cb::SortKey*)ws.f_sort.p, n, p.dk, p.dko, s,
                                  p.dvo, (ulonglong2*)ws.f_vsp.p, tsum, &dr->flags[3]));
  } else
    HIP_TRY(cb::launch_entry_sort(nullptr, (cb::SortKey*)ws.f_sk2.p, (cb::SortKey*)ws.f_sort.p, n, p.dk, p.dko, s,
                                  p.dvo, (ulonglong2*)ws.f_vsp.p, tsum, &dr->flags[0]));
  if ((rc = enqueue_format(t.get(), ws, p, dr, s))) return rc;
  HIP_TRY(hipMemcpyAsync(p.hres, dr, sizeof(cb::CreateResult), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipEventRecord(p.ev, s));
  lk.unlock();
  t->dmap = t->dir ? dmap_slot(t.get()) : nullptr;
  t->pend = std::move(pend);
  t->ready.store(false, std::memory_order_release);
  on_error.ok = true;
  if (bloom_out) *bloom_out = f.release();
  *table_out = t.release();
  return CB_OK;
}

// Release what a finalised (or destroyed) table no longer needs.
void drop_pending(cb_table* t) {
  t->pend.reset();  // (~TablePending returns the staged block and the result slot)
}

int finalize_locked(cb_table* t) {
  TablePending& p = *t->pend;
  DeviceGuard dg(t->device);
  if (p.ev) HIP_TRY(hipEventSynchronize(p.ev));
  if (!p.n) return CB_OK;
  cb::CreateResult* hr = p.hres;
  if (hr->flags[4]) {
    t->ferr = CB_EINVAL;
    t->ferr_msg = "SsTable::create: the batch's key or value bytes exceed the bounds the table was sized from";
    return CB_OK;
  }
  // (hr->flags[3]: the bin sort could not place the batch and the merge sort
  // ran after it on the create's stream; the file is already written)
  t->len = hr->len;
  // zone map: ZoneMap::update over the sorted keys = first / last line
  t->zidx[0] = hr->idx_min;
  t->zidx[1] = hr->idx_max;
  for (int w = 0; w < 2; ++w) {
    const uint64_t kl = hr->zlen[w];
    std::string& z = w ? t->zmax : t->zmin;
    z.assign((const char*)hr->zkey[w], (size_t)std::min<uint64_t>(kl, cb::kZoneInline));
    if (kl > cb::kZoneInline) {  // a long key: the rest in one more copy
      const uint64_t i = w ? hr->idx_max : hr->idx_min;
      uint64_t o = 0;
      HIP_TRY(hipMemcpy(&o, p.dko + i, 8, hipMemcpyDeviceToHost));
      z.resize(kl);
      HIP_TRY(hipMemcpy(&z[cb::kZoneInline], p.dk + o + cb::kZoneInline, kl - cb::kZoneInline,
                        hipMemcpyDeviceToHost));
    }
  }
  t->has_zone = true;
  if (hr->flags[1]) {
    // a key holds '\n' or '\t': the file's lines are not the entries, so
    // index it the way SsTable::get splits it (src/sstable.rs:142-146)
    pool_release(t->device, t->rec, t->rec_cap);
    t->rec = nullptr;
    t->pfx = t->fence = nullptr;
    t->llen = nullptr;
    t->dir = nullptr;
    t->dmap = nullptr;
    t->nlines = 0;
    int rc = index_table(t, nullptr);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(nullptr));
  } else {
    t->fast = !hr->flags[2] && !g_table_exact;
  }
  return CB_OK;
}

}  // namespace

namespace cbx {

int finalize_table(cb_table* t) {
  if (!t->ready.load(std::memory_order_acquire)) {
    std::lock_guard<std::mutex> lk(t->fin_mu);
    if (!t->ready.load(std::memory_order_acquire)) {
      const int rc = finalize_locked(t);
      drop_pending(t);
      if (rc && !t->ferr) {
        t->ferr = rc;
        t->ferr_msg = cbx::g_err;
      }
      t->ready.store(true, std::memory_order_release);
    }
  }
  return t->ferr ? fail(t->ferr, t->ferr_msg.c_str()) : CB_OK;
}

}  // namespace cbx

namespace {
}  // namespace

extern "C" {

// ---- SSTable data files and the batched read path ----

int cb_table_destroy(cb_table* t) {
  if (!t) return CB_OK;
  {
    DeviceGuard dg(t->device);
    if (t->pend) {  // enqueued work may still be running: let it finish first
      std::lock_guard<std::mutex> lk(t->fin_mu);
      if (t->pend->ev && !t->ready.load()) (void)hipEventSynchronize(t->pend->ev);
      drop_pending(t);
    }
    pool_release(t->device, t->data, t->data_cap);
    pool_release(t->device, t->rec, t->rec_cap);  // rec heads the one index allocation
    if (t->bkt) pool_release(t->device, t->bkt, t->bkt_cap);
    if (t->bkt_ev) (void)hipEventDestroy(t->bkt_ev);
  }
  delete t;
  return CB_OK;
}

int cb_table_create(const uint8_t* data, uint64_t len, int device, void* stream, cb_table** out) {
  if (!out || (!data && len)) return fail(CB_EINVAL, "null argument");
  *out = nullptr;
  int rc = cb_init(device);
  if (rc) return rc;
  DeviceGuard dg(device);
  hipStream_t s = (hipStream_t)stream;
  note_stream(device, s);
  std::unique_ptr<cb_table, int (*)(cb_table*)> t(new cb_table(), cb_table_destroy);
  t->device = device;
  t->len = len;
  if (pool_alloc(device, len + 16, (void**)&t->data, &t->data_cap) != hipSuccess) {
    t->data = nullptr;
    return fail(CB_ENOMEM, "device allocation failed for an SSTable buffer");
  }
  HIP_TRY(hipMemsetAsync(t->data + len, 0, 16, s));
  if (len) HIP_TRY(hipMemcpyAsync(t->data, data, len, hipMemcpyDefault, s));
  if ((rc = index_table(t.get(), s))) return rc;
  HIP_TRY(hipStreamSynchronize(s));
  *out = t.release();
  return CB_OK;
}

int cb_table_data(const cb_table* t, const uint8_t** data, uint64_t* len) {
  if (!t) return fail(CB_EINVAL, "null table");
  if (int rc = finalize_table(const_cast<cb_table*>(t))) return rc;
  if (data) *data = t->data;
  if (len) *len = t->len;
  return CB_OK;
}

int cb_table_copy(const cb_table* t, uint64_t offset, uint64_t len, uint8_t* out) {
  if (!t || (!out && len)) return fail(CB_EINVAL, "null argument");
  if (int rc = finalize_table(const_cast<cb_table*>(t))) return rc;
  if (offset > t->len || len > t->len - offset) return fail(CB_EINVAL, "range outside the file");
  if (!len) return CB_OK;
  DeviceGuard dg(t->device);
  HIP_TRY(hipMemcpy(out, t->data + offset, len, hipMemcpyDefault));
  return CB_OK;
}

int cb_sstable_create(const uint8_t* keys, const uint64_t* key_off, const uint8_t* vals,
                      const uint64_t* val_off, uint64_t n, uint64_t m_bits, int device, void* stream,
                      cb_table** table_out, cb_filter** bloom_out, uint64_t* zone_min_idx,
                      uint64_t* zone_max_idx) {
  if (!table_out || !key_off || !val_off) return fail(CB_EINVAL, "null argument");
  if (zone_min_idx) *zone_min_idx = ~0ull;
  if (zone_max_idx) *zone_max_idx = ~0ull;
  // byte totals: host offsets carry them; device offsets are read back (one
  // round trip: cb_sstable_create_bounded takes the bounds instead)
  uint64_t kt = 0, vt = 0;
  const bool kdev = is_device_ptr(key_off), vdev = is_device_ptr(val_off);
  if (kdev || vdev) {
    int rc = cb_init(device);
    if (rc) return rc;
    DeviceGuard dg(device);
    hipStream_t s = (hipStream_t)stream;
    uint64_t tot[2] = {0, 0};
    if (kdev) HIP_TRY(hipMemcpyAsync(&tot[0], key_off + n, 8, hipMemcpyDeviceToHost, s));
    if (vdev) HIP_TRY(hipMemcpyAsync(&tot[1], val_off + n, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    kt = tot[0];
    vt = tot[1];
  }
  if (!kdev) kt = key_off[n];
  if (!vdev) vt = val_off[n];
  int rc = sstable_enqueue(keys, key_off, kt, vals, val_off, vt, n, m_bits, device, (hipStream_t)stream, table_out,
                           bloom_out);
  if (rc || !(zone_min_idx || zone_max_idx) || !n) return rc;
  // the zone map's input indices are host values: wait for them
  cb_table* t = *table_out;
  if ((rc = finalize_table(t))) {
    cb_table_destroy(t);
    *table_out = nullptr;
    if (bloom_out && *bloom_out) {
      cb_filter_destroy(*bloom_out);
      *bloom_out = nullptr;
    }
    return rc;
  }
  if (zone_min_idx) *zone_min_idx = t->zidx[0];
  if (zone_max_idx) *zone_max_idx = t->zidx[1];
  return CB_OK;
}

int cb_sstable_create_bounded(const uint8_t* keys, const uint64_t* key_off, uint64_t key_bytes, const uint8_t* vals,
                              const uint64_t* val_off, uint64_t val_bytes, uint64_t n, uint64_t m_bits, int device,
                              void* stream, cb_table** table_out, cb_filter** bloom_out) {
  if (!table_out || !key_off || !val_off) return fail(CB_EINVAL, "null argument");
  if (!is_device_ptr(key_off) && key_off[n] > key_bytes) return fail(CB_EINVAL, "key bytes exceed key_bytes");
  if (!is_device_ptr(val_off) && val_off[n] > val_bytes) return fail(CB_EINVAL, "value bytes exceed val_bytes");
  return sstable_enqueue(keys, key_off, key_bytes, vals, val_off, val_bytes, n, m_bits, device, (hipStream_t)stream,
                         table_out, bloom_out);
}

int cb_table_wait(const cb_table* t) {
  if (!t) return fail(CB_EINVAL, "null table");
  return finalize_table(const_cast<cb_table*>(t));
}

int cb_table_rebuild(const cb_table* t, uint64_t m_bits, void* stream, cb_filter** bloom_out,
                     uint64_t* zone_min_line, uint64_t* zone_max_line) {
  if (!t || !bloom_out) return fail(CB_EINVAL, "null argument");
  *bloom_out = nullptr;
  if (int rc = finalize_table(const_cast<cb_table*>(t))) return rc;
  if (zone_min_line) *zone_min_line = ~0ull;
  if (zone_max_line) *zone_max_line = ~0ull;
  hipStream_t s = (hipStream_t)stream;
  cb_filter* fp = nullptr;
  int rc = cb_filter_create(m_bits, t->device, &fp);  // BloomFilter::new(1024) (src/sstable.rs:111)
  if (rc) return rc;
  std::unique_ptr<cb_filter, int (*)(cb_filter*)> f(fp, cb_filter_destroy);
  const uint64_t nl = t->nlines;
  if (nl) {
    DeviceGuard dg(t->device);
    Workspace& ws = workspace(t->device, s);
    std::lock_guard<std::mutex> lk(ws.mu);
    HIP_TRY(ws.i_cnt.reserve((nl + 1) * 8, s));
    HIP_TRY(ws.i_base.reserve((nl + 1) * 8, s));
    HIP_TRY(ws.i_start.reserve((nl + 1) * 8, s));
    HIP_TRY(ws.i_end.reserve((nl + 1) * 8, s));
    HIP_TRY(ws.i_tmp.reserve(cb::scan_tmp_words(nl) * 8, s));
    HIP_TRY(ws.i_err.reserve(8, s));
    uint64_t* has = (uint64_t*)ws.i_cnt.p;
    uint64_t* has_scan = (uint64_t*)ws.i_base.p;
    uint64_t* klen = (uint64_t*)ws.i_start.p;
    uint64_t* len_scan = (uint64_t*)ws.i_end.p;
    uint64_t* bad = (uint64_t*)ws.i_err.p;
    HIP_TRY(hipMemsetAsync(bad, 0xFF, 8, s));
    HIP_TRY(cb::launch_rebuild_mark(t->data, t->rec, nl, has, klen, bad, s));
    HIP_TRY(cb::launch_scan_u64(has, has_scan, nl, (uint64_t*)ws.i_tmp.p, s));
    HIP_TRY(cb::launch_scan_u64(klen, len_scan, nl, (uint64_t*)ws.i_tmp.p, s));
    uint64_t h[3];
    HIP_TRY(hipMemcpyAsync(&h[0], bad, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&h[1], has_scan + nl, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&h[2], len_scan + nl, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (h[0] != ~0ull) {  // std::str::from_utf8(..).map_err(..)? (src/sstable.rs:115-116)
      char msg[96];
      std::snprintf(msg, sizeof msg, "SsTable::load: the key on line %llu is not UTF-8",
                    (unsigned long long)h[0]);
      return fail(CB_EUTF8, msg);
    }
    const uint64_t nk = h[1], kbytes = h[2];
    if (nk) {
      HIP_TRY(ws.lkey.reserve(kbytes + 16, s));
      HIP_TRY(ws.t_line.reserve((nk + 1) * 8, s));
      HIP_TRY(ws.t_which.reserve(nk * 8, s));
      uint8_t* kb = (uint8_t*)ws.lkey.p;
      uint64_t* ko = (uint64_t*)ws.t_line.p;
      uint64_t* lmap = (uint64_t*)ws.t_which.p;
      HIP_TRY(cb::launch_rebuild_gather(t->data, t->rec, nl, has_scan, len_scan, kb, ko, lmap, s));
      // bloom.insert(key) for every TAB line (src/sstable.rs:117)
      if ((rc = insert_locked(ws, f.get(), kb, ko, 0, nk, s))) return rc;
      // zone_map.update(key) for every TAB line (src/sstable.rs:118)
      HIP_TRY(ws.zone.reserve((2 * 1024 + 2) * 8, s));
      uint64_t* dtmp = (uint64_t*)ws.zone.p;
      uint64_t* didx = dtmp + 2 * 1024;
      HIP_TRY(cb::launch_zone_bounds(cb::KEY_VAR, cb::KeySrc{kb, ko, 0}, nk, dtmp, didx, s));
      uint64_t idx[2], line[2];
      HIP_TRY(hipMemcpyAsync(idx, didx, 16, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      HIP_TRY(hipMemcpyAsync(&line[0], lmap + idx[0], 8, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipMemcpyAsync(&line[1], lmap + idx[1], 8, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      if (zone_min_line) *zone_min_line = line[0];
      if (zone_max_line) *zone_max_line = line[1];
    }
  }
  *bloom_out = f.release();
  return CB_OK;
}

int cb_table_zone(const cb_table* t, int which, uint8_t* out, uint64_t cap, uint64_t* len) {
  if (!t || !len || (which != 0 && which != 1)) return fail(CB_EINVAL, "bad argument");
  if (int rc = finalize_table(const_cast<cb_table*>(t))) return rc;
  if (!t->has_zone) return fail(CB_EINVAL, "table has no zone bounds (not made by cb_sstable_create, or empty)");
  const std::string& z = which ? t->zmax : t->zmin;
  *len = z.size();
  if (out && cap) std::memcpy(out, z.data(), (size_t)std::min<uint64_t>(cap, z.size()));
  return CB_OK;
}

int cb_table_info(const cb_table* t, uint64_t* nlines, uint64_t* bytes) {
  if (!t) return fail(CB_EINVAL, "null table");
  if (int rc = finalize_table(const_cast<cb_table*>(t))) return rc;
  if (nlines) *nlines = t->nlines;
  if (bytes) *bytes = t->len;
  return CB_OK;
}

int cb_table_well_formed(const cb_table* t, int* out) {
  if (!t || !out) return fail(CB_EINVAL, "null argument");
  if (int rc = finalize_table(const_cast<cb_table*>(t))) return rc;
  *out = t->fast ? 1 : 0;
  return CB_OK;
}

int cb_table_force_exact(int on) {
  g_table_exact = on != 0;
  return CB_OK;
}

int cb_table_bucket_limit(uint64_t max_bytes) {
  g_bucket_limit.store(max_bytes, std::memory_order_relaxed);
  return CB_OK;
}

int cb_table_lines(const cb_table* t, uint64_t* start, uint32_t* key_len, uint32_t* line_len) {
  if (!t) return fail(CB_EINVAL, "null table");
  if (int rc = finalize_table(const_cast<cb_table*>(t))) return rc;
  DeviceGuard dg(t->device);
  if (!t->nlines) return CB_OK;
  // strided copies out of the 32-byte records
  const size_t pitch = sizeof(cb::LineRec);
  const uint8_t* r = (const uint8_t*)t->rec;
  if (start)
    HIP_TRY(hipMemcpy2D(start, 8, r + offsetof(cb::LineRec, start), pitch, 8, t->nlines, hipMemcpyDefault));
  if (key_len)
    HIP_TRY(hipMemcpy2D(key_len, 4, r + offsetof(cb::LineRec, klen), pitch, 4, t->nlines, hipMemcpyDefault));
  if (line_len) HIP_TRY(hipMemcpy(line_len, t->llen, t->nlines * 4, hipMemcpyDefault));
  return CB_OK;
}

int cb_table_search_fixed(const cb_table* t, const uint8_t* keys, uint32_t key_len, uint64_t n,
                          int64_t* line_out, void* stream) {
  return table_search_impl(t, keys, nullptr, key_len, n, line_out, (hipStream_t)stream);
}

int cb_table_search_var(const cb_table* t, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                        int64_t* line_out, void* stream) {
  if (!offsets) return fail(CB_EINVAL, "null offsets");
  return table_search_impl(t, bytes, offsets, 0, n, line_out, (hipStream_t)stream);
}

int cb_get_many_fixed(const cb_table* const* tables, uint32_t nt, const uint64_t* hits,
                      const uint32_t* hit_rows, const uint8_t* keys, uint32_t key_len, uint64_t n,
                      int32_t* which, uint64_t* val_off, uint8_t* vals, uint64_t cap,
                      uint64_t* total, void* stream) {
  return get_many_impl(tables, nt, hits, hit_rows, keys, nullptr, key_len, n, which, val_off, vals,
                       cap, total, (hipStream_t)stream);
}

int cb_get_many_var(const cb_table* const* tables, uint32_t nt, const uint64_t* hits,
                    const uint32_t* hit_rows, const uint8_t* bytes, const uint64_t* offsets,
                    uint64_t n, int32_t* which, uint64_t* val_off, uint8_t* vals, uint64_t cap,
                    uint64_t* total, void* stream) {
  if (!offsets) return fail(CB_EINVAL, "null offsets");
  return get_many_impl(tables, nt, hits, hit_rows, bytes, offsets, 0, n, which, val_off, vals, cap,
                       total, (hipStream_t)stream);
}

int cb_set_get_many_fixed(const cb_filterset* set, const cb_table* const* tables, uint32_t nt,
                          const uint32_t* slots, const uint8_t* keys, uint32_t key_len, uint64_t n,
                          int32_t* which, uint64_t* val_off, uint8_t* vals, uint64_t cap, uint64_t* total,
                          void* stream) {
  if (!set) return fail(CB_EINVAL, "null set");
  return get_many_impl(tables, nt, nullptr, slots, keys, nullptr, key_len, n, which, val_off, vals, cap, total,
                       (hipStream_t)stream, set);
}

int cb_set_get_many_var(const cb_filterset* set, const cb_table* const* tables, uint32_t nt,
                        const uint32_t* slots, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                        int32_t* which, uint64_t* val_off, uint8_t* vals, uint64_t cap, uint64_t* total,
                        void* stream) {
  if (!set) return fail(CB_EINVAL, "null set");
  if (!offsets) return fail(CB_EINVAL, "null offsets");
  return get_many_impl(tables, nt, nullptr, slots, bytes, offsets, 0, n, which, val_off, vals, cap, total,
                       (hipStream_t)stream, set);
}

}  // extern "C"
