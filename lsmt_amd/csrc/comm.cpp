// comm.cpp — the multi-GPU hit-bitmap exchange on the C ABI:
// a communicator per rank (one process per GPU) and cb_hits_allgather, which
// assembles the global [total_rows][words] hit map that Database::get's
// fan-out reads (/root/reference/src/lib.rs:129-134) from every rank's rows.
//
// Filters shard one contiguous subset per rank (shard_rows below, the same
// split as lsmt_amd/shard.py:shard_range), so rank r's rows are one
// contiguous slice of the global filter-major map:
//   dense  — one all-gather of the rows (padded to the largest shard when
//            the shards are uneven, then each rank's rows copied into place);
//   sparse — cb_hits_compress of the rows into a fixed-size pack of set-bit
//            positions, one all-gather of the packs, cb_hits_expand into
//            the dense map (every word written once). At BASELINE densities a
//            pack is ~1/10 of the dense rows.
// Everything is enqueued on the caller's stream; nothing is read back unless
// the caller asks for the synchronous overflow check (ok == NULL).
//
// The all-gather of bytes is the only step that depends on the transport:
//   RCCL     — ncclAllGather over xGMI (the product path);
//   loopback — every rank in one process (one host thread per rank), device
//              copies between the ranks' buffers (tests at world > 1 on one GPU);
//   host     — a caller-supplied all-gather of host bytes.
// Collectives of one communicator run one after another in issue order even
// when they come from several streams (pipeline lanes): each waits on an
// event recorded after the previous one, and each stream has its own packs.
#include <rccl/rccl.h>

#include <condition_variable>

#include "capi_internal.hpp"

namespace {

enum Transport { kRccl = 0, kLoopback = 1, kHost = 2 };

// Loopback group: the rendezvous of `world` host threads, one per rank.
struct LoopGroup {
  int world = 1;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;  // cb_comm_abort on any rank: every waiter returns, every later call fails
  std::vector<const void*> send;
  std::vector<size_t> bytes;
  std::vector<hipEvent_t> ready, done;  // per rank: its send data written / its copies issued
  std::vector<int> err;                 // per rank: a step failed (every rank then fails the call)

  // false: the group was aborted (the rendezvous will not complete)
  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) return false;
    const uint64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g || aborted; });
    }
    return !aborted;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
  }
  ~LoopGroup() {
    for (hipEvent_t e : ready)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : done)
      if (e) (void)hipEventDestroy(e);
  }
};

}  // namespace

struct cb_comm {
  int transport = kRccl;
  ncclComm_t comm = nullptr;
  std::shared_ptr<LoopGroup> loop;
  cb_host_allgather_fn host_fn = nullptr;
  void* host_user = nullptr;
  std::vector<uint8_t> host_send, host_recv;
  int rank = 0, world = 1, device = 0;
  std::mutex mu;  // one exchange call at a time per communicator (host side)
  struct Bufs {
    cbx::DevBuf pack, packs, pad;  // this rank's pack, the gathered packs, padded rows
  };
  std::map<hipStream_t, Bufs> bufs;  // per calling stream: pipelined lanes never share a pack
  hipEvent_t order = nullptr;        // recorded after the last collective
  hipStream_t order_stream = nullptr;
  bool order_set = false;
  std::vector<uint32_t> counts;  // host: the gathered pack counts (sync overflow check)
  // cb_comm_abort (any thread, even while another is inside a collective):
  // RCCL's communicator is aborted and freed, every later call fails
  std::atomic<bool> aborted{false};
};

namespace {

using namespace cbx;

int nccl_fail(ncclResult_t r, const char* where) {
  std::string m = std::string(where) + ": " + ncclGetErrorString(r);
  const char* last = ncclGetLastError(nullptr);
  if (last && *last) m += std::string(" (") + last + ")";
  return fail(CB_EHIP, m.c_str());
}

#define NCCL_TRY(expr)                                   \
  do {                                                   \
    ncclResult_t _r = (expr);                            \
    if (_r != ncclSuccess) return nccl_fail(_r, #expr);  \
  } while (0)

// Rows of rank r when n rows are split over world ranks: contiguous, sizes
// differing by at most one, the larger shards first.
void shard_rows(uint64_t n, int world, int r, uint64_t* lo, uint64_t* cnt) {
  const uint64_t base = n / (uint64_t)world, extra = n % (uint64_t)world;
  *lo = (uint64_t)r * base + std::min<uint64_t>((uint64_t)r, extra);
  *cnt = base + ((uint64_t)r < extra ? 1 : 0);
}

// Loopback all-gather: three rendezvous per call. (1) every rank publishes
// its send pointer and an event after its send data; (2) every rank's stream
// waits for every sender's event and copies the senders' bytes into its own
// receive buffer, then records an event after its copies; (3) every rank's
// stream waits for every other rank's copies (so it never overwrites its
// send buffer while a peer still reads it). No early return between the
// rendezvous: a rank that fails a step still takes part, and every rank then
// reports the failure.
int loop_allgather(cb_comm* c, const void* send, void* recv, size_t bytes, hipStream_t s) {
  LoopGroup& g = *c->loop;
  const int me = c->rank;
  hipError_t e = hipEventRecord(g.ready[me], s);
  {
    std::lock_guard<std::mutex> lk(g.mu);
    g.send[me] = send;
    g.bytes[me] = bytes;
    g.err[me] = e != hipSuccess;
  }
  if (!g.barrier()) return fail(CB_EINVAL, "loopback all-gather: the communicator was aborted");
  bool bad = false;
  for (int r = 0; r < g.world; ++r) bad |= g.err[r] || g.bytes[r] != bytes;
  if (!g.barrier()) return fail(CB_EINVAL, "loopback all-gather: the communicator was aborted");
  if (!bad) {
    for (int r = 0; r < g.world && e == hipSuccess; ++r) {
      e = hipStreamWaitEvent(s, g.ready[r], 0);
      if (e == hipSuccess && bytes)
        e = hipMemcpyAsync((uint8_t*)recv + (size_t)r * bytes, g.send[r], bytes, hipMemcpyDeviceToDevice, s);
    }
    if (e == hipSuccess) e = hipEventRecord(g.done[me], s);
  }
  {
    std::lock_guard<std::mutex> lk(g.mu);
    g.err[me] = e != hipSuccess;
  }
  if (!g.barrier()) return fail(CB_EINVAL, "loopback all-gather: the communicator was aborted");
  for (int r = 0; r < g.world; ++r) bad |= g.err[r] != 0;
  if (!bad)
    for (int r = 0; r < g.world && e == hipSuccess; ++r)
      if (r != me) e = hipStreamWaitEvent(s, g.done[r], 0);
  if (!g.barrier()) return fail(CB_EINVAL, "loopback all-gather: the communicator was aborted");  // events reusable after
  if (e != hipSuccess) return hip_fail(e, "loopback all-gather");
  if (bad) return fail(CB_EINVAL, "loopback all-gather: a rank failed or the ranks' sizes differ");
  return CB_OK;
}

int host_allgather(cb_comm* c, const void* send, void* recv, size_t bytes, hipStream_t s) {
  c->host_send.resize(bytes);
  c->host_recv.resize(bytes * (size_t)c->world);
  if (bytes) HIP_TRY(hipMemcpyAsync(c->host_send.data(), send, bytes, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const int rc = c->host_fn(c->host_user, c->host_send.data(), c->host_recv.data(), (uint64_t)bytes);
  if (rc) return fail(CB_EINVAL, "the caller's host all-gather failed");
  if (bytes)
    HIP_TRY(hipMemcpyAsync(recv, c->host_recv.data(), bytes * (size_t)c->world, hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));  // host_recv is reused by the next call
  return CB_OK;
}

// The all-gather of `bytes` per rank from send into recv (world * bytes), on
// stream s, after the communicator's previous collective (any stream).
int allgather_bytes(cb_comm* c, const void* send, void* recv, size_t bytes, hipStream_t s) {
  if (c->aborted.load()) return fail(CB_EINVAL, "the communicator was aborted (cb_comm_abort)");
  if (c->order_set && c->order_stream != s) HIP_TRY(hipStreamWaitEvent(s, c->order, 0));
  int rc = CB_OK;
  switch (c->transport) {
    case kRccl:
      if (bytes % 4 == 0) {
        NCCL_TRY(ncclAllGather(send, recv, bytes / 4, ncclUint32, c->comm, s));
      } else {
        NCCL_TRY(ncclAllGather(send, recv, bytes, ncclUint8, c->comm, s));
      }
      break;
    case kLoopback:
      rc = loop_allgather(c, send, recv, bytes, s);
      break;
    default:
      rc = host_allgather(c, send, recv, bytes, s);
  }
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c->order, s));
  c->order_stream = s;
  c->order_set = true;
  return CB_OK;
}

int allgather_dense(cb_comm* c, cb_comm::Bufs& b, const uint64_t* local, uint64_t rows, uint64_t words,
                    uint64_t total_rows, uint64_t* full, hipStream_t s) {
  const uint64_t max_rows = (total_rows + (uint64_t)c->world - 1) / (uint64_t)c->world;
  const bool even = total_rows % (uint64_t)c->world == 0;
  if (even)  // every slice has max_rows rows: gather straight into the map
    return allgather_bytes(c, local, full, rows * words * 8, s);
  const size_t slab = (size_t)max_rows * words * 8;
  HIP_TRY(b.pad.reserve(slab * (size_t)(c->world + 1), s));
  uint8_t* mine = (uint8_t*)b.pad.p;  // this rank's rows, padded to max_rows
  uint8_t* all = mine + slab;         // world slabs of max_rows rows
  if (rows) HIP_TRY(hipMemcpyAsync(mine, local, rows * words * 8, hipMemcpyDeviceToDevice, s));
  if (rows < max_rows)  // the padding row is not part of any rank's map, but keep it defined
    HIP_TRY(hipMemsetAsync(mine + rows * words * 8, 0, (max_rows - rows) * words * 8, s));
  int rc = allgather_bytes(c, mine, all, slab, s);
  if (rc) return rc;
  for (int r = 0; r < c->world; ++r) {
    uint64_t lo, cnt;
    shard_rows(total_rows, c->world, r, &lo, &cnt);
    if (cnt)
      HIP_TRY(hipMemcpyAsync(full + lo * words, all + (size_t)r * slab, cnt * words * 8,
                             hipMemcpyDeviceToDevice, s));
  }
  return CB_OK;
}

// The synchronous overflow check after the packs' all-gather: every rank
// reads the same gathered counts and takes the same decision.
int any_overflow(cb_comm* c, const uint32_t* packs, size_t pack_words, uint64_t cap, hipStream_t s,
                 bool* over) {
  c->counts.assign((size_t)c->world, 0);
  HIP_TRY(hipMemcpy2DAsync(c->counts.data(), 4, packs, pack_words * 4, 4, (size_t)c->world,
                           hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  *over = false;
  for (uint32_t v : c->counts) *over |= v > cap;
  return CB_OK;
}

int new_comm(int rank, int world, int device, std::unique_ptr<cb_comm>* out) {
  std::unique_ptr<cb_comm> c(new cb_comm());
  c->rank = rank;
  c->world = world;
  c->device = device;
  // the order event is only waited on by other streams of the same device
  // (hipStreamWaitEvent before the next collective): a device-scope release
  // is enough, so no system-scope fence (an L2 write-back per record, paid
  // in GPU time every step; round 3 measured the zone-read events' fence)
  unsigned order_flags = hipEventDisableTiming | hipEventDisableSystemFence;
#ifdef CB_EXPERIMENTS
  if (const char* e = getenv("CB_ORDER_FENCE"); e && e[0] == '1')  // A/B: the fenced event
    order_flags = hipEventDisableTiming;
#endif
  HIP_TRY(hipEventCreateWithFlags(&c->order, order_flags));
  *out = std::move(c);
  return CB_OK;
}

// cb_set_probe_allgather_fixed's pack format: the fused probe's
// per-probe-block pack, or the separate compress's. Every rank must choose
// the same, since the two all-gather different byte counts in different
// layouts (a choice read from the rank's own set, whose zone
// state or width may differ, can split the ranks and hang the collective).
// So the choice reads only what every rank of one call shares: max_rows
// (from total_rows and world), n, the caller's gated flag and m (uniform over
// a store's tables: every SSTable filter has the same m,
// /root/reference/src/sstable.rs:44,59). A gated call always takes the fused
// pack (the dense probe does not gate); an ungated dense-shaped batch takes
// the separate compress, whichever kernel each rank's probe then runs (the
// density test is priced at the width the shard would use).
bool sparse_separate(uint64_t max_rows, uint64_t m, uint64_t n, bool gated) {
  if (max_rows > 64) return true;
  return !gated && cb::set_probe_dense_ok(max_rows <= 32 ? 32u : 64u, m, n);
}

int check_world(int rank, int world) {
  if (world < 1 || (uint32_t)world > cb::kMaxRanks || rank < 0 || rank >= world)
    return fail(CB_EINVAL, "need 0 <= rank < world <= 64");
  return CB_OK;
}

}  // namespace

extern "C" {

int cb_comm_unique_id(uint8_t* id) {
  if (!id) return fail(CB_EINVAL, "null id");
  static_assert(sizeof(ncclUniqueId) == CB_COMM_ID_BYTES, "RCCL unique id size");
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u));
  std::memcpy(id, &u, sizeof(u));
  return CB_OK;
}

int cb_comm_init(int rank, int world, const uint8_t* id, int device, cb_comm** out) {
  if (!out || !id) return fail(CB_EINVAL, "null argument");
  *out = nullptr;
  int rc = check_world(rank, world);
  if (rc) return rc;
  rc = cb_init(device);
  if (rc) return rc;
  DeviceGuard dg(device);  // ncclCommInitRank binds the communicator to the current device
  std::unique_ptr<cb_comm> c;
  rc = new_comm(rank, world, device, &c);
  if (rc) return rc;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  NCCL_TRY(ncclCommInitRank(&c->comm, world, u, rank));
  *out = c.release();
  return CB_OK;
}

int cb_comm_init_loopback(int world, int device, cb_comm** ranks) {
  if (!ranks) return fail(CB_EINVAL, "null argument");
  int rc = check_world(0, world);
  if (rc) return rc;
  for (int r = 0; r < world; ++r) ranks[r] = nullptr;
  rc = cb_init(device);
  if (rc) return rc;
  DeviceGuard dg(device);
  auto g = std::make_shared<LoopGroup>();
  g->world = world;
  g->send.assign((size_t)world, nullptr);
  g->bytes.assign((size_t)world, 0);
  g->err.assign((size_t)world, 0);
  g->ready.assign((size_t)world, nullptr);
  g->done.assign((size_t)world, nullptr);
  for (int r = 0; r < world; ++r) {
    HIP_TRY(hipEventCreateWithFlags(&g->ready[r], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&g->done[r], hipEventDisableTiming));
  }
  std::vector<std::unique_ptr<cb_comm>> made((size_t)world);
  for (int r = 0; r < world; ++r) {
    rc = new_comm(r, world, device, &made[r]);
    if (rc) return rc;
    made[r]->transport = kLoopback;
    made[r]->loop = g;
  }
  for (int r = 0; r < world; ++r) ranks[r] = made[r].release();
  return CB_OK;
}

int cb_comm_init_host(int rank, int world, int device, cb_host_allgather_fn fn, void* user, cb_comm** out) {
  if (!out || !fn) return fail(CB_EINVAL, "null argument");
  *out = nullptr;
  int rc = check_world(rank, world);
  if (rc) return rc;
  rc = cb_init(device);
  if (rc) return rc;
  DeviceGuard dg(device);
  std::unique_ptr<cb_comm> c;
  rc = new_comm(rank, world, device, &c);
  if (rc) return rc;
  c->transport = kHost;
  c->host_fn = fn;
  c->host_user = user;
  *out = c.release();
  return CB_OK;
}

int cb_comm_abort(cb_comm* c) {
  if (!c) return fail(CB_EINVAL, "null comm");
  if (c->aborted.exchange(true)) return CB_OK;  // once
  if (c->loop) c->loop->abort();
  if (c->transport == kRccl && c->comm) {
    DeviceGuard dg(c->device);
    // ncclCommAbort may run while another thread is blocked in a collective
    // of this communicator (its documented use): the collective returns an
    // error, the kernels it queued end, and the communicator is freed
    NCCL_TRY(ncclCommAbort(c->comm));
  }
  return CB_OK;
}

int cb_comm_destroy(cb_comm* c) {
  if (!c) return CB_OK;
  {
    DeviceGuard dg(c->device);
    (void)hipDeviceSynchronize();  // queued exchanges may still use the buffers
    if (c->comm && !c->aborted.load()) (void)ncclCommDestroy(c->comm);  // (an aborted one is already freed)
    for (auto& kv : c->bufs)
      for (DevBuf* b : {&kv.second.pack, &kv.second.packs, &kv.second.pad})
        if (b->p) (void)hipFree(b->p);
    if (c->order) (void)hipEventDestroy(c->order);
  }
  delete c;
  return CB_OK;
}

int cb_comm_info(const cb_comm* c, int* rank, int* world, int* device) {
  if (!c) return fail(CB_EINVAL, "null comm");
  if (rank) *rank = c->rank;
  if (world) *world = c->world;
  if (device) *device = c->device;
  return CB_OK;
}

int cb_comm_shard(uint64_t total_rows, int world, int rank, uint64_t* first_row, uint64_t* rows) {
  if (world < 1 || rank < 0 || rank >= world) return fail(CB_EINVAL, "need 0 <= rank < world");
  uint64_t lo, cnt;
  shard_rows(total_rows, world, rank, &lo, &cnt);
  if (first_row) *first_row = lo;
  if (rows) *rows = cnt;
  return CB_OK;
}

int cb_hits_allgather(cb_comm* c, const uint64_t* local, uint64_t rows, uint64_t words,
                      uint64_t total_rows, uint64_t* full, int mode, uint64_t cap, uint32_t* ok,
                      int* sparse_used, void* stream) {
  if (!c) return fail(CB_EINVAL, "null comm");
  if (sparse_used) *sparse_used = 0;
  if (!full || (rows && words && !local)) return fail(CB_EINVAL, "null argument");
  if (mode != CB_XCHG_DENSE && mode != CB_XCHG_SPARSE) return fail(CB_EINVAL, "mode must be dense or sparse");
  uint64_t lo, want;
  shard_rows(total_rows, c->world, c->rank, &lo, &want);
  if (rows != want) return fail(CB_EINVAL, "rows differ from this rank's shard of total_rows");
  if (!words || !total_rows) return CB_OK;
  if (!is_device_ptr(full) || (rows && !is_device_ptr(local)))
    return fail(CB_EINVAL, "local and full must be device memory on the communicator's device");
  if (mode == CB_XCHG_SPARSE && !cap) return fail(CB_EINVAL, "sparse exchange needs cap > 0");
  const uint64_t max_rows = (total_rows + (uint64_t)c->world - 1) / (uint64_t)c->world;
  if (mode == CB_XCHG_SPARSE && max_rows * words > cb::kMaxCompressWords)
    return fail(CB_EINVAL, "rows * words * 64 must be below 2^32");
  hipStream_t s = (hipStream_t)stream;
  DeviceGuard dg(c->device);
  std::lock_guard<std::mutex> lk(c->mu);
  cb_comm::Bufs& b = c->bufs[s];
  if (mode == CB_XCHG_DENSE) return allgather_dense(c, b, local, rows, words, total_rows, full, s);

  const size_t pack_words = cb::pack_words(max_rows * words, cap);  // equal on every rank
  HIP_TRY(b.pack.reserve(pack_words * 4, s));
  HIP_TRY(b.packs.reserve(pack_words * 4 * (size_t)c->world, s));
  uint32_t* pack = (uint32_t*)b.pack.p;
  uint32_t* packs = (uint32_t*)b.packs.p;
  {
    Workspace& ws = workspace(c->device, s);
    std::lock_guard<std::mutex> wl(ws.mu);
    cb::CompressState* st = nullptr;
    int rc = compress_state(ws, s, &st);
    if (rc) return rc;
    HIP_TRY(cb::launch_hits_compress(local, rows, words, pack, cap, *st, s));
  }
  int rc = allgather_bytes(c, pack, packs, pack_words * 4, s);
  if (rc) return rc;
  if (!ok) {
    bool over = false;
    rc = any_overflow(c, packs, pack_words, cap, s, &over);
    if (rc) return rc;
    if (over) return allgather_dense(c, b, local, rows, words, total_rows, full, s);
  }
  cb::RankRows rr{};
  for (int r = 0; r < c->world; ++r) {
    uint64_t cnt;
    shard_rows(total_rows, c->world, r, &rr.row_off[r], &cnt);
  }
  HIP_TRY(cb::launch_hits_expand(packs, (uint32_t)c->world, cap, rr, words, total_rows, full, ok, s));
  if (sparse_used) *sparse_used = 1;
  return CB_OK;
}

int cb_set_probe_allgather_fixed(cb_comm* c, const cb_filterset* set, const uint8_t* keys, uint32_t key_len,
                                 uint64_t n, int gated, uint64_t* local_hits, uint64_t total_rows, uint64_t* full,
                                 int mode, uint64_t cap, uint32_t* ok, int* sparse_used, void* stream) {
  if (!c || !set) return fail(CB_EINVAL, "null comm or set");
  if (sparse_used) *sparse_used = 0;
  if (mode != CB_XCHG_DENSE && mode != CB_XCHG_SPARSE) return fail(CB_EINVAL, "mode must be dense or sparse");
  if (set->device != c->device) return fail(CB_EINVAL, "the set and the communicator live on different devices");
  uint64_t lo, rows;
  shard_rows(total_rows, c->world, c->rank, &lo, &rows);
  if (rows != set->used) return fail(CB_EINVAL, "the set's used slots differ from this rank's shard of total_rows");
  if (!n || !total_rows) return CB_OK;
  if (!local_hits || !full) return fail(CB_EINVAL, "null hits");
  const uint64_t hwords = (n + 63) / 64;
  hipStream_t s = (hipStream_t)stream;
  if (mode == CB_XCHG_DENSE) {
    int rc = set_probe_device(set, keys, key_len, n, gated != 0, local_hits, nullptr, 0, s);
    if (rc) return rc;
    return cb_hits_allgather(c, local_hits, rows, hwords, total_rows, full, CB_XCHG_DENSE, 0, nullptr, nullptr,
                             stream);
  }
  if (!cap) return fail(CB_EINVAL, "sparse exchange needs cap > 0");
  const uint64_t max_rows = (total_rows + (uint64_t)c->world - 1) / (uint64_t)c->world;
  if (sparse_separate(max_rows, set->m, n, gated != 0)) {
    // shards past 64 tables (wide sets: the product's hundreds of m = 1024
    // tables over a few GPUs), and dense batches (C5: the region-partitioned
    // probe writes no pack): the probe writes the rows, then the separate
    // compress and the same sparse all-gather. The branch depends only on
    // values every rank shares (sparse_separate); each rank's own probe
    // still picks its kernel from its own set.
    int rc = set_probe_device(set, keys, key_len, n, gated != 0, local_hits, nullptr, 0, s);
    if (rc) return rc;
    return cb_hits_allgather(c, local_hits, rows, hwords, total_rows, full, CB_XCHG_SPARSE, cap, ok, sparse_used,
                             stream);
  }
  if (max_rows * hwords * 64 >= (1ull << 32)) return fail(CB_EINVAL, "rows * ceil(n/64) * 64 must be below 2^32");
  const uint64_t nblk = cb::set_probe_blocks(n);
  const size_t pack_words = 2 + cap + 2 * nblk;  // equal on every rank
  DeviceGuard dg(c->device);
  std::lock_guard<std::mutex> lk(c->mu);
  cb_comm::Bufs& b = c->bufs[s];
  HIP_TRY(b.pack.reserve(pack_words * 4, s));
  HIP_TRY(b.packs.reserve(pack_words * 4 * (size_t)c->world, s));
  uint32_t* pack = (uint32_t*)b.pack.p;
  uint32_t* packs = (uint32_t*)b.packs.p;
  // the probe writes this rank's rows and its pack in one launch
  int rc = set_probe_device(set, keys, key_len, n, gated != 0, local_hits, pack, cap, s);
  if (rc) return rc;
  rc = allgather_bytes(c, pack, packs, pack_words * 4, s);
  if (rc) return rc;
  if (!ok) {  // synchronous overflow check (as cb_hits_allgather): dense redo on every rank
    bool over = false;
    rc = any_overflow(c, packs, pack_words, cap, s, &over);
    if (rc) return rc;
    if (over) return allgather_dense(c, b, local_hits, rows, hwords, total_rows, full, s);
  }
  cb::RankRows rr{};
  for (int r = 0; r < c->world; ++r) {
    uint64_t cnt;
    shard_rows(total_rows, c->world, r, &rr.row_off[r], &cnt);
  }
  HIP_TRY(cb::launch_hits_expand_blocks(packs, (uint32_t)c->world, cap, pack_words, rr, hwords, total_rows,
                                        (uint32_t)nblk, cb::kSetWords, full, ok, s));
  if (sparse_used) *sparse_used = 1;
  return CB_OK;
}

}  // extern "C"
