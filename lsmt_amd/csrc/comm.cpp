// comm.cpp — the multi-GPU hit-bitmap exchange on the C ABI:
// an RCCL communicator per rank (one process per GPU) and cb_hits_allgather,
// which assembles the global [total_rows][words] hit map that Database::get's
// fan-out reads (/root/reference/src/lib.rs:129-134) from every rank's rows.
//
// Filters shard one contiguous subset per rank (shard_rows below, the same
// split as lsmt_amd/shard.py:shard_range), so rank r's rows are one
// contiguous slice of the global filter-major map:
//   dense  — one ncclAllGather of the rows (padded to the largest shard when
//            the shards are uneven, then each rank's rows copied into place);
//   sparse — cb_hits_compress of the rows into a fixed-size pack of set-bit
//            positions, one ncclAllGather of the packs, cb_hits_expand into
//            the dense map (every word written once). At BASELINE densities a
//            pack is ~1/10 of the dense rows.
// Everything is enqueued on the caller's stream; nothing is read back unless
// the caller asks for the synchronous overflow check (ok == NULL).
#include <rccl/rccl.h>

#include "capi_internal.hpp"

struct cb_comm {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1, device = 0;
  std::mutex mu;                  // one exchange at a time per communicator
  cbx::DevBuf pack, packs, pad;   // this rank's pack, the gathered packs, padded rows
  std::vector<uint32_t> counts;   // host: the gathered pack counts (sync overflow check)
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

int allgather_dense(cb_comm* c, const uint64_t* local, uint64_t rows, uint64_t words,
                    uint64_t total_rows, uint64_t* full, hipStream_t s) {
  const uint64_t max_rows = (total_rows + (uint64_t)c->world - 1) / (uint64_t)c->world;
  const bool even = total_rows % (uint64_t)c->world == 0;
  if (even) {  // every slice has max_rows rows: gather straight into the map
    NCCL_TRY(ncclAllGather(local, full, rows * words, ncclUint64, c->comm, s));
    return CB_OK;
  }
  const size_t slab = (size_t)max_rows * words * 8;
  HIP_TRY(c->pad.reserve(slab * (size_t)(c->world + 1), s));
  uint8_t* mine = (uint8_t*)c->pad.p;  // this rank's rows, padded to max_rows
  uint8_t* all = mine + slab;          // world slabs of max_rows rows
  if (rows) HIP_TRY(hipMemcpyAsync(mine, local, rows * words * 8, hipMemcpyDeviceToDevice, s));
  NCCL_TRY(ncclAllGather(mine, all, max_rows * words, ncclUint64, c->comm, s));
  for (int r = 0; r < c->world; ++r) {
    uint64_t lo, cnt;
    shard_rows(total_rows, c->world, r, &lo, &cnt);
    if (cnt)
      HIP_TRY(hipMemcpyAsync(full + lo * words, all + (size_t)r * slab, cnt * words * 8,
                             hipMemcpyDeviceToDevice, s));
  }
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
  if (world < 1 || (uint32_t)world > cb::kMaxRanks || rank < 0 || rank >= world)
    return fail(CB_EINVAL, "need 0 <= rank < world <= 64");
  int rc = cb_init(device);
  if (rc) return rc;
  DeviceGuard dg(device);  // ncclCommInitRank binds the communicator to the current device
  std::unique_ptr<cb_comm> c(new cb_comm());
  c->rank = rank;
  c->world = world;
  c->device = device;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  NCCL_TRY(ncclCommInitRank(&c->comm, world, u, rank));
  *out = c.release();
  return CB_OK;
}

int cb_comm_destroy(cb_comm* c) {
  if (!c) return CB_OK;
  {
    DeviceGuard dg(c->device);
    (void)hipDeviceSynchronize();  // queued exchanges may still use the buffers
    if (c->comm) (void)ncclCommDestroy(c->comm);
    for (DevBuf* b : {&c->pack, &c->packs, &c->pad})
      if (b->p) (void)hipFree(b->p);
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
  hipStream_t s = (hipStream_t)stream;
  DeviceGuard dg(c->device);
  std::lock_guard<std::mutex> lk(c->mu);
  if (mode == CB_XCHG_DENSE) return allgather_dense(c, local, rows, words, total_rows, full, s);

  if (!cap) return fail(CB_EINVAL, "sparse exchange needs cap > 0");
  const uint64_t max_rows = (total_rows + (uint64_t)c->world - 1) / (uint64_t)c->world;
  if (max_rows * words > cb::kMaxCompressWords) return fail(CB_EINVAL, "rows * words * 64 must be below 2^32");
  const size_t pack_words = cb::pack_words(max_rows * words, cap);  // equal on every rank
  HIP_TRY(c->pack.reserve(pack_words * 4, s));
  HIP_TRY(c->packs.reserve(pack_words * 4 * (size_t)c->world, s));
  uint32_t* pack = (uint32_t*)c->pack.p;
  uint32_t* packs = (uint32_t*)c->packs.p;
  {
    Workspace& ws = workspace(c->device, s);
    std::lock_guard<std::mutex> wl(ws.mu);
    cb::CompressState* st = nullptr;
    int rc = compress_state(ws, s, &st);
    if (rc) return rc;
    HIP_TRY(cb::launch_hits_compress(local, rows, words, pack, cap, *st, s));
  }
  NCCL_TRY(ncclAllGather(pack, packs, pack_words, ncclUint32, c->comm, s));
  cb::RankRows rr{};
  for (int r = 0; r < c->world; ++r) {
    uint64_t cnt;
    shard_rows(total_rows, c->world, r, &rr.row_off[r], &cnt);
  }
  if (!ok) {
    // synchronous check: every rank reads the same gathered counts and takes
    // the same decision, so either all expand or all redo the batch densely
    c->counts.assign((size_t)c->world, 0);
    HIP_TRY(hipMemcpy2DAsync(c->counts.data(), 4, packs, pack_words * 4, 4, (size_t)c->world,
                             hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (uint32_t v : c->counts)
      if (v > cap) return allgather_dense(c, local, rows, words, total_rows, full, s);
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
  if (max_rows > 64) return fail(CB_EINVAL, "more than 64 rows per rank");
  const uint64_t nblk = cb::set_probe_blocks(n);
  const size_t pack_words = 2 + cap + 2 * nblk;  // equal on every rank
  DeviceGuard dg(c->device);
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(c->pack.reserve(pack_words * 4, s));
  HIP_TRY(c->packs.reserve(pack_words * 4 * (size_t)c->world, s));
  uint32_t* pack = (uint32_t*)c->pack.p;
  uint32_t* packs = (uint32_t*)c->packs.p;
  // the probe writes this rank's rows and its pack in one launch
  int rc = set_probe_device(set, keys, key_len, n, gated != 0, local_hits, pack, cap, s);
  if (rc) return rc;
  NCCL_TRY(ncclAllGather(pack, packs, pack_words, ncclUint32, c->comm, s));
  if (!ok) {  // synchronous overflow check (as cb_hits_allgather): dense redo on every rank
    c->counts.assign((size_t)c->world, 0);
    HIP_TRY(hipMemcpy2DAsync(c->counts.data(), 4, packs, pack_words * 4, 4, (size_t)c->world,
                             hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (uint32_t v : c->counts)
      if (v > cap) return allgather_dense(c, local_hits, rows, hwords, total_rows, full, s);
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
