// create_host.hip — host cost of the product's flush (cb_sstable_create_bounded
// of a 1024-entry sorted memtable, m = 1024) from C, without Python: the
// per-call host time of K enqueue-only creates, and beside it the host cost of
// the HIP calls a create is made of (an empty kernel launch, a small
// hipMemsetAsync, a D2H copy into pinned memory, hipEventRecord). Output: one
// JSON object. Diagnostic only. Build: hipcc --offload-arch=gfx950 -O3 -Iinclude tools/create_host.hip -o build/create_host
// -Llsmt_amd -lcassbloom -Wl,-rpath,'$ORIGIN/../lsmt_amd'.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "cassbloom.h"

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

__global__ void k_nop(int* p) {
  if (p && threadIdx.x == 1023) p[0] = 1;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 200;
  const uint64_t n = argc > 2 ? strtoull(argv[2], nullptr, 10) : 1024;
  if (cb_init(0)) return 1;
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // sorted 16-byte hex keys and 16-byte values
  std::vector<uint8_t> kh(n * 16), vh(n * 16);
  std::vector<uint64_t> oh(n + 1);
  for (uint64_t i = 0; i < n; ++i) {
    snprintf((char*)&kh[i * 16], 17, "%016llx", (unsigned long long)(i * 2654435761ull));
    for (int j = 0; j < 16; ++j) vh[i * 16 + j] = (uint8_t)(i + j);
  }
  // sort the keys (as MemTable::scan hands them over)
  std::vector<std::vector<uint8_t>> rows(n);
  for (uint64_t i = 0; i < n; ++i) rows[i].assign(&kh[i * 16], &kh[i * 16] + 16);
  std::sort(rows.begin(), rows.end());
  for (uint64_t i = 0; i < n; ++i) memcpy(&kh[i * 16], rows[i].data(), 16);
  for (uint64_t i = 0; i <= n; ++i) oh[i] = 16 * i;
  uint8_t *kd, *vd;
  uint64_t* od;
  CHECK(hipMalloc(&kd, n * 16));
  CHECK(hipMalloc(&vd, n * 16));
  CHECK(hipMalloc(&od, (n + 1) * 8));
  CHECK(hipMemcpy(kd, kh.data(), n * 16, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(vd, vh.data(), n * 16, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(od, oh.data(), (n + 1) * 8, hipMemcpyHostToDevice));

  std::vector<cb_table*> ts(K);
  std::vector<cb_filter*> fs(K);
  auto creates = [&](int k, std::vector<double>* per) {
    for (int i = 0; i < k; ++i) {
      const double a = now_us();
      if (cb_sstable_create_bounded(kd, od, n * 16, vd, od, n * 16, n, 1024, 0, s, &ts[i], &fs[i])) {
        fprintf(stderr, "create failed: %s\n", cb_last_error());
        return 1;
      }
      if (per) per->push_back(now_us() - a);
    }
    for (int i = 0; i < k; ++i) {
      cb_table_wait(ts[i]);
      cb_table_destroy(ts[i]);
      cb_filter_destroy(fs[i]);
    }
    return 0;
  };
  if (creates(K, nullptr)) return 1;  // warm: pools, workspaces, result slots
  std::vector<double> per;
  if (creates(K, &per)) return 1;
  std::sort(per.begin(), per.end());
  double sum = 0;
  for (double v : per) sum += v;

  // the pieces
  auto host_per = [&](auto f) -> double {
    (void)hipStreamSynchronize(s);
    const double a = now_us();
    for (int i = 0; i < K; ++i) f();
    const double b = now_us();
    (void)hipStreamSynchronize(s);
    return (b - a) / K;
  };
  int* dflag;
  CHECK(hipMalloc(&dflag, 256));
  void* pinned;
  CHECK(hipHostMalloc(&pinned, 256, hipHostMallocDefault));
  hipEvent_t ev;
  CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const double t_launch = host_per([&] { hipLaunchKernelGGL(k_nop, dim3(4), dim3(256), 0, s, dflag); });
  const double t_memset = host_per([&] { (void)hipMemsetAsync(dflag, 0, 64, s); });
  const double t_d2h = host_per([&] { (void)hipMemcpyAsync(pinned, dflag, 64, hipMemcpyDeviceToHost, s); });
  const double t_event = host_per([&] { (void)hipEventRecord(ev, s); });
  const double t_query = host_per([&] { (void)hipEventQuery(ev); });
  printf("{\"n\": %llu, \"K\": %d, \"create_host_us\": {\"median\": %.2f, \"mean\": %.2f, \"p90\": %.2f}, "
         "\"api_host_us\": {\"kernel_launch\": %.2f, \"memset_async\": %.2f, \"d2h_pinned_async\": %.2f, "
         "\"event_record\": %.2f, \"event_query\": %.2f}}\n",
         (unsigned long long)n, K, per[per.size() / 2], sum / per.size(), per[per.size() * 9 / 10], t_launch, t_memset,
         t_d2h, t_event, t_query);
  return 0;
}
