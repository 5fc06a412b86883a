// ubench_host.hip — host-side cost of the C2 build call and of the HIP
// primitives inside it (hipPointerGetAttributes, hipEventRecord, a kernel
// launch), each timed over 1000 back-to-back calls on one stream without a
// wait. Answers whether a pipelined build leg is bound by the host's issue
// rate. Diagnostic only; prints one JSON object.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "cassbloom.h"

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void k_nop(int* p) {
  if (p && threadIdx.x == 1024) p[0] = 1;
}

template <class F>
static double per_call_us(F f, int reps = 1000) {
  for (int i = 0; i < 20; ++i) f();
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; ++i) f();
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int main() {
  const uint64_t n = 1u << 20, m = 1ull << 27;
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint8_t* keys;
  CHECK(hipMalloc(&keys, n * 16));
  CHECK(hipMemset(keys, 7, n * 16));
  cb_filter* f = nullptr;
  if (cb_filter_create(m, 0, &f)) return 1;
  hipEvent_t ev;
  CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  hipPointerAttribute_t attr;
  const double t_attr = per_call_us([&] { (void)hipPointerGetAttributes(&attr, keys); });
  const double t_event = per_call_us([&] { (void)hipEventRecord(ev, s); });
  CHECK(hipStreamSynchronize(s));
  const double t_launch = per_call_us([&] { hipLaunchKernelGGL(k_nop, dim3(256), dim3(1024), 0, s, nullptr); });
  CHECK(hipStreamSynchronize(s));
  const double t_insert = per_call_us([&] { (void)cb_filter_insert_fixed(f, keys, 16, n, s); }, 300);
  CHECK(hipStreamSynchronize(s));
  const double t_clear = per_call_us([&] { (void)cb_filter_clear(f, s); });
  CHECK(hipStreamSynchronize(s));
  printf("{\"hipPointerGetAttributes_us\": %.2f, \"hipEventRecord_us\": %.2f, \"launch_us\": %.2f, "
         "\"cb_filter_insert_fixed_us\": %.2f, \"cb_filter_clear_us\": %.2f}\n",
         t_attr, t_event, t_launch, t_insert, t_clear);
  cb_filter_destroy(f);
  return 0;
}
