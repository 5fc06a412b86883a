// ubench_pcie.hip — the host<->device legs of the end-to-end probe (SURVEY.md
// §8d: 16 MiB of keys in, a 4 MiB hit bitmap out, pinned host memory), timed
// in the forms the library could use:
//   h2d / d2h          one hipMemcpyAsync (SDMA)
//   d2h_2d             the [32][2048]-word column block of a [32][16384] map
//                      as one hipMemcpy2DAsync (what a chunked pipeline does)
//   d2h_rows           the same block as 32 row copies
//   both               h2d and d2h on two streams at once (full duplex?)
//   k_write_host       a kernel storing 4 MiB straight into pinned memory
//   k_read_host        a kernel loading 16 MiB straight from pinned memory
// Output: one JSON object, microseconds and GB/s. Diagnostic only.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__global__ void k_write(uint4* dst, size_t n16) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
    dst[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

__global__ void k_read(const uint4* src, size_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

template <class F>
static double us(F f, int reps) {
  f();
  CHECK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  double tot = 0;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(a, 0));
    f();
    CHECK(hipEventRecord(b, 0));
    CHECK(hipDeviceSynchronize());
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    tot += ms;
  }
  return tot * 1e3 / reps;
}

int main() {
  const size_t KB = 16u << 20, HB = 4u << 20;
  void *hk, *hh, *dk, *dh;
  uint32_t* dout;
  CHECK(hipHostMalloc(&hk, KB, hipHostMallocDefault));
  CHECK(hipHostMalloc(&hh, HB, hipHostMallocDefault));
  CHECK(hipMalloc(&dk, KB));
  CHECK(hipMalloc(&dh, HB));
  CHECK(hipMalloc(&dout, 64));
  hipStream_t s1, s2;
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const int reps = 10;
  const double t_h2d = us([&] { CHECK(hipMemcpyAsync(dk, hk, KB, hipMemcpyHostToDevice, 0)); }, reps);
  const double t_d2h = us([&] { CHECK(hipMemcpyAsync(hh, dh, HB, hipMemcpyDeviceToHost, 0)); }, reps);
  // one 2048-word column block of a [32][16384] uint64 map
  const double t_2d = us([&] {
    CHECK(hipMemcpy2DAsync(hh, 16384 * 8, dh, 2048 * 8, 2048 * 8, 32, hipMemcpyDeviceToHost, 0));
  }, reps);
  const double t_rows = us([&] {
    for (int r = 0; r < 32; ++r)
      CHECK(hipMemcpyAsync((char*)hh + r * 16384 * 8, (char*)dh + r * 2048 * 8, 2048 * 8,
                           hipMemcpyDeviceToHost, 0));
  }, reps);
  hipEvent_t e0;
  CHECK(hipEventCreate(&e0));
  const double t_both = us([&] {
    CHECK(hipEventRecord(e0, 0));
    CHECK(hipStreamWaitEvent(s1, e0, 0));
    CHECK(hipStreamWaitEvent(s2, e0, 0));
    CHECK(hipMemcpyAsync(dk, hk, KB, hipMemcpyHostToDevice, s1));
    CHECK(hipMemcpyAsync(hh, dh, HB, hipMemcpyDeviceToHost, s2));
    hipEvent_t x1, x2;
    CHECK(hipEventCreateWithFlags(&x1, hipEventDisableTiming));
    CHECK(hipEventCreateWithFlags(&x2, hipEventDisableTiming));
    CHECK(hipEventRecord(x1, s1));
    CHECK(hipEventRecord(x2, s2));
    CHECK(hipStreamWaitEvent(0, x1, 0));
    CHECK(hipStreamWaitEvent(0, x2, 0));
  }, reps);
  // chunked pipelines over the same 16 MiB in / 4 MiB out, 4 chunks
  const int NC = 4;
  const size_t kc = KB / NC, hc = HB / NC;
  hipEvent_t ein[NC], erun[NC];
  for (int c = 0; c < NC; ++c) {
    CHECK(hipEventCreateWithFlags(&ein[c], hipEventDisableTiming));
    CHECK(hipEventCreateWithFlags(&erun[c], hipEventDisableTiming));
  }
  // P0: everything on one stream, chunk by chunk (no overlap possible)
  const double t_p0 = us([&] {
    for (int c = 0; c < NC; ++c) {
      CHECK(hipMemcpyAsync((char*)dk + c * kc, (char*)hk + c * kc, kc, hipMemcpyHostToDevice, 0));
      hipLaunchKernelGGL(k_read, dim3(256), dim3(256), 0, 0, (const uint4*)((char*)dk + c * kc), kc / 16, dout);
      CHECK(hipMemcpyAsync((char*)hh + c * hc, (char*)dh + c * hc, hc, hipMemcpyDeviceToHost, 0));
    }
  }, reps);
  // P1: H2D on s1, kernel on the null stream, D2H on s2, events between
  const double t_p1 = us([&] {
    CHECK(hipEventRecord(e0, 0));
    CHECK(hipStreamWaitEvent(s1, e0, 0));
    for (int c = 0; c < NC; ++c) {
      CHECK(hipMemcpyAsync((char*)dk + c * kc, (char*)hk + c * kc, kc, hipMemcpyHostToDevice, s1));
      CHECK(hipEventRecord(ein[c], s1));
      CHECK(hipStreamWaitEvent(0, ein[c], 0));
      hipLaunchKernelGGL(k_read, dim3(256), dim3(256), 0, 0, (const uint4*)((char*)dk + c * kc), kc / 16, dout);
      CHECK(hipEventRecord(erun[c], 0));
      CHECK(hipStreamWaitEvent(s2, erun[c], 0));
      CHECK(hipMemcpyAsync((char*)hh + c * hc, (char*)dh + c * hc, hc, hipMemcpyDeviceToHost, s2));
    }
    CHECK(hipStreamSynchronize(s2));
  }, reps);
  // P2: H2D on s1, the kernel writes its output straight into pinned memory
  const double t_p2 = us([&] {
    CHECK(hipEventRecord(e0, 0));
    CHECK(hipStreamWaitEvent(s1, e0, 0));
    for (int c = 0; c < NC; ++c) {
      CHECK(hipMemcpyAsync((char*)dk + c * kc, (char*)hk + c * kc, kc, hipMemcpyHostToDevice, s1));
      CHECK(hipEventRecord(ein[c], s1));
      CHECK(hipStreamWaitEvent(0, ein[c], 0));
      hipLaunchKernelGGL(k_read, dim3(256), dim3(256), 0, 0, (const uint4*)((char*)dk + c * kc), kc / 16, dout);
      hipLaunchKernelGGL(k_write, dim3(256), dim3(256), 0, 0, (uint4*)((char*)hh + c * hc), hc / 16);
    }
  }, reps);
  printf("{\"pipe4_one_stream_us\": %.1f, \"pipe4_three_streams_us\": %.1f, \"pipe4_h2d_stream_kernel_writes_host_us\": %.1f}\n",
         t_p0, t_p1, t_p2);
  void *dhk = nullptr, *dhh = nullptr;
  CHECK(hipHostGetDevicePointer(&dhk, hk, 0));
  CHECK(hipHostGetDevicePointer(&dhh, hh, 0));
  const double t_kw = us([&] { hipLaunchKernelGGL(k_write, dim3(1024), dim3(256), 0, 0, (uint4*)dhh, HB / 16); }, reps);
  const double t_kr = us([&] { hipLaunchKernelGGL(k_read, dim3(2048), dim3(256), 0, 0, (const uint4*)dhk, KB / 16, dout); }, reps);
  printf("{\"h2d_16MiB_us\": %.1f, \"h2d_GBps\": %.1f, \"d2h_4MiB_us\": %.1f, \"d2h_GBps\": %.1f, "
         "\"d2h_2d_block_us\": %.1f, \"d2h_32rows_block_us\": %.1f, \"h2d_and_d2h_two_streams_us\": %.1f, "
         "\"k_write_host_4MiB_us\": %.1f, \"k_write_GBps\": %.1f, \"k_read_host_16MiB_us\": %.1f, \"k_read_GBps\": %.1f, "
         "\"host_ptr_is_device_ptr\": %s}\n",
         t_h2d, KB / t_h2d / 1e3, t_d2h, HB / t_d2h / 1e3, t_2d, t_rows, t_both, t_kw, HB / t_kw / 1e3, t_kr,
         KB / t_kr / 1e3, (dhk == hk && dhh == hh) ? "true" : "false");
  return 0;
}
