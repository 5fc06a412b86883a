// c2_lane.hip — one C2 build at a time (2^20 16-byte keys
// key(1, i) -> one fresh 2^27-bit filter), against any build of the library
// named on the command line (dlopen), so builds from different commits can be
// timed on one box with one harness (the round-5 bisect of the one-lane C2
// regression). Per library: K steps of cb_filter_clear + cb_filter_insert_fixed
// on one stream, bracketed by HIP events (= bench.py's build.one_lane), and the
// same with a 1 GiB device write before each of 8 reps (the cold protocol).
// Uses only entry points whose signatures have not changed since round 3.
// Output: one JSON line per library. Diagnostic only; not part of the product.
#include <hip/hip_runtime.h>
#include <dlfcn.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef int (*fn_init)(int);
typedef int (*fn_create)(uint64_t, int, void**);
typedef int (*fn_clear)(void*, void*);
typedef int (*fn_insert)(void*, const uint8_t*, uint32_t, uint64_t, void*);
typedef int (*fn_destroy)(void*);

static uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s lib.so [lib.so ...] (env C2_STEPS, C2_REPS)\n", argv[0]);
    return 2;
  }
  const int K = getenv("C2_STEPS") ? atoi(getenv("C2_STEPS")) : 200;
  const int reps = getenv("C2_REPS") ? atoi(getenv("C2_REPS")) : 3;
  const uint64_t n = 1u << 20, m = 1ull << 27;
  // key(1, i): 16 lowercase hex chars of splitmix64(1 << 32 | i), MSB nibble first
  std::vector<uint8_t> h(n * 16);
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t v = splitmix64((1ull << 32) + i);
    for (int c = 0; c < 16; ++c) h[i * 16 + c] = "0123456789abcdef"[(v >> (60 - 4 * c)) & 15];
  }
  uint8_t* keys;
  CHECK(hipMalloc(&keys, n * 16));
  CHECK(hipMemcpy(keys, h.data(), n * 16, hipMemcpyHostToDevice));
  void* junk;
  const size_t junk_bytes = 1ull << 30;
  CHECK(hipMalloc(&junk, junk_bytes));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int li = 1; li < argc; ++li) {
    void* L = dlopen(argv[li], RTLD_NOW | RTLD_LOCAL);
    if (!L) {
      fprintf(stderr, "dlopen %s: %s\n", argv[li], dlerror());
      return 1;
    }
    auto init = (fn_init)dlsym(L, "cb_init");
    auto create = (fn_create)dlsym(L, "cb_filter_create");
    auto clear = (fn_clear)dlsym(L, "cb_filter_clear");
    auto insert = (fn_insert)dlsym(L, "cb_filter_insert_fixed");
    auto destroy = (fn_destroy)dlsym(L, "cb_filter_destroy");
    if (!init || !create || !clear || !insert || !destroy) {
      fprintf(stderr, "%s: missing symbols\n", argv[li]);
      return 1;
    }
    if (init(0)) return 1;
    // C2_FUSED=-1 / 0: the two-launch or the one-launch single build
    // (cb_set_build_fused: round 5's one-launch experiment, since removed;
    // DESIGN.md §5 "Why the build stays two launches")
    if (const char* fz = getenv("C2_FUSED")) {
      auto set_fused = (int (*)(int))dlsym(L, "cb_set_build_fused");
      if (!set_fused || set_fused(atoi(fz))) {
        fprintf(stderr, "%s: cb_set_build_fused(%s) unavailable\n", argv[li], fz);
        return 1;
      }
    }
    void* f = nullptr;
    if (create(m, 0, &f)) return 1;
    auto step = [&]() {
      if (clear(f, s) || insert(f, keys, 16, n, s)) {
        fprintf(stderr, "build failed\n");
        exit(1);
      }
    };
    for (int i = 0; i < 5; ++i) step();
    CHECK(hipStreamSynchronize(s));
    // C2_GRAPH=1: the same build (clear + the partition and tile launches)
    // captured once into a hipGraph and replayed per step (VERDICT r5 Next 6:
    // the launch pair as a graph against plain launches). A replay repeats
    // the captured launches, a fresh build from zero each time, as every step
    // here is.
    const bool graph = getenv("C2_GRAPH") && getenv("C2_GRAPH")[0] == '1';
    hipGraphExec_t gx = nullptr;
    if (graph) {
      hipGraph_t g;
      CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
      step();
      CHECK(hipStreamEndCapture(s, &g));
      CHECK(hipGraphInstantiate(&gx, g, nullptr, nullptr, 0));
      CHECK(hipGraphDestroy(g));
      for (int i = 0; i < 5; ++i) CHECK(hipGraphLaunch(gx, s));
      CHECK(hipStreamSynchronize(s));
    }
    auto run = [&]() {
      if (gx)
        CHECK(hipGraphLaunch(gx, s));
      else
        step();
    };
    std::vector<float> warm;
    for (int r = 0; r < reps; ++r) {
      CHECK(hipEventRecord(a, s));
      for (int i = 0; i < K; ++i) run();
      CHECK(hipEventRecord(b, s));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      warm.push_back(ms * 1e3f / K);
    }
    std::vector<float> cold;
    for (int r = 0; r < 8; ++r) {
      CHECK(hipMemsetAsync(junk, r, junk_bytes, s));
      CHECK(hipEventRecord(a, s));
      run();
      CHECK(hipEventRecord(b, s));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      cold.push_back(ms * 1e3f);
    }
    std::sort(cold.begin(), cold.end());
    printf("{\"lib\": \"%s\", \"fused\": \"%s\", \"graph\": %s, \"one_lane_us\": [", argv[li],
           getenv("C2_FUSED") ? getenv("C2_FUSED") : "default", graph ? "true" : "false");
    for (size_t i = 0; i < warm.size(); ++i) printf("%s%.2f", i ? ", " : "", warm[i]);
    printf("], \"cold_us_median\": %.2f}\n", (cold[3] + cold[4]) / 2);
    fflush(stdout);
    if (gx) CHECK(hipGraphExecDestroy(gx));
    destroy(f);
    CHECK(hipStreamSynchronize(s));
    // the library stays loaded (its device state and RCCL hooks stay valid)
  }
  return 0;
}
