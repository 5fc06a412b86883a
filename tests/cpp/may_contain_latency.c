/*
 * Single-key may_contain latency through the C ABI, as the drop-in shim calls
 * it: SsTable::get asks `bloom.may_contain(key)` once per key per table
 * (/root/reference/src/sstable.rs:138, inside Database::get's table loop,
 * src/lib.rs:130-134). One host thread, a filter of m bits holding n keys,
 * probed with half present / half absent 16-byte keys:
 *   - host mirror on (cb_filter_host_mirror 1): the first call after the
 *     build (the one D2H of the words) and the steady-state mean;
 *   - host mirror off: every call is a one-key GPU probe (launch, copy, sync).
 * Both answer every probe key; the answers must agree key for key.
 *
 *   may_contain_latency M_BITS N_KEYS [CALLS]   -> one JSON line on stdout
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "cassbloom.h"

static uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* key(seed, i) of SURVEY.md §8d: 16 lowercase hex chars of splitmix64(seed*2^32 + i) */
static void key16(uint64_t seed, uint64_t i, uint8_t* out) {
  static const char hex[] = "0123456789abcdef";
  const uint64_t v = splitmix64((seed << 32) + i);
  for (int j = 0; j < 16; ++j) out[j] = (uint8_t)hex[(v >> (60 - 4 * j)) & 15];
}

static double now_ns(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec * 1e9 + (double)t.tv_nsec;
}

#define CHECK(x)                                                                   \
  do {                                                                             \
    int rc_ = (x);                                                                 \
    if (rc_) {                                                                     \
      fprintf(stderr, "%s failed: %d %s\n", #x, rc_, cb_last_error());             \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s M_BITS N_KEYS [CALLS]\n", argv[0]);
    return 2;
  }
  const uint64_t m = strtoull(argv[1], NULL, 10), n = strtoull(argv[2], NULL, 10);
  const uint64_t calls = argc > 3 ? strtoull(argv[3], NULL, 10) : 400000;
  const uint64_t nprobe = 4096, gpu_calls = 2000;
  uint8_t* keys = (uint8_t*)malloc(16 * (n ? n : 1));
  uint8_t* probe = (uint8_t*)malloc(16 * nprobe);
  for (uint64_t i = 0; i < n; ++i) key16(11, i, keys + 16 * i);
  for (uint64_t i = 0; i < nprobe; ++i) {
    if (i % 2 == 0 && n)
      key16(11, (i / 2 * 7919) % n, probe + 16 * i); /* present */
    else
      key16(12, i, probe + 16 * i); /* absent */
  }
  cb_filter* f = NULL;
  CHECK(cb_filter_create(m, 0, &f));
  CHECK(cb_filter_insert_fixed(f, keys, 16, n, NULL));

  int* mirror = (int*)malloc(sizeof(int) * nprobe);
  int* device = (int*)malloc(sizeof(int) * nprobe);

  /* mirror on: the first call refreshes the mirror (waits for the build, one D2H) */
  CHECK(cb_filter_host_mirror(f, 1));
  double t0 = now_ns();
  CHECK(cb_may_contain(f, probe, 16, &mirror[0]));
  const double first_ns = now_ns() - t0;
  for (uint64_t i = 0; i < nprobe; ++i) CHECK(cb_may_contain(f, probe + 16 * i, 16, &mirror[i]));
  int sink = 0, v = 0;
  t0 = now_ns();
  for (uint64_t c = 0; c < calls; ++c) {
    CHECK(cb_may_contain(f, probe + 16 * (c & (nprobe - 1)), 16, &v));
    sink += v;
  }
  const double mirror_ns = (now_ns() - t0) / (double)calls;

  /* mirror off: one-key GPU probe per call */
  CHECK(cb_filter_host_mirror(f, 0));
  for (uint64_t i = 0; i < nprobe; ++i) CHECK(cb_may_contain(f, probe + 16 * i, 16, &device[i]));
  t0 = now_ns();
  for (uint64_t c = 0; c < gpu_calls; ++c) {
    CHECK(cb_may_contain(f, probe + 16 * (c & (nprobe - 1)), 16, &v));
    sink += v;
  }
  const double gpu_ns = (now_ns() - t0) / (double)gpu_calls;

  uint64_t agree = 0, hits = 0;
  for (uint64_t i = 0; i < nprobe; ++i) {
    agree += mirror[i] == device[i];
    hits += (uint64_t)mirror[i];
  }
  printf("{\"m_bits\": %llu, \"keys\": %llu, \"probe_keys\": %llu, \"hits\": %llu, "
         "\"mirror_first_call_us\": %.3f, \"mirror_ns_per_call\": %.1f, \"mirror_calls\": %llu, "
         "\"gpu_ns_per_call\": %.1f, \"gpu_calls\": %llu, \"agree\": %s, \"sink\": %d}\n",
         (unsigned long long)m, (unsigned long long)n, (unsigned long long)nprobe, (unsigned long long)hits,
         first_ns / 1e3, mirror_ns, (unsigned long long)calls, gpu_ns, (unsigned long long)gpu_calls,
         agree == nprobe ? "true" : "false", sink);
  CHECK(cb_filter_destroy(f));
  free(keys);
  free(probe);
  free(mirror);
  free(device);
  return agree == nprobe ? 0 : 1;
}
