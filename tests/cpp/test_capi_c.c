/* Compiles include/cassbloom.h as plain C11 and links libcassbloom.so from C:
 * the boundary is a real C ABI (no C++ or HIP types). Without a GPU it only
 * exercises calls that need no device; with one it runs a tiny build+probe. */
#include <stdio.h>
#include <string.h>

#include "cassbloom.h"

int main(int argc, char** argv) {
  int n = 0;
  if (cb_filter_bits(NULL, NULL) != CB_EINVAL) return 1;
  printf("version: %s\n", cb_version());
  if (argc > 1 && strcmp(argv[1], "--gpu") == 0) {
    cb_filter* f = NULL;
    if (cb_device_count(&n) || n < 1) return 2;
    if (cb_filter_create(128, 0, &f)) return 3;
    const char* key = "hello";
    if (cb_filter_insert_fixed(f, (const uint8_t*)key, 5, 1, NULL)) return 4;
    uint64_t hits = 0;
    const cb_filter* fs[1] = {f};
    if (cb_probe_fixed(fs, 1, (const uint8_t*)key, 5, 1, &hits, NULL)) return 5;
    if (hits != 1) return 6;
    cb_filter_destroy(f);
    printf("c abi gpu ok\n");
  }
  return 0;
}
