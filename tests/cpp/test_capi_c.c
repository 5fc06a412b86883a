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
    /* SsTable::create from host buffers, enqueue-only (null zone pointers),
     * then the first read finalises it: the file of src/sstable.rs:57-72 */
    const char* kb = "ba";
    const uint64_t ko[3] = {0, 1, 2};
    const char* vb = "12";
    const uint64_t vo[3] = {0, 1, 2};
    cb_table* t = NULL;
    cb_filter* bloom = NULL;
    if (cb_sstable_create((const uint8_t*)kb, ko, (const uint8_t*)vb, vo, 2, 1024, 0, NULL, &t, &bloom, NULL,
                          NULL))
      return 7;
    if (cb_table_wait(t)) return 8;
    uint64_t len = 0, zl = 0;
    uint8_t file[32], z[4];
    if (cb_table_info(t, NULL, &len) || len != 14) return 9;
    if (cb_table_copy(t, 0, len, file) || memcmp(file, "a\tMg==\nb\tMQ==\n", 14)) return 10;
    if (cb_table_zone(t, 1, z, sizeof z, &zl) || zl != 1 || z[0] != 'b') return 11;
    /* a wide set (more than 64 slots) and Database::get over it in one call */
    cb_filterset* set = NULL;
    if (cb_set_create(1024, 128, 0, &set)) return 12;
    if (cb_set_assign(set, 100, bloom, NULL)) return 13;
    const cb_table* tabs[1] = {t};
    const uint32_t slots[1] = {100};
    int32_t which = -2;
    uint64_t voff[2] = {0, 0}, total = 0;
    uint8_t val[4];
    if (cb_set_get_many_fixed(set, tabs, 1, slots, (const uint8_t*)"a", 1, 1, &which, voff, val, sizeof val,
                              &total, NULL))
      return 14;
    if (which != 0 || total != 1 || val[0] != '2') return 15;
    cb_set_destroy(set);
    cb_table_destroy(t);
    cb_filter_destroy(bloom);
    printf("c abi gpu ok\n");
  }
  return 0;
}
