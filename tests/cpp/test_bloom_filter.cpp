// C++ host-mirror tests (lsmt_amd/csrc/bloom_filter.hpp over the C ABI),
// mirroring the reference's own tests that touch the Bloom path. Expected
// values come from tests/golden/golden.json ("scenarios"). Needs a GPU; run by
// tests/test_cpp_mirror.py. Exit code 0 = pass.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "bloom_filter.hpp"

static int failures = 0;
#define EXPECT(c)                                                  \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                  \
    }                                                              \
  } while (0)

int main() {
  using cass::BloomFilter;
  // tests/bloom_test.rs:3-8
  {
    BloomFilter b = BloomFilter::create(128);
    b.insert("hello");
    EXPECT(b.may_contain("hello"));
    EXPECT(!b.may_contain("world"));
    EXPECT(!b.may_contain(""));
    auto p = b.to_proto();
    std::vector<int> set;
    for (size_t i = 0; i < p.bits.size(); ++i)
      if (p.bits[i]) set.push_back((int)i);
    EXPECT((set == std::vector<int>{25, 82}));
  }
  // tests/sstable_test.rs: keys a, b, c at m = 1024 (SsTable::new's size)
  {
    BloomFilter b(1024);
    for (const char* k : {"b", "a", "c"}) b.insert(k);
    EXPECT(b.may_contain("a") && b.may_contain("b") && b.may_contain("c"));
    EXPECT(!b.may_contain("d"));
  }
  // tests/sstable_local_test.rs:12 — to_bytes survives from_bytes unchanged
  {
    BloomFilter b(1024);
    b.insert("k");
    auto bytes = b.to_bytes();
    EXPECT(bytes.size() == 1 + 2 + 1024 && bytes[0] == 0x0A);
    BloomFilter c = BloomFilter::from_bytes(bytes);
    EXPECT(c.to_bytes() == bytes);
    BloomFilter d = BloomFilter::from_proto(b.to_proto());
    EXPECT(d.to_bytes() == bytes);
    EXPECT(c.may_contain("k") && !c.may_contain("v"));
  }
  // tests/lsm_flush_test.rs: k1, k2 present, "missing" absent
  {
    BloomFilter b(1024);
    b.insert_batch({"k1", "k2"});
    EXPECT(b.may_contain("k1") && b.may_contain("k2") && !b.may_contain("missing"));
  }
  // batched multi-filter probe == per-filter may_contain (Database::get fan-out)
  {
    std::vector<BloomFilter> fs;
    std::vector<std::string> keys;
    for (int t = 0; t < 3; ++t) {
      fs.emplace_back(1 << 16);
      std::vector<std::string> ks;
      for (int i = 0; i < 500; ++i) ks.push_back("ns:" + std::to_string(t) + "|" + std::to_string(i));
      fs.back().insert_batch(ks);
      keys.insert(keys.end(), ks.begin(), ks.begin() + 50);
    }
    for (int i = 0; i < 100; ++i) keys.push_back("absent-" + std::to_string(i));
    std::vector<const BloomFilter*> ptrs;
    for (auto& f : fs) ptrs.push_back(&f);
    auto hits = BloomFilter::probe(ptrs, keys);
    for (size_t f = 0; f < fs.size(); ++f)
      for (size_t k = 0; k < keys.size(); ++k) EXPECT(hits[f][k] == fs[f].may_contain(keys[k]));
    for (size_t k = 0; k < 150; ++k) EXPECT(hits[k / 50][k]);  // no false negatives
  }
  // m == 0 panics in the reference (`% 0`, bloom.rs:36)
  {
    BloomFilter z(0);
    bool threw = false;
    try {
      z.insert("x");
    } catch (const std::domain_error&) {
      threw = true;
    }
    EXPECT(threw);
    threw = false;
    try {
      BloomFilter::from_bytes({0x0A, 0x05, 0x01});
    } catch (const std::invalid_argument&) {
      threw = true;
    }
    EXPECT(threw);
  }
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("cpp mirror ok\n");
  return 0;
}
