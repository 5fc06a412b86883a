// bloom_filter.hpp — C++ mirror of the reference's BloomFilter
// (/root/reference/src/bloom.rs) over the C ABI in include/cassbloom.h.
//
// Surface, one for one with the Rust type:
//   BloomFilter::create(size)        BloomFilter::new            bloom.rs:17-21
//   insert(item)                     insert(&mut self, &str)     bloom.rs:40-44
//   may_contain(item)                may_contain(&self, &str)    bloom.rs:48-51
//   to_proto() / from_proto(p)       bloom.rs:54-63
//   to_bytes() / from_bytes(b)       bloom.rs:66-77
// plus the batched entry points the callers use on the GPU path
// (insert_batch for SsTable::create's loop, src/sstable.rs:62-65; probe for
// Database::get's fan-out, src/lib.rs:129-134).
//
// Per-key insert() calls are queued on the host and flushed as one batched
// build before the filter is next read, so a caller that inserts key by key
// (as SsTable::create does) gets one GPU launch per flush, not per key.
// The reference's panics become exceptions: m == 0 -> std::domain_error,
// malformed proto -> std::invalid_argument, anything else -> std::runtime_error.
#pragma once

#include <cstdint>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

#include "cassbloom.h"

namespace cass {

inline void cb_check(int rc) {
  if (rc == CB_OK) return;
  const std::string msg = cb_last_error();
  if (rc == CB_EZEROM) throw std::domain_error(msg);
  if (rc == CB_EDECODE) throw std::invalid_argument(msg);
  throw std::runtime_error("cassbloom error " + std::to_string(rc) + ": " + msg);
}

// BloomProto { repeated bool bits = 1; } (bloom.rs:9-13). uint8_t per bit
// keeps the Vec<bool> byte layout.
struct BloomProto {
  std::vector<uint8_t> bits;
};

class BloomFilter {
 public:
  explicit BloomFilter(uint64_t size, int device = 0) {
    cb_filter* h = nullptr;
    cb_check(cb_filter_create(size, device, &h));
    h_.reset(h);
    m_ = size;
  }
  static BloomFilter create(uint64_t size, int device = 0) { return BloomFilter(size, device); }

  BloomFilter(BloomFilter&&) noexcept = default;
  BloomFilter& operator=(BloomFilter&&) noexcept = default;

  uint64_t len() const { return m_; }
  const cb_filter* handle() const {
    flush();
    return h_.get();
  }

  void insert(std::string_view item) {
    if (m_ == 0) throw std::domain_error("attempt to calculate the remainder with a divisor of zero");
    std::lock_guard<std::mutex> lk(*mu_);
    pend_bytes_.append(item.data(), item.size());
    pend_offs_.push_back(pend_bytes_.size());
  }

  // Inserts every key at once (one build launch).
  void insert_batch(const std::vector<std::string>& keys) {
    std::string bytes;
    std::vector<uint64_t> offs{0};
    for (const auto& k : keys) {
      bytes += k;
      offs.push_back(bytes.size());
    }
    flush();
    cb_check(cb_filter_insert_var(h_.get(), reinterpret_cast<const uint8_t*>(bytes.data()),
                                  offs.data(), keys.size(), nullptr));
  }

  bool may_contain(std::string_view item) const {
    flush();
    int out = 0;
    cb_check(cb_may_contain(h_.get(), reinterpret_cast<const uint8_t*>(item.data()), item.size(), &out));
    return out != 0;
  }

  BloomProto to_proto() const {
    flush();
    BloomProto p;
    p.bits.resize(m_);
    if (m_) cb_check(cb_filter_export_bools(h_.get(), p.bits.data(), nullptr));
    return p;
  }

  static BloomFilter from_proto(BloomProto proto, int device = 0) {
    BloomFilter f(proto.bits.size(), device);
    if (!proto.bits.empty())
      cb_check(cb_filter_import_bools(f.h_.get(), proto.bits.data(), proto.bits.size(), nullptr));
    return f;
  }

  std::vector<uint8_t> to_bytes() const {
    flush();
    uint64_t n = 0;
    cb_check(cb_filter_to_bytes(h_.get(), nullptr, 0, &n));
    std::vector<uint8_t> out(n);
    cb_check(cb_filter_to_bytes(h_.get(), out.data(), n, &n));
    return out;
  }

  static BloomFilter from_bytes(const std::vector<uint8_t>& data, int device = 0) {
    cb_filter* h = nullptr;
    cb_check(cb_filter_from_bytes(data.data(), data.size(), device, &h));
    uint64_t m = 0;
    cb_check(cb_filter_bits(h, &m));
    return BloomFilter(h, m);
  }

  // may_contain of every key against every filter: result[f][k].
  static std::vector<std::vector<bool>> probe(const std::vector<const BloomFilter*>& filters,
                                              const std::vector<std::string>& keys) {
    std::string bytes;
    std::vector<uint64_t> offs{0};
    for (const auto& k : keys) {
      bytes += k;
      offs.push_back(bytes.size());
    }
    std::vector<const cb_filter*> hs;
    for (const auto* f : filters) hs.push_back(f->handle());
    const uint64_t words = (keys.size() + 63) / 64;
    std::vector<uint64_t> hits(filters.size() * words + 1);
    cb_check(cb_probe_var(hs.data(), (uint32_t)hs.size(), reinterpret_cast<const uint8_t*>(bytes.data()),
                          offs.data(), keys.size(), hits.data(), nullptr));
    std::vector<std::vector<bool>> out(filters.size(), std::vector<bool>(keys.size()));
    for (size_t f = 0; f < filters.size(); ++f)
      for (size_t k = 0; k < keys.size(); ++k) out[f][k] = (hits[f * words + k / 64] >> (k % 64)) & 1;
    return out;
  }

  // Flushes queued per-key inserts as one batched build.
  void flush() const {
    std::lock_guard<std::mutex> lk(*mu_);
    if (pend_offs_.size() <= 1) return;
    const uint64_t n = pend_offs_.size() - 1;
    cb_check(cb_filter_insert_var(h_.get(), reinterpret_cast<const uint8_t*>(pend_bytes_.data()),
                                  pend_offs_.data(), n, nullptr));
    pend_bytes_.clear();
    pend_offs_.assign(1, 0);
  }

 private:
  BloomFilter(cb_filter* h, uint64_t m) : h_(h), m_(m) {}
  struct Del {
    void operator()(cb_filter* f) const { cb_filter_destroy(f); }
  };
  std::unique_ptr<cb_filter, Del> h_;
  uint64_t m_ = 0;
  mutable std::string pend_bytes_;
  mutable std::vector<uint64_t> pend_offs_{0};
  std::unique_ptr<std::mutex> mu_ = std::make_unique<std::mutex>();
};

}  // namespace cass
