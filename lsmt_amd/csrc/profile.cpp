// profile.cpp — accumulates per-kernel durations from HIP event pairs.
#include "profile.hpp"

#include <atomic>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "cassbloom.h"

namespace cb {
namespace {
std::atomic<bool> g_on{false};
std::mutex g_mu;
struct Rec {
  std::string name;
  hipEvent_t e0, e1;
};
std::vector<Rec> g_pending;
struct Acc {
  double ms = 0;
  uint64_t n = 0;
};
std::map<std::string, Acc> g_acc;

void drain_locked() {
  for (auto& r : g_pending) {
    float ms = 0;
    if (hipEventSynchronize(r.e1) == hipSuccess && hipEventElapsedTime(&ms, r.e0, r.e1) == hipSuccess) {
      auto& a = g_acc[r.name];
      a.ms += ms;
      a.n += 1;
    }
    (void)hipEventDestroy(r.e0);
    (void)hipEventDestroy(r.e1);
  }
  g_pending.clear();
}
}  // namespace

bool prof_enabled() { return g_on.load(std::memory_order_relaxed); }

void prof_record(const char* name, hipEvent_t start, hipEvent_t stop) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_pending.push_back({name, start, stop});
}

}  // namespace cb

extern "C" {

int cb_profile_enable(int on) {
  cb::g_on.store(on != 0);
  return CB_OK;
}

int cb_profile_reset(void) {
  std::lock_guard<std::mutex> lk(cb::g_mu);
  cb::drain_locked();
  cb::g_acc.clear();
  return CB_OK;
}

int cb_profile_read(const char* kernel, double* total_ms, uint64_t* launches) {
  if (!kernel || !total_ms || !launches) return CB_EINVAL;
  std::lock_guard<std::mutex> lk(cb::g_mu);
  cb::drain_locked();
  auto it = cb::g_acc.find(kernel);
  *total_ms = it == cb::g_acc.end() ? 0.0 : it->second.ms;
  *launches = it == cb::g_acc.end() ? 0 : it->second.n;
  return CB_OK;
}

}  // extern "C"
