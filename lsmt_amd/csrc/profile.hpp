// profile.hpp — optional per-kernel timing with HIP events recorded on the
// launch stream (bench.py's roofline leg). Off by default: zero cost.
#pragma once
#include <hip/hip_runtime.h>

namespace cb {

bool prof_enabled();
void prof_record(const char* name, hipEvent_t start, hipEvent_t stop);

// Records an event pair around the launches in its scope, on stream s.
struct ProfScope {
  const char* name;
  hipStream_t s;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  ProfScope(const char* n, hipStream_t st) : name(n), s(st) {
    if (!prof_enabled()) return;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
      e0 = e1 = nullptr;
      return;
    }
    (void)hipEventRecord(e0, s);
  }
  ~ProfScope() {
    if (!e0) return;
    (void)hipEventRecord(e1, s);
    prof_record(name, e0, e1);
  }
};

}  // namespace cb
