// launch_log.hip — per-kernel launch counters of the library (diagnostics, no reference counterpart).
//
// EEGF_LAUNCH (eegfusion_internal.h) calls eegf_note_launch with the kernel's host stub before every
// launch.  eegf_launch_log_read lists "count<TAB>kernel name" lines, the name being the runtime's
// (demangled) device symbol, e.g. "(anonymous namespace)::gemm4r_kernel<true, 1, false>(...)".  The
// route-coverage test (tests/test_production_gpu.py) compares the kernel sets of two steps with it,
// instead of a profiler that can drop records.
#include "common.h"
#include "eegfusion_internal.h"

#include <cxxabi.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>

namespace {
std::mutex g_log_mu;
std::map<const void*, unsigned long long>& counts() {
  static std::map<const void*, unsigned long long> m;
  return m;
}

std::string kernel_name(const void* fn) {
  const char* mangled = hipKernelNameRefByPtr(fn, nullptr);
  if (!mangled) {
    char buf[32];
    snprintf(buf, sizeof buf, "kernel@%p", fn);
    return buf;
  }
  int st = 0;
  char* d = abi::__cxa_demangle(mangled, nullptr, nullptr, &st);
  std::string out = (st == 0 && d) ? d : mangled;
  free(d);
  return out;
}
}  // namespace

void eegf_note_launch(const void* kernel) {
  std::lock_guard<std::mutex> g(g_log_mu);
  ++counts()[kernel];
}

extern "C" int eegf_launch_log_reset(void) {
  std::lock_guard<std::mutex> g(g_log_mu);
  counts().clear();
  return 0;
}

extern "C" long eegf_launch_log_read(char* buf, long cap) {
  std::string text;
  {
    std::lock_guard<std::mutex> g(g_log_mu);
    for (const auto& kv : counts()) {
      text += std::to_string(kv.second);
      text += '\t';
      text += kernel_name(kv.first);
      text += '\n';
    }
  }
  const long need = (long)text.size() + 1;
  if (buf && cap > 0) {
    const long n = need <= cap ? need - 1 : cap - 1;
    memcpy(buf, text.data(), (size_t)n);
    buf[n] = '\0';
  }
  return need;
}
