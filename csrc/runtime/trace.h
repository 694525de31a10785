// roctx ranges of the native runtime (the owner's apply batches of the asynchronous PS), so they
// appear next to the Python-side Get / Add / Clock / collective ranges in a
// `rocprofv3 --marker-trace` timeline (minips_amd/utils/metrics.py: range). Off unless
// MINIPS_ROCTX=1: the library is dlopen-ed then, so the runtime has no link dependency on the
// profiler SDK and a disabled range costs one predictable branch.
#pragma once

#include <dlfcn.h>

#include <cstdlib>
#include <cstring>

namespace minips {

struct RoctxApi {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;

  static const RoctxApi& Get() {
    static const RoctxApi api = [] {
      RoctxApi a;
      const char* on = std::getenv("MINIPS_ROCTX");
      if (!on || std::strcmp(on, "1") != 0) return a;
      for (const char* name : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so"}) {
        void* h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
        if (!h) continue;
        a.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
        a.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
        if (a.push && a.pop) break;
        a.push = nullptr;
        a.pop = nullptr;
      }
      return a;
    }();
    return api;
  }
};

// RAII roctx range on the calling thread
class TraceRange {
 public:
  explicit TraceRange(const char* name) : api_(RoctxApi::Get()) {
    if (api_.push) api_.push(name);
  }
  ~TraceRange() {
    if (api_.pop) api_.pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  const RoctxApi& api_;
};

}  // namespace minips
