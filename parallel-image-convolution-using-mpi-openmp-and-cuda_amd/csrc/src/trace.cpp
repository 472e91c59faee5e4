// roctx bridge (see trace.hpp).
#include "pconv/trace.hpp"

#include <dlfcn.h>

#include <cstdlib>
#include <mutex>

namespace pconv {

namespace {

using PushFn = int (*)(const char*);
using PopFn = int (*)();
using MarkFn = void (*)(const char*);

struct Roctx {
  bool on = false;
  PushFn push = nullptr;
  PopFn pop = nullptr;
  MarkFn mark = nullptr;
};

const Roctx& roctx() {
  static Roctx r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = std::getenv("PCONV_TRACE");
    if (!e || e[0] == '\0' || e[0] == '0') return;
    void* h = nullptr;
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                            "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"}) {
      h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
      if (h) break;
    }
    if (!h) return;
    r.push = reinterpret_cast<PushFn>(dlsym(h, "roctxRangePushA"));
    r.pop = reinterpret_cast<PopFn>(dlsym(h, "roctxRangePop"));
    r.mark = reinterpret_cast<MarkFn>(dlsym(h, "roctxMarkA"));
    r.on = r.push && r.pop;
  });
  return r;
}

}  // namespace

bool trace_enabled() { return roctx().on; }
void trace_push(const char* name) {
  if (roctx().on) roctx().push(name);
}
void trace_pop() {
  if (roctx().on) roctx().pop();
}
void trace_mark(const char* name) {
  if (roctx().on && roctx().mark) roctx().mark(name);
}

}  // namespace pconv
