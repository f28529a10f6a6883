#include "real.h"

#include "common.h"

namespace vgpu {

static void* open_noload(const char* const* names) {
  for (const char* const* n = names; *n; ++n) {
    void* h = dlopen(*n, RTLD_NOLOAD | RTLD_LAZY);
    if (h) return h;
  }
  return nullptr;
}

static void* open_any(const char* const* names) {
  void* h = open_noload(names);
  if (h) return h;
  for (const char* const* n = names; *n; ++n) {
    h = dlopen(*n, RTLD_LAZY | RTLD_GLOBAL);
    if (h) return h;
  }
  return nullptr;
}

void* hip_lib_handle() {
  static void* h = nullptr;
  void* v = __atomic_load_n(&h, __ATOMIC_ACQUIRE);
  if (v) return v;
  static const char* names[] = {"libamdhip64.so.7", "libamdhip64.so", nullptr};
  v = open_any(names);
  if (!v) v = RTLD_NEXT;
  __atomic_store_n(&h, v, __ATOMIC_RELEASE);
  return v;
}

void* hsa_lib_handle() {
  static void* h = nullptr;
  void* v = __atomic_load_n(&h, __ATOMIC_ACQUIRE);
  if (v) return v;
  static const char* names[] = {"libhsa-runtime64.so.1", "libhsa-runtime64.so", nullptr};
  v = open_any(names);
  if (!v) v = RTLD_NEXT;
  __atomic_store_n(&h, v, __ATOMIC_RELEASE);
  return v;
}

void* resolve_real(void* handle, const char* name) {
  void* p = dlsym(handle, name);
  if (!p && handle != RTLD_NEXT) p = dlsym(RTLD_NEXT, name);
  // Never resolve to ourselves (would recurse forever).
  Dl_info self_info, sym_info;
  if (p && dladdr((void*)&resolve_real, &self_info) && dladdr(p, &sym_info) &&
      self_info.dli_fbase == sym_info.dli_fbase) {
    p = dlsym(RTLD_NEXT, name);
  }
  if (!p) VLOG_ERR("cannot resolve real %s: %s", name, dlerror());
  return p;
}

}  // namespace vgpu
