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

void* amdsmi_lib_handle() {
  static void* h = nullptr;
  void* v = __atomic_load_n(&h, __ATOMIC_ACQUIRE);
  if (v) return v;
  // Only ever called from a hook the application reached, i.e. once the
  // application has loaded the library itself.
  static const char* names[] = {"libamd_smi.so.26", "libamd_smi.so.25", "libamd_smi.so.24",
                                "libamd_smi.so", nullptr};
  v = open_noload(names);
  if (!v) v = RTLD_NEXT;
  __atomic_store_n(&h, v, __ATOMIC_RELEASE);
  return v;
}

void* rsmi_lib_handle() {
  static void* h = nullptr;
  void* v = __atomic_load_n(&h, __ATOMIC_ACQUIRE);
  if (v) return v;
  // libamd_smi bundles rocm-smi and calls its rsmi_* entry points through the
  // GOT — i.e. through our interposers — even when librocm_smi64 is not loaded.
  static const char* names[] = {"librocm_smi64.so.1", "librocm_smi64.so", nullptr};
  v = open_noload(names);
  if (!v && amdsmi_lib_handle() != RTLD_NEXT) v = amdsmi_lib_handle();
  if (!v) v = RTLD_NEXT;
  __atomic_store_n(&h, v, __ATOMIC_RELEASE);
  return v;
}

bool called_from_smi_lib(void* ret_addr) {
  Dl_info di;
  return ret_addr && dladdr(ret_addr, &di) && di.dli_fname && strstr(di.dli_fname, "smi") &&
         !is_own_address(ret_addr);
}

void* smi_real(const char* name, void* ret_addr, void* (*fallback_handle)()) {
  // 1. A call from inside an smi library (libamd_smi calling its bundled
  //    rsmi_* through the GOT): that library's own definition.
  Dl_info di;
  if (ret_addr && dladdr(ret_addr, &di) && di.dli_fname && strstr(di.dli_fname, "smi") &&
      !is_own_address(ret_addr)) {
    if (void* h = dlopen(di.dli_fname, RTLD_NOLOAD | RTLD_LAZY)) {
      void* p = real_dlsym(h, name);
      dlclose(h);
      if (p && !is_own_address(p)) return p;
    }
  }
  // 2. The definition the application's dlsym(handle, name) found.
  if (void* p = recorded_real(name)) return p;
  // 3. By library name.
  return resolve_real(fallback_handle(), name);
}

void* resolve_real(void* handle, const char* name) {
  void* p = real_dlsym(handle, name);
  if (!p && handle != RTLD_NEXT) p = real_dlsym(RTLD_NEXT, name);
  // Never resolve to ourselves (would recurse forever).
  Dl_info self_info, sym_info;
  if (p && dladdr((void*)&resolve_real, &self_info) && dladdr(p, &sym_info) &&
      self_info.dli_fbase == sym_info.dli_fbase) {
    p = real_dlsym(RTLD_NEXT, name);
  }
  if (!p) VLOG_ERR("cannot resolve real %s: %s", name, dlerror());
  return p;
}

}  // namespace vgpu
