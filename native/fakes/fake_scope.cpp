// Two tiny libraries for the dlsym-scope regression test
// (tests/test_shim_native.py::test_dlsym_default_keeps_the_callers_scope).
//
// libscope_user.so depends on libscope_dep.so and is dlopen'ed RTLD_LOCAL, the
// way ctypes loads libamdhip64 (whose libhsa-runtime64 then lives only in the
// local scope).  Inside it, dlsym(RTLD_DEFAULT, "scope_dep_fn") must find the
// dependency's symbol: glibc searches the CALLER's scope, so the shim's dlsym
// interposer must hand RTLD_DEFAULT lookups to glibc with the caller's return
// address (HIP's stream-ordered pool resolves optional ROCr entry points this
// way and failed hipMallocAsync without it).
#include <dlfcn.h>

extern "C" {
#ifdef SCOPE_DEP
__attribute__((visibility("default"))) int scope_dep_fn() { return 42; }
#else
int scope_dep_fn();
__attribute__((visibility("default"))) int scope_lookup() {
  auto f = (int (*)())dlsym(RTLD_DEFAULT, "scope_dep_fn");
  return f ? f() : -1;
}
__attribute__((visibility("default"))) int scope_linked() { return scope_dep_fn(); }
#endif
}
