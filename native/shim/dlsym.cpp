// dlsym interposition: symbol lookups by handle must land on our hooks too.
//
// Reference behaviour: libvgpu.so overrides `dlsym` (856 B) and keeps a
// `real_dlsym` so that lookups made through dlopen handles — the CUDA runtime
// resolving driver entry points, NVML users loading libnvidia-ml by hand — go
// to its hooks.
//
// On ROCm the lookups that bypass LD_PRELOAD are ctypes users of libamd_smi
// (amd-smi CLI, torch.cuda's amdsmi queries), tools that dlopen
// librocm_smi64/libamdhip64 and dlsym their entry points, and anything that
// resolves HSA entry points by hand.  A lookup of a hooked name through a
// handle of one of those libraries returns our interposer instead.
//
// RTLD_NEXT and RTLD_DEFAULT must keep their meaning: glibc derives the caller
// from the return address ("the next object after the caller"; "the caller's
// lookup scope", which for a library dlopen'ed RTLD_LOCAL includes its own
// dependencies — ctypes loads libamdhip64 that way, and HIP's stream-ordered
// pool resolves optional ROCr entry points with RTLD_DEFAULT).  So `dlsym`
// below is a two-way x86-64 trampoline: both pseudo-handles tail-jump straight
// into glibc's dlsym with the caller's return address untouched, every real
// handle tail-jumps into vgpu_dlsym_hook.  Our own code resolves through
// vgpu::real_dlsym (never the exported dlsym), so the shim never sees itself.
#include <dlfcn.h>
#include <link.h>
#include <pthread.h>

#include <mutex>
#include <string>
#include <unordered_map>

#include "common.h"

typedef void* (*dlsym_fn)(void*, const char*);

// Sanitizer runtimes resolve their interceptors with dlsym(RTLD_NEXT) before
// any instrumented code may run, so sanitizer builds of the shim (host-side
// race / address checking, tests/test_shim_robustness.py) keep glibc's dlsym.
#if defined(__SANITIZE_THREAD__) || defined(__SANITIZE_ADDRESS__)
#define VGPU_NO_DLSYM_OVERRIDE 1
#endif

extern "C" {
__attribute__((visibility("hidden"))) dlsym_fn vgpu_real_dlsym_ptr = nullptr;
__attribute__((visibility("hidden"))) void* vgpu_dlsym_hook(void* handle, const char* name);
__attribute__((visibility("hidden"))) void* vgpu_dlsym_next_slow(void* handle, const char* name);
}

#ifndef VGPU_NO_DLSYM_OVERRIDE
// RTLD_NEXT == (void*)-1, RTLD_DEFAULT == 0 on glibc.
__asm__(
    ".text\n"
    ".globl dlsym\n"
    ".type dlsym,@function\n"
    ".p2align 4\n"
    "dlsym:\n"
    "  cmpq $-1, %rdi\n"
    "  je 3f\n"
    "  testq %rdi, %rdi\n"
    "  jne 1f\n"
    "3:\n"
    "  movq vgpu_real_dlsym_ptr(%rip), %rax\n"
    "  testq %rax, %rax\n"
    "  jz 2f\n"
    "  jmp *%rax\n"
    "1:\n"
    "  jmp vgpu_dlsym_hook\n"
    "2:\n"
    "  jmp vgpu_dlsym_next_slow\n"
    ".size dlsym, .-dlsym\n");
#endif

namespace vgpu {

static dlsym_fn resolve_glibc_dlsym() {
#ifdef VGPU_NO_DLSYM_OVERRIDE
  return &::dlsym;
#endif
  dlsym_fn f = __atomic_load_n(&vgpu_real_dlsym_ptr, __ATOMIC_ACQUIRE);
  if (f) return f;
  // dlvsym is not interposed; 2.34 moved dlsym into libc proper.
  f = (dlsym_fn)dlvsym(RTLD_NEXT, "dlsym", "GLIBC_2.34");
  if (!f) f = (dlsym_fn)dlvsym(RTLD_NEXT, "dlsym", "GLIBC_2.2.5");
  __atomic_store_n(&vgpu_real_dlsym_ptr, f, __ATOMIC_RELEASE);
  return f;
}

void* real_dlsym(void* handle, const char* name) {
  dlsym_fn f = resolve_glibc_dlsym();
  return f ? f(handle, name) : nullptr;
}

__attribute__((constructor(101))) static void dlsym_ctor() { resolve_glibc_dlsym(); }

// Base address of this shared object (to tell our definitions from others).
static void* self_base() {
  static void* base = nullptr;
  void* b = __atomic_load_n(&base, __ATOMIC_ACQUIRE);
  if (b) return b;
  Dl_info di;
  if (dladdr((void*)&self_base, &di)) b = di.dli_fbase;
  __atomic_store_n(&base, b, __ATOMIC_RELEASE);
  return b;
}

static void* self_handle() {
  static void* h = nullptr;
  void* v = __atomic_load_n(&h, __ATOMIC_ACQUIRE);
  if (v) return v;
  Dl_info di;
  if (dladdr((void*)&self_handle, &di) && di.dli_fname) v = dlopen(di.dli_fname, RTLD_NOLOAD | RTLD_LAZY);
  __atomic_store_n(&h, v, __ATOMIC_RELEASE);
  return v;
}

static bool hookable_prefix(const char* n) {
  return !strncmp(n, "hip", 3) || !strncmp(n, "hsa_", 4) || !strncmp(n, "amdsmi_", 7) ||
         !strncmp(n, "rsmi_", 5);
}

// Our own definition of `name`, or nullptr when the shim does not hook it.
void* own_hook(const char* name) {
  if (!name || !hookable_prefix(name)) return nullptr;
  void* h = self_handle();
  if (!h) return nullptr;
  void* p = real_dlsym(h, name);  // searches us first, then our dependencies
  if (!p) return nullptr;
  Dl_info di;
  if (!dladdr(p, &di) || di.dli_fbase != self_base()) return nullptr;
  return p;
}

// What the application's own lookup would have returned, per hooked name
// (handle-specific lookups only): the smi hooks call exactly that function,
// not whichever copy of the library a by-name lookup finds first (PyTorch
// ships its own librocm_smi64 / libamd_smi beside the system ones).
static std::mutex g_rec_mu;
static std::unordered_map<std::string, void*> g_recorded;

static void record_real(const char* name, void* p) {
  std::lock_guard<std::mutex> g(g_rec_mu);
  g_recorded[name] = p;
}

void* recorded_real(const char* name) {
  std::lock_guard<std::mutex> g(g_rec_mu);
  auto it = g_recorded.find(name);
  return it == g_recorded.end() ? nullptr : it->second;
}

bool is_own_address(void* p) {
  Dl_info di;
  return p && dladdr(p, &di) && di.dli_fbase == self_base();
}

}  // namespace vgpu

extern "C" void* vgpu_dlsym_hook(void* handle, const char* name) {
  void* p = vgpu::real_dlsym(handle, name);
  if (!p || handle == RTLD_DEFAULT || !name || !vgpu::hookable_prefix(name)) return p;
  void* mine = vgpu::own_hook(name);
  if (mine && mine != p) {
    VLOG_DEBUG("dlsym(%p, %s) -> interposer", handle, name);
    vgpu::record_real(name, p);
    return mine;
  }
  return p;
}

// RTLD_NEXT / RTLD_DEFAULT before our constructor ran (another preload's
// constructor): the lookup is made relative to this object, which is at most
// one object off.
extern "C" void* vgpu_dlsym_next_slow(void* handle, const char* name) {
  return vgpu::real_dlsym(handle, name);
}
