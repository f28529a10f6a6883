// Event trace ring (VGPU_TRACE=<dir>); layout in include/vgpu/trace.h.
#include "vgpu/trace.h"

#include <fcntl.h>
#include <sys/mman.h>

#include "common.h"
#include "state.h"

namespace vgpu {

static vgpu_trace_header_t* g_hdr = nullptr;
static vgpu_trace_event_t* g_ev = nullptr;

void trace_open() {
  const char* dir = env_first("VGPU_TRACE");
  if (!dir || !*dir || g_hdr) return;
  const char* cap_s = env_first("VGPU_TRACE_EVENTS");
  uint64_t cap = cap_s ? strtoull(cap_s, nullptr, 10) : 65536;
  if (cap < 64) cap = 64;
  char path[512];
  snprintf(path, sizeof path, "%s/vgpu-trace-%d.bin", dir, (int)getpid());
  int fd = open(path, O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) {
    VLOG_WARN("VGPU_TRACE: cannot create %s", path);
    return;
  }
  const size_t bytes = sizeof(vgpu_trace_header_t) + cap * sizeof(vgpu_trace_event_t);
  if (ftruncate(fd, (off_t)bytes) != 0) {
    close(fd);
    return;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return;
  auto* h = static_cast<vgpu_trace_header_t*>(p);
  h->magic = VGPU_TRACE_MAGIC;
  h->version = VGPU_TRACE_VERSION;
  h->header_size = sizeof(vgpu_trace_header_t);
  h->event_size = sizeof(vgpu_trace_event_t);
  h->capacity = cap;
  h->head = 0;
  h->pid = getpid();
  h->host_pid = self_host_pid(nullptr);
  h->start_ns = mono_ns();
  g_ev = reinterpret_cast<vgpu_trace_event_t*>(h + 1);
  __atomic_store_n(&g_hdr, h, __ATOMIC_RELEASE);
  VLOG_INFO("VGPU_TRACE: %s (%llu events)", path, (unsigned long long)cap);
}

void trace_after_fork() {
  // The child inherits the parent's mapping; it gets a file of its own.
  __atomic_store_n(&g_hdr, (vgpu_trace_header_t*)nullptr, __ATOMIC_RELEASE);
  g_ev = nullptr;
  trace_open();
}

bool trace_on() { return __atomic_load_n(&g_hdr, __ATOMIC_RELAXED) != nullptr; }

void trace_emit(uint32_t type, int dev, uint64_t a, uint64_t b) {
  vgpu_trace_header_t* h = __atomic_load_n(&g_hdr, __ATOMIC_ACQUIRE);
  if (!h) return;
  const uint64_t i = __atomic_fetch_add(&h->head, 1, __ATOMIC_RELAXED) % h->capacity;
  vgpu_trace_event_t& e = g_ev[i];
  __atomic_store_n(&e.ts_ns, (uint64_t)0, __ATOMIC_RELAXED);
  e.type = type;
  e.dev = dev;
  e.a = a;
  e.b = b;
  __atomic_store_n(&e.ts_ns, mono_ns(), __ATOMIC_RELEASE);
}

}  // namespace vgpu
