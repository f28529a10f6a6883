// Fake HIP runtime (SONAME libamdhip64.so.7, symbol versions copied from the
// real library at build time) for CPU-only tests of the enforcement library.
//
// Device memory is a bump allocator over a fake address space (nothing is
// actually allocated, so a 288 GB device costs no host RAM).  Like the real
// CLR, the first API call creates one HSA queue per device through
// hsa_queue_create — resolved through the global scope, i.e. through the
// preloaded libvgpu.so hook, exactly as in a PyTorch process.
//
// Device buffers come from the GPU agent's HSA memory pool
// (hsa_amd_memory_pool_allocate through the global scope, as CLR does), and
// VGPU_FAKE_RUNTIME_ALLOC bytes per device are allocated at init the way CLR
// allocates its device kernarg / staging pools outside any hipMalloc.
//
// Fixture env: VGPU_FAKE_GPUS (1), VGPU_FAKE_MEM (bytes, default 288 GiB),
// VGPU_FAKE_CUS (256), VGPU_FAKE_RUNTIME_ALLOC (bytes, default 0).
#include <hip/hip_runtime_api.h>
#include <dlfcn.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/file.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <set>
#include <mutex>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <vector>

namespace {

struct Dev {
  uint64_t total = 0;
  uint64_t used = 0;
  uint64_t imported = 0;  // bytes mapped from other processes (IPC)
  hsa_queue_t* queue = nullptr;
  hsa_amd_memory_pool_t pool{0};
  void* runtime_buf = nullptr;
};

std::mutex g_mu;
std::vector<Dev> g_devs;
std::map<uintptr_t, std::pair<int, uint64_t>> g_allocs;  // ptr -> (dev, size)
uintptr_t g_next = 0x7f0000000000ull;
thread_local int tl_dev = 0;
// Launch counters sharded per thread: a launch from one thread touches no
// cache line another launching thread writes (the shim's launch-path cost is
// measured on this runtime, `shim_driver launchcost`).
struct alignas(64) Shard {
  std::atomic<uint64_t> v{0};
};
struct Sharded {
  Shard s[64];
  void add(uint64_t n) {
    static std::atomic<unsigned> next{0};
    thread_local unsigned me = next.fetch_add(1) & 63;
    s[me].v.fetch_add(n, std::memory_order_relaxed);
  }
  uint64_t load() const {
    uint64_t t = 0;
    for (const Shard& x : s) t += x.v.load(std::memory_order_relaxed);
    return t;
  }
  void fetch_add(uint64_t n) { add(n); }
};
Sharded g_launches;
std::atomic<uint64_t> g_branchy_single_queue{0};  // graph launches the real runtime would crash on
Sharded g_launch_blocks;
std::atomic<uint64_t> g_graph_launches{0};
bool g_inited = false;

int env_int(const char* n, int d) {
  const char* v = getenv(n);
  return v && *v ? atoi(v) : d;
}

// ---- fake GPU timeline -------------------------------------------------------
// VGPU_FAKE_KERNEL_US > 0 gives every launch that much GPU time.  Launches run
// in FIFO order on one timeline: per process, or — with VGPU_FAKE_GPU_TIMELINE
// naming a file — shared by every process using that file (time-sharing one
// device).  Events complete when the process's last launch before the record
// has finished.
uint64_t now_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + ts.tv_nsec;
}
std::mutex g_tl_mu;
uint64_t g_busy_until = 0;   // private timeline
std::atomic<uint64_t> g_my_last_end{0};  // end of this process's latest launch
std::atomic<uint64_t> g_exec_ns{0};

void sleep_until(uint64_t t) {
  for (uint64_t n = now_ns(); n < t; n = now_ns()) {
    struct timespec ts{0, (long)std::min<uint64_t>(t - n, 1000000)};
    nanosleep(&ts, nullptr);
  }
}

void timeline_launch() {
  static const int us = env_int("VGPU_FAKE_KERNEL_US", 0);
  if (us <= 0) return;
  const uint64_t dur = (uint64_t)us * 1000;
  // A full AQL queue blocks the submitter: keep at most ~20 ms queued.
  uint64_t last;
  last = g_my_last_end.load();
  if (last > 20000000ull) sleep_until(last - 20000000ull);
  std::lock_guard<std::mutex> g(g_tl_mu);
  const uint64_t now = now_ns();
  static const char* shared = getenv("VGPU_FAKE_GPU_TIMELINE");
  // VGPU_FAKE_MASK_FACTOR: a process whose queue has a CU mask runs on CUs of
  // its own (a private timeline), each launch taking dur x (256 / its CUs) x
  // factor -- < 1 models workloads that run better spatially, > 1 worse.
  static const char* mf = getenv("VGPU_FAKE_MASK_FACTOR");
  if (mf && *mf) {
    using qm_t = int (*)(int, uint32_t*, int, uint64_t*);
    static qm_t qm = (qm_t)dlsym(RTLD_DEFAULT, "fake_hsa_queue_mask");
    uint32_t m[8] = {};
    uint64_t agent = 0;
    const int words = qm ? qm(0, m, 8, &agent) : -1;
    int bits = 0;
    for (int w = 0; w < words && w < 8; ++w) bits += __builtin_popcount(m[w]);
    if (bits > 0 && bits < 256) {
      const uint64_t d = (uint64_t)(dur * (256.0 / bits) * atof(mf));
      const uint64_t start = g_busy_until > now ? g_busy_until : now;
      g_busy_until = start + d;
      g_my_last_end = g_busy_until;
      g_exec_ns.fetch_add(d);
      return;
    }
  }
  if (shared && *shared) {
    int fd = open(shared, O_RDWR | O_CREAT, 0666);
    if (fd >= 0) {
      flock(fd, LOCK_EX);
      uint64_t until = 0;
      if (pread(fd, &until, sizeof until, 0) != sizeof until) until = 0;
      const uint64_t start = until > now ? until : now;
      until = start + dur;
      if (pwrite(fd, &until, sizeof until, 0) != sizeof until) {}
      flock(fd, LOCK_UN);
      close(fd);
      g_my_last_end = until;
      g_exec_ns.fetch_add(dur);
      return;
    }
  }
  const uint64_t start = g_busy_until > now ? g_busy_until : now;
  g_busy_until = start + dur;
  g_my_last_end = g_busy_until;
  g_exec_ns.fetch_add(dur);
}

uint64_t timeline_last_end() { return g_my_last_end.load(std::memory_order_acquire); }


struct FakeEvent {
  uint64_t at = 0;
  hipStream_t stream = nullptr;  // where it was last recorded
};

// Stream capture, as the runtime behaves: a capture is invalidated when an
// event recorded on the capturing stream is queried before the capture ends
// (hipErrorStreamCaptureInvalidated at hipStreamEndCapture).
// VGPU_FAKE_QUERY_US widens hipEventQuery so tests can hit that window.
std::mutex g_cap_mu;
std::map<hipStream_t, bool> g_capturing;  // stream -> invalidated
std::map<hipStream_t, unsigned long long> g_capture_id;  // stream -> capture id

hsa_status_t pick_gpu(hsa_agent_t a, void* data) {
  auto* v = (std::vector<hsa_agent_t>*)data;
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS &&
      t == HSA_DEVICE_TYPE_GPU)
    v->push_back(a);
  return HSA_STATUS_SUCCESS;
}

hsa_status_t first_pool(hsa_amd_memory_pool_t p, void* data) {
  *(hsa_amd_memory_pool_t*)data = p;
  return HSA_STATUS_SUCCESS;
}

void kfd_publish(int dev);

// Fake KFD cu_occupancy (VGPU_FAKE_KFD_OCC with VGPU_KFD_PROC_DIR and
// VGPU_FAKE_HOST_PID): a thread keeps <dir>/<host pid>/stats_<gpu id>/cu_occupancy
// at 64 while this process's timeline has work in flight, else 0.
void occ_thread_start(int ndev) {
  const char* on = getenv("VGPU_FAKE_KFD_OCC");
  const char* dir = getenv("VGPU_KFD_PROC_DIR");
  const char* hp = getenv("VGPU_FAKE_HOST_PID");
  if (!on || !dir || !hp) return;
  std::string base = std::string(dir) + "/" + hp;
  std::thread([base, ndev] {
    std::vector<std::string> files;
    for (int d = 0; d < ndev; ++d) {
      const std::string sd = base + "/stats_" + std::to_string(1000 + d);
      mkdir(base.c_str(), 0755);
      mkdir(sd.c_str(), 0755);
      files.push_back(sd + "/cu_occupancy");
    }
    int last = -1;
    for (;;) {
      const int v = timeline_last_end() > now_ns() ? 64 : 0;
      if (v != last) {
        for (auto& f : files)
          if (FILE* fp = fopen(f.c_str(), "w")) {
            fprintf(fp, "%d\n", v);
            fclose(fp);
          }
        last = v;
      }
      usleep(200);
    }
  }).detach();
}

void init_locked() {
  if (g_inited) return;
  g_inited = true;
  hsa_init();
  int n = env_int("VGPU_FAKE_GPUS", 1);
  const char* m = getenv("VGPU_FAKE_MEM");
  uint64_t mem = m ? strtoull(m, nullptr, 10) : (288ull << 30);
  const char* ra = getenv("VGPU_FAKE_RUNTIME_ALLOC");
  uint64_t runtime_alloc = ra ? strtoull(ra, nullptr, 10) : 0;
  g_devs.assign(n, Dev{});
  occ_thread_start(n);
  std::vector<hsa_agent_t> gpus;
  hsa_iterate_agents(pick_gpu, &gpus);
  for (int i = 0; i < n; ++i) {
    g_devs[i].total = mem;
    if (i < (int)gpus.size()) {
      hsa_queue_create(gpus[i], 4096, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, 0, 0,
                       &g_devs[i].queue);
      hsa_amd_agent_iterate_memory_pools(gpus[i], first_pool, &g_devs[i].pool);
      if (runtime_alloc &&
          hsa_amd_memory_pool_allocate(g_devs[i].pool, runtime_alloc, 0, &g_devs[i].runtime_buf) ==
              HSA_STATUS_SUCCESS)
        g_devs[i].used += runtime_alloc;
    }
    kfd_publish(i);
  }
}

std::atomic<int> g_init_done{0};
void init() {
  if (g_init_done.load(std::memory_order_acquire)) return;  // launch path: no lock once initialised
  std::lock_guard<std::mutex> g(g_mu);
  init_locked();
  g_init_done.store(1, std::memory_order_release);
}

// Fake KFD per-process VRAM counter (/sys/class/kfd/kfd/proc/<pid>/vram_<gpu id>):
// with VGPU_FAKE_KFD_RUNTIME=<bytes> the device's used bytes plus that much
// runtime-owned memory the HIP hooks never see (queues' context-save areas).
void kfd_publish(int dev) {
  static const char* rt = getenv("VGPU_FAKE_KFD_RUNTIME");
  const char* dir = getenv("VGPU_KFD_PROC_DIR");
  const char* hp = getenv("VGPU_FAKE_HOST_PID");
  if (!rt || !dir || !hp) return;
  char path[512];
  snprintf(path, sizeof path, "%s/%s/vram_%d", dir, hp, 1000 + dev);
  if (FILE* f = fopen(path, "w")) {
    // KFD counts buffers mapped from other processes (IPC imports) as well
    fprintf(f, "%llu\n", (unsigned long long)(g_devs[dev].used + g_devs[dev].imported + strtoull(rt, nullptr, 10)));
    fclose(f);
  }
}

hipError_t dev_alloc(void** p, size_t size, int dev) {
  std::lock_guard<std::mutex> g(g_mu);
  init_locked();
  if (dev < 0 || dev >= (int)g_devs.size()) return hipErrorInvalidDevice;
  if (g_devs[dev].used + size > g_devs[dev].total) return hipErrorOutOfMemory;
  void* hp = nullptr;
  if (hsa_amd_memory_pool_allocate(g_devs[dev].pool, size, 0, &hp) != HSA_STATUS_SUCCESS || !hp)
    return hipErrorOutOfMemory;
  g_devs[dev].used += size;
  kfd_publish(dev);
  uintptr_t a = (uintptr_t)hp;
  g_allocs[a] = {dev, size};
  *p = (void*)a;
  return hipSuccess;
}

hipError_t dev_free(void* p) {
  if (!p) return hipSuccess;
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_allocs.find((uintptr_t)p);
  if (it == g_allocs.end()) return hipErrorInvalidValue;
  g_devs[it->second.first].used -= it->second.second;
  kfd_publish(it->second.first);
  g_allocs.erase(it);
  hsa_amd_memory_pool_free(p);
  return hipSuccess;
}

void count_launch(uint64_t blocks) {
  init();
  g_launches.fetch_add(1);
  g_launch_blocks.fetch_add(blocks);
  timeline_launch();
}

}  // namespace

extern "C" {

hipError_t hipInit(unsigned int) { init(); return hipSuccess; }
hipError_t hipSetDevice(int d) {
  init();
  if (d < 0 || d >= (int)g_devs.size()) return hipErrorInvalidDevice;
  tl_dev = d;
  return hipSuccess;
}
hipError_t hipGetDevice(int* d) { *d = tl_dev; return hipSuccess; }
// Streams remember the device they were created on (hipStreamGetDevice);
// handles never created here (a test's made-up stream) belong to the current device.
std::mutex g_stream_mu;
std::map<hipStream_t, int> g_stream_dev;
std::atomic<uintptr_t> g_next_stream{0x7000000};
hipError_t hipStreamCreateWithFlags(hipStream_t* st, unsigned int) {
  if (!st) return hipErrorInvalidValue;
  *st = reinterpret_cast<hipStream_t>(g_next_stream.fetch_add(64));
  std::lock_guard<std::mutex> g(g_stream_mu);
  g_stream_dev[*st] = tl_dev;
  return hipSuccess;
}
hipError_t hipStreamCreate(hipStream_t* st) { return hipStreamCreateWithFlags(st, 0); }
hipError_t hipStreamGetDevice(hipStream_t st, hipDevice_t* d) {
  if (!d) return hipErrorInvalidValue;
  std::lock_guard<std::mutex> g(g_stream_mu);
  auto it = g_stream_dev.find(st);
  *d = it == g_stream_dev.end() ? tl_dev : it->second;
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t st) {
  std::lock_guard<std::mutex> g(g_stream_mu);
  g_stream_dev.erase(st);
  return hipSuccess;
}
hipError_t hipGetDeviceCount(int* n) { init(); *n = (int)g_devs.size(); return hipSuccess; }
hipError_t hipGetLastError() { return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t) { sleep_until(timeline_last_end()); return hipSuccess; }
hipError_t hipDeviceSynchronize() { sleep_until(timeline_last_end()); return hipSuccess; }
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
  *e = reinterpret_cast<hipEvent_t>(new FakeEvent);
  return hipSuccess;
}
hipError_t hipEventCreate(hipEvent_t* e) { return hipEventCreateWithFlags(e, 0); }
// VGPU_FAKE_EARLY_EVENTS=f: an event completes once a fraction f of the work
// queued before it has run (a profiler that rewrites completion signals).
hipError_t hipEventRecord(hipEvent_t e, hipStream_t stream) {
  if (!e) return hipErrorInvalidHandle;
  static const double early = getenv("VGPU_FAKE_EARLY_EVENTS") ? atof(getenv("VGPU_FAKE_EARLY_EVENTS")) : 1.0;
  const uint64_t end = timeline_last_end(), now = now_ns();
  reinterpret_cast<FakeEvent*>(e)->at = end > now && early < 1.0 ? now + (uint64_t)(early * (end - now)) : end;
  reinterpret_cast<FakeEvent*>(e)->stream = stream;
  return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t e) {
  if (!e) return hipErrorInvalidHandle;
  static const int delay_us = getenv("VGPU_FAKE_QUERY_US") ? atoi(getenv("VGPU_FAKE_QUERY_US")) : 0;
  if (delay_us > 0) usleep(delay_us);
  {
    std::lock_guard<std::mutex> g(g_cap_mu);
    auto it = g_capturing.find(reinterpret_cast<FakeEvent*>(e)->stream);
    if (it != g_capturing.end()) {
      it->second = true;
      return hipErrorStreamCaptureUnsupported;
    }
  }
  return now_ns() >= reinterpret_cast<FakeEvent*>(e)->at ? hipSuccess : hipErrorNotReady;
}
hipError_t hipEventSynchronize(hipEvent_t e) {
  if (!e) return hipErrorInvalidHandle;
  sleep_until(reinterpret_cast<FakeEvent*>(e)->at);
  return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) {
  delete reinterpret_cast<FakeEvent*>(e);
  return hipSuccess;
}
hipError_t hipStreamIsCapturing(hipStream_t s, hipStreamCaptureStatus* st) {
  std::lock_guard<std::mutex> g(g_cap_mu);
  auto it = g_capturing.find(s);
  if (st)
    *st = it == g_capturing.end() ? hipStreamCaptureStatusNone
                                  : (it->second ? hipStreamCaptureStatusInvalidated : hipStreamCaptureStatusActive);
  return hipSuccess;
}
hipError_t hipThreadExchangeStreamCaptureMode(hipStreamCaptureMode*) { return hipSuccess; }

// Arrays / 3D / mipmaps: device memory from the pool like any buffer (the
// real runtime sizes image rows at a 256-byte pitch).
static size_t fake_array_bytes(size_t elem, size_t w, size_t h, size_t d) {
  return ((w ? w : 1) * elem + 255) / 256 * 256 * (h ? h : 1) * (d ? d : 1);
}
hipError_t hipMalloc3D(hipPitchedPtr* pp, hipExtent e) {
  void* p = nullptr;
  hipError_t rc = dev_alloc(&p, fake_array_bytes(1, e.width, e.height, e.depth), tl_dev);
  if (rc == hipSuccess) *pp = hipPitchedPtr{p, (e.width + 255) / 256 * 256, e.width, e.height};
  return rc;
}
hipError_t hipMallocArray(hipArray_t* a, const hipChannelFormatDesc* d, size_t w, size_t h, unsigned int) {
  size_t elem = d ? (size_t)(d->x + d->y + d->z + d->w + 7) / 8 : 4;
  return dev_alloc((void**)a, fake_array_bytes(elem, w, h, 1), tl_dev);
}
hipError_t hipArray3DCreate(hipArray_t* a, const HIP_ARRAY3D_DESCRIPTOR* d) {
  return dev_alloc((void**)a, fake_array_bytes(4 * d->NumChannels, d->Width, d->Height, d->Depth), tl_dev);
}
hipError_t hipArrayCreate(hipArray_t* a, const HIP_ARRAY_DESCRIPTOR* d) {
  return dev_alloc((void**)a, fake_array_bytes(4 * d->NumChannels, d->Width, d->Height, 1), tl_dev);
}
hipError_t hipFreeArray(hipArray_t a) { return dev_free((void*)a); }
hipError_t hipArrayDestroy(hipArray_t a) { return dev_free((void*)a); }
// Code objects: the loaded image occupies device memory of its own size.
hipError_t hipModuleLoadData(hipModule_t* m, const void* image) {
  size_t n = 0;
  const unsigned char* p = (const unsigned char*)image;
  if (p && p[0] == 0x7f && p[1] == 'E') {
    uint64_t shoff;
    uint16_t shentsize, shnum;
    memcpy(&shoff, p + 0x28, 8);
    memcpy(&shentsize, p + 0x3a, 2);
    memcpy(&shnum, p + 0x3c, 2);
    n = shoff + (size_t)shentsize * shnum;
  }
  return dev_alloc((void**)m, n ? n : 4096, tl_dev);
}
hipError_t hipModuleUnload(hipModule_t m) { return dev_free((void*)m); }
// IPC: a handle carries (address, size); opening it maps the exporter's
// buffer at a new address without allocating device memory.
std::map<uintptr_t, std::pair<int, size_t>> g_imports;  // address -> (device, size)
uintptr_t g_import_next = 0x7e0000000000ull;
hipError_t hipIpcGetMemHandle(hipIpcMemHandle_t* h, void* p) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_allocs.find((uintptr_t)p);
  if (it == g_allocs.end()) return hipErrorInvalidValue;
  memset(h, 0, sizeof *h);
  uint64_t a = (uint64_t)(uintptr_t)p, sz = it->second.second;
  memcpy(h->reserved, &a, 8);
  memcpy(h->reserved + 8, &sz, 8);
  return hipSuccess;
}
hipError_t hipIpcOpenMemHandle(void** p, hipIpcMemHandle_t h, unsigned int) {
  std::lock_guard<std::mutex> g(g_mu);
  uint64_t sz;
  memcpy(&sz, h.reserved + 8, 8);
  uintptr_t a = g_import_next;
  g_import_next += (sz + (1 << 21)) & ~((uintptr_t)(1 << 21) - 1);
  g_imports[a] = {tl_dev, sz};
  if (tl_dev >= 0 && tl_dev < (int)g_devs.size()) {
    g_devs[tl_dev].imported += sz;
    kfd_publish(tl_dev);
  }
  *p = (void*)a;
  return hipSuccess;
}
hipError_t hipIpcCloseMemHandle(void* p) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_imports.find((uintptr_t)p);
  if (it == g_imports.end()) return hipErrorInvalidValue;
  const int d = it->second.first;
  if (d >= 0 && d < (int)g_devs.size()) {
    g_devs[d].imported -= it->second.second;
    kfd_publish(d);
  }
  g_imports.erase(it);
  return hipSuccess;
}
hipError_t hipMemGetAddressRange(hipDeviceptr_t* base, size_t* size, hipDeviceptr_t p) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_allocs.find((uintptr_t)p);
  if (it != g_allocs.end()) {
    *base = p;
    *size = it->second.second;
    return hipSuccess;
  }
  auto jt = g_imports.find((uintptr_t)p);
  if (jt == g_imports.end()) return hipErrorInvalidValue;
  *base = p;
  *size = jt->second.second;
  return hipSuccess;
}
static hipError_t begin_capture_impl(hipStream_t s) {
  std::lock_guard<std::mutex> g(g_cap_mu);
  if (g_capturing.count(s)) return hipErrorIllegalState;
  g_capturing[s] = false;
  static unsigned long long next_id = 100;
  g_capture_id[s] = ++next_id;
  return hipSuccess;
}
hipError_t hipStreamBeginCapture(hipStream_t s, hipStreamCaptureMode) { return begin_capture_impl(s); }
hipError_t hipStreamBeginCapture_spt(hipStream_t s, hipStreamCaptureMode) { return begin_capture_impl(s); }
hipError_t hipStreamGetCaptureInfo(hipStream_t s, hipStreamCaptureStatus* st, unsigned long long* id) {
  std::lock_guard<std::mutex> lk(g_cap_mu);
  auto it = g_capturing.find(s);
  if (st)
    *st = it == g_capturing.end() ? hipStreamCaptureStatusNone
                                  : (it->second ? hipStreamCaptureStatusInvalidated : hipStreamCaptureStatusActive);
  if (id) *id = it == g_capturing.end() ? 0 : g_capture_id[s];
  return hipSuccess;
}

hipError_t hipMalloc(void** p, size_t size) { return dev_alloc(p, size, tl_dev); }
hipError_t hipExtMallocWithFlags(void** p, size_t size, unsigned int) { return dev_alloc(p, size, tl_dev); }
// Stream-ordered pool (one per device): freed blocks stay reserved for reuse
// until hipMemPoolTrimTo; allocations made while a stream is being captured
// become the graph's alloc bytes (drawn from the graph pool at launch).
struct FakePool {
  std::map<uintptr_t, uint64_t> live, freed;  // block -> size
  uint64_t reserved = 0;
};
std::map<int, FakePool> g_pools;
// capture id -> peak bytes live at once (free nodes let the graph pool reuse memory)
struct CapAlloc {
  uint64_t live = 0, peak = 0;
};
std::map<unsigned long long, CapAlloc> g_cap_alloc;
std::map<uintptr_t, std::pair<unsigned long long, uint64_t>> g_cap_ptr;  // captured block -> (cid, size)
uint64_t g_graph_mem[16] = {};
hipError_t pool_alloc(void** p, size_t size, hipStream_t s) {
  {
    std::lock_guard<std::mutex> lk(g_cap_mu);
    auto it = g_capturing.find(s);
    if (it != g_capturing.end()) {  // graph alloc node: a VA now, memory at launch
      CapAlloc& ca = g_cap_alloc[g_capture_id[s]];
      ca.live += size;
      ca.peak = std::max(ca.peak, ca.live);
      std::lock_guard<std::mutex> g(g_mu);
      uintptr_t a = g_next | (1ull << 44);
      g_next += ((size + 4095) / 4096) * 4096 + 4096;
      g_cap_ptr[a] = {g_capture_id[s], size};
      *p = (void*)a;
      return hipSuccess;
    }
  }
  std::lock_guard<std::mutex> g(g_mu);
  init_locked();
  FakePool& fp = g_pools[tl_dev];
  for (auto it = fp.freed.begin(); it != fp.freed.end(); ++it)
    if (it->second >= size) {  // reuse a freed block: no new memory
      fp.live[it->first] = it->second;
      *p = (void*)it->first;
      fp.freed.erase(it);
      return hipSuccess;
    }
  Dev& d = g_devs[tl_dev];
  if (d.used + size > d.total) return hipErrorOutOfMemory;
  d.used += size;
  fp.reserved += size;
  uintptr_t a = g_next | (1ull << 43);
  g_next += ((size + 4095) / 4096) * 4096 + 4096;
  fp.live[a] = size;
  *p = (void*)a;
  return hipSuccess;
}
bool cap_free(void* p) {  // a free node of the capture that allocated the block
  std::lock_guard<std::mutex> lk(g_cap_mu);
  auto it = g_cap_ptr.find((uintptr_t)p);
  if (it == g_cap_ptr.end()) return false;
  auto ca = g_cap_alloc.find(it->second.first);
  if (ca != g_cap_alloc.end()) ca->second.live -= std::min(ca->second.live, it->second.second);
  g_cap_ptr.erase(it);
  return true;
}
bool pool_free(void* p) {
  std::lock_guard<std::mutex> g(g_mu);
  for (auto& kv : g_pools) {
    auto it = kv.second.live.find((uintptr_t)p);
    if (it != kv.second.live.end()) {
      kv.second.freed[it->first] = it->second;
      kv.second.live.erase(it);
      return true;
    }
  }
  return false;
}
hipError_t hipMallocAsync(void** p, size_t size, hipStream_t s) { return pool_alloc(p, size, s); }
hipError_t hipMallocFromPoolAsync(void** p, size_t size, hipMemPool_t, hipStream_t s) {
  return pool_alloc(p, size, s);
}
hipError_t hipDeviceGetMemPool(hipMemPool_t* pool, int dev) {
  *pool = reinterpret_cast<hipMemPool_t>((uintptr_t)0x9000 + dev);
  return hipSuccess;
}
hipError_t hipMemPoolGetAttribute(hipMemPool_t pool, hipMemPoolAttr attr, void* value) {
  std::lock_guard<std::mutex> g(g_mu);
  const int dev = (int)((uintptr_t)pool - 0x9000);
  if (attr != hipMemPoolAttrReservedMemCurrent) return hipErrorInvalidValue;
  *(uint64_t*)value = g_pools.count(dev) ? g_pools[dev].reserved : 0;
  return hipSuccess;
}
hipError_t hipMemPoolTrimTo(hipMemPool_t pool, size_t) {
  std::lock_guard<std::mutex> g(g_mu);
  const int dev = (int)((uintptr_t)pool - 0x9000);
  FakePool& fp = g_pools[dev];
  for (auto& kv : fp.freed) {
    fp.reserved -= kv.second;
    g_devs[dev].used -= kv.second;
  }
  fp.freed.clear();
  return hipSuccess;
}
hipError_t hipDeviceGetGraphMemAttribute(int dev, hipGraphMemAttributeType attr, void* value) {
  if (attr != hipGraphMemAttrReservedMemCurrent) return hipErrorInvalidValue;
  std::lock_guard<std::mutex> g(g_mu);
  *(uint64_t*)value = g_graph_mem[dev];
  return hipSuccess;
}
hipError_t hipDeviceGraphMemTrim(int dev) {
  std::lock_guard<std::mutex> g(g_mu);
  g_devs[dev].used -= g_graph_mem[dev];
  g_graph_mem[dev] = 0;
  return hipSuccess;
}
hipError_t hipMallocHost(void** p, size_t size);
hipError_t hipHostAlloc(void** p, size_t size, unsigned int flags);
hipError_t hipFreeHost(void*) { return hipSuccess; }
hipError_t hipHostRegister(void*, size_t, unsigned int) { return hipSuccess; }
hipError_t hipHostUnregister(void*) { return hipSuccess; }
// Managed (KFD SVM) ranges start host-resident and take no VRAM until the
// fake HSA's hsa_amd_svm_prefetch_async moves them (fake_hip_svm_move).
struct Managed {
  int dev;
  uint64_t size;
  uint64_t gpu_bytes;
};
std::map<uintptr_t, Managed> g_managed;
hipError_t hipMallocManaged(void** p, size_t size, unsigned int) {
  std::lock_guard<std::mutex> g(g_mu);
  init_locked();
  uintptr_t a = g_next | (1ull << 45);
  g_next += ((size + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1)) + (2u << 20);
  g_managed[a] = Managed{tl_dev, size, 0};
  *p = (void*)a;
  return hipSuccess;
}
hipError_t hipMemAdvise(const void*, size_t, hipMemoryAdvise, int) { return hipSuccess; }
// hipMemPrefetchAsync on a managed range (resident part = a prefix).  Asked for
// more VRAM than is free, the real KFD evicts the process's own buffers to make
// room (profiles/vmem_r2.md); the fake moves what fits and counts the request
// (fake_hip_prefetch_overflows), so tests can assert that none reaches it.
static uint64_t g_prefetch_over = 0;
static hipError_t prefetch_locked(const void* p, size_t n, int device) {
  auto it = g_managed.upper_bound((uintptr_t)p);
  if (it == g_managed.begin()) return hipErrorInvalidValue;
  --it;
  Managed& m = it->second;
  const uint64_t off = (uintptr_t)p - it->first;
  if (off >= m.size) return hipErrorInvalidValue;
  Dev& d = g_devs[m.dev];
  if (device < 0) {
    const uint64_t keep = std::min<uint64_t>(m.gpu_bytes, off);
    d.used -= m.gpu_bytes - keep;
    m.gpu_bytes = keep;
    return hipSuccess;
  }
  const uint64_t want = std::min<uint64_t>(m.size, off + n);
  uint64_t add = want > m.gpu_bytes ? want - m.gpu_bytes : 0;
  if (d.used + add > d.total) {
    ++g_prefetch_over;
    add = d.total - d.used;
  }
  m.gpu_bytes += add;
  d.used += add;
  return hipSuccess;
}
hipError_t hipMemPrefetchAsync(const void* p, size_t n, int device, hipStream_t) {
  std::lock_guard<std::mutex> g(g_mu);
  return prefetch_locked(p, n, device);
}
hipError_t hipMemPrefetchAsync_v2(const void* p, size_t n, hipMemLocation loc, unsigned int, hipStream_t) {
  std::lock_guard<std::mutex> g(g_mu);
  return prefetch_locked(p, n, loc.type == hipMemLocationTypeDevice ? loc.id : -1);
}
// A host<->device copy touching a managed range: KFD migrates the touched pages
// to system memory (native/probes/managed_access.hip); device-to-device copies
// run on the GPU and move nothing.  No bytes are copied (fake addresses).
static uint64_t g_host_touch_bytes = 0;  // bytes of managed ranges moved to host by copies
uint64_t g_copies2d = 0;
std::atomic<uint64_t> g_memsets{0};
static void host_copy_touch_locked(const void* p, size_t n) {
  auto it = g_managed.upper_bound((uintptr_t)p);
  if (it == g_managed.begin()) return;
  --it;
  Managed& m = it->second;
  if ((uintptr_t)p >= it->first + m.size) return;
  const uint64_t lo = ((uintptr_t)p - it->first) & ~((2ull << 20) - 1);
  const uint64_t hi = std::min<uint64_t>(m.size, ((uintptr_t)p - it->first + n + (2ull << 20) - 1) & ~((2ull << 20) - 1));
  const uint64_t moved = m.gpu_bytes > lo ? std::min<uint64_t>(m.gpu_bytes, hi) - lo : 0;
  m.gpu_bytes -= moved;
  g_devs[m.dev].used -= moved;
  g_host_touch_bytes += moved;
}
static bool device_mem_locked(const void* p) {
  auto it = g_allocs.upper_bound((uintptr_t)p);
  if (it != g_allocs.begin() && (uintptr_t)p < std::prev(it)->first + std::prev(it)->second.second) return true;
  auto jt = g_managed.upper_bound((uintptr_t)p);
  return jt != g_managed.begin() && (uintptr_t)p < std::prev(jt)->first + std::prev(jt)->second.size;
}
// A host<->device copy moves every managed page it touches to system memory
// (KFD); device-to-device copies (explicit, or Default between device
// memory) move nothing.
// VMM (hipMemAddressReserve / hipMemMap): reserved ranges are PROT_NONE
// anonymous memory, a mapping makes them read/write zero pages (the handle's
// contents do not survive an unmap: tests only map fresh handles), and copies
// between a mapped range and fake host memory (addresses with no storage)
// keep the bytes in g_host_data, so data that goes out and comes back can be
// checked.
static std::map<uintptr_t, size_t> g_vmm_mapped;
static std::map<uintptr_t, std::vector<char>> g_host_data;  // fake host address -> bytes copied there
static bool vmm_mapped_locked(const void* p, size_t n) {
  auto it = g_vmm_mapped.upper_bound((uintptr_t)p);
  return it != g_vmm_mapped.begin() && (uintptr_t)p + n <= std::prev(it)->first + std::prev(it)->second;
}
static bool vmm_copy_locked(void* dst, const void* src, size_t n) {
  const bool din = vmm_mapped_locked(dst, n), sin = vmm_mapped_locked(src, n);
  if (!din && !sin) return false;
  if (din && sin) {
    memmove(dst, src, n);
  } else if (sin) {  // range -> host: keep the bytes under the host address
    std::vector<char> v((const char*)src, (const char*)src + n);
    g_host_data[(uintptr_t)dst] = std::move(v);
  } else {  // host -> range: from bytes stored at (or inside) a host copy
    auto it = g_host_data.upper_bound((uintptr_t)src);
    if (it != g_host_data.begin()) {
      --it;
      const size_t off = (uintptr_t)src - it->first;
      if (off + n <= it->second.size()) memcpy(dst, it->second.data() + off, n);
    }
  }
  return true;
}
static hipError_t fake_copy(void* dst, const void* src, size_t n, hipMemcpyKind kind) {
  if (kind == hipMemcpyDeviceToDevice) return hipSuccess;
  std::lock_guard<std::mutex> g(g_mu);
  if (vmm_copy_locked(dst, src, n)) return hipSuccess;
  if (kind == hipMemcpyDefault && device_mem_locked(dst) && device_mem_locked(src)) return hipSuccess;
  host_copy_touch_locked(dst, n);
  host_copy_touch_locked(src, n);
  return hipSuccess;
}
static size_t span2d(size_t pitch, size_t w, size_t h) { return h ? pitch * (h - 1) + w : 0; }
// (Entry points call static helpers, never each other: an exported call would
// resolve to a preloaded interposer and be counted twice.)
static hipError_t copy2d(void* d, size_t dp, const void* s, size_t sp, size_t w, size_t h, hipMemcpyKind k) {
  if (k == hipMemcpyDeviceToDevice) return hipSuccess;
  std::lock_guard<std::mutex> g(g_mu);
  host_copy_touch_locked(d, span2d(dp, w, h));
  host_copy_touch_locked(s, span2d(sp, w, h));
  g_copies2d++;
  return hipSuccess;
}
hipError_t hipMemcpy2D(void* d, size_t dp, const void* s, size_t sp, size_t w, size_t h, hipMemcpyKind k) {
  return copy2d(d, dp, s, sp, w, h, k);
}
hipError_t hipMemcpy2DAsync(void* d, size_t dp, const void* s, size_t sp, size_t w, size_t h, hipMemcpyKind k,
                            hipStream_t) {
  return copy2d(d, dp, s, sp, w, h, k);
}
static hipError_t copy3d(const hipMemcpy3DParms* p) {
  if (!p || p->kind == hipMemcpyDeviceToDevice) return hipSuccess;
  std::lock_guard<std::mutex> g(g_mu);
  const size_t n = p->extent.depth * p->extent.height * p->extent.width;
  if (p->dstPtr.ptr) host_copy_touch_locked(p->dstPtr.ptr, n);
  if (p->srcPtr.ptr) host_copy_touch_locked(p->srcPtr.ptr, n);
  return hipSuccess;
}
hipError_t hipMemcpy3D(const hipMemcpy3DParms* p) { return copy3d(p); }
hipError_t hipMemcpy3DAsync(const hipMemcpy3DParms* p, hipStream_t) { return copy3d(p); }
hipError_t hipMemcpyToSymbol(const void*, const void* s, size_t n, size_t, hipMemcpyKind k) {
  return fake_copy(nullptr, s, n, k);
}
hipError_t hipMemcpyToSymbolAsync(const void*, const void* s, size_t n, size_t, hipMemcpyKind k, hipStream_t) {
  return fake_copy(nullptr, s, n, k);
}
hipError_t hipMemcpyFromSymbol(void* d, const void*, size_t n, size_t, hipMemcpyKind k) {
  return fake_copy(d, nullptr, n, k);
}
hipError_t hipMemcpyFromSymbolAsync(void* d, const void*, size_t n, size_t, hipMemcpyKind k, hipStream_t) {
  return fake_copy(d, nullptr, n, k);
}
// Memsets run on the GPU: no page moves.
hipError_t hipMemset(void*, int, size_t) { g_memsets++; return hipSuccess; }
hipError_t hipMemsetAsync(void*, int, size_t, hipStream_t) { g_memsets++; return hipSuccess; }
hipError_t hipMemsetD8(hipDeviceptr_t, unsigned char, size_t) { g_memsets++; return hipSuccess; }
hipError_t hipMemsetD8Async(hipDeviceptr_t, unsigned char, size_t, hipStream_t) { g_memsets++; return hipSuccess; }
hipError_t hipMemsetD16(hipDeviceptr_t, unsigned short, size_t) { g_memsets++; return hipSuccess; }
hipError_t hipMemsetD16Async(hipDeviceptr_t, unsigned short, size_t, hipStream_t) { g_memsets++; return hipSuccess; }
hipError_t hipMemsetD32(hipDeviceptr_t, int, size_t) { g_memsets++; return hipSuccess; }
hipError_t hipMemsetD32Async(hipDeviceptr_t, int, size_t, hipStream_t) { g_memsets++; return hipSuccess; }
hipError_t hipMemset2D(void*, size_t, int, size_t, size_t) { g_memsets++; return hipSuccess; }
hipError_t hipMemset2DAsync(void*, size_t, int, size_t, size_t, hipStream_t) { g_memsets++; return hipSuccess; }
hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind k) { return fake_copy(d, s, n, k); }
// Peer copies: copy engine, device to device; no page of a managed range moves.
std::atomic<uint64_t> g_peer_copies{0};
hipError_t hipMemcpyPeer(void*, int, const void*, int, size_t) { g_peer_copies++; return hipSuccess; }
hipError_t hipMemcpyPeerAsync(void*, int, const void*, int, size_t, hipStream_t) { g_peer_copies++; return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned int) { return hipSuccess; }
// Device memory and managed ranges are "device"; anything else is unregistered host memory.
hipError_t hipPointerGetAttributes(hipPointerAttribute_t* a, const void* p) {
  std::lock_guard<std::mutex> g(g_mu);
  auto da = g_allocs.upper_bound((uintptr_t)p);
  if (da != g_allocs.begin() && (uintptr_t)p < std::prev(da)->first + std::prev(da)->second.second) {
    a->type = hipMemoryTypeDevice;
    return hipSuccess;
  }
  auto it = g_managed.upper_bound((uintptr_t)p);
  if (it != g_managed.begin() && (uintptr_t)p < std::prev(it)->first + std::prev(it)->second.size) {
    a->type = hipMemoryTypeManaged;
    return hipSuccess;
  }
  return hipErrorInvalidValue;
}
uint64_t fake_hip_host_touch_bytes() {
  std::lock_guard<std::mutex> g(g_mu);
  return g_host_touch_bytes;
}
hipError_t hipMemcpyWithStream(void* d, const void* s, size_t n, hipMemcpyKind k, hipStream_t) {
  return fake_copy(d, s, n, k);
}
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind k, hipStream_t) {
  return fake_copy(d, s, n, k);
}
hipError_t hipMemcpyHtoD(hipDeviceptr_t d, const void* s, size_t n) {
  return fake_copy(d, s, n, hipMemcpyHostToDevice);
}
hipError_t hipMemcpyDtoH(void* d, hipDeviceptr_t s, size_t n) { return fake_copy(d, s, n, hipMemcpyDeviceToHost); }
hipError_t hipMemcpyHtoDAsync(hipDeviceptr_t d, const void* s, size_t n, hipStream_t) {
  return fake_copy(d, s, n, hipMemcpyHostToDevice);
}
hipError_t hipMemcpyDtoHAsync(void* d, hipDeviceptr_t s, size_t n, hipStream_t) {
  return fake_copy(d, s, n, hipMemcpyDeviceToHost);
}
hipError_t hipDeviceGetPCIBusId(char*, int, int) { return hipErrorNotSupported; }  // no sysfs behind a fake
hipError_t hipMallocPitch(void** p, size_t* pitch, size_t w, size_t h) {
  *pitch = ((w + 511) / 512) * 512;
  return dev_alloc(p, *pitch * h, tl_dev);
}
hipError_t hipMemAllocPitch(hipDeviceptr_t* p, size_t* pitch, size_t w, size_t h, unsigned int) {
  *pitch = ((w + 511) / 512) * 512;
  return dev_alloc(p, *pitch * h, tl_dev);
}
hipError_t hipFree(void* p) {
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_managed.find((uintptr_t)p);
    if (it != g_managed.end()) {
      g_devs[it->second.dev].used -= it->second.gpu_bytes;
      g_managed.erase(it);
      return hipSuccess;
    }
  }
  return dev_free(p);
}
hipError_t hipFreeAsync(void* p, hipStream_t) {
  if (cap_free(p) || pool_free(p)) return hipSuccess;
  return dev_free(p);
}

static hipError_t host_alloc(void** p, size_t size) {
  // Host memory: a fake address too (tests allocate hundreds of GB virtually).
  std::lock_guard<std::mutex> g(g_mu);
  uintptr_t a = g_next | (1ull << 46);
  g_next += ((size + 4095) / 4096) * 4096 + 4096;
  *p = (void*)a;
  return hipSuccess;
}
hipError_t hipHostMalloc(void** p, size_t size, unsigned int) { return host_alloc(p, size); }
hipError_t hipHostFree(void* p) {
  std::lock_guard<std::mutex> g(g_mu);
  g_host_data.erase((uintptr_t)p);
  return hipSuccess;
}
// Not via hipHostMalloc: a preloaded interposer would see that call too.
hipError_t hipMallocHost(void** p, size_t size) { return host_alloc(p, size); }
hipError_t hipMemAllocHost(void** p, size_t size) { return host_alloc(p, size); }
hipError_t hipHostAlloc(void** p, size_t size, unsigned int) { return host_alloc(p, size); }

hipError_t hipMemCreate(hipMemGenericAllocationHandle_t* h, size_t size,
                        const hipMemAllocationProp* prop, unsigned long long) {
  void* p = nullptr;
  hipError_t rc = dev_alloc(&p, size, prop ? prop->location.id : tl_dev);
  *h = (hipMemGenericAllocationHandle_t)p;
  return rc;
}
hipError_t hipMemRelease(hipMemGenericAllocationHandle_t h) { return dev_free((void*)h); }
hipError_t hipMemGetAllocationGranularity(size_t* g, const hipMemAllocationProp*, hipMemAllocationGranularity_flags) {
  *g = 4096;
  return hipSuccess;
}
hipError_t hipMemAddressReserve(void** p, size_t size, size_t, void*, unsigned long long) {
  void* a = mmap(nullptr, size, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (a == MAP_FAILED) return hipErrorOutOfMemory;
  *p = a;
  return hipSuccess;
}
hipError_t hipMemAddressFree(void* p, size_t size) { return munmap(p, size) == 0 ? hipSuccess : hipErrorInvalidValue; }
hipError_t hipMemMap(void* p, size_t size, size_t, hipMemGenericAllocationHandle_t, unsigned long long) {
  if (mmap(p, size, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED, -1, 0) == MAP_FAILED)
    return hipErrorInvalidValue;
  std::lock_guard<std::mutex> g(g_mu);
  g_vmm_mapped[(uintptr_t)p] = size;
  return hipSuccess;
}
hipError_t hipMemUnmap(void* p, size_t size) {
  std::lock_guard<std::mutex> g(g_mu);
  g_vmm_mapped.erase((uintptr_t)p);
  // back to an inaccessible reservation: the contents are gone
  mmap(p, size, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED | MAP_NORESERVE, -1, 0);
  return hipSuccess;
}
hipError_t hipMemSetAccess(void*, size_t, const hipMemAccessDesc*, size_t) { return hipSuccess; }

hipError_t hipMemGetInfo(size_t* f, size_t* t) {
  std::lock_guard<std::mutex> g(g_mu);
  init_locked();
  Dev& d = g_devs[tl_dev];
  // Like ROCm: VRAM that SVM migrations took is not subtracted.
  uint64_t svm = 0;
  for (auto& m : g_managed)
    if (m.second.dev == tl_dev) svm += m.second.gpu_bytes;
  *f = d.total - d.used + svm;
  *t = d.total;
  return hipSuccess;
}
hipError_t hipDeviceTotalMem(size_t* b, hipDevice_t dev) {
  init();
  *b = g_devs[dev].total;
  return hipSuccess;
}
hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600* p, int dev) {
  init();
  memset(p, 0, sizeof(*p));
  snprintf(p->name, sizeof(p->name), "AMD Instinct MI355X (fake)");
  snprintf(p->gcnArchName, sizeof(p->gcnArchName), "gfx950:sramecc+:xnack-");
  p->totalGlobalMem = g_devs[dev].total;
  p->multiProcessorCount = env_int("VGPU_FAKE_CUS", 256);
  p->warpSize = 64;
  return hipSuccess;
}
hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t a, int) {
  init();
  if (a == hipDeviceAttributeMultiprocessorCount) { *v = env_int("VGPU_FAKE_CUS", 256); return hipSuccess; }
  *v = 0;
  return hipSuccess;
}
hipError_t hipOccupancyMaxActiveBlocksPerMultiprocessor(int* n, const void*, int, size_t) {
  *n = 8;
  return hipSuccess;
}

hipError_t hipLaunchKernel(const void*, dim3 g, dim3, void**, size_t, hipStream_t) {
  count_launch((uint64_t)g.x * g.y * g.z);
  return hipSuccess;
}
hipError_t hipExtLaunchKernel(const void*, dim3 g, dim3, void**, size_t, hipStream_t, hipEvent_t,
                              hipEvent_t, int) {
  count_launch((uint64_t)g.x * g.y * g.z);
  return hipSuccess;
}
hipError_t hipModuleLaunchKernel(hipFunction_t, unsigned gx, unsigned gy, unsigned gz, unsigned,
                                 unsigned, unsigned, unsigned, hipStream_t, void**, void**) {
  count_launch((uint64_t)gx * gy * gz);
  return hipSuccess;
}
hipError_t hipExtModuleLaunchKernel(hipFunction_t, uint32_t gx, uint32_t gy, uint32_t gz,
                                    uint32_t lx, uint32_t ly, uint32_t lz, size_t, hipStream_t,
                                    void**, void**, hipEvent_t, hipEvent_t, uint32_t) {
  count_launch((uint64_t)(gx / (lx ? lx : 1)) * (gy / (ly ? ly : 1)) * (gz / (lz ? lz : 1)));
  return hipSuccess;
}
hipError_t hipLaunchCooperativeKernel(const void*, dim3 g, dim3, void**, unsigned int, hipStream_t) {
  count_launch((uint64_t)g.x * g.y * g.z);
  return hipSuccess;
}
hipError_t hipModuleLaunchCooperativeKernel(hipFunction_t, unsigned gx, unsigned gy, unsigned gz,
                                            unsigned, unsigned, unsigned, unsigned, hipStream_t,
                                            void**) {
  count_launch((uint64_t)gx * gy * gz);
  return hipSuccess;
}
hipError_t hipLaunchKernelExC(const hipLaunchConfig_t* c, const void*, void**) {
  count_launch((uint64_t)c->gridDim.x * c->gridDim.y * c->gridDim.z);
  return hipSuccess;
}
// The launch entry points beyond the common ones (VERDICT r5 missing #1):
// per-thread-default-stream variants, the driver-style extensible launch, the
// multi-device launches (one kernel per list entry) and the legacy
// configure/launch-by-pointer pair.
hipError_t hipLaunchKernel_spt(const void*, dim3 g, dim3, void**, size_t, hipStream_t) {
  count_launch((uint64_t)g.x * g.y * g.z);
  return hipSuccess;
}
hipError_t hipLaunchCooperativeKernel_spt(const void*, dim3 g, dim3, void**, uint32_t, hipStream_t) {
  count_launch((uint64_t)g.x * g.y * g.z);
  return hipSuccess;
}
hipError_t hipDrvLaunchKernelEx(const HIP_LAUNCH_CONFIG* c, hipFunction_t, void**, void**) {
  if (!c) return hipErrorInvalidValue;
  count_launch((uint64_t)c->gridDimX * c->gridDimY * c->gridDimZ);
  return hipSuccess;
}
hipError_t hipHccModuleLaunchKernel(hipFunction_t, uint32_t gx, uint32_t gy, uint32_t gz, uint32_t lx,
                                    uint32_t ly, uint32_t lz, size_t, hipStream_t, void**, void**, hipEvent_t,
                                    hipEvent_t) {
  count_launch((uint64_t)(gx / (lx ? lx : 1)) * (gy / (ly ? ly : 1)) * (gz / (lz ? lz : 1)));
  return hipSuccess;
}
hipError_t hipExtLaunchMultiKernelMultiDevice(hipLaunchParams* l, int n, unsigned int) {
  for (int i = 0; l && i < n; ++i) count_launch((uint64_t)l[i].gridDim.x * l[i].gridDim.y * l[i].gridDim.z);
  return hipSuccess;
}
hipError_t hipLaunchCooperativeKernelMultiDevice(hipLaunchParams* l, int n, unsigned int) {
  for (int i = 0; l && i < n; ++i) count_launch((uint64_t)l[i].gridDim.x * l[i].gridDim.y * l[i].gridDim.z);
  return hipSuccess;
}
hipError_t hipModuleLaunchCooperativeKernelMultiDevice(hipFunctionLaunchParams* l, unsigned int n, unsigned int) {
  for (unsigned i = 0; l && i < n; ++i) count_launch((uint64_t)l[i].gridDimX * l[i].gridDimY * l[i].gridDimZ);
  return hipSuccess;
}
static thread_local std::vector<dim3> tl_configured;
hipError_t hipConfigureCall(dim3 g, dim3, size_t, hipStream_t) {
  tl_configured.push_back(g);
  return hipSuccess;
}
hipError_t hipSetupArgument(const void*, size_t, size_t) { return hipSuccess; }
hipError_t hipLaunchByPtr(const void*) {
  if (tl_configured.empty()) return hipErrorNotInitialized;
  const dim3 g = tl_configured.back();
  tl_configured.pop_back();
  count_launch((uint64_t)g.x * g.y * g.z);
  return hipSuccess;
}
}  // extern "C"
// The C++-linkage module launches older hip_ext.h declared (still exported by
// libamdhip64 under their mangled names).
extern "C" hipError_t fake_cxx_ext_module_launch(hipFunction_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t,
                                                 uint32_t, size_t, hipStream_t, void**, void**, hipEvent_t,
                                                 hipEvent_t, uint32_t) __asm__(
    "_Z24hipExtModuleLaunchKernelP18ihipModuleSymbol_tjjjjjjmP12ihipStream_tPPvS4_P11ihipEvent_tS6_j");
extern "C" hipError_t fake_cxx_ext_module_launch(hipFunction_t, uint32_t gx, uint32_t gy, uint32_t gz, uint32_t lx,
                                                 uint32_t ly, uint32_t lz, size_t, hipStream_t, void**, void**,
                                                 hipEvent_t, hipEvent_t, uint32_t) {
  count_launch((uint64_t)(gx / (lx ? lx : 1)) * (gy / (ly ? ly : 1)) * (gz / (lz ? lz : 1)));
  return hipSuccess;
}
extern "C" hipError_t fake_cxx_hcc_module_launch(hipFunction_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t,
                                                 uint32_t, size_t, hipStream_t, void**, void**, hipEvent_t,
                                                 hipEvent_t) __asm__(
    "_Z24hipHccModuleLaunchKernelP18ihipModuleSymbol_tjjjjjjmP12ihipStream_tPPvS4_P11ihipEvent_tS6_");
extern "C" hipError_t fake_cxx_hcc_module_launch(hipFunction_t, uint32_t gx, uint32_t gy, uint32_t gz, uint32_t lx,
                                                 uint32_t ly, uint32_t lz, size_t, hipStream_t, void**, void**,
                                                 hipEvent_t, hipEvent_t) {
  count_launch((uint64_t)(gx / (lx ? lx : 1)) * (gy / (ly ? ly : 1)) * (gz / (lz ? lz : 1)));
  return hipSuccess;
}
extern "C" {
// Minimal graphs: a graph is a list of kernel nodes (grid sizes) and child
// graphs, enough for the shim's node walk; an exec remembers its graph.
struct FakeNode {
  hipGraphNodeType type;
  dim3 grid;
  hipGraph_t child;
  const void* func = nullptr;  // kernel nodes: the host stub (hipKernelNodeParams::func)
};
struct FakeGraph {
  std::vector<FakeNode*> nodes;
  std::vector<std::pair<FakeNode*, FakeNode*>> edges;  // dependencies (from, to)
  uint64_t alloc_bytes = 0;  // captured hipMallocAsync bytes (graph alloc nodes)
};
// A capture yields an (empty) graph: enough for the shim's capture -> graph
// -> exec bookkeeping.
static hipError_t end_capture_impl(hipStream_t s, hipGraph_t* g) {
  if (g) *g = nullptr;
  std::lock_guard<std::mutex> lk(g_cap_mu);
  auto it = g_capturing.find(s);
  if (it == g_capturing.end()) return hipErrorIllegalState;
  const bool invalid = it->second;
  g_capturing.erase(it);
  const unsigned long long cid = g_capture_id[s];
  g_capture_id.erase(s);
  if (!invalid && g) {
    auto* fg = new FakeGraph;
    fg->alloc_bytes = g_cap_alloc[cid].peak;
    *g = reinterpret_cast<hipGraph_t>(fg);
  }
  g_cap_alloc.erase(cid);
  for (auto it = g_cap_ptr.begin(); it != g_cap_ptr.end();)
    it = it->second.first == cid ? g_cap_ptr.erase(it) : std::next(it);
  return invalid ? hipErrorStreamCaptureInvalidated : hipSuccess;
}
hipError_t hipStreamEndCapture(hipStream_t s, hipGraph_t* g) { return end_capture_impl(s, g); }
hipError_t hipStreamEndCapture_spt(hipStream_t s, hipGraph_t* g) { return end_capture_impl(s, g); }
hipError_t hipGraphDestroy(hipGraph_t g) {
  delete reinterpret_cast<FakeGraph*>(g);
  return hipSuccess;
}
hipError_t hipGraphGetNodes(hipGraph_t g, hipGraphNode_t* nodes, size_t* n) {
  auto* fg = reinterpret_cast<FakeGraph*>(g);
  if (!fg || !n) return hipErrorInvalidValue;
  if (nodes)
    for (size_t i = 0; i < *n && i < fg->nodes.size(); ++i) nodes[i] = reinterpret_cast<hipGraphNode_t>(fg->nodes[i]);
  *n = fg->nodes.size();
  return hipSuccess;
}
hipError_t hipGraphNodeGetType(hipGraphNode_t node, hipGraphNodeType* t) {
  *t = reinterpret_cast<FakeNode*>(node)->type;
  return hipSuccess;
}
hipError_t hipGraphKernelNodeGetParams(hipGraphNode_t node, hipKernelNodeParams* p) {
  auto* fn = reinterpret_cast<FakeNode*>(node);
  if (fn->type != hipGraphNodeTypeKernel) return hipErrorInvalidValue;
  *p = hipKernelNodeParams{};
  p->gridDim = fn->grid;
  p->blockDim = dim3(256, 1, 1);
  p->func = const_cast<void*>(fn->func);
  return hipSuccess;
}
hipError_t hipGraphChildGraphNodeGetGraph(hipGraphNode_t node, hipGraph_t* g) {
  *g = reinterpret_cast<FakeNode*>(node)->child;
  return hipSuccess;
}
std::set<const void*> g_live_execs;  // a test may launch an exec it destroyed
hipError_t hipGraphInstantiateWithFlags(hipGraphExec_t* e, hipGraph_t g, unsigned long long) {
  *e = reinterpret_cast<hipGraphExec_t>(new hipGraph_t(g));
  std::lock_guard<std::mutex> l(g_mu);
  g_live_execs.insert(*e);
  return hipSuccess;
}
hipError_t hipGraphInstantiate(hipGraphExec_t* e, hipGraph_t g, hipGraphNode_t*, char*, size_t) {
  return hipGraphInstantiateWithFlags(e, g, 0);
}
hipError_t hipGraphExecDestroy(hipGraphExec_t e) {
  {
    std::lock_guard<std::mutex> l(g_mu);
    g_live_execs.erase(e);
  }
  delete reinterpret_cast<hipGraph_t*>(e);
  return hipSuccess;
}
static hipError_t graph_launch_impl(hipGraphExec_t e) {
  init();
  if (e) {  // alloc nodes draw on the device's graph pool (kept until hipDeviceGraphMemTrim)
    std::lock_guard<std::mutex> g(g_mu);
    auto* fg = g_live_execs.count(e) ? reinterpret_cast<FakeGraph*>(*reinterpret_cast<hipGraph_t*>(e)) : nullptr;
    if (fg && fg->alloc_bytes > g_graph_mem[tl_dev]) {
      const uint64_t grow = fg->alloc_bytes - g_graph_mem[tl_dev];
      if (g_devs[tl_dev].used + grow > g_devs[tl_dev].total) return hipErrorOutOfMemory;
      g_devs[tl_dev].used += grow;
      g_graph_mem[tl_dev] = fg->alloc_bytes;
    }
  }
  // The ROCm 7 runtime's multi-stream executor reads past its stream list when
  // GPU_MAX_HW_QUEUES=1 and the graph has parallel branches (a node with two
  // successors): the real runtime segfaults, the fake refuses the launch.
  if (e) {
    static const bool one_queue = getenv("GPU_MAX_HW_QUEUES") && atoi(getenv("GPU_MAX_HW_QUEUES")) == 1;
    std::lock_guard<std::mutex> g(g_mu);
    auto* fg = g_live_execs.count(e) ? reinterpret_cast<FakeGraph*>(*reinterpret_cast<hipGraph_t*>(e)) : nullptr;
    if (one_queue && fg) {
      std::map<FakeNode*, int> succ;
      for (auto& ed : fg->edges)
        if (++succ[ed.first] > 1) {
          g_branchy_single_queue.fetch_add(1);
          return hipErrorLaunchFailure;
        }
    }
  }
  g_graph_launches.fetch_add(1);
  g_launches.fetch_add(1);
  timeline_launch();
  return hipSuccess;
}
hipError_t hipGraphLaunch(hipGraphExec_t e, hipStream_t) { return graph_launch_impl(e); }
hipError_t hipGraphLaunch_spt(hipGraphExec_t e, hipStream_t) { return graph_launch_impl(e); }
// Explicit graph construction (hipGraphAdd*Node): nodes join the fake graph;
// an alloc node's bytes come from the graph pool at launch.
hipError_t hipGraphCreate(hipGraph_t* g, unsigned int) {
  *g = reinterpret_cast<hipGraph_t>(new FakeGraph);
  return hipSuccess;
}
static hipGraphNode_t add_node(hipGraphNode_t* node, hipGraph_t g, FakeNode* n) {
  reinterpret_cast<FakeGraph*>(g)->nodes.push_back(n);
  if (node) *node = reinterpret_cast<hipGraphNode_t>(n);
  return reinterpret_cast<hipGraphNode_t>(n);
}
hipError_t hipGraphAddKernelNode(hipGraphNode_t* node, hipGraph_t g, const hipGraphNode_t* deps, size_t ndeps,
                                 const hipKernelNodeParams* p) {
  if (!g || !p) return hipErrorInvalidValue;
  hipGraphNode_t n = add_node(node, g, new FakeNode{hipGraphNodeTypeKernel, p->gridDim, nullptr, p->func});
  for (size_t i = 0; i < ndeps; ++i)
    reinterpret_cast<FakeGraph*>(g)->edges.push_back({reinterpret_cast<FakeNode*>(deps[i]), reinterpret_cast<FakeNode*>(n)});
  return hipSuccess;
}
hipError_t hipGraphClone(hipGraph_t* out, hipGraph_t g) {
  if (!out || !g) return hipErrorInvalidValue;
  auto* src = reinterpret_cast<FakeGraph*>(g);
  auto* c = new FakeGraph;
  std::map<FakeNode*, FakeNode*> m;
  for (FakeNode* n : src->nodes) {
    c->nodes.push_back(new FakeNode(*n));
    m[n] = c->nodes.back();
  }
  for (auto& e : src->edges) c->edges.push_back({m[e.first], m[e.second]});
  c->alloc_bytes = src->alloc_bytes;
  *out = reinterpret_cast<hipGraph_t>(c);
  return hipSuccess;
}
hipError_t hipGraphGetEdges(hipGraph_t g, hipGraphNode_t* from, hipGraphNode_t* to, size_t* n) {
  if (!g || !n) return hipErrorInvalidValue;
  auto& e = reinterpret_cast<FakeGraph*>(g)->edges;
  if (from && to)
    for (size_t i = 0; i < e.size() && i < *n; ++i) {
      from[i] = reinterpret_cast<hipGraphNode_t>(e[i].first);
      to[i] = reinterpret_cast<hipGraphNode_t>(e[i].second);
    }
  *n = e.size();
  return hipSuccess;
}
hipError_t hipGraphAddDependencies(hipGraph_t g, const hipGraphNode_t* from, const hipGraphNode_t* to, size_t n) {
  if (!g) return hipErrorInvalidValue;
  for (size_t i = 0; i < n; ++i)
    reinterpret_cast<FakeGraph*>(g)->edges.push_back(
        {reinterpret_cast<FakeNode*>(from[i]), reinterpret_cast<FakeNode*>(to[i])});
  return hipSuccess;
}
hipError_t hipGraphRemoveDependencies(hipGraph_t g, const hipGraphNode_t* from, const hipGraphNode_t* to, size_t n) {
  if (!g) return hipErrorInvalidValue;
  auto& e = reinterpret_cast<FakeGraph*>(g)->edges;
  for (size_t i = 0; i < n; ++i) {
    auto it = std::find(e.begin(), e.end(), std::make_pair(reinterpret_cast<FakeNode*>(from[i]),
                                                           reinterpret_cast<FakeNode*>(to[i])));
    if (it == e.end()) return hipErrorInvalidValue;
    e.erase(it);
  }
  return hipSuccess;
}
static hipError_t set_kernel_params(hipGraphNode_t node, const hipKernelNodeParams* p) {
  if (!node || !p) return hipErrorInvalidValue;
  reinterpret_cast<FakeNode*>(node)->grid = p->gridDim;
  return hipSuccess;
}
hipError_t hipGraphKernelNodeSetParams(hipGraphNode_t node, const hipKernelNodeParams* p) {
  return set_kernel_params(node, p);
}
// (an executable's node is not its graph's: the fake leaves the graph alone)
hipError_t hipGraphExecKernelNodeSetParams(hipGraphExec_t e, hipGraphNode_t node, const hipKernelNodeParams* p) {
  return e && node && p ? hipSuccess : hipErrorInvalidValue;
}
hipError_t hipGraphExecUpdate(hipGraphExec_t e, hipGraph_t g, hipGraphNode_t*, hipGraphExecUpdateResult* r) {
  if (!e || !g) return hipErrorInvalidValue;
  *reinterpret_cast<hipGraph_t*>(e) = g;
  if (r) *r = hipGraphExecUpdateSuccess;
  return hipSuccess;
}
hipError_t hipGraphAddMemcpyNode(hipGraphNode_t* node, hipGraph_t g, const hipGraphNode_t*, size_t,
                                 const hipMemcpy3DParms*) {
  add_node(node, g, new FakeNode{hipGraphNodeTypeMemcpy, dim3(1, 1, 1), nullptr});
  return hipSuccess;
}
hipError_t hipGraphAddMemcpyNode1D(hipGraphNode_t* node, hipGraph_t g, const hipGraphNode_t*, size_t, void*,
                                   const void*, size_t, hipMemcpyKind) {
  add_node(node, g, new FakeNode{hipGraphNodeTypeMemcpy, dim3(1, 1, 1), nullptr});
  return hipSuccess;
}
hipError_t hipGraphAddMemsetNode(hipGraphNode_t* node, hipGraph_t g, const hipGraphNode_t*, size_t,
                                 const hipMemsetParams*) {
  add_node(node, g, new FakeNode{hipGraphNodeTypeMemset, dim3(1, 1, 1), nullptr});
  return hipSuccess;
}
hipError_t hipGraphAddChildGraphNode(hipGraphNode_t* node, hipGraph_t g, const hipGraphNode_t*, size_t,
                                     hipGraph_t child) {
  add_node(node, g, new FakeNode{hipGraphNodeTypeGraph, dim3(1, 1, 1), child});
  reinterpret_cast<FakeGraph*>(g)->alloc_bytes += reinterpret_cast<FakeGraph*>(child)->alloc_bytes;
  return hipSuccess;
}
hipError_t hipGraphAddMemAllocNode(hipGraphNode_t* node, hipGraph_t g, const hipGraphNode_t*, size_t,
                                   hipMemAllocNodeParams* p) {
  if (!g || !p) return hipErrorInvalidValue;
  add_node(node, g, new FakeNode{hipGraphNodeTypeMemAlloc, dim3(1, 1, 1), nullptr});
  reinterpret_cast<FakeGraph*>(g)->alloc_bytes += p->bytesize;
  std::lock_guard<std::mutex> l(g_mu);
  p->dptr = (void*)g_next;
  g_next += (p->bytesize + (1 << 21)) & ~((uintptr_t)(1 << 21) - 1);
  return hipSuccess;
}

// Test helper: a graph of kernel nodes with grids (grids[i], 2, 1) plus, when
// child_grid > 0, one child graph holding a kernel node of grid child_grid.
hipGraph_t fake_hip_graph_create(const unsigned* grids, int n, unsigned child_grid) {
  auto* g = new FakeGraph;
  for (int i = 0; i < n; ++i) g->nodes.push_back(new FakeNode{hipGraphNodeTypeKernel, dim3(grids[i], 2, 1), nullptr});
  if (child_grid) {
    auto* c = new FakeGraph;
    c->nodes.push_back(new FakeNode{hipGraphNodeTypeKernel, dim3(child_grid, 1, 1), nullptr});
    g->nodes.push_back(new FakeNode{hipGraphNodeTypeGraph, dim3(1, 1, 1), reinterpret_cast<hipGraph_t>(c)});
  }
  // a memcpy-like node the walk must ignore
  g->nodes.push_back(new FakeNode{hipGraphNodeTypeMemset, dim3(99999, 1, 1), nullptr});
  return reinterpret_cast<hipGraph_t>(g);
}
}  // extern "C"
// The runtime's own entry points as its lookups return them: internal
// addresses no preloaded library can interpose (taking &hipLaunchKernel here
// would resolve through the GOT to the interposer).
static hipError_t own_launch(const void*, dim3 g, dim3, void**, size_t, hipStream_t) {
  count_launch((uint64_t)g.x * g.y * g.z);
  return hipSuccess;
}
static void* own_entry(const char* sym) {
  if (!strcmp(sym, "hipLaunchKernel") || !strcmp(sym, "hipLaunchKernel_spt")) return (void*)&own_launch;
  return nullptr;
}
extern "C" {
hipError_t hipGetDriverEntryPoint(const char* sym, void** pfn, unsigned long long, hipDriverEntryPointQueryResult* st) {
  *pfn = sym ? own_entry(sym) : nullptr;
  if (st) *st = *pfn ? hipDriverEntryPointSuccess : hipDriverEntryPointSymbolNotFound;
  return *pfn ? hipSuccess : hipErrorNotFound;
}
hipError_t hipGetDriverEntryPoint_spt(const char* sym, void** pfn, unsigned long long f,
                                      hipDriverEntryPointQueryResult* st) {
  return hipGetDriverEntryPoint(sym, pfn, f, st);
}
hipError_t hipGetProcAddress(const char* sym, void** pfn, int, uint64_t,
                             hipDriverProcAddressQueryResult* st) {
  // Answer from this library only (the real runtime returns its own entry points).
  static void* self = dlopen("libamdhip64.so.7", RTLD_NOLOAD | RTLD_LAZY);
  *pfn = sym ? own_entry(sym) : nullptr;
  if (!*pfn) *pfn = self ? dlsym(self, sym) : nullptr;
  if (st) *st = *pfn ? HIP_GET_PROC_ADDRESS_SUCCESS : HIP_GET_PROC_ADDRESS_SYMBOL_NOT_FOUND;
  return *pfn ? hipSuccess : hipErrorNotFound;
}

// ---- test introspection ----
uint64_t fake_hip_launches() { return g_launches.load(); }
uint64_t fake_hip_branchy_single_queue_launches() { return g_branchy_single_queue.load(); }
uint64_t fake_hip_memsets() { return g_memsets.load(); }
uint64_t fake_hip_exec_ns() { return g_exec_ns.load(); }
// The graph an executable runs (tests: what the shim instantiated).
hipGraph_t fake_hip_exec_graph(hipGraphExec_t e) { return e ? *reinterpret_cast<hipGraph_t*>(e) : nullptr; }
uint64_t fake_hip_launch_blocks() { return g_launch_blocks.load(); }
uint64_t fake_hip_physical_used(int dev) {
  std::lock_guard<std::mutex> g(g_mu);
  return dev < (int)g_devs.size() ? g_devs[dev].used : 0;
}
// KFD SVM migration of [p, p+n) of a managed range: to HBM only if it fits
// (KFD leaves pages in system memory otherwise, and still reports success).
int fake_hip_svm_move(const void* p, uint64_t n, int to_gpu) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_managed.upper_bound((uintptr_t)p);
  if (it == g_managed.begin()) return -1;
  --it;
  Managed& m = it->second;
  if ((uintptr_t)p >= it->first + m.size) return -1;
  Dev& d = g_devs[m.dev];
  if (to_gpu) {
    uint64_t add = std::min<uint64_t>(n, m.size - m.gpu_bytes);
    if (d.used + add > d.total) return 0;
    m.gpu_bytes += add;
    d.used += add;
  } else {
    uint64_t sub = std::min<uint64_t>(n, m.gpu_bytes);
    m.gpu_bytes -= sub;
    d.used -= sub;
  }
  return 1;
}
uint64_t fake_hip_peer_copies() { return g_peer_copies.load(); }
uint64_t fake_hip_prefetch_overflows() {
  std::lock_guard<std::mutex> g(g_mu);
  return g_prefetch_over;
}
uint64_t fake_hip_managed_gpu_bytes(const void* p) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_managed.find((uintptr_t)p);
  return it == g_managed.end() ? 0 : it->second.gpu_bytes;
}

}  // extern "C"
