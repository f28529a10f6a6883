// Migration-rate probe for the shim's virtual device memory (native/shim/vmem.cpp).
// KFD SVM (hipMallocManaged) ranges are the only VA-stable vehicle between HBM
// and host memory with XNACK off (profiles/vmem_r2.md); round 2 measured
// 4-6.5 GB/s host->HBM with 1 GiB pieces.  This probe measures what moves it
// faster:
//   fresh   : never-touched range -> HBM (allocation-time residency)
//   piece   : host-filled range -> HBM in pieces of 256 MiB / 1 GiB / whole
//   thp     : the same with MADV_HUGEPAGE on the host pages before first touch
//   conc    : 4 ranges prefetched concurrently (4 signals in flight)
//   down    : HBM -> host
//   read    : kernel read bandwidth of a promoted range; data check
// Output: one "key=value" line per measurement (GB/s), parsed by scripts.
// Build: hipcc --offload-arch=gfx950 -O2 -o svm_rate svm_rate.hip -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) printf("err %s -> %d (%s)\n", #x, e_, hipGetErrorString(e_)); \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void sum_k(const uint4* p, size_t n, unsigned long long* out) {
  unsigned long long s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint4 q = p[i];
    s += q.x ^ q.w;
  }
  if (s == 0x1234567) atomicAdd(out, s);  // keeps the loads alive
}

static hsa_agent_t g_gpu{}, g_cpu{};
static hsa_status_t agent_cb(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
  if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
  return HSA_STATUS_SUCCESS;
}

// Prefetch [p, p+n) in `piece`-sized chunks with up to `depth` in flight.
static double prefetch(void* p, size_t n, bool to_gpu, size_t piece, int depth) {
  std::vector<hsa_signal_t> sig(depth);
  for (auto& s : sig) hsa_signal_create(1, 0, nullptr, &s);
  double t0 = now();
  size_t off = 0;
  int k = 0;
  std::vector<bool> busy(depth, false);
  while (off < n) {
    if (busy[k]) hsa_signal_wait_scacquire(sig[k], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    hsa_signal_store_relaxed(sig[k], 1);
    size_t m = n - off < piece ? n - off : piece;
    hsa_status_t st = hsa_amd_svm_prefetch_async((char*)p + off, m, to_gpu ? g_gpu : g_cpu, 0, nullptr, sig[k]);
    if (st != HSA_STATUS_SUCCESS) printf("err prefetch %d\n", (int)st);
    busy[k] = true;
    off += m;
    k = (k + 1) % depth;
  }
  for (int i = 0; i < depth; ++i)
    if (busy[i]) hsa_signal_wait_scacquire(sig[i], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
  double dt = now() - t0;
  for (auto& s : sig) hsa_signal_destroy(s);
  return n / dt / 1e9;
}

static void* managed(size_t n, bool thp, bool fill) {
  void* p = nullptr;
  CK(hipMallocManaged(&p, n, hipMemAttachGlobal));
  CK(hipMemAdvise(p, n, hipMemAdviseSetCoarseGrain, 0));
  if (thp) madvise(p, n, MADV_HUGEPAGE);
  if (fill) memset(p, 0x5a, n);
  return p;
}

static double read_bw(void* p, size_t n, unsigned long long* out) {
  sum_k<<<8192, 256>>>((const uint4*)p, n / 16, out);
  CK(hipDeviceSynchronize());
  double t0 = now();
  for (int i = 0; i < 3; ++i) sum_k<<<8192, 256>>>((const uint4*)p, n / 16, out);
  CK(hipDeviceSynchronize());
  return 3.0 * n / (now() - t0) / 1e9;
}

int main(int argc, char** argv) {
  const size_t G = 1ull << 30;
  const size_t n = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 4) * G;
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  hsa_iterate_agents(agent_cb, nullptr);
  unsigned long long* out;
  CK(hipMalloc(&out, 8));

  {  // pinned copy reference
    void *h, *d;
    CK(hipHostMalloc(&h, n, hipHostMallocDefault));
    CK(hipMalloc(&d, n));
    memset(h, 1, n);
    CK(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
    double t0 = now();
    CK(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
    printf("pinned_h2d=%.2f\n", n / (now() - t0) / 1e9);
    t0 = now();
    CK(hipMemcpy(h, d, n, hipMemcpyDeviceToHost));
    printf("pinned_d2h=%.2f\n", n / (now() - t0) / 1e9);
    CK(hipFree(d));
    CK(hipHostFree(h));
  }
  {  // never-touched range straight to HBM
    void* p = managed(n, false, false);
    printf("fresh_up=%.2f\n", prefetch(p, n, true, n, 1));
    printf("fresh_read=%.1f\n", read_bw(p, n, out));
    CK(hipFree(p));
  }
  {  // never-touched, THP
    void* p = managed(n, true, false);
    printf("fresh_thp_up=%.2f\n", prefetch(p, n, true, n, 1));
    CK(hipFree(p));
  }
  const size_t pieces[] = {256ull << 20, G, n};
  for (size_t pc : pieces) {
    void* p = managed(n, false, true);
    printf("up_piece%zuM=%.2f\n", pc >> 20, prefetch(p, n, true, pc, 1));
    if (pc == G) {
      printf("read_promoted=%.1f\n", read_bw(p, n, out));
      printf("down_piece%zuM=%.2f\n", pc >> 20, prefetch(p, n, false, pc, 1));
      printf("read_host=%.1f\n", read_bw(p, n, out));
      printf("up_again=%.2f\n", prefetch(p, n, true, pc, 1));
    }
    CK(hipFree(p));
  }
  {
    void* p = managed(n, true, true);
    printf("thp_up_whole=%.2f\n", prefetch(p, n, true, n, 1));
    printf("thp_down_whole=%.2f\n", prefetch(p, n, false, n, 1));
    printf("thp_up_again=%.2f\n", prefetch(p, n, true, n, 1));
    CK(hipFree(p));
  }
  {  // 4 concurrent pieces
    void* p = managed(n, true, true);
    printf("thp_up_conc4_256M=%.2f\n", prefetch(p, n, true, 256ull << 20, 4));
    printf("thp_down_conc4_256M=%.2f\n", prefetch(p, n, false, 256ull << 20, 4));
    CK(hipFree(p));
  }
  printf("done=1\n");
  return 0;
}
