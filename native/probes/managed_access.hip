// Access-cost probe for the shim's managed-by-default ranges (native/shim/vmem.cpp):
// a VGG-16 pod under the vgpu-vmem knobs ran some hipBLASLt GEMMs and the
// optimizer's multi_tensor_apply 10-55x slower on promoted (HBM-resident)
// managed ranges than on hipMalloc memory, while a plain streaming read of a
// promoted range runs at full bandwidth (svm_rate.hip).  This probe times, on
// 512 MiB buffers of each kind,
//   stream : one read pass (float4)
//   reuse  : every block re-reads the same 4 MiB window 16x (L2 reuse, like GEMM tiles)
//   write  : one write pass
//   pages  : one 16-byte read per 4 KiB page in a scattered page order (TLB reach)
//   atomic : float atomicAdd into a 256 KiB window (split-K reductions)
// for hipMalloc, managed + coarse-grain advice + prefetch, and managed +
// prefetch without the advice, then a promoted range after host<->device copies.  Output: "kind op us" lines.
// Build: hipcc --offload-arch=gfx950 -O2 -o managed_access managed_access.hip -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) printf("err %s -> %d (%s)\n", #x, e_, hipGetErrorString(e_)); \
  } while (0)

constexpr size_t kBytes = 512ull << 20;
constexpr size_t kN4 = kBytes / 16;

__global__ void stream_k(const float4* p, size_t n, float* out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float4 q = p[i];
    s += q.x + q.w;
  }
  if (s == 12345.f) out[0] = s;
}

__global__ void reuse_k(const float4* p, float* out) {
  constexpr size_t win = (4u << 20) / 16;
  float s = 0.f;
  for (int r = 0; r < 16; ++r)
    for (size_t i = threadIdx.x + (size_t)(blockIdx.x % 64) * 256; i < win; i += 64 * 256) {
      float4 q = p[i];
      s += q.y * (float)r;
    }
  if (s == 12345.f) out[0] = s;
}

__global__ void write_k(float4* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

// One 16-byte read per 4 KiB page, pages visited in a scattered order: a new
// page (and translation) per access, like a transposed GEMM operand.
__global__ void pages_k(const float4* p, size_t n, float* out) {
  const size_t pages = n / 256;
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t pg = (i * 2654435761ull) % pages, off = (i / pages) % 256;
    s += p[pg * 256 + off].z;
  }
  if (s == 12345.f) out[0] = s;
}

__global__ void atomic_k(float* p) {
  const size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) % (64 * 1024);
  atomicAdd(p + i, 1.f);
}

static float time_us(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f;
}

static void run(const char* kind, void* buf, float* out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep) {  // first pass warms (page tables, code)
    const bool pr = rep == 1;
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i) stream_k<<<4096, 256>>>((const float4*)buf, kN4, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    if (pr) printf("%s stream %.1f us (%.0f GB/s)\n", kind, time_us(a, b) / 10, kBytes / (time_us(a, b) / 10) / 1e3);
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i) reuse_k<<<4096, 256>>>((const float4*)buf, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    if (pr) printf("%s reuse %.1f us\n", kind, time_us(a, b) / 10);
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i) pages_k<<<4096, 256>>>((const float4*)buf, kN4, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    if (pr) printf("%s pages %.1f us\n", kind, time_us(a, b) / 10);
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i) write_k<<<4096, 256>>>((float4*)buf, kN4);
    hipEventRecord(b);
    hipEventSynchronize(b);
    if (pr) printf("%s write %.1f us (%.0f GB/s)\n", kind, time_us(a, b) / 10, kBytes / (time_us(a, b) / 10) / 1e3);
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i) atomic_k<<<4096, 256>>>((float*)buf);
    hipEventRecord(b);
    hipEventSynchronize(b);
    if (pr) printf("%s atomic %.1f us\n", kind, time_us(a, b) / 10);
  }
  CK(hipDeviceSynchronize());
  hipEventDestroy(a);
  hipEventDestroy(b);
}

static void prefetch_gpu(void* p) {
  hsa_agent_t gpu{};
  hsa_iterate_agents(
      [](hsa_agent_t ag, void* d) {
        hsa_device_type_t t;
        hsa_agent_get_info(ag, HSA_AGENT_INFO_DEVICE, &t);
        if (t == HSA_DEVICE_TYPE_GPU) {
          *(hsa_agent_t*)d = ag;
          return HSA_STATUS_INFO_BREAK;
        }
        return HSA_STATUS_SUCCESS;
      },
      &gpu);
  hsa_signal_t sig;
  hsa_signal_create(1, 0, nullptr, &sig);
  hsa_status_t st = hsa_amd_svm_prefetch_async(p, kBytes, gpu, 0, nullptr, sig);
  if (st == HSA_STATUS_SUCCESS)
    hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
  else
    printf("prefetch failed %d\n", (int)st);
  hsa_signal_destroy(sig);
}

int main() {
  CK(hipSetDevice(0));
  float* out;
  CK(hipMalloc(&out, 64));
  void* d;
  CK(hipMalloc(&d, kBytes));
  CK(hipMemset(d, 0, kBytes));
  run("hipMalloc", d, out);
  void* m;
  CK(hipMallocManaged(&m, kBytes, hipMemAttachGlobal));
  hipError_t adv = hipMemAdvise(m, kBytes, hipMemAdviseSetCoarseGrain, 0);
  printf("advise coarse rc=%d\n", (int)adv);
  prefetch_gpu(m);
  run("managed_coarse", m, out);
  void* f;
  CK(hipMallocManaged(&f, kBytes, hipMemAttachGlobal));
  prefetch_gpu(f);
  run("managed_plain", f, out);
  void* g;
  CK(hipMallocManaged(&g, kBytes, hipMemAttachGlobal));
  (void)hipMemAdvise(g, kBytes, hipMemAdviseSetCoarseGrain, 0);
  CK(hipMemAdvise(g, kBytes, hipMemAdviseSetPreferredLocation, 0));
  prefetch_gpu(g);
  run("managed_coarse_pref", g, out);
  // A promoted range written by hipMemcpy from pageable host memory, then
  // read back to pageable host memory: does either move its pages to the host?
  {
    void* h = malloc(kBytes);
    memset(h, 1, kBytes);
    void* c;
    CK(hipMallocManaged(&c, kBytes, hipMemAttachGlobal));
    (void)hipMemAdvise(c, kBytes, hipMemAdviseSetCoarseGrain, 0);
    prefetch_gpu(c);
    run("promoted", c, out);
    CK(hipMemcpy(c, h, kBytes, hipMemcpyHostToDevice));
    run("after_h2d", c, out);
    prefetch_gpu(c);
    run("after_h2d_reprefetch", c, out);
    CK(hipMemcpy(h, c, kBytes, hipMemcpyDeviceToHost));
    run("after_d2h", c, out);
    prefetch_gpu(c);
    CK(hipMemcpy(c, h, 4096, hipMemcpyDefault));
    run("after_small_default", c, out);
    prefetch_gpu(c);
    void* ph;
    CK(hipHostMalloc(&ph, kBytes, hipHostMallocDefault));
    CK(hipMemcpyAsync(c, ph, kBytes, hipMemcpyHostToDevice, 0));
    CK(hipDeviceSynchronize());
    run("after_pinned_h2d", c, out);
    // Device-to-device copies from plain HBM into the promoted range: the
    // staging route for host uploads, if they leave the pages in HBM.
    prefetch_gpu(c);
    CK(hipMemcpy(c, d, kBytes, hipMemcpyDeviceToDevice));
    run("after_d2d", c, out);
    CK(hipMemcpyAsync(c, d, kBytes, hipMemcpyDeviceToDevice, 0));
    CK(hipDeviceSynchronize());
    run("after_d2d_async", c, out);
    CK(hipMemcpyAsync(c, d, kBytes, hipMemcpyDefault, 0));
    CK(hipDeviceSynchronize());
    run("after_d2d_default", c, out);
    CK(hipMemcpyAsync(d, c, kBytes, hipMemcpyDeviceToDevice, 0));
    CK(hipDeviceSynchronize());
    run("after_d2d_from", c, out);
  }
  printf("done\n");
  return 0;
}
