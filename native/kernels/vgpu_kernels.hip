// Hand-written gfx950 (MI355X / CDNA4) kernels used by the vGPU stack itself.
// The reference ships no kernel source at all; these are the
// device-side tools the MI355X design needs:
//
//  K1 vgpu_census / vgpu_busy  — placement census + calibrated busy-spin.
//     Each workgroup records the XCD (HW_REG_XCC_ID) and SE/SH/CU (HW_REG_HW_ID)
//     it ran on, then spins for a fixed number of shader-clock ticks
//     (s_memtime).  Used to (a) verify which physical CUs a CU mask maps to and
//     (b) measure compute-share accuracy: with 1 wave per workgroup the kernel
//     time is ⌈workgroups / (usable CUs × waves/CU)⌉ × spin, so the ratio of two
//     runs gives the effective CU share directly.
//  K2 vgpu_gather_pages / vgpu_scatter_pages — page-granular copy engine for
//     virtual device memory (HBM ↔ pinned host).  One workgroup per 64 KiB slab,
//     16 B per lane per access (global_load_dwordx4 / global_store_dwordx4),
//     nontemporal stores so a migration does not evict the tenant's L2 / MALL.
//  K3 vgpu_fill_pattern / vgpu_verify_pattern — position-hashed fill and check,
//     used to prove every byte of a capped allocation is real and to validate
//     page migration end to end.
//
// Launch geometry: 256-thread workgroups (4 waves), grid-stride loops capped at
// 256 CUs × 8 workgroups so launches fill all 8 XCDs (≫256 workgroups) without
// oversubscribing the dispatcher.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VGPU_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kThreads = 256;
constexpr int kMaxGrid = 256 * 8;

__device__ __forceinline__ uint32_t read_xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v;
}

__device__ __forceinline__ uint32_t read_hw_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
  return v;
}

__device__ __forceinline__ uint64_t memtime() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// K1 --------------------------------------------------------------------------------
// out[2*b+0] = xcc id, out[2*b+1] = raw HW_ID of workgroup b's first wave.
__global__ void __launch_bounds__(64) census_kernel(uint32_t* __restrict__ out, uint64_t spin_ticks,
                                                     uint64_t* __restrict__ ticks_out) {
  const uint64_t t0 = memtime();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x + 0] = read_xcc_id();
    out[2 * blockIdx.x + 1] = read_hw_id();
  }
  // Bounded spin: every wave exits after spin_ticks shader clocks.
  uint64_t t = t0;
  while (t - t0 < spin_ticks) {
    __builtin_amdgcn_s_sleep(1);
    t = memtime();
  }
  if (threadIdx.x == 0 && ticks_out) ticks_out[blockIdx.x] = t - t0;
}

// Busy kernel without census bookkeeping: `iters` dependent FMAs per lane keep
// the VALU busy (not sleeping), so concurrent tenants actually contend.
__global__ void __launch_bounds__(kThreads) busy_kernel(float* __restrict__ sink, uint32_t iters) {
  float a = 1.0f + threadIdx.x * 1e-7f, b = 0.999999f, c = 1e-7f;
  for (uint32_t i = 0; i < iters; ++i) {
    a = __builtin_fmaf(a, b, c);
    b = __builtin_fmaf(b, a, c);
  }
  if (a == 1234.5f && b == 0.0f) sink[threadIdx.x] = a;  // keep the loop alive
}

// K2 --------------------------------------------------------------------------------
// Copies npages pages of page_bytes (multiple of 16) between a scattered and a
// packed layout.  gather: dst[k] <- src[idx[k]];  scatter: dst[idx[k]] <- src[k].
template <bool kGather>
__global__ void __launch_bounds__(kThreads) page_copy_kernel(uint4* __restrict__ dst,
                                                             const uint4* __restrict__ src,
                                                             const int64_t* __restrict__ idx,
                                                             uint64_t page_vecs, uint64_t npages) {
  const uint64_t total = page_vecs * npages;
  const uint64_t stride = (uint64_t)gridDim.x * kThreads;
  for (uint64_t v = (uint64_t)blockIdx.x * kThreads + threadIdx.x; v < total; v += stride) {
    const uint64_t page = v / page_vecs;
    const uint64_t off = v - page * page_vecs;
    const uint64_t sp = kGather ? (uint64_t)idx[page] : page;
    const uint64_t dp = kGather ? page : (uint64_t)idx[page];
    const uint4 x = src[sp * page_vecs + off];
    __builtin_nontemporal_store(x.x, &dst[dp * page_vecs + off].x);
    __builtin_nontemporal_store(x.y, &dst[dp * page_vecs + off].y);
    __builtin_nontemporal_store(x.z, &dst[dp * page_vecs + off].z);
    __builtin_nontemporal_store(x.w, &dst[dp * page_vecs + off].w);
  }
}

// K3 --------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix(uint64_t x, uint32_t seed) {
  x ^= (uint64_t)seed * 0x9E3779B97F4A7C15ull;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (uint32_t)x;
}

__global__ void __launch_bounds__(kThreads) fill_kernel(uint4* __restrict__ p, uint64_t nvec,
                                                        uint32_t seed) {
  const uint64_t stride = (uint64_t)gridDim.x * kThreads;
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += stride) {
    uint4 v;
    v.x = mix(4 * i + 0, seed);
    v.y = mix(4 * i + 1, seed);
    v.z = mix(4 * i + 2, seed);
    v.w = mix(4 * i + 3, seed);
    p[i] = v;
  }
}

__global__ void __launch_bounds__(kThreads) verify_kernel(const uint4* __restrict__ p, uint64_t nvec,
                                                          uint32_t seed,
                                                          unsigned long long* __restrict__ errors) {
  const uint64_t stride = (uint64_t)gridDim.x * kThreads;
  uint32_t bad = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += stride) {
    const uint4 v = p[i];
    bad += (v.x != mix(4 * i + 0, seed)) + (v.y != mix(4 * i + 1, seed)) +
           (v.z != mix(4 * i + 2, seed)) + (v.w != mix(4 * i + 3, seed));
  }
  // wave reduction (64 lanes) then one atomic per wave
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(errors, (unsigned long long)bad);
}

inline unsigned grid_for(uint64_t work_items) {
  uint64_t g = (work_items + kThreads - 1) / kThreads;
  if (g < 1) g = 1;
  if (g > kMaxGrid) g = kMaxGrid;
  return (unsigned)g;
}

}  // namespace

// ---- C ABI (ctypes) ------------------------------------------------------------------
// All entry points are asynchronous on `stream` and return a hipError_t.

VGPU_API int vgpu_census(uint32_t* out, uint32_t blocks, uint64_t spin_ticks, uint64_t* ticks_out,
                         void* stream) {
  if (!out || blocks == 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(census_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream, out, spin_ticks,
                     ticks_out);
  return (int)hipGetLastError();
}

VGPU_API int vgpu_busy(float* sink, uint32_t blocks, uint32_t iters, void* stream) {
  if (!sink || blocks == 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(busy_kernel, dim3(blocks), dim3(kThreads), 0, (hipStream_t)stream, sink, iters);
  return (int)hipGetLastError();
}

// The same busy kernel launched through another runtime entry point (GPU
// tests of the enforcement library's hooks): 1 = hipLaunchKernel_spt (what
// -fgpu-default-stream=per-thread code calls), 2 = a one-entry
// hipExtLaunchMultiKernelMultiDevice.
VGPU_API int vgpu_busy_via(float* sink, uint32_t blocks, uint32_t iters, void* stream, int path) {
  if (!sink || blocks == 0) return (int)hipErrorInvalidValue;
  void* args[] = {&sink, &iters};
  if (path == 1)
    return (int)hipLaunchKernel_spt((const void*)busy_kernel, dim3(blocks), dim3(kThreads), args, 0,
                                    (hipStream_t)stream);
  if (path == 2) {
    // the multi-device launch wants a real stream per entry (not the null stream)
    static hipStream_t own = nullptr;
    if (!stream && !own && hipStreamCreateWithFlags(&own, hipStreamNonBlocking) != hipSuccess) return -1;
    if (!stream) stream = own;
    hipLaunchParams p{};
    p.func = (void*)busy_kernel;
    p.gridDim = dim3(blocks);
    p.blockDim = dim3(kThreads);
    p.args = args;
    p.sharedMem = 0;
    p.stream = (hipStream_t)stream;
    return (int)hipExtLaunchMultiKernelMultiDevice(&p, 1, 0);
  }
  return (int)hipLaunchKernel((const void*)busy_kernel, dim3(blocks), dim3(kThreads), args, 0, (hipStream_t)stream);
}

VGPU_API int vgpu_gather_pages(void* dst, const void* src, const int64_t* idx, uint64_t page_bytes,
                               uint64_t npages, void* stream) {
  if (page_bytes % 16 || !dst || !src || !idx) return (int)hipErrorInvalidValue;
  const uint64_t pv = page_bytes / 16;
  hipLaunchKernelGGL(page_copy_kernel<true>, dim3(grid_for(pv * npages)), dim3(kThreads), 0,
                     (hipStream_t)stream, (uint4*)dst, (const uint4*)src, idx, pv, npages);
  return (int)hipGetLastError();
}

VGPU_API int vgpu_scatter_pages(void* dst, const void* src, const int64_t* idx, uint64_t page_bytes,
                                uint64_t npages, void* stream) {
  if (page_bytes % 16 || !dst || !src || !idx) return (int)hipErrorInvalidValue;
  const uint64_t pv = page_bytes / 16;
  hipLaunchKernelGGL(page_copy_kernel<false>, dim3(grid_for(pv * npages)), dim3(kThreads), 0,
                     (hipStream_t)stream, (uint4*)dst, (const uint4*)src, idx, pv, npages);
  return (int)hipGetLastError();
}

VGPU_API int vgpu_fill_pattern(void* p, uint64_t bytes, uint32_t seed, void* stream) {
  if (bytes % 16 || !p) return (int)hipErrorInvalidValue;
  const uint64_t n = bytes / 16;
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream,
                     (uint4*)p, n, seed);
  return (int)hipGetLastError();
}

VGPU_API int vgpu_verify_pattern(const void* p, uint64_t bytes, uint32_t seed,
                                 unsigned long long* errors, void* stream) {
  if (bytes % 16 || !p || !errors) return (int)hipErrorInvalidValue;
  const uint64_t n = bytes / 16;
  hipLaunchKernelGGL(verify_kernel, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream,
                     (const uint4*)p, n, seed, errors);
  return (int)hipGetLastError();
}

VGPU_API int vgpu_kernels_abi_version() { return 1; }
