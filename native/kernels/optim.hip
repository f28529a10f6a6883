// SGD with momentum for bf16 parameters in one launch per ≤ 48 tensors
// (vgpu.ops.optim.SGD; the training workloads of the ai-benchmark suite).
//
// PyTorch's fused SGD walks its tensor lists with multi_tensor_apply: VGG-16's
// 138M parameters took 7 launches of ~50 us, ≈ 3.9 TB/s over the 10 B per
// parameter the update must move (read p, g, m; write p, m) — 15 % of the
// batch-2 training step (profiles/r5/train/vgg_b2_kernels.md).  Here the
// segment table (pointers, sizes, first block of each tensor) travels in the
// kernel arguments, so a captured hipGraph replays it with no host copy; each
// block owns 8192 elements of one tensor, 16-B vector loads of all three
// operands issued before any math.
//
//   g' = g + wd·p ;  m = first ? g' : mom·m + (1 − damp)·g' ;
//   d = nesterov ? g' + mom·m : m ;  p = p − lr·d         (fp32 math, bf16 storage)
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VGPU_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kThreads = 256;
constexpr int kVec = 8;                      // bf16 per 16-B access
constexpr int kIters = 4;                    // accesses per thread per block
constexpr int kChunk = kThreads * kVec * kIters;  // 8192 elements per block
constexpr int kMaxSeg = 48;

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

struct SgdSegs {
  uint16_t* p[kMaxSeg];
  const uint16_t* g[kMaxSeg];
  uint16_t* m[kMaxSeg];
  int64_t n[kMaxSeg];
  int first_blk[kMaxSeg + 1];
  int nseg;
};

__device__ __forceinline__ float lo(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float hi(uint32_t v) { return __uint_as_float(v & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) float f2;
  typedef __attribute__((ext_vector_type(2))) __bf16 b2;
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{a, b}, b2));
}

template <bool FIRST, bool NESTEROV>
__device__ __forceinline__ void step2(uint32_t pv, uint32_t gv, uint32_t mv, float lr, float mom, float damp1,
                                      float wd, uint32_t& po, uint32_t& mo) {
  float p[2] = {lo(pv), hi(pv)}, g[2] = {lo(gv), hi(gv)}, m[2] = {lo(mv), hi(mv)};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float gg = fmaf(wd, p[k], g[k]);
    m[k] = FIRST ? gg : fmaf(mom, m[k], damp1 * gg);
    const float d = NESTEROV ? fmaf(mom, m[k], gg) : m[k];
    p[k] = fmaf(-lr, d, p[k]);
  }
  po = pack2(p[0], p[1]);
  mo = pack2(m[0], m[1]);
}

template <bool FIRST, bool NESTEROV>
__global__ void __launch_bounds__(kThreads) sgd_bf16_kernel(const SgdSegs s, float lr, float mom, float damp1,
                                                            float wd) {
  const int b = blockIdx.x;
  int seg = 0;
  while (seg + 1 < s.nseg && s.first_blk[seg + 1] <= b) ++seg;  // ≤ 48 uniform compares
  const int64_t n = s.n[seg];
  const int64_t base = (int64_t)(b - s.first_blk[seg]) * kChunk;
  u32x4* P = reinterpret_cast<u32x4*>(s.p[seg] + base);
  const u32x4* G = reinterpret_cast<const u32x4*>(s.g[seg] + base);
  u32x4* M = reinterpret_cast<u32x4*>(s.m[seg] + base);
  const int64_t nv = (n - base) / kVec;  // whole vectors left in this tensor from base (n % 8 == 0)
  u32x4 pv[kIters], gv[kIters], mv[kIters];
#pragma unroll
  for (int u = 0; u < kIters; ++u) {
    const int i = u * kThreads + threadIdx.x;
    if (i < nv) {
      // every byte is touched once: nontemporal, so the stream does not evict
      // what the next step's first kernels would find in L2 / MALL
      pv[u] = __builtin_nontemporal_load(&P[i]);
      gv[u] = __builtin_nontemporal_load(&G[i]);
      if (!FIRST) mv[u] = __builtin_nontemporal_load(&M[i]);
    }
  }
#pragma unroll
  for (int u = 0; u < kIters; ++u) {
    const int i = u * kThreads + threadIdx.x;
    if (i >= nv) continue;
    uint32_t po[4], mo[4];
    const uint32_t pw[4] = {pv[u].x, pv[u].y, pv[u].z, pv[u].w}, gw[4] = {gv[u].x, gv[u].y, gv[u].z, gv[u].w};
    uint32_t mw[4] = {0u, 0u, 0u, 0u};
    if (!FIRST) { mw[0] = mv[u].x; mw[1] = mv[u].y; mw[2] = mv[u].z; mw[3] = mv[u].w; }
#pragma unroll
    for (int k = 0; k < 4; ++k) step2<FIRST, NESTEROV>(pw[k], gw[k], mw[k], lr, mom, damp1, wd, po[k], mo[k]);
    __builtin_nontemporal_store(u32x4{po[0], po[1], po[2], po[3]}, &P[i]);
    __builtin_nontemporal_store(u32x4{mo[0], mo[1], mo[2], mo[3]}, &M[i]);
  }
}

}  // namespace

VGPU_API int vgpu_sgd_max_segments() { return kMaxSeg; }

// One SGD step over nseg ≤ 48 bf16 tensors: p[i], g[i], m[i] of n[i] elements
// each (n % 8 == 0, 16-B aligned; checked here).  first: the momentum buffers
// are initialised from the gradient (PyTorch's first step).  Returns 0, -1 for
// unsupported arguments, or a hipError_t.
VGPU_API int vgpu_sgd_bf16(void* const* p, const void* const* g, void* const* m, const int64_t* n, int nseg,
                           float lr, float momentum, float dampening, float weight_decay, int nesterov, int first,
                           hipStream_t stream) {
  if (nseg < 1 || nseg > kMaxSeg) return -1;
  SgdSegs s{};
  s.nseg = nseg;
  int64_t blocks = 0;
  for (int i = 0; i < nseg; ++i) {
    if (n[i] < 1 || n[i] % kVec || ((uintptr_t)p[i] | (uintptr_t)g[i] | (uintptr_t)m[i]) & 15) return -1;
    s.p[i] = static_cast<uint16_t*>(p[i]);
    s.g[i] = static_cast<const uint16_t*>(g[i]);
    s.m[i] = static_cast<uint16_t*>(m[i]);
    s.n[i] = n[i];
    s.first_blk[i] = (int)blocks;
    blocks += (n[i] + kChunk - 1) / kChunk;
    if (blocks >= ((int64_t)1 << 31)) return -1;
  }
  s.first_blk[nseg] = (int)blocks;
  const float damp1 = first ? 1.0f : 1.0f - dampening;
  const dim3 grid((unsigned)blocks), block(kThreads);
  if (first && nesterov)
    hipLaunchKernelGGL((sgd_bf16_kernel<true, true>), grid, block, 0, stream, s, lr, momentum, damp1, weight_decay);
  else if (first)
    hipLaunchKernelGGL((sgd_bf16_kernel<true, false>), grid, block, 0, stream, s, lr, momentum, damp1, weight_decay);
  else if (nesterov)
    hipLaunchKernelGGL((sgd_bf16_kernel<false, true>), grid, block, 0, stream, s, lr, momentum, damp1, weight_decay);
  else
    hipLaunchKernelGGL((sgd_bf16_kernel<false, false>), grid, block, 0, stream, s, lr, momentum, damp1, weight_decay);
  return (int)hipGetLastError();
}
