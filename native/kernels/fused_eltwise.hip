// Fused NHWC bf16 epilogue kernels for the ai-benchmark CNN workloads on MI355X.
//
// Why: with BatchNorm folded into the convolution weights, a pre-activation
// ResNet bottleneck still needs bias → ReLU after conv1 and conv2 and
// residual-add → BN → ReLU after conv3.  As separate PyTorch / MIOpen ops that
// is 7 full passes over the activation per block (MIOpen's bias kernel alone
// costs ~4x the 1x1 convolution it follows on gfx950, measured in
// vgpu/bench/convbench.py).  These kernels do it in 3 passes:
//
//   bias_act:             x <- act(x + bias[c])                      (in place)
//   scale_shift_act:      y <- act(x * scale[c] + shift[c])
//   add_scale_shift_act:  s <- a + b ; y <- act(s * scale[c] + shift[c])  (dual output)
//
// Memory-bound: 16 B per lane per access (8 bf16), fp32 math, per-channel
// parameters read through the vector L1 (tiny, shared by every row), grid
// capped at 256 CUs x 8 workgroups with a grid-stride loop.  Requires C % 8 == 0
// and 16-B aligned tensors (checked on the host).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VGPU_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kThreads = 256;
constexpr int kMaxGrid = 256 * 8;

struct alignas(16) bf16x8 {
  uint16_t v[8];
};

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  // v_cvt_pk_bf16_f32 on gfx950 (round-to-nearest-even, NaN-preserving)
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

template <int kAct>
__device__ __forceinline__ float act(float x) {
  if constexpr (kAct == 1) return fmaxf(x, 0.0f);
  if constexpr (kAct == 2) return fminf(fmaxf(x, 0.0f), 6.0f);
  return x;
}

__device__ __forceinline__ void load8(const float* __restrict__ p, float (&o)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

// Channel-group index tracked incrementally: one 64-bit modulo per thread,
// then a compare-and-subtract per grid-stride step.
#define VGPU_GRID_LOOP(i, ci, nvec, cvec)                                          \
  const uint64_t stride_ = (uint64_t)gridDim.x * kThreads;                         \
  const uint32_t cstep_ = (uint32_t)(stride_ % (cvec));                            \
  uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;                      \
  uint32_t ci = (uint32_t)(i % (cvec));                                            \
  for (; i < (nvec); i += stride_, ci = (ci + cstep_ >= (cvec)) ? ci + cstep_ - (cvec) : ci + cstep_)

template <int kAct>
__global__ void __launch_bounds__(kThreads) bias_act_kernel(bf16x8* __restrict__ x,
                                                            const float* __restrict__ bias,
                                                            uint64_t nvec, uint32_t cvec) {
  VGPU_GRID_LOOP(i, ci, nvec, cvec) {
    bf16x8 v = x[i];
    float bb[8];
    load8(bias + ci * 8, bb);
#pragma unroll
    for (int k = 0; k < 8; ++k) v.v[k] = f2bf(act<kAct>(bf2f(v.v[k]) + bb[k]));
    x[i] = v;
  }
}

template <int kAct>
__global__ void __launch_bounds__(kThreads) scale_shift_act_kernel(
    const bf16x8* __restrict__ x, bf16x8* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, uint64_t nvec, uint32_t cvec) {
  VGPU_GRID_LOOP(i, ci, nvec, cvec) {
    const bf16x8 v = x[i];
    float sc[8], sh[8];
    load8(scale + ci * 8, sc);
    load8(shift + ci * 8, sh);
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o.v[k] = f2bf(act<kAct>(bf2f(v.v[k]) * sc[k] + sh[k]));
    y[i] = o;
  }
}

template <int kAct>
__global__ void __launch_bounds__(kThreads) add_scale_shift_act_kernel(
    const bf16x8* __restrict__ a, const bf16x8* __restrict__ b, bf16x8* __restrict__ s_out,
    bf16x8* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
    uint64_t nvec, uint32_t cvec) {
  VGPU_GRID_LOOP(i, ci, nvec, cvec) {
    const bf16x8 va = a[i];
    const bf16x8 vb = b[i];
    float sc[8], sh[8];
    load8(scale + ci * 8, sc);
    load8(shift + ci * 8, sh);
    bf16x8 s, o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      // the residual stream is stored in bf16: round the sum once, and derive
      // the activation from the rounded value (what an unfused graph computes)
      const uint16_t sk = f2bf(bf2f(va.v[k]) + bf2f(vb.v[k]));
      s.v[k] = sk;
      o.v[k] = f2bf(act<kAct>(bf2f(sk) * sc[k] + sh[k]));
    }
    s_out[i] = s;
    y[i] = o;
  }
}

inline unsigned grid_for(uint64_t nvec) {
  uint64_t g = (nvec + kThreads - 1) / kThreads;
  if (g < 1) g = 1;
  if (g > kMaxGrid) g = kMaxGrid;
  return (unsigned)g;
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

// act: 0 = identity, 1 = relu, 2 = relu6.  n = total elements, c = channels.
VGPU_API int vgpu_bias_act_nhwc(void* x, const float* bias, uint64_t n, uint32_t c, int act,
                                void* stream) {
  if (c % 8 || n % c || !aligned16(x) || !aligned16(bias)) return (int)hipErrorInvalidValue;
  const uint64_t nvec = n / 8;
  const uint32_t cvec = c / 8;
  auto* xv = (bf16x8*)x;
  switch (act) {
    case 0: hipLaunchKernelGGL(bias_act_kernel<0>, dim3(grid_for(nvec)), dim3(kThreads), 0, (hipStream_t)stream, xv, bias, nvec, cvec); break;
    case 1: hipLaunchKernelGGL(bias_act_kernel<1>, dim3(grid_for(nvec)), dim3(kThreads), 0, (hipStream_t)stream, xv, bias, nvec, cvec); break;
    case 2: hipLaunchKernelGGL(bias_act_kernel<2>, dim3(grid_for(nvec)), dim3(kThreads), 0, (hipStream_t)stream, xv, bias, nvec, cvec); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

VGPU_API int vgpu_scale_shift_act_nhwc(const void* x, void* y, const float* scale, const float* shift,
                                       uint64_t n, uint32_t c, int act, void* stream) {
  if (c % 8 || n % c || !aligned16(x) || !aligned16(y) || !aligned16(scale) || !aligned16(shift)) return (int)hipErrorInvalidValue;
  const uint64_t nvec = n / 8;
  const uint32_t cvec = c / 8;
  auto* xv = (const bf16x8*)x;
  auto* yv = (bf16x8*)y;
  switch (act) {
    case 0: hipLaunchKernelGGL(scale_shift_act_kernel<0>, dim3(grid_for(nvec)), dim3(kThreads), 0, (hipStream_t)stream, xv, yv, scale, shift, nvec, cvec); break;
    case 1: hipLaunchKernelGGL(scale_shift_act_kernel<1>, dim3(grid_for(nvec)), dim3(kThreads), 0, (hipStream_t)stream, xv, yv, scale, shift, nvec, cvec); break;
    case 2: hipLaunchKernelGGL(scale_shift_act_kernel<2>, dim3(grid_for(nvec)), dim3(kThreads), 0, (hipStream_t)stream, xv, yv, scale, shift, nvec, cvec); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

VGPU_API int vgpu_add_scale_shift_act_nhwc(const void* a, const void* b, void* s_out, void* y,
                                           const float* scale, const float* shift, uint64_t n,
                                           uint32_t c, int act, void* stream) {
  if (c % 8 || n % c || !aligned16(a) || !aligned16(b) || !aligned16(s_out) || !aligned16(y) ||
      !aligned16(scale) || !aligned16(shift))
    return (int)hipErrorInvalidValue;
  const uint64_t nvec = n / 8;
  const uint32_t cvec = c / 8;
  auto* av = (const bf16x8*)a;
  auto* bv = (const bf16x8*)b;
  auto* sv = (bf16x8*)s_out;
  auto* yv = (bf16x8*)y;
  switch (act) {
    case 0: hipLaunchKernelGGL(add_scale_shift_act_kernel<0>, dim3(grid_for(nvec)), dim3(kThreads), 0, (hipStream_t)stream, av, bv, sv, yv, scale, shift, nvec, cvec); break;
    case 1: hipLaunchKernelGGL(add_scale_shift_act_kernel<1>, dim3(grid_for(nvec)), dim3(kThreads), 0, (hipStream_t)stream, av, bv, sv, yv, scale, shift, nvec, cvec); break;
    case 2: hipLaunchKernelGGL(add_scale_shift_act_kernel<2>, dim3(grid_for(nvec)), dim3(kThreads), 0, (hipStream_t)stream, av, bv, sv, yv, scale, shift, nvec, cvec); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// ---- ReLU backward + bias gradient (training conv + bias + ReLU, VGG-16) ------------
//   g <- (y > 0) ? dy : 0 ;  db[c] = Σ_rows g[., c]   (fp32, deterministic)
// One pass over dy and y instead of a threshold kernel and a PyTorch column
// reduction that re-reads g (profiles/r5/train).  Block = one slab of
// kIters · (256 / cv) rows: thread t owns channel group t % cv and every
// (256 / cv)-th row from t / cv, kIters of them with all loads issued first;
// lanes of one group are merged through LDS into part[slab][C]; the reduce
// kernel sums the slabs in a fixed order, 16 threads per channel.
namespace {
constexpr int kIters = 8;

// Pooled variant (POOL): dy is the gradient of a k×k / stride-k max pool of y
// ([N][H/k][W/k][C]) with its one-byte-per-element argmax (pool_train.hip);
// the row's gradient is gathered from its window (the pool backward fused in).
struct PoolGeo {
  const bf16x8* dyp;
  const uint2* idx;
  int H, W, OH, OW, k;
  int nchw;  // dyp is [N][C][OH][OW] (the gradient of an NCHW-written pool output)
};

template <bool POOL>
__global__ void __launch_bounds__(kThreads) relu_bias_grad_kernel(const bf16x8* __restrict__ dy,
                                                                  const bf16x8* __restrict__ y,
                                                                  bf16x8* __restrict__ g, float* __restrict__ part,
                                                                  uint64_t rows, uint32_t cv, const PoolGeo pg) {
  __shared__ float red[kThreads][9];  // 8 sums + pad (bank spread)
  const uint32_t t = threadIdx.x;
  const uint32_t per = kThreads / cv;  // rows in flight per block pass
  const uint32_t cg = t % cv, r0 = t / cv;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (r0 < per) {
    const uint64_t row0 = (uint64_t)blockIdx.x * per * kIters + r0;
    bf16x8 a[kIters], b[kIters];
    uint32_t tap[kIters];
#pragma unroll
    for (int k = 0; k < kIters; ++k) {
      const uint64_t r = row0 + (uint64_t)k * per;
      if (r < rows) {
        if constexpr (POOL) {
          // 32-bit index math (rows < 2^31, checked on the host): the 64-bit
          // div / mod pair per row made this pass ~1.8x the unpooled one
          const uint32_t r32 = (uint32_t)r, W = (uint32_t)pg.W, H = (uint32_t)pg.H;
          const uint32_t t2 = r32 / W, iw = r32 - t2 * W, n = t2 / H, ih = t2 - n * H;
          const uint32_t oh = ih / pg.k, ow = iw / pg.k;
          tap[k] = 0xffu;  // rows past the last full window receive no gradient
          if (oh < (uint32_t)pg.OH && ow < (uint32_t)pg.OW) {
            const uint64_t o = (uint64_t)((n * (uint32_t)pg.OH + oh) * (uint32_t)pg.OW + ow) * cv + cg;
            if (pg.nchw) {
              const uint16_t* d = reinterpret_cast<const uint16_t*>(pg.dyp);
              const uint64_t hw = (uint64_t)pg.OH * pg.OW;
              const uint64_t base = ((uint64_t)n * cv * 8 + cg * 8) * hw + (uint64_t)oh * pg.OW + ow;
#pragma unroll
              for (int j = 0; j < 8; ++j) a[k].v[j] = d[base + j * hw];
            } else {
              a[k] = pg.dyp[o];
            }
            const uint2 t = pg.idx[o];
            tap[k] = (ih - oh * pg.k) * pg.k + (iw - ow * pg.k);
            // per channel j: keep dy where the window's argmax is this row
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if ((((j < 4 ? t.x : t.y) >> (8 * (j & 3))) & 0xffu) != tap[k]) a[k].v[j] = 0;
          }
        } else {
          a[k] = dy[r * cv + cg];
        }
        b[k] = y[r * cv + cg];
      }
    }
#pragma unroll
    for (int k = 0; k < kIters; ++k) {
      const uint64_t r = row0 + (uint64_t)k * per;
      if (r >= rows) continue;
      if constexpr (POOL) {
        if (tap[k] == 0xffu) {
#pragma unroll
          for (int j = 0; j < 8; ++j) a[k].v[j] = 0;
        }
      }
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool on = bf2f(b[k].v[j]) > 0.0f;
        o.v[j] = on ? a[k].v[j] : (uint16_t)0;
        s[j] += on ? bf2f(a[k].v[j]) : 0.0f;
      }
      g[r * cv + cg] = o;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[t][j] = s[j];
  __syncthreads();
  if (t < cv) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (uint32_t k = 0; k < per; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += red[k * cv + t][j];
    float* out = part + (uint64_t)blockIdx.x * cv * 8 + t * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = acc[j];
  }
}

// 16 channels per block, 16 threads per channel (slab residues mod 16), merged in order.
template <typename T>
__global__ void __launch_bounds__(kThreads) relu_bias_grad_reduce_kernel(const float* __restrict__ part,
                                                                         T* __restrict__ db, uint32_t c,
                                                                         uint32_t slabs) {
  __shared__ float red[16][17];
  const uint32_t cl = threadIdx.x % 16, q = threadIdx.x / 16, ch = blockIdx.x * 16 + cl;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (ch < c) {
    uint32_t k = q;
    for (; k + 48 < slabs; k += 64) {
      a0 += part[(uint64_t)k * c + ch];
      a1 += part[(uint64_t)(k + 16) * c + ch];
      a2 += part[(uint64_t)(k + 32) * c + ch];
      a3 += part[(uint64_t)(k + 48) * c + ch];
    }
    for (; k < slabs; k += 16) a0 += part[(uint64_t)k * c + ch];
  }
  red[q][cl] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (q == 0 && ch < c) {
    float a = 0.f;
    for (int i = 0; i < 16; ++i) a += red[i][cl];
    if constexpr (sizeof(T) == 2) db[ch] = f2bf(a);  // a bf16 bias's gradient, no cast pass
    else db[ch] = a;
  }
}

uint32_t rbg_slabs(uint64_t rows, uint32_t cv) {
  const uint64_t slab_rows = (uint64_t)(kThreads / cv) * kIters;
  return (uint32_t)((rows + slab_rows - 1) / slab_rows);
}
}  // namespace

VGPU_API int64_t vgpu_relu_bias_grad_workspace(uint64_t rows, uint32_t c) {
  if (c % 8 || c / 8 > kThreads || c == 0) return -1;
  return (int64_t)rbg_slabs(rows, c / 8) * c * 4;
}

// dy, y, g: [rows, c] bf16 (NHWC); db: [c] fp32, or bf16 when db_bf16; ws:
// vgpu_relu_bias_grad_workspace bytes.
VGPU_API int vgpu_relu_bias_grad_nhwc(const void* dy, const void* y, void* g, void* db, void* ws, uint64_t rows,
                                      uint32_t c, int db_bf16, hipStream_t stream) {
  if (c % 8 || c / 8 > kThreads || rows == 0) return -1;
  const uint32_t cv = c / 8;
  const uint32_t slabs = rbg_slabs(rows, cv);
  hipLaunchKernelGGL(relu_bias_grad_kernel<false>, dim3(slabs), dim3(kThreads), 0, stream, (const bf16x8*)dy,
                     (const bf16x8*)y, (bf16x8*)g, (float*)ws, rows, cv, PoolGeo{});
  if (db_bf16)
    hipLaunchKernelGGL(relu_bias_grad_reduce_kernel<uint16_t>, dim3((c + 15) / 16), dim3(kThreads), 0, stream,
                       (const float*)ws, (uint16_t*)db, c, slabs);
  else
    hipLaunchKernelGGL(relu_bias_grad_reduce_kernel<float>, dim3((c + 15) / 16), dim3(kThreads), 0, stream,
                       (const float*)ws, (float*)db, c, slabs);
  return (int)hipGetLastError();
}

// The same with the gradient arriving through a k×k / stride-k max pool of y
// (no padding): dyp [N][H/k][W/k][c] and its argmax bytes idx (the layout of
// vgpu_maxpool_fwd_idx_nhwc); y, g: [N][H][W][c].  One pass instead of the
// pool backward plus this one (VGG-16's five conv + ReLU + pool blocks).
VGPU_API int vgpu_pool_relu_bias_grad_nhwc(const void* dyp, const void* idx, const void* y, void* g, void* db,
                                           void* ws, int N, int H, int W, uint32_t c, int k, int db_bf16,
                                           hipStream_t stream) {
  if (c % 8 || c / 8 > kThreads || N < 1 || H < 1 || W < 1 || k < 1 || k > 15 || H < k || W < k) return -1;
  if ((uint64_t)N * H * W >= (1ull << 31)) return -1;
  const uint32_t cv = c / 8;
  const uint64_t rows = (uint64_t)N * H * W;
  const uint32_t slabs = rbg_slabs(rows, cv);
  const PoolGeo pg{(const bf16x8*)dyp, (const uint2*)idx, H, W, H / k, W / k, k};
  hipLaunchKernelGGL(relu_bias_grad_kernel<true>, dim3(slabs), dim3(kThreads), 0, stream, nullptr,
                     (const bf16x8*)y, (bf16x8*)g, (float*)ws, rows, cv, pg);
  if (db_bf16)
    hipLaunchKernelGGL(relu_bias_grad_reduce_kernel<uint16_t>, dim3((c + 15) / 16), dim3(kThreads), 0, stream,
                       (const float*)ws, (uint16_t*)db, c, slabs);
  else
    hipLaunchKernelGGL(relu_bias_grad_reduce_kernel<float>, dim3((c + 15) / 16), dim3(kThreads), 0, stream,
                       (const float*)ws, (float*)db, c, slabs);
  return (int)hipGetLastError();
}

VGPU_API int vgpu_relu_bias_grad_partial2(const void* dy, const void* idx, const void* y, void* g, void* ws, int N,
                                          int H, int W, uint32_t c, int k, int dy_nchw, int* slabs_out,
                                          hipStream_t stream);

// Partials only (no reduce launch): ws receives [slabs][c] fp32 and *slabs_out
// their count; the bias gradient is summed by vgpu_conv_wgrad_db_nhwc's reduce
// launch (or vgpu_bias_grad_reduce).  pooled: dy is [N][H/k][W/k][c] with its
// argmax idx, as in vgpu_pool_relu_bias_grad_nhwc (k = 0: not pooled).
VGPU_API int vgpu_relu_bias_grad_partial_nhwc(const void* dy, const void* idx, const void* y, void* g, void* ws,
                                              int N, int H, int W, uint32_t c, int k, int* slabs_out,
                                              hipStream_t stream) {
  return vgpu_relu_bias_grad_partial2(dy, idx, y, g, ws, N, H, W, c, k, 0, slabs_out, stream);
}

// k > 0 and dy_nchw: the pooled gradient is NCHW-contiguous (a flatten's).
VGPU_API int vgpu_relu_bias_grad_partial2(const void* dy, const void* idx, const void* y, void* g, void* ws, int N,
                                          int H, int W, uint32_t c, int k, int dy_nchw, int* slabs_out,
                                          hipStream_t stream) {
  if (c % 8 || c / 8 > kThreads || N < 1 || H < 1 || W < 1 || k < 0 || k > 15 || (k && (H < k || W < k)))
    return -1;
  if ((uint64_t)N * H * W >= (1ull << 31)) return -1;
  const uint32_t cv = c / 8;
  const uint64_t rows = (uint64_t)N * H * W;
  const uint32_t slabs = rbg_slabs(rows, cv);
  if (k) {
    const PoolGeo pg{(const bf16x8*)dy, (const uint2*)idx, H, W, H / k, W / k, k, dy_nchw};
    hipLaunchKernelGGL(relu_bias_grad_kernel<true>, dim3(slabs), dim3(kThreads), 0, stream, nullptr,
                       (const bf16x8*)y, (bf16x8*)g, (float*)ws, rows, cv, pg);
  } else {
    hipLaunchKernelGGL(relu_bias_grad_kernel<false>, dim3(slabs), dim3(kThreads), 0, stream, (const bf16x8*)dy,
                       (const bf16x8*)y, (bf16x8*)g, (float*)ws, rows, cv, PoolGeo{});
  }
  if (slabs_out) *slabs_out = (int)slabs;
  return (int)hipGetLastError();
}

// ---- zero-pad the channel dimension of a [rows][c] bf16 tensor to cp ---------------
// One pass (F.pad is a fill plus a copy): VGG-16's 3-channel first layer runs
// the MFMA conv on 64 channels, its input and weight padded every step.
namespace {
__global__ void __launch_bounds__(kThreads) pad_channels_kernel(const uint16_t* __restrict__ x,
                                                                bf16x8* __restrict__ y, uint64_t rows, uint32_t c,
                                                                uint32_t cpv) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= rows * cpv) return;
  const uint64_t r = i / cpv;
  const uint32_t c0 = (uint32_t)(i - r * cpv) * 8;
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o.v[j] = c0 + j < c ? x[r * c + c0 + j] : (uint16_t)0;
  y[i] = o;
}
}  // namespace

VGPU_API int vgpu_pad_channels(const void* x, void* y, uint64_t rows, uint32_t c, uint32_t cp, hipStream_t stream) {
  if (cp % 8 || cp < c || rows == 0 || !aligned16(y)) return -1;
  const uint64_t n = rows * (cp / 8);
  hipLaunchKernelGGL(pad_channels_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0, stream,
                     (const uint16_t*)x, (bf16x8*)y, rows, c, cp / 8);
  return (int)hipGetLastError();
}
