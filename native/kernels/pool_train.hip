// Training max pool for NHWC bf16 activations (the ResNet stem's 3x3/s2/p1):
// forward writes y and, per output element, the window tap that won (one
// byte); backward gathers — each input pixel sums dy over the (at most
// ceil(k/s)² ) windows whose saved tap is that pixel — so no atomics and no
// zero-fill pass.  PyTorch's max_pool2d backward over the same 76 MB stem
// activation cost 82 µs + its forward 82 µs per ResNet-V2-50 b=20 step
// (profiles/r4/train/bnfuse/rocprof_train_1.2_fused_r4.md).
//
// Semantics follow at::max_pool2d: the first maximum in (kh, kw) scan order
// wins, a NaN wins over numbers (the last NaN of a window), padding never wins.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define VGPU_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kThreads = 256;

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;

__device__ __forceinline__ void unpack8(const u32x4 v, float (&f)[8]) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  typedef __attribute__((ext_vector_type(2))) float f2;
  typedef __attribute__((ext_vector_type(2))) __bf16 b2;
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{lo, hi}, b2));
}

// One thread per (output pixel, 8 channels); grid-stride over N·OH·OW·C/8.
// nchw: y is written [N][C][OH][OW] (the layout a following flatten reads
// without a copy; idx stays NHWC).
__global__ void __launch_bounds__(kThreads) maxpool_fwd_idx_kernel(const u32x4* __restrict__ x,
                                                                   u32x4* __restrict__ y,
                                                                   u32x2* __restrict__ idx, int H, int W,
                                                                   int cv, int OH, int OW, int k, int stride,
                                                                   int pad, int64_t total, int nchw) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kThreads) {
    const int c = (int)(i % cv);
    int64_t r = i / cv;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int n = (int)(r / OH);
    const int h0 = oh * stride - pad, w0 = ow * stride - pad;
    const u32x4* xn = x + (int64_t)n * H * W * cv + c;
    float m[8];
    uint32_t t8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m[j] = -INFINITY;
      t8[j] = 0xff;
    }
    for (int dh = 0; dh < k; ++dh) {
      const int ih = h0 + dh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int dw = 0; dw < k; ++dw) {
        const int iw = w0 + dw;
        if ((unsigned)iw >= (unsigned)W) continue;
        float e[8];
        unpack8(xn[((int64_t)ih * W + iw) * cv], e);
        const uint32_t tap = (uint32_t)(dh * k + dw);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (e[j] > m[j] || isnan(e[j]) || t8[j] == 0xff) {
            m[j] = e[j];
            t8[j] = tap;
          }
      }
    }
    if (nchw) {
      uint16_t* yh = reinterpret_cast<uint16_t*>(y);
      const int64_t hw = (int64_t)OH * OW, base = ((int64_t)n * cv * 8 + c * 8) * hw + (int64_t)oh * OW + ow;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        __bf16 b = (__bf16)m[j];
        yh[base + j * hw] = __builtin_bit_cast(uint16_t, b);
      }
    } else {
      y[i] = u32x4{pack2(m[0], m[1]), pack2(m[2], m[3]), pack2(m[4], m[5]), pack2(m[6], m[7])};
    }
    idx[i] = u32x2{t8[0] | t8[1] << 8 | t8[2] << 16 | t8[3] << 24, t8[4] | t8[5] << 8 | t8[6] << 16 | t8[7] << 24};
  }
}

// One thread per (input pixel, 8 channels): dx = Σ dy over the windows that
// chose this pixel, in fp32, rounded once.
__global__ void __launch_bounds__(kThreads) maxpool_bwd_kernel(const u32x4* __restrict__ dy,
                                                               const u32x2* __restrict__ idx,
                                                               u32x4* __restrict__ dx, int H, int W, int cv,
                                                               int OH, int OW, int k, int stride, int pad,
                                                               int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kThreads) {
    const int c = (int)(i % cv);
    int64_t r = i / cv;
    const int iw = (int)(r % W);
    r /= W;
    const int ih = (int)(r % H);
    const int n = (int)(r / H);
    // windows oh with oh·s - pad <= ih <= oh·s - pad + k - 1
    const int ohi = (ih + pad) / stride, owi = (iw + pad) / stride;
    int olo = ih + pad - k + 1, wlo = iw + pad - k + 1;
    olo = olo <= 0 ? 0 : (olo + stride - 1) / stride;
    wlo = wlo <= 0 ? 0 : (wlo + stride - 1) / stride;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.0f;
    for (int oh = olo; oh <= ohi && oh < OH; ++oh)
      for (int ow = wlo; ow <= owi && ow < OW; ++ow) {
        const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * cv + c;
        const u32x2 t = idx[o];
        const uint32_t tap = (uint32_t)((ih - (oh * stride - pad)) * k + (iw - (ow * stride - pad)));
        float g[8];
        unpack8(dy[o], g);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t tj = ((j < 4 ? t.x : t.y) >> (8 * (j & 3))) & 0xffu;
          if (tj == tap) acc[j] += g[j];
        }
      }
    dx[i] = u32x4{pack2(acc[0], acc[1]), pack2(acc[2], acc[3]), pack2(acc[4], acc[5]), pack2(acc[6], acc[7])};
  }
}

inline unsigned grid_for(int64_t total) {
  int64_t g = (total + kThreads - 1) / kThreads;
  if (g > 256 * 16) g = 256 * 16;
  return (unsigned)(g < 1 ? 1 : g);
}

inline bool shape_ok(int N, int H, int W, int C, int k, int stride, int pad, int& OH, int& OW) {
  if (N < 1 || H < 1 || W < 1 || C % 8 || k < 1 || k > 15 || stride < 1 || pad < 0 || 2 * pad > k) return false;
  OH = (H + 2 * pad - k) / stride + 1;
  OW = (W + 2 * pad - k) / stride + 1;
  return OH >= 1 && OW >= 1;
}

}  // namespace

// y [N][OH][OW][C] bf16 and idx [N][OH][OW][C] uint8 (the winning tap dh·k + dw)
// of a k×k max pool over x [N][H][W][C] bf16 (C % 8 == 0, pad ≤ k/2).
VGPU_API int vgpu_maxpool_fwd_idx_nhwc(const void* x, void* y, void* idx, int N, int H, int W, int C, int k,
                                       int stride, int pad, hipStream_t s) {
  int OH, OW;
  if (!shape_ok(N, H, W, C, k, stride, pad, OH, OW)) return -1;
  const int cv = C / 8;
  const int64_t total = (int64_t)N * OH * OW * cv;
  hipLaunchKernelGGL(maxpool_fwd_idx_kernel, dim3(grid_for(total)), dim3(kThreads), 0, s,
                     static_cast<const u32x4*>(x), static_cast<u32x4*>(y), static_cast<u32x2*>(idx), H, W, cv, OH,
                     OW, k, stride, pad, total, 0);
  return (int)hipGetLastError();
}

// The same with y written NCHW-contiguous (x and idx stay NHWC).
VGPU_API int vgpu_maxpool_fwd_idx_nchw_out(const void* x, void* y, void* idx, int N, int H, int W, int C, int k,
                                           int stride, int pad, hipStream_t s) {
  int OH, OW;
  if (!shape_ok(N, H, W, C, k, stride, pad, OH, OW)) return -1;
  const int cv = C / 8;
  const int64_t total = (int64_t)N * OH * OW * cv;
  hipLaunchKernelGGL(maxpool_fwd_idx_kernel, dim3(grid_for(total)), dim3(kThreads), 0, s,
                     static_cast<const u32x4*>(x), static_cast<u32x4*>(y), static_cast<u32x2*>(idx), H, W, cv, OH,
                     OW, k, stride, pad, total, 1);
  return (int)hipGetLastError();
}

// dx [N][H][W][C] bf16 from dy [N][OH][OW][C] and the forward's idx.
VGPU_API int vgpu_maxpool_bwd_nhwc(const void* dy, const void* idx, void* dx, int N, int H, int W, int C, int k,
                                   int stride, int pad, hipStream_t s) {
  int OH, OW;
  if (!shape_ok(N, H, W, C, k, stride, pad, OH, OW)) return -1;
  const int cv = C / 8;
  const int64_t total = (int64_t)N * H * W * cv;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for(total)), dim3(kThreads), 0, s,
                     static_cast<const u32x4*>(dy), static_cast<const u32x2*>(idx), static_cast<u32x4*>(dx), H, W,
                     cv, OH, OW, k, stride, pad, total);
  return (int)hipGetLastError();
}
