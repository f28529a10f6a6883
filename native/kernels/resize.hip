// Bilinear resize (align_corners=False) of NHWC bf16 activations, forward
// (vgpu.ops.interp).  DeepLab-v3 upsamples its 21-channel logits 16x (24² ->
// 384² at 4.2, 32² -> 512² at 4.1): PyTorch's channels-last kernel took
// 26 us a dispatch at 4.1 for ~22 MB of output (profiles/r6/train).
//
// One thread per output pixel: the source coordinates and the four weights
// are computed once, then the pixel's C channels are interpolated from the
// four source pixels (contiguous C-runs, L2-resident: the input is tiny) and
// written as one contiguous C-run -- adjacent threads write adjacent runs.
// C % 8 == 0 moves 16-byte vectors, else bf16 pairs / singles.  The weights
// and the arithmetic order follow PyTorch's upsample_bilinear2d (fp32
// lambdas from scale = in / out, src = max(scale·(o + 0.5) - 0.5, 0), result
// h0λ·(w0λ·x00 + w1λ·x01) + h1λ·(w0λ·x10 + w1λ·x11), one bf16 rounding).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VGPU_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float bf(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ uint16_t tobf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

struct Src {
  int i0, i1;
  float l0, l1;
};

__device__ __forceinline__ Src src_index(int o, int in, float scale) {
  float r = scale * ((float)o + 0.5f) - 0.5f;
  r = r < 0.0f ? 0.0f : r;
  Src s;
  s.i0 = (int)r;
  if (s.i0 > in - 1) s.i0 = in - 1;
  s.i1 = s.i0 + (s.i0 < in - 1 ? 1 : 0);
  s.l1 = r - (float)s.i0;
  s.l0 = 1.0f - s.l1;
  return s;
}

template <bool kVec>
__global__ void __launch_bounds__(kThreads) resize_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                          int N, int IH, int IW, int C, int OH, int OW, float sh,
                                                          float sw) {
  const int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const int64_t P = (int64_t)N * OH * OW;
  if (p >= P) return;
  const int ox = (int)(p % OW);
  const int64_t r = p / OW;
  const int oy = (int)(r % OH);
  const int n = (int)(r / OH);
  const Src h = src_index(oy, IH, sh), w = src_index(ox, IW, sw);
  const uint16_t* xn = x + (int64_t)n * IH * IW * C;
  const uint16_t* x00 = xn + ((int64_t)h.i0 * IW + w.i0) * C;
  const uint16_t* x01 = xn + ((int64_t)h.i0 * IW + w.i1) * C;
  const uint16_t* x10 = xn + ((int64_t)h.i1 * IW + w.i0) * C;
  const uint16_t* x11 = xn + ((int64_t)h.i1 * IW + w.i1) * C;
  uint16_t* out = y + p * C;
  if constexpr (kVec) {
    typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
    for (int c = 0; c < C; c += 8) {
      const u32x4 a = *reinterpret_cast<const u32x4*>(x00 + c), b = *reinterpret_cast<const u32x4*>(x01 + c);
      const u32x4 d = *reinterpret_cast<const u32x4*>(x10 + c), e = *reinterpret_cast<const u32x4*>(x11 + c);
      const uint16_t* pa = reinterpret_cast<const uint16_t*>(&a);
      const uint16_t* pb = reinterpret_cast<const uint16_t*>(&b);
      const uint16_t* pd = reinterpret_cast<const uint16_t*>(&d);
      const uint16_t* pe = reinterpret_cast<const uint16_t*>(&e);
      u32x4 o;
      uint16_t* po = reinterpret_cast<uint16_t*>(&o);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        po[k] = tobf(h.l0 * (w.l0 * bf(pa[k]) + w.l1 * bf(pb[k])) + h.l1 * (w.l0 * bf(pd[k]) + w.l1 * bf(pe[k])));
      *reinterpret_cast<u32x4*>(out + c) = o;
    }
  } else {
    for (int c = 0; c < C; ++c)
      out[c] = tobf(h.l0 * (w.l0 * bf(x00[c]) + w.l1 * bf(x01[c])) + h.l1 * (w.l0 * bf(x10[c]) + w.l1 * bf(x11[c])));
  }
}

}  // namespace

// x [N][IH][IW][C], y [N][OH][OW][C] bf16 (channels-last storage of NCHW
// tensors).  Returns 0, -1 (bad arguments) or a hipError_t.
VGPU_API int vgpu_resize_bilinear_nhwc(const void* x, void* y, int N, int IH, int IW, int C, int OH, int OW,
                                       hipStream_t s) {
  if (N < 1 || IH < 1 || IW < 1 || C < 1 || OH < 1 || OW < 1) return -1;
  const int64_t P = (int64_t)N * OH * OW;
  const int64_t blocks = (P + kThreads - 1) / kThreads;
  if (blocks > 0x7fffffffll) return -1;
  const float sh = (float)IH / (float)OH, sw = (float)IW / (float)OW;
  const bool vec = C % 8 == 0 && ((uintptr_t)x & 15u) == 0 && ((uintptr_t)y & 15u) == 0;
  if (vec)
    hipLaunchKernelGGL(resize_kernel<true>, dim3((unsigned)blocks), dim3(kThreads), 0, s, (const uint16_t*)x,
                       (uint16_t*)y, N, IH, IW, C, OH, OW, sh, sw);
  else
    hipLaunchKernelGGL(resize_kernel<false>, dim3((unsigned)blocks), dim3(kThreads), 0, s, (const uint16_t*)x,
                       (uint16_t*)y, N, IH, IW, C, OH, OW, sh, sw);
  return (int)hipGetLastError();
}
