// Cross-entropy over bf16 (or fp32) logits with integer targets, forward and
// gradient in one pass (vgpu.ops.loss; the training pods).  PyTorch's
// CrossEntropyLoss on bf16 logits runs a cast, log-softmax, NLL forward, and
// in the backward a fill, NLL backward, log-softmax backward and a cast —
// eight launches of ~4.7 us each in a replayed training step (VGG-16 b=2,
// profiles/r5/train); DeepLab's per-pixel loss (nll_loss2d) was ~224 us a step.
//
// Logits are [rows][C] in any of three layouts, addressed as
//   x[row, c] = base(row) + c * cstride,  base(row) = (row / hw) * bstride + (row % hw) * pstride
// — a 2-D [rows, C] matrix, a channels-last [B, H, W, C] map or an NCHW map
// (rows = B·H·W) — so the per-pixel loss reads the convolution's output in
// place.  A row whose target is outside [0, C) or equals ignore_index is
// ignored as torch.nn.functional.cross_entropy ignores it: loss 0, gradient
// 0, not counted in the mean.
//
// The forward writes the unscaled gradient (softmax − onehot) of every valid
// row and the reciprocal of the valid-row count; the backward multiplies by
// (incoming gradient × that reciprocal).  Per-row work is mapped by C: one
// workgroup per row for wide rows (ImageNet's 1000 classes), one lane per row
// for narrow ones (DeepLab's 21: a wave covers 64 pixels, its NCHW reads are
// coalesced across lanes).  The mean is taken in a fixed order: by one
// workgroup over the row losses (wide rows), or over per-workgroup partials
// the narrow kernel writes (no atomics: the result is deterministic).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VGPU_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float ld(const uint16_t* p, int64_t i) { return __uint_as_float((uint32_t)p[i] << 16); }
__device__ __forceinline__ float ld(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ void st(uint16_t* p, int64_t i, float v) {
  __bf16 b = (__bf16)v;
  p[i] = __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ void st(float* p, int64_t i, float v) { p[i] = v; }

struct Layout {
  int64_t hw, bstride, pstride, cstride;
  __device__ __forceinline__ int64_t base(int64_t row) const { return (row / hw) * bstride + (row % hw) * pstride; }
};

__device__ __forceinline__ bool valid_target(int64_t t, int C, int64_t ignore) { return t >= 0 && t < C && t != ignore; }

template <typename T>
__device__ float block_reduce(float v, float* sh, bool is_max) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float u = __shfl_xor(v, o, 64);
    v = is_max ? fmaxf(v, u) : v + u;
  }
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  float r = sh[0];
#pragma unroll
  for (int w = 1; w < kThreads / 64; ++w) r = is_max ? fmaxf(r, sh[w]) : r + sh[w];
  __syncthreads();
  return r;
}

// One workgroup per row (wide rows).
template <typename T>
__device__ float xent_row_block(const T* __restrict__ x, const int64_t* __restrict__ tgt, T* __restrict__ dx,
                                int64_t row, int C, int64_t ignore, Layout L, float* sh) {
  const int64_t b = L.base(row);
  const int64_t t = tgt[row];
  const bool ok = valid_target(t, C, ignore);
  float m = -INFINITY;
  for (int c = threadIdx.x; c < C; c += kThreads) m = fmaxf(m, ld(x, b + c * L.cstride));
  m = block_reduce<T>(m, sh, true);
  float s = 0.0f;
  for (int c = threadIdx.x; c < C; c += kThreads) s += __expf(ld(x, b + c * L.cstride) - m);
  s = block_reduce<T>(s, sh, false);
  const float lse = m + __logf(s), inv = 1.0f / s;
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float p = __expf(ld(x, b + c * L.cstride) - m) * inv;
    st(dx, b + c * L.cstride, ok ? p - (c == t ? 1.0f : 0.0f) : 0.0f);
  }
  return ok ? lse - ld(x, b + t * L.cstride) : 0.0f;
}

template <typename T>
__global__ void __launch_bounds__(kThreads) xent_wide_kernel(const T* __restrict__ x, const int64_t* __restrict__ tgt,
                                                             float* __restrict__ loss_rows, T* __restrict__ dx, int C,
                                                             int64_t ignore, Layout L) {
  __shared__ float sh[kThreads / 64];
  const float l = xent_row_block(x, tgt, dx, blockIdx.x, C, ignore, L, sh);
  if (threadIdx.x == 0) loss_rows[blockIdx.x] = l;
}

// One lane per row (C <= 64): two passes over the row's C logits (max, then
// Σexp and the gradient), all in registers' reach of L1/L2.
// Also writes the block's (Σ loss, valid rows) to part[blockIdx.x] for mean_part_kernel
// (a single-block mean over DeepLab's 147k pixel rows took 158 us).
template <typename T>
__global__ void __launch_bounds__(kThreads) xent_narrow_kernel(const T* __restrict__ x, const int64_t* __restrict__ tgt,
                                                               float* __restrict__ loss_rows, T* __restrict__ dx,
                                                               int64_t rows, int C, int64_t ignore, Layout L,
                                                               float2* __restrict__ part) {
  __shared__ float sh[kThreads / 64];
  const int64_t row0 = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const bool in = row0 < rows;
  const int64_t row = in ? row0 : rows - 1;  // every lane takes part in the block sums
  const int64_t b = L.base(row);
  const int64_t t = tgt[row];
  const bool ok = valid_target(t, C, ignore);
  float m = -INFINITY;
  for (int c = 0; c < C; ++c) m = fmaxf(m, ld(x, b + c * L.cstride));
  float s = 0.0f, xt = 0.0f;
  for (int c = 0; c < C; ++c) {
    const float v = ld(x, b + c * L.cstride);
    s += __expf(v - m);
    if (c == t) xt = v;
  }
  const float inv = 1.0f / s;
  if (in)
    for (int c = 0; c < C; ++c) {
      const float p = __expf(ld(x, b + c * L.cstride) - m) * inv;
      st(dx, b + c * L.cstride, ok ? p - (c == t ? 1.0f : 0.0f) : 0.0f);
    }
  const float l = (in && ok) ? m + __logf(s) - xt : 0.0f;
  if (in) loss_rows[row] = l;
  const float bl = block_reduce<float>(l, sh, false);
  const float bn = block_reduce<float>((in && ok) ? 1.0f : 0.0f, sh, false);
  if (threadIdx.x == 0) part[blockIdx.x] = float2{bl, bn};
}

// out[0] = Σ part.x / Σ part.y, out[1] = 1 / Σ part.y (block partials summed in order).
__global__ void __launch_bounds__(kThreads) mean_part_kernel(const float2* __restrict__ part, float* __restrict__ out,
                                                             int n) {
  __shared__ float sh[kThreads / 64];
  float s = 0.0f, k = 0.0f;
  for (int i = threadIdx.x; i < n; i += kThreads) {
    s += part[i].x;
    k += part[i].y;
  }
  s = block_reduce<float>(s, sh, false);
  k = block_reduce<float>(k, sh, false);
  if (threadIdx.x == 0) {
    out[0] = s / k;
    out[1] = k > 0.0f ? 1.0f / k : 0.0f;
  }
}

// Up to 64 wide rows: one block does every row and the mean (one launch in all).
template <typename T>
__global__ void __launch_bounds__(kThreads) xent_small_kernel(const T* __restrict__ x, const int64_t* __restrict__ tgt,
                                                              float* __restrict__ loss_rows, float* __restrict__ out,
                                                              T* __restrict__ dx, int rows, int C, int64_t ignore,
                                                              Layout L) {
  __shared__ float sh[kThreads / 64];
  float total = 0.0f;
  int valid = 0;
  for (int row = 0; row < rows; ++row) {
    const float l = xent_row_block(x, tgt, dx, row, C, ignore, L, sh);
    total += l;
    valid += valid_target(tgt[row], C, ignore) ? 1 : 0;
    if (threadIdx.x == 0) loss_rows[row] = l;
  }
  if (threadIdx.x == 0) {  // rows summed in order
    out[0] = total / (float)valid;
    out[1] = valid ? 1.0f / (float)valid : 0.0f;
  }
}

// out[0] = Σ loss_rows / valid rows (in a fixed order), out[1] = 1 / valid rows.
__global__ void __launch_bounds__(kThreads) mean_kernel(const float* __restrict__ v, const int64_t* __restrict__ tgt,
                                                        float* __restrict__ out, int64_t n, int C, int64_t ignore) {
  __shared__ float sh[kThreads / 64];
  float s = 0.0f, k = 0.0f;
  for (int64_t i = threadIdx.x; i < n; i += kThreads) {
    s += v[i];
    k += valid_target(tgt[i], C, ignore) ? 1.0f : 0.0f;
  }
  s = block_reduce<float>(s, sh, false);
  k = block_reduce<float>(k, sh, false);  // exact: counts below 2^24 per lane sum
  if (threadIdx.x == 0) {
    out[0] = s / k;
    out[1] = k > 0.0f ? 1.0f / k : 0.0f;
  }
}

template <typename T>
int launch(const T* x, const int64_t* tgt, float* loss_rows, float* out, T* dx, int64_t rows, int C, int64_t ignore,
           Layout L, hipStream_t s) {
  if (C > 64 && rows <= 64) {
    hipLaunchKernelGGL(xent_small_kernel<T>, dim3(1), dim3(kThreads), 0, s, x, tgt, loss_rows, out, dx, (int)rows, C,
                       ignore, L);
    return (int)hipGetLastError();
  }
  if (C > 64) {
    if (rows > 0x7fffffffll) return -1;
    hipLaunchKernelGGL(xent_wide_kernel<T>, dim3((unsigned)rows), dim3(kThreads), 0, s, x, tgt, loss_rows, dx, C,
                       ignore, L);
  } else {
    // block partials live behind the row losses (the caller sizes loss_rows for both)
    const int64_t blocks = (rows + kThreads - 1) / kThreads;
    if (blocks > 0x7fffffffll) return -1;
    float2* part = reinterpret_cast<float2*>(loss_rows + ((rows + 1) & ~int64_t(1)));
    hipLaunchKernelGGL(xent_narrow_kernel<T>, dim3((unsigned)blocks), dim3(kThreads), 0, s, x, tgt, loss_rows, dx,
                       rows, C, ignore, L, part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(mean_part_kernel, dim3(1), dim3(kThreads), 0, s, (const float2*)part, out, (int)blocks);
    return (int)hipGetLastError();
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(kThreads), 0, s, (const float*)loss_rows, tgt, out, rows, C, ignore);
  return (int)hipGetLastError();
}

}  // namespace

// fp32 elements loss_rows must hold for vgpu_cross_entropy_fwd_bwd2 (row losses,
// and for narrow rows the per-block partials behind them).
VGPU_API int64_t vgpu_cross_entropy_rows_workspace(int64_t rows, int C) {
  if (rows < 1 || C < 1) return -1;
  return C > 64 ? rows : ((rows + 1) & ~int64_t(1)) + 2 * ((rows + kThreads - 1) / kThreads);
}

// logits (bf16 when is_bf16, else fp32) addressed by (hw, bstride, pstride,
// cstride) as above; targets int64 [rows].  Writes loss_rows fp32 [rows],
// out fp32 [2] = {mean loss over valid rows, 1 / valid rows}, and dlogits
// (same dtype and layout as the logits) = unscaled ∂loss_row/∂logits.
// loss_rows holds vgpu_cross_entropy_rows_workspace(rows, C) floats.
// Returns 0, -1 (bad arguments) or a hipError_t.
VGPU_API int vgpu_cross_entropy_fwd_bwd2(const void* logits, const int64_t* tgt, float* loss_rows, float* out,
                                         void* dlogits, int64_t rows, int C, int64_t ignore_index, int64_t hw,
                                         int64_t bstride, int64_t pstride, int64_t cstride, int is_bf16,
                                         hipStream_t s) {
  if (rows < 1 || C < 1 || hw < 1 || cstride < 1) return -1;
  const Layout L{hw, bstride, pstride, cstride};
  if (is_bf16)
    return launch((const uint16_t*)logits, tgt, loss_rows, out, (uint16_t*)dlogits, rows, C, ignore_index, L, s);
  return launch((const float*)logits, tgt, loss_rows, out, (float*)dlogits, rows, C, ignore_index, L, s);
}
