// Cross-entropy over bf16 (or fp32) logits with integer targets, forward and
// gradient in ONE kernel (vgpu.ops.loss; the training pods).  PyTorch's
// CrossEntropyLoss on bf16 logits runs a cast, log-softmax, NLL forward, and
// in the backward a fill, NLL backward, log-softmax backward and a cast —
// eight launches of ~4.7 us each in a replayed training step (VGG-16 b=2,
// profiles/r5/train).  Here each row is one workgroup: max, Σ exp, the row's
// loss and dlogits = (softmax − onehot) / rows in one pass (fp32 math), then
// one block takes the mean of the row losses in a fixed order.  The backward
// only scales the saved dlogits by the incoming gradient.
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

// One block per row.  loss_rows[r] = logsumexp(x_r) − x_r[t_r]; dx = (softmax − onehot) · scale.
template <typename T>
__global__ void __launch_bounds__(kThreads) xent_kernel(const T* __restrict__ x, const int64_t* __restrict__ tgt,
                                                        float* __restrict__ loss_rows, T* __restrict__ dx, int C,
                                                        float scale) {
  __shared__ float sh[kThreads / 64];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * C;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < C; c += kThreads) m = fmaxf(m, ld(xr, c));
  m = block_reduce<T>(m, sh, true);
  float s = 0.0f;
  for (int c = threadIdx.x; c < C; c += kThreads) s += __expf(ld(xr, c) - m);
  s = block_reduce<T>(s, sh, false);
  const int64_t t = tgt[row];
  const float lse = m + __logf(s), inv = 1.0f / s;
  if (threadIdx.x == 0) loss_rows[row] = (t >= 0 && t < C) ? lse - ld(xr, t) : 0.0f;
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float p = __expf(ld(xr, c) - m) * inv;
    st(dx, row * C + c, (p - (c == t ? 1.0f : 0.0f)) * scale);
  }
}

// Up to 64 rows: one block does every row and the mean (one launch in all).
template <typename T>
__global__ void __launch_bounds__(kThreads) xent_small_kernel(const T* __restrict__ x, const int64_t* __restrict__ tgt,
                                                              float* __restrict__ loss_rows, float* __restrict__ loss,
                                                              T* __restrict__ dx, int rows, int C, float scale) {
  __shared__ float sh[kThreads / 64];
  float total = 0.0f;
  for (int row = 0; row < rows; ++row) {
    const T* xr = x + (int64_t)row * C;
    float m = -INFINITY;
    for (int c = threadIdx.x; c < C; c += kThreads) m = fmaxf(m, ld(xr, c));
    m = block_reduce<T>(m, sh, true);
    float s = 0.0f;
    for (int c = threadIdx.x; c < C; c += kThreads) s += __expf(ld(xr, c) - m);
    s = block_reduce<T>(s, sh, false);
    const int64_t t = tgt[row];
    const float lse = m + __logf(s), inv = 1.0f / s;
    const float l = (t >= 0 && t < C) ? lse - ld(xr, t) : 0.0f;
    total += l;
    if (threadIdx.x == 0) loss_rows[row] = l;
    for (int c = threadIdx.x; c < C; c += kThreads) {
      const float p = __expf(ld(xr, c) - m) * inv;
      st(dx, (int64_t)row * C + c, (p - (c == t ? 1.0f : 0.0f)) * scale);
    }
  }
  if (threadIdx.x == 0) loss[0] = total / (float)rows;  // rows summed in order
}

// mean of the row losses in a fixed order (one block)
__global__ void __launch_bounds__(kThreads) mean_kernel(const float* __restrict__ v, float* __restrict__ out,
                                                        int n) {
  __shared__ float sh[kThreads / 64];
  float s = 0.0f;
  for (int i = threadIdx.x; i < n; i += kThreads) s += v[i];
  s = block_reduce<float>(s, sh, false);
  if (threadIdx.x == 0) out[0] = s / (float)n;
}

}  // namespace

// logits [rows][C] (bf16 when is_bf16, else fp32), targets int64 [rows];
// writes loss_rows fp32 [rows], loss fp32 [1] (mean) and dlogits (the logits'
// dtype) = ∂mean/∂logits.  Returns 0, -1 (bad arguments) or a hipError_t.
VGPU_API int vgpu_cross_entropy_fwd_bwd(const void* logits, const int64_t* tgt, float* loss_rows, float* loss,
                                        void* dlogits, int rows, int C, int is_bf16, hipStream_t s) {
  if (rows < 1 || C < 1) return -1;
  const float scale = 1.0f / (float)rows;
  if (rows <= 64) {
    if (is_bf16)
      hipLaunchKernelGGL(xent_small_kernel<uint16_t>, dim3(1), dim3(kThreads), 0, s, (const uint16_t*)logits, tgt,
                         loss_rows, loss, (uint16_t*)dlogits, rows, C, scale);
    else
      hipLaunchKernelGGL(xent_small_kernel<float>, dim3(1), dim3(kThreads), 0, s, (const float*)logits, tgt,
                         loss_rows, loss, (float*)dlogits, rows, C, scale);
    return (int)hipGetLastError();
  }
  if (is_bf16)
    hipLaunchKernelGGL(xent_kernel<uint16_t>, dim3(rows), dim3(kThreads), 0, s, (const uint16_t*)logits, tgt,
                       loss_rows, (uint16_t*)dlogits, C, scale);
  else
    hipLaunchKernelGGL(xent_kernel<float>, dim3(rows), dim3(kThreads), 0, s, (const float*)logits, tgt, loss_rows,
                       (float*)dlogits, C, scale);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(kThreads), 0, s, (const float*)loss_rows, loss, rows);
  return (int)hipGetLastError();
}
