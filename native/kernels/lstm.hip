// Fused LSTM recurrence for inference on gfx950 (ai-benchmark 5.1, LSTM-Sentiment:
// hidden 128, 2 layers, 1024 steps, batch 100).
//
// Why: PyTorch-ROCm runs nn.LSTM as MIOpen's per-timestep kernel sequence —
// about 4 000 dispatches of a few microseconds per 2-layer forward.  One pod is then
// bound by dispatch latency, and several pods sharing a GPU contend for the
// command processor instead of for CUs (docs/benchmarks.md, round 2).  Here one
// layer is one GEMM for the input projection of all timesteps (hipBLASLt, outside)
// plus ONE persistent kernel for the recurrence:
//
//   gates_t = Xp_t + h_{t-1} · W_hhᵀ          Xp = X · W_ihᵀ + b_ih + b_hh  (precomputed)
//   c_t = σ(f)·c_{t-1} + σ(i)·tanh(g),  h_t = σ(o)·tanh(c_t)      (gate order i, f, g, o)
//
// A workgroup owns 16 batch rows for the whole sequence.  Its 4 waves own the
// 4 gate blocks (128 columns each); each wave keeps its 128x128 slice of W_hh
// as MFMA B fragments in registers (32 x bf16x8 = 128 VGPRs) for all 1024 steps,
// so a timestep is 32 mfma_f32_16x16x32_bf16 per wave on h_{t-1} (16x128 bf16
// in LDS, rows padded to 272 B), the gate activations through LDS (fp32), and
// the cell update with c_t held in registers (8 cells per thread).  The Xp
// values of step t+1 are loaded while step t computes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VGPU_API extern "C" __attribute__((visibility("default")))

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

constexpr int kH = 128;            // hidden size (one wave's gate block)
constexpr int kRows = 16;          // batch rows per workgroup
constexpr int kHStride = kH + 8;   // h rows in LDS: 272 B (bank spread)

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) { return 2.0f / (1.0f + __expf(-2.0f * x)) - 1.0f; }

// xp: [T][B][4H] bf16 (biases folded in); whh: [4H][H] bf16 (PyTorch weight_hh_l*);
// y: [B][T][H] bf16 or nullptr; hlast: [B][H] bf16 or nullptr.
__global__ void __launch_bounds__(256, 1) lstm_recurrence_kernel(const uint16_t* __restrict__ xp,
                                                                 const uint16_t* __restrict__ whh,
                                                                 uint16_t* __restrict__ y,
                                                                 uint16_t* __restrict__ hlast, int B, int T) {
  __shared__ __attribute__((aligned(16))) uint16_t sh[kRows * kHStride];   // h_{t-1}, bf16
  __shared__ __attribute__((aligned(16))) float sg[4 * kRows * kH];          // activated gates

  const int t_ = threadIdx.x, lane = t_ & 63, w = t_ >> 6;  // wave w owns gate block w
  const int fr = lane & 15, fk = lane >> 4;
  const int b0 = blockIdx.x * kRows;

  // W_hh slice of gate block w as B fragments: tile jn (16 gate columns) x k step kk (32 hidden).
  bf16x8_t wf[8][4];
#pragma unroll
  for (int jn = 0; jn < 8; ++jn)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      wf[jn][kk] = *reinterpret_cast<const bf16x8_t*>(whh + (size_t)(w * kH + jn * 16 + fr) * kH + kk * 32 + fk * 8);

  // h_0 = 0, c_0 = 0
  for (int i = t_; i < kRows * kHStride; i += 256) sh[i] = 0;
  float c[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) c[q] = 0.0f;
  const int cm = t_ >> 4, cn = (t_ & 15) * 8;  // this thread's 8 cells: row cm, units cn..cn+7

  // Xp of one step in accumulator layout: tile jn, row 4*fk+e, column w*128 + 16*jn + fr.
  uint16_t xn[8][4];
  auto load_xp = [&](int t) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = b0 + fk * 4 + e;
      const bool ok = r < B;
      const uint16_t* p = xp + ((size_t)t * B + (ok ? r : 0)) * (4 * kH) + w * kH + fr;
#pragma unroll
      for (int jn = 0; jn < 8; ++jn) xn[jn][e] = ok ? p[jn * 16] : (uint16_t)0;
    }
  };
  load_xp(0);
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    f32x4_t acc[8];
#pragma unroll
    for (int jn = 0; jn < 8; ++jn)
      acc[jn] = f32x4_t{bf2f(xn[jn][0]), bf2f(xn[jn][1]), bf2f(xn[jn][2]), bf2f(xn[jn][3])};
    if (t + 1 < T) load_xp(t + 1);  // lands while this step computes
    bf16x8_t hf[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      hf[kk] = *reinterpret_cast<const bf16x8_t*>(sh + fr * kHStride + kk * 32 + fk * 8);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int jn = 0; jn < 8; ++jn)
        acc[jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hf[kk], wf[jn][kk], acc[jn], 0, 0, 0);
    // activations: sigmoid for i, f, o; tanh for g (block 2)
#pragma unroll
    for (int jn = 0; jn < 8; ++jn)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = acc[jn][e];
        sg[(w * kRows + fk * 4 + e) * kH + jn * 16 + fr] = (w == 2) ? tanh_f(v) : sigm(v);
      }
    __syncthreads();  // gates complete; every wave's reads of h_{t-1} done
    const float* gi = sg + (0 * kRows + cm) * kH + cn;
    const float* gf = sg + (1 * kRows + cm) * kH + cn;
    const float* gg = sg + (2 * kRows + cm) * kH + cn;
    const float* go = sg + (3 * kRows + cm) * kH + cn;
    uint16_t hv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      c[q] = gf[q] * c[q] + gi[q] * gg[q];
      hv[q] = f2bf(go[q] * tanh_f(c[q]));
    }
    const u32x4 packed{(uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16),
                       (uint32_t)hv[4] | ((uint32_t)hv[5] << 16), (uint32_t)hv[6] | ((uint32_t)hv[7] << 16)};
    *reinterpret_cast<u32x4*>(sh + cm * kHStride + cn) = packed;
    const int row = b0 + cm;
    if (row < B) {
      if (y) *reinterpret_cast<u32x4*>(y + ((size_t)row * T + t) * kH + cn) = packed;
      if (hlast && t == T - 1) *reinterpret_cast<u32x4*>(hlast + (size_t)row * kH + cn) = packed;
    }
    __syncthreads();  // h_t published; gate buffer free
  }
}

}  // namespace

// Returns 0, or -1 for an unsupported shape (hidden size must be 128).
VGPU_API int vgpu_lstm_recurrence(const void* xp, const void* whh, void* y, void* hlast, int B, int T, int H,
                                  hipStream_t s) {
  if (H != kH || B < 1 || T < 1) return -1;
  const int grid = (B + kRows - 1) / kRows;
  hipLaunchKernelGGL(lstm_recurrence_kernel, dim3(grid), dim3(256), 0, s, static_cast<const uint16_t*>(xp),
                     static_cast<const uint16_t*>(whh), static_cast<uint16_t*>(y), static_cast<uint16_t*>(hlast), B,
                     T);
  return (int)hipGetLastError();
}
