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
// Training: gates (activated, bf16 [T][B][4H]) and cells (fp32 [T][B][H]) are
// also written for the backward kernel.
__global__ void __launch_bounds__(256, 1) lstm_recurrence_kernel(const uint16_t* __restrict__ xp,
                                                                 const uint16_t* __restrict__ whh,
                                                                 uint16_t* __restrict__ y,
                                                                 uint16_t* __restrict__ hlast,
                                                                 uint16_t* __restrict__ gates_out,
                                                                 float* __restrict__ cells_out, int B, int T) {
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
    if (row < B && gates_out) {
      const float* gsrc[4] = {gi, gf, gg, go};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t pk[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) pk[q] = (uint32_t)f2bf(gsrc[k][2 * q]) | ((uint32_t)f2bf(gsrc[k][2 * q + 1]) << 16);
        *reinterpret_cast<u32x4*>(gates_out + ((size_t)t * B + row) * (4 * kH) + k * kH + cn) =
            u32x4{pk[0], pk[1], pk[2], pk[3]};
      }
      float* cd = cells_out + ((size_t)t * B + row) * kH + cn;
      *reinterpret_cast<float4*>(cd) = float4{c[0], c[1], c[2], c[3]};
      *reinterpret_cast<float4*>(cd + 4) = float4{c[4], c[5], c[6], c[7]};
    }
    if (row < B) {
      if (y) *reinterpret_cast<u32x4*>(y + ((size_t)row * T + t) * kH + cn) = packed;
      if (hlast && t == T - 1) *reinterpret_cast<u32x4*>(hlast + (size_t)row * kH + cn) = packed;
    }
    __syncthreads();  // h_t published; gate buffer free
  }
}

// Backward through time of one layer.  dgates_t (pre-activation) from the saved
// activated gates and cells, dh_t = dY_t + dh_next, and
//   dh_next = dgates_t · W_hh          (16 x 512) · (512 x 128) on MFMA
// with wave w owning hidden columns [32w, 32w+32) and its W_hh slice (k = all
// 512 gate rows) as B fragments in registers.  dgates go to global (bf16
// [T][B][4H]) for the weight-gradient GEMMs done outside.
constexpr int kGStride = 4 * kH + 8;  // dgates rows in LDS: 1040 B

__global__ void __launch_bounds__(256, 1) lstm_backward_kernel(const uint16_t* __restrict__ gates,
                                                               const float* __restrict__ cells,
                                                               const uint16_t* __restrict__ dy,
                                                               const uint16_t* __restrict__ whh,
                                                               uint16_t* __restrict__ dgates, int B, int T) {
  __shared__ __attribute__((aligned(16))) uint16_t sdg[kRows * kGStride];  // dgates_t, bf16
  __shared__ __attribute__((aligned(16))) float sdh[kRows * kH];            // dh_next, fp32

  const int t_ = threadIdx.x, lane = t_ & 63, w = t_ >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int b0 = blockIdx.x * kRows;
  // B operand: B[k][n] = W_hh[k][n], k = gate row (0..511), n = hidden column of this wave's tiles.
  bf16x8_t wf[2][16];
#pragma unroll
  for (int jn = 0; jn < 2; ++jn)
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      uint16_t v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = whh[(size_t)(ks * 32 + fk * 8 + j) * kH + w * 32 + jn * 16 + fr];
      wf[jn][ks] = __builtin_bit_cast(bf16x8_t, u32x4{(uint32_t)v[0] | ((uint32_t)v[1] << 16),
                                                       (uint32_t)v[2] | ((uint32_t)v[3] << 16),
                                                       (uint32_t)v[4] | ((uint32_t)v[5] << 16),
                                                       (uint32_t)v[6] | ((uint32_t)v[7] << 16)});
    }
  for (int i = t_; i < kRows * kH; i += 256) sdh[i] = 0.0f;
  const int cm = t_ >> 4, cn = (t_ & 15) * 8;  // this thread's 8 cells
  const int row = b0 + cm;
  const bool live = row < B;
  float dcn[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) dcn[q] = 0.0f;
  __syncthreads();

  for (int t = T - 1; t >= 0; --t) {
    float dg_i[8], dg_f[8], dg_g[8], dg_o[8];
    if (live) {
      const uint16_t* gp = gates + ((size_t)t * B + row) * (4 * kH) + cn;
      const float* cp = cells + ((size_t)t * B + row) * kH + cn;
      const float* cpp = t > 0 ? cells + ((size_t)(t - 1) * B + row) * kH + cn : nullptr;
      const uint16_t* dyp = dy + ((size_t)row * T + t) * kH + cn;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float i = bf2f(gp[q]), f = bf2f(gp[kH + q]), g = bf2f(gp[2 * kH + q]), o = bf2f(gp[3 * kH + q]);
        const float c = cp[q], cprev = cpp ? cpp[q] : 0.0f;
        const float dh = bf2f(dyp[q]) + sdh[cm * kH + cn + q];
        const float tc = tanh_f(c);
        const float dc = dh * o * (1.0f - tc * tc) + dcn[q];
        dg_o[q] = dh * tc * o * (1.0f - o);
        dg_i[q] = dc * g * i * (1.0f - i);
        dg_g[q] = dc * i * (1.0f - g * g);
        dg_f[q] = dc * cprev * f * (1.0f - f);
        dcn[q] = dc * f;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) dg_i[q] = dg_f[q] = dg_g[q] = dg_o[q] = 0.0f;
    }
    const float* dsrc[4] = {dg_i, dg_f, dg_g, dg_o};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t pk[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) pk[q] = (uint32_t)f2bf(dsrc[k][2 * q]) | ((uint32_t)f2bf(dsrc[k][2 * q + 1]) << 16);
      const u32x4 v{pk[0], pk[1], pk[2], pk[3]};
      *reinterpret_cast<u32x4*>(sdg + cm * kGStride + k * kH + cn) = v;
      if (live) *reinterpret_cast<u32x4*>(dgates + ((size_t)t * B + row) * (4 * kH) + k * kH + cn) = v;
    }
    __syncthreads();  // dgates_t complete; every read of dh_next done
    f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(sdg + fr * kGStride + ks * 32 + fk * 8);
#pragma unroll
      for (int jn = 0; jn < 2; ++jn) acc[jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[jn][ks], acc[jn], 0, 0, 0);
    }
#pragma unroll
    for (int jn = 0; jn < 2; ++jn)
#pragma unroll
      for (int e = 0; e < 4; ++e) sdh[(fk * 4 + e) * kH + w * 32 + jn * 16 + fr] = acc[jn][e];
    __syncthreads();  // dh_next published; dgates buffer free
  }
}

}  // namespace

VGPU_API int vgpu_lstm_forward_train(const void* xp, const void* whh, void* y, void* gates, void* cells, int B,
                                     int T, int H, hipStream_t s) {
  if (H != kH || B < 1 || T < 1 || !gates || !cells) return -1;
  hipLaunchKernelGGL(lstm_recurrence_kernel, dim3((B + kRows - 1) / kRows), dim3(256), 0, s,
                     static_cast<const uint16_t*>(xp), static_cast<const uint16_t*>(whh), static_cast<uint16_t*>(y),
                     static_cast<uint16_t*>(nullptr), static_cast<uint16_t*>(gates), static_cast<float*>(cells), B, T);
  return (int)hipGetLastError();
}

VGPU_API int vgpu_lstm_backward(const void* gates, const void* cells, const void* dy, const void* whh, void* dgates,
                                int B, int T, int H, hipStream_t s) {
  if (H != kH || B < 1 || T < 1) return -1;
  hipLaunchKernelGGL(lstm_backward_kernel, dim3((B + kRows - 1) / kRows), dim3(256), 0, s,
                     static_cast<const uint16_t*>(gates), static_cast<const float*>(cells),
                     static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(whh),
                     static_cast<uint16_t*>(dgates), B, T);
  return (int)hipGetLastError();
}

// Returns 0, or -1 for an unsupported shape (hidden size must be 128).
VGPU_API int vgpu_lstm_recurrence(const void* xp, const void* whh, void* y, void* hlast, int B, int T, int H,
                                  hipStream_t s) {
  if (H != kH || B < 1 || T < 1) return -1;
  const int grid = (B + kRows - 1) / kRows;
  hipLaunchKernelGGL(lstm_recurrence_kernel, dim3(grid), dim3(256), 0, s, static_cast<const uint16_t*>(xp),
                     static_cast<const uint16_t*>(whh), static_cast<uint16_t*>(y), static_cast<uint16_t*>(hlast),
                     static_cast<uint16_t*>(nullptr), static_cast<float*>(nullptr), B, T);
  return (int)hipGetLastError();
}
