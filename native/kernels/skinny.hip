// Fully connected layers at a handful of rows (batch ≤ 8: VGG-16 training at
// b=2, ai-benchmark test 3.2).  Each of the three GEMMs of a training step is
// a stream over the [N][K] weight with the batch rows riding along:
//
//   forward  y[b][n]  = act(Σ_k x[b][k]·W[n][k] + bias[n])       reads W once
//   dgrad    dx[b][k] = Σ_n g[b][n]·W[n][k]                      reads W once
//   wgrad    dW[n][k] = Σ_b g[b][n]·x[b][k],  db[n] = Σ_b g[b][n] writes dW once
//
// with g = dy·act'(y) formed on the fly from the layer's own output (no mask
// pass).  hipBLASLt ran fc1 (25088 → 4096, 205 MB of bf16 weights) at 75 / 50
// / 66 us for these three (profiles/r5/train/vgg_b2_kernels.md); each is one
// pass over 205 MB, 26 us at 8 TB/s.  The MFMA is of no use at 2 rows: the
// math is 2 FLOP per weight byte, so these are VALU dot products fed by 16-B
// loads, sized for bytes in flight.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VGPU_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kThreads = 256;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

__device__ __forceinline__ void unpack8(const u32x4 v, float (&f)[8]) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) float f2;
  typedef __attribute__((ext_vector_type(2))) __bf16 b2;
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{a, b}, b2));
}
__device__ __forceinline__ float act_f(int act, float v) {
  return act == 1 ? fmaxf(v, 0.0f) : act == 2 ? fminf(fmaxf(v, 0.0f), 6.0f) : v;
}
// d act / d z from the stored output y (relu: y > 0; relu6: 0 < y < 6)
__device__ __forceinline__ float act_grad(int act, float y) {
  return act == 1 ? (y > 0.0f ? 1.0f : 0.0f) : act == 2 ? ((y > 0.0f && y < 6.0f) ? 1.0f : 0.0f) : 1.0f;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---- forward: a block per R = 4 output rows, its 4 waves splitting K ---------------
// Each wave streams every 4th 512-column chunk of the R rows (U = 4 chunks'
// loads in flight), the four partial dot products meet in LDS.  4096 waves for
// fc1: one wave per SIMD with the whole K each ran the pass at ~3.5 TB/s in a
// training step, loads and math strictly alternating (68 us for 205 MB).
// Two rows per block: 2048 blocks for fc1, 31.2 / 7.6 / 4.0 us for VGG-16's fc1-3
// against 32.6 / 8.6 / 4.8 with four rows; eight chunks in flight lost (44.6 us).
constexpr int kFwdRows = 2, kFwdWaves = kThreads / 64;
template <int B, int kR, int kU>
__global__ void __launch_bounds__(kThreads) skinny_fwd_kernel(const uint16_t* __restrict__ x,
                                                              const uint16_t* __restrict__ w,
                                                              const uint16_t* __restrict__ bias,
                                                              uint16_t* __restrict__ y, int N, int K, int act) {
  __shared__ float part[kFwdWaves][kR * B];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * kR;
  float acc[kR][B];
#pragma unroll
  for (int r = 0; r < kR; ++r)
#pragma unroll
    for (int b = 0; b < B; ++b) acc[r][b] = 0.0f;
  const int kv = K >> 3;  // 16-B chunks per row
  const u32x4* W0 = reinterpret_cast<const u32x4*>(w + (int64_t)n0 * K);
  const u32x4* X = reinterpret_cast<const u32x4*>(x);
  for (int c0 = wave * 64 + lane; c0 < kv; c0 += 64 * kFwdWaves * kU) {
    u32x4 wv[kU][kR], xv[kU][B];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int c = c0 + 64 * kFwdWaves * u;
      if (c < kv) {
#pragma unroll
        for (int r = 0; r < kR; ++r) wv[u][r] = W0[(int64_t)r * kv + c];
#pragma unroll
        for (int b = 0; b < B; ++b) xv[u][b] = X[(int64_t)b * kv + c];
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (c0 + 64 * kFwdWaves * u >= kv) continue;
      float xf[B][8];
#pragma unroll
      for (int b = 0; b < B; ++b) unpack8(xv[u][b], xf[b]);
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        float wf[8];
        unpack8(wv[u][r], wf);
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[r][b] = fmaf(wf[j], xf[b][j], acc[r][b]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < kR; ++r)
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const float v = wave_sum(acc[r][b]);
      if (lane == 0) part[wave][r * B + b] = v;
    }
  __syncthreads();
  if (threadIdx.x < kR * B && n0 + (int)threadIdx.x / B < N) {  // thread (r, b) stores one output
    const int r = threadIdx.x / B, b = threadIdx.x % B;
    float v = 0.0f;
#pragma unroll
    for (int q = 0; q < kFwdWaves; ++q) v += part[q][threadIdx.x];  // fixed order
    if (bias) v += bf2f(bias[n0 + r]);
    y[(int64_t)b * N + n0 + r] = f2bf(act_f(act, v));
  }
}

// ---- data gradient: blocks own 64 chunks of 8 columns × an N range -------------
// 4 waves split the block's rows; thread = 8 consecutive k.  g for the block's
// rows is formed into LDS first.  Partials of the NS row splits go to ws and
// skinny_dgrad_reduce sums them in order.
// Optimizer-in-backward (skinny_dgrad_kernel<..., SGD = true>): the weight gradient never reaches memory.
// Each bf16-rounded dW element updates p and its momentum buffer m exactly as
// sgd_bf16_kernel (native/kernels/optim.hip) would, saving the dW write and
// its read back (2 x 205 MB for VGG-16's fc1).
struct SgdJob {
  uint16_t* p;
  uint16_t* m;
  float lr, mom, damp1, wd;
  int nesterov, first;
};

constexpr int kDgRows = 256;  // rows per block (64 per wave); 128 rows or 16 loads in flight ran no faster
// The SGD form writes as much as it reads: 128 rows x 4 loads in flight ran VGG-16 b=2 at
// 1 591-1 610 images/s against 1 563-1 572 for 256 x 8 / 256 x 4, 1 600-1 604 for 128 x 8, 1 581-1 588 for
// 128 x 2, 1 588-1 601 for 64 x 8 / 64 x 4 and 1 554 for 32 x 4 (profiles/r5/train).
constexpr int kSgdRows = 128;
// bf16(gg) -> SGD on one weight element (sgd_bf16_kernel's math)
__device__ __forceinline__ void sgd_elem(const SgdJob& sj, float gg, float& p, float& m) {
  gg = fmaf(sj.wd, p, gg);
  m = sj.first ? gg : fmaf(sj.mom, m, sj.damp1 * gg);
  const float d = sj.nesterov ? fmaf(sj.mom, m, gg) : m;
  p = fmaf(-sj.lr, d, p);
}

// SGD = true: the block also takes the SGD step of the weights it streams (the
// weight gradient of its rows x its 64 chunks needs only x and g): the weight is
// read once for both, dx from its value before the step; db from grid column 0.
template <int B, int kDgRows, int RU, bool SGD = false>
__global__ void __launch_bounds__(kThreads) skinny_dgrad_kernel(const uint16_t* __restrict__ dy,
                                                                const uint16_t* __restrict__ yout,
                                                                const uint16_t* __restrict__ w,
                                                                float* __restrict__ ws, int N, int K, int act,
                                                                const uint16_t* __restrict__ x = nullptr,
                                                                uint16_t* __restrict__ db = nullptr,
                                                                const SgdJob sj = SgdJob{}) {
  __shared__ float sg[B][kDgRows];
  __shared__ float red[3][B][64][9];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int kv = K >> 3;
  const int c = blockIdx.x * 64 + lane;
  const int nb = blockIdx.y * kDgRows;
  for (int i = t; i < B * kDgRows; i += kThreads) {
    const int b = i / kDgRows, r = i - b * kDgRows, n = nb + r;
    float g = 0.0f;
    if (n < N) {
      g = bf2f(dy[(int64_t)b * N + n]);
      if (yout) g *= act_grad(act, bf2f(yout[(int64_t)b * N + n]));
    }
    sg[b][r] = g;
  }
  __syncthreads();
  float xf[SGD ? B : 1][8];
  if (SGD) {
    if (db && blockIdx.x == 0 && nb + t < N && t < kDgRows) {
      float sb = 0.0f;
#pragma unroll
      for (int b = 0; b < B; ++b) sb += sg[b][t];
      db[nb + t] = f2bf(sb);
    }
    if (c < kv)
#pragma unroll
      for (int b = 0; b < (SGD ? B : 1); ++b) unpack8(reinterpret_cast<const u32x4*>(x)[(int64_t)b * kv + c], xf[b]);
  }
  float acc[B][8];
#pragma unroll
  for (int b = 0; b < B; ++b)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[b][j] = 0.0f;
  if (c < kv) {
    const int r0 = wave * (kDgRows / 4);
    const u32x4* W = reinterpret_cast<const u32x4*>(w) + c;
    for (int r = r0; r < r0 + kDgRows / 4; r += RU) {
      u32x4 wv[RU], mv[SGD ? RU : 1];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int n = nb + r + u;
        wv[u] = n < N ? (SGD ? __builtin_nontemporal_load(W + (int64_t)n * kv) : W[(int64_t)n * kv])
                      : u32x4{0u, 0u, 0u, 0u};
        if (SGD && n < N && !sj.first)
          mv[SGD ? u : 0] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sj.m) + c + (int64_t)n * kv);
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        float wf[8];
        unpack8(wv[u], wf);
#pragma unroll
        for (int b = 0; b < B; ++b) {
          const float g = sg[b][r + u];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[b][j] = fmaf(g, wf[j], acc[b][j]);
        }
        if (SGD && nb + r + u < N) {
          float mf[8] = {};
          if (!sj.first) unpack8(mv[SGD ? u : 0], mf);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float o = 0.0f;
#pragma unroll
            for (int b = 0; b < (SGD ? B : 1); ++b) o = fmaf(sg[b][r + u], xf[b][j], o);
            sgd_elem(sj, bf2f(f2bf(o)), wf[j], mf[j]);  // the gradient as bf16, as unfused
          }
          const int64_t at = c + (int64_t)(nb + r + u) * kv;
          __builtin_nontemporal_store(
              u32x4{pack2(wf[0], wf[1]), pack2(wf[2], wf[3]), pack2(wf[4], wf[5]), pack2(wf[6], wf[7])},
              reinterpret_cast<u32x4*>(sj.p) + at);
          __builtin_nontemporal_store(
              u32x4{pack2(mf[0], mf[1]), pack2(mf[2], mf[3]), pack2(mf[4], mf[5]), pack2(mf[6], mf[7])},
              reinterpret_cast<u32x4*>(sj.m) + at);
        }
      }
    }
  }
  // waves 1-3 hand their partial sums to wave 0 (fixed order)
  if (wave > 0) {
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wave - 1][b][lane][j] = acc[b][j];
  }
  __syncthreads();
  if (wave == 0 && c < kv) {
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int b = 0; b < B; ++b)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[b][j] += red[q][b][lane][j];
    float* out = ws + (int64_t)blockIdx.y * B * K;
#pragma unroll
    for (int b = 0; b < B; ++b) {
      float4* o = reinterpret_cast<float4*>(out + (int64_t)b * K + c * 8);
      o[0] = float4{acc[b][0], acc[b][1], acc[b][2], acc[b][3]};
      o[1] = float4{acc[b][4], acc[b][5], acc[b][6], acc[b][7]};
    }
  }
}

// dx = bf16(Σ_split ws[split]) — one thread per 8 values.
__global__ void __launch_bounds__(kThreads) skinny_dgrad_reduce_kernel(const float* __restrict__ ws,
                                                                       uint16_t* __restrict__ dx, int64_t total8,
                                                                       int splits) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= total8) return;
  const float4* p = reinterpret_cast<const float4*>(ws) + i * 2;
  float4 a = p[0], b = p[1];
  for (int s = 1; s < splits; ++s) {
    const float4* q = p + (int64_t)s * total8 * 2;
    const float4 c = q[0], d = q[1];
    a.x += c.x; a.y += c.y; a.z += c.z; a.w += c.w;
    b.x += d.x; b.y += d.y; b.z += d.z; b.w += d.w;
  }
  reinterpret_cast<u32x4*>(dx)[i] = u32x4{pack2(a.x, a.y), pack2(a.z, a.w), pack2(b.x, b.y), pack2(b.z, b.w)};
}

// ---- weight gradient: thread = 8 columns of kRows rows; x chunk held in registers
constexpr int kWgRows = 8;
// The data gradient's split sum rides along: blocks of the extra grid row
// (blockIdx.y == row_groups) reduce ws into dx instead (one launch fewer).
struct DxJob {
  const float* ws;
  uint16_t* dx;
  int64_t total8;
  int splits;
};

template <int B>
__global__ void __launch_bounds__(kThreads) skinny_wgrad_kernel(const uint16_t* __restrict__ dy,
                                                                const uint16_t* __restrict__ yout,
                                                                const uint16_t* __restrict__ x,
                                                                uint16_t* __restrict__ dw, uint16_t* __restrict__ db,
                                                                int N, int K, int act, const DxJob job,
                                                                int row_groups) {
  if ((int)blockIdx.y >= row_groups) {  // block-uniform: the dx reduce job
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < job.total8;
         i += (int64_t)gridDim.x * kThreads) {
      const float4* p = reinterpret_cast<const float4*>(job.ws) + i * 2;
      float4 a = p[0], b = p[1];
      for (int sp = 1; sp < job.splits; ++sp) {
        const float4* q = p + (int64_t)sp * job.total8 * 2;
        const float4 c = q[0], d = q[1];
        a.x += c.x; a.y += c.y; a.z += c.z; a.w += c.w;
        b.x += d.x; b.y += d.y; b.z += d.z; b.w += d.w;
      }
      reinterpret_cast<u32x4*>(job.dx)[i] =
          u32x4{pack2(a.x, a.y), pack2(a.z, a.w), pack2(b.x, b.y), pack2(b.z, b.w)};
    }
    return;
  }
  const int kv = K >> 3;
  const int c = blockIdx.x * kThreads + threadIdx.x;
  const int n0 = blockIdx.y * kWgRows;
  float g[kWgRows][B];
#pragma unroll
  for (int r = 0; r < kWgRows; ++r)
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const int n = n0 + r;
      float v = 0.0f;
      if (n < N) {
        v = bf2f(dy[(int64_t)b * N + n]);
        if (yout) v *= act_grad(act, bf2f(yout[(int64_t)b * N + n]));
      }
      g[r][b] = v;
    }
  if (db && blockIdx.x == 0 && threadIdx.x < kWgRows && n0 + (int)threadIdx.x < N) {
    float s = 0.0f;
#pragma unroll
    for (int r = 0; r < kWgRows; ++r)
      if (r == (int)threadIdx.x)
#pragma unroll
        for (int b = 0; b < B; ++b) s += g[r][b];
    db[n0 + threadIdx.x] = f2bf(s);
  }
  if (c >= kv) return;
  float xf[B][8];
#pragma unroll
  for (int b = 0; b < B; ++b) unpack8(reinterpret_cast<const u32x4*>(x)[(int64_t)b * kv + c], xf[b]);
#pragma unroll
  for (int r = 0; r < kWgRows; ++r) {
    if (n0 + r >= N) break;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = 0.0f;
#pragma unroll
      for (int b = 0; b < B; ++b) s = fmaf(g[r][b], xf[b][j], s);
      o[j] = s;
    }
    // nontemporal: dW (205 MB for fc1) would otherwise push W out of the MALL
    // between this layer's data gradient and the optimizer
    __builtin_nontemporal_store(u32x4{pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7])},
                                &reinterpret_cast<u32x4*>(dw)[(int64_t)(n0 + r) * kv + c]);
  }
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

#define VGPU_SKINNY_SWITCH_T(B, KERNEL, P, Q, GRID, ...)                                                  \
  switch (B) {                                                                                            \
    case 1: hipLaunchKernelGGL((KERNEL<1, P, Q>), GRID, dim3(kThreads), 0, s, __VA_ARGS__); break;        \
    case 2: hipLaunchKernelGGL((KERNEL<2, P, Q>), GRID, dim3(kThreads), 0, s, __VA_ARGS__); break;        \
    case 3: hipLaunchKernelGGL((KERNEL<3, P, Q>), GRID, dim3(kThreads), 0, s, __VA_ARGS__); break;        \
    case 4: hipLaunchKernelGGL((KERNEL<4, P, Q>), GRID, dim3(kThreads), 0, s, __VA_ARGS__); break;        \
    case 8: hipLaunchKernelGGL((KERNEL<8, P, Q>), GRID, dim3(kThreads), 0, s, __VA_ARGS__); break;        \
    default: return -1;                                                                                   \
  }

#define VGPU_SKINNY_SGD_CASE(ROWS, RU, GRID, ...)                                                          \
  switch (B) {                                                                                            \
    case 1: hipLaunchKernelGGL((skinny_dgrad_kernel<1, ROWS, RU, true>), GRID, dim3(kThreads), 0, s, __VA_ARGS__); break; \
    case 2: hipLaunchKernelGGL((skinny_dgrad_kernel<2, ROWS, RU, true>), GRID, dim3(kThreads), 0, s, __VA_ARGS__); break; \
    case 3: hipLaunchKernelGGL((skinny_dgrad_kernel<3, ROWS, RU, true>), GRID, dim3(kThreads), 0, s, __VA_ARGS__); break; \
    case 4: hipLaunchKernelGGL((skinny_dgrad_kernel<4, ROWS, RU, true>), GRID, dim3(kThreads), 0, s, __VA_ARGS__); break; \
    case 8: hipLaunchKernelGGL((skinny_dgrad_kernel<8, ROWS, RU, true>), GRID, dim3(kThreads), 0, s, __VA_ARGS__); break; \
    default: return -1;                                                                                   \
  }

#define VGPU_SKINNY_SWITCH(B, KERNEL, GRID, ...)                                                          \
  switch (B) {                                                                                            \
    case 1: hipLaunchKernelGGL(KERNEL<1>, GRID, dim3(kThreads), 0, s, __VA_ARGS__); break;                \
    case 2: hipLaunchKernelGGL(KERNEL<2>, GRID, dim3(kThreads), 0, s, __VA_ARGS__); break;                \
    case 3: hipLaunchKernelGGL(KERNEL<3>, GRID, dim3(kThreads), 0, s, __VA_ARGS__); break;                \
    case 4: hipLaunchKernelGGL(KERNEL<4>, GRID, dim3(kThreads), 0, s, __VA_ARGS__); break;                \
    case 8: hipLaunchKernelGGL(KERNEL<8>, GRID, dim3(kThreads), 0, s, __VA_ARGS__); break;                \
    default: return -1;                                                                                   \
  }

static int launch_dgrad(int B, dim3 grid, const void* dy, const void* yout, const void* w, void* ws, int N, int K,
                        int act, hipStream_t s) {
  VGPU_SKINNY_SWITCH_T(B, skinny_dgrad_kernel, kDgRows, 8, grid, (const uint16_t*)dy, (const uint16_t*)yout,
                       (const uint16_t*)w, (float*)ws, N, K, act)
  return 0;
}

VGPU_API int vgpu_skinny_supported(int B, int N, int K) {
  return (B == 1 || B == 2 || B == 3 || B == 4 || B == 8) && N % 4 == 0 && K % 8 == 0 && N > 0 && K > 0;
}

// y [B][N] = act(x [B][K] · W[N][K]ᵀ + bias) (bf16; bias bf16 or null; act 0/1/2).
VGPU_API int vgpu_skinny_fwd(const void* x, const void* w, const void* bias, void* y, int B, int N, int K, int act,
                             hipStream_t s) {
  if (!vgpu_skinny_supported(B, N, K) || !al16(x) || !al16(w) || act < 0 || act > 2) return -1;
  const dim3 grid(N / kFwdRows);
  VGPU_SKINNY_SWITCH_T(B, skinny_fwd_kernel, kFwdRows, 4, grid, (const uint16_t*)x, (const uint16_t*)w,
                       (const uint16_t*)bias, (uint16_t*)y, N, K, act)
  return (int)hipGetLastError();
}

// Workspace (bytes) of vgpu_skinny_dgrad: fp32 partials of the row splits.
VGPU_API int64_t vgpu_skinny_dgrad_workspace(int B, int N, int K) {
  return (int64_t)((N + kSgdRows - 1) / kSgdRows) * B * K * 4;  // the SGD form's row split
}

// dx [B][K] = (dy·act'(y)) [B][N] · W [N][K]; yout = the layer's output (null: no activation).
VGPU_API int vgpu_skinny_dgrad(const void* dy, const void* yout, const void* w, void* dx, void* ws, int64_t ws_bytes,
                               int B, int N, int K, int act, hipStream_t s) {
  if (!vgpu_skinny_supported(B, N, K) || !al16(w) || !al16(dx) || !al16(ws)) return -1;
  if (ws_bytes < vgpu_skinny_dgrad_workspace(B, N, K)) return -1;
  const int splits = (N + kDgRows - 1) / kDgRows;
  const dim3 grid((K / 8 + 63) / 64, splits);
  if (launch_dgrad(B, grid, dy, yout, w, ws, N, K, act, s)) return -1;
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const int64_t total8 = (int64_t)B * K / 8;
  hipLaunchKernelGGL(skinny_dgrad_reduce_kernel, dim3((unsigned)((total8 + kThreads - 1) / kThreads)), dim3(kThreads),
                     0, s, (const float*)ws, (uint16_t*)dx, total8, splits);
  return (int)hipGetLastError();
}

// dW [N][K] = gᵀ · x, db [N] = Σ_b g (db may be null), g = dy·act'(y).
VGPU_API int vgpu_skinny_wgrad(const void* dy, const void* yout, const void* x, void* dw, void* db, int B, int N,
                               int K, int act, hipStream_t s) {
  if (!vgpu_skinny_supported(B, N, K) || !al16(x) || !al16(dw)) return -1;
  const int rg = (N + kWgRows - 1) / kWgRows;
  const dim3 grid((K / 8 + kThreads - 1) / kThreads, rg);
  VGPU_SKINNY_SWITCH(B, skinny_wgrad_kernel, grid, (const uint16_t*)dy, (const uint16_t*)yout, (const uint16_t*)x,
                     (uint16_t*)dw, (uint16_t*)db, N, K, act, DxJob{}, rg)
  return (int)hipGetLastError();
}

// The whole backward of a skinny layer in two launches: the data gradient's
// row splits into ws, then dW / db with the split sum into dx riding along.
VGPU_API int vgpu_skinny_backward(const void* dy, const void* yout, const void* x, const void* w, void* dx, void* dw,
                                  void* db, void* ws, int64_t ws_bytes, int B, int N, int K, int act,
                                  hipStream_t s) {
  if (!vgpu_skinny_supported(B, N, K) || !al16(x) || !al16(dw) || !al16(w) || !al16(dx) || !al16(ws)) return -1;
  if (ws_bytes < vgpu_skinny_dgrad_workspace(B, N, K)) return -1;
  const int splits = (N + kDgRows - 1) / kDgRows;
  const dim3 g1((K / 8 + 63) / 64, splits);
  if (launch_dgrad(B, g1, dy, yout, w, ws, N, K, act, s)) return -1;
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const int rg = (N + kWgRows - 1) / kWgRows;
  const dim3 g2((K / 8 + kThreads - 1) / kThreads, rg + 1);
  const DxJob job{(const float*)ws, (uint16_t*)dx, (int64_t)B * K / 8, splits};
  VGPU_SKINNY_SWITCH(B, skinny_wgrad_kernel, g2, (const uint16_t*)dy, (const uint16_t*)yout, (const uint16_t*)x,
                     (uint16_t*)dw, (uint16_t*)db, N, K, act, job, rg)
  return (int)hipGetLastError();
}

// The backward with the weight's SGD step fused in (no dW): w and its momentum
// buffer m are updated in place after the data gradient has read w.  first:
// m is written from the gradient (PyTorch's first step).  db is still a gradient.
VGPU_API int vgpu_skinny_backward_sgd(const void* dy, const void* yout, const void* x, void* w, void* dx, void* m,
                                      void* db, void* ws, int64_t ws_bytes, int B, int N, int K, int act, float lr,
                                      float momentum, float dampening, float weight_decay, int nesterov, int first,
                                      hipStream_t s) {
  if (!w || !m || !vgpu_skinny_supported(B, N, K) || !al16(x) || !al16(w) || !al16(m) || !al16(dx) || !al16(ws))
    return -1;
  if (ws_bytes < vgpu_skinny_dgrad_workspace(B, N, K)) return -1;
  const SgdJob sj{(uint16_t*)w, (uint16_t*)m, lr, momentum, first ? 1.0f : 1.0f - dampening, weight_decay,
                  nesterov, first};
  const int splits = (N + kSgdRows - 1) / kSgdRows;
  const dim3 grid((K / 8 + 63) / 64, splits);
  VGPU_SKINNY_SGD_CASE(kSgdRows, 4, grid, (const uint16_t*)dy, (const uint16_t*)yout, (const uint16_t*)w, (float*)ws,
                       N, K, act, (const uint16_t*)x, (uint16_t*)db, sj)
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const int64_t total8 = (int64_t)B * K / 8;
  hipLaunchKernelGGL(skinny_dgrad_reduce_kernel, dim3((unsigned)((total8 + kThreads - 1) / kThreads)), dim3(kThreads),
                     0, s, (const float*)ws, (uint16_t*)dx, total8, splits);
  return (int)hipGetLastError();
}
