// Training-mode BatchNorm (+ ReLU / ReLU6) for NHWC bf16 activations on MI355X.
//
// Why: a ResNet-V2-50 training step (ai-benchmark 1.2, b=20 346²) spent 53% of
// its steady-state GPU time in PyTorch's channels-last BatchNorm reductions
// (batch_norm_collect_statistics + batch_norm_backward_reduce, ~110 µs each per
// layer; profiles/rocprof_train_r1.md).  These kernels are bandwidth-shaped:
//
//   forward:  reduce  (shifted sums of x per channel, fp32 per block)
//             finalize (fp64 merge of the block partials -> mean / invstd,
//                      running-stat update, folded scale/shift)
//             apply   y = act(x * s[c] + t[c])
//   backward: reduce  (Σ dz, Σ dz·x̂ with dz = dy · act'(x * s + t))
//             finalize (dβ, dγ, folded dx coefficients)
//             apply   dx = s·dz + cc·x + b          (one pass, no dz tensor)
//
// The reduction grid is ≈1024 workgroups (4 per CU) of 256 threads; a thread
// owns 8 channels (one 16-B load per row) and walks rows with 4 loads in
// flight, all addresses clamped in range so the loop has no exec branches.
// Variance uses sums shifted by the first row's value (one shift for every
// block, so partials merge by plain addition) and an fp64 merge: no E[x²]-E[x]²
// cancellation at 600k rows/channel.
//
// Parameters (γ, β, running stats, dγ, dβ) are fp32 or bf16 (a model cast with
// .to(bfloat16)); the saved mean / invstd are always fp32.  Requires C % 8 == 0
// and 16-B aligned tensors (checked on the host).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define VGPU_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kThreads = 256;
constexpr int kUnroll = 4;           // rows in flight per thread (default; 8 via vgpu_bn_set_tuning)
constexpr int kMaxChunk = 512;       // channels per reduction workgroup
constexpr int kTargetBlocks = 1024;  // reduction grid ≈ 4 workgroups per CU (default)
int g_target_blocks = kTargetBlocks;  // A/B: vgpu_bn_set_tuning
int g_unroll = kUnroll;
constexpr int kFinC = 8;             // finalize: channels per workgroup
constexpr int kFinG = 128;           //           partial groups per workgroup (tree-merged):
                                     // ≤ 8 loads per thread at G = 1024, ≤ 19 at the epilogue
                                     // statistics' G = M / 64 of ResNet stage 1 (2366)
constexpr int kMaxGrid = 256 * 8;

struct alignas(16) bf16x8 {
  uint16_t v[8];
};

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

// Parameter access: P = float or uint16_t (bf16 bits); a null pointer reads as dflt.
__device__ __forceinline__ float ldp(const float* p, int i, float dflt) { return p ? p[i] : dflt; }
__device__ __forceinline__ float ldp(const uint16_t* p, int i, float dflt) { return p ? bf2f(p[i]) : dflt; }
__device__ __forceinline__ void stp(float* p, int i, float v) { p[i] = v; }
__device__ __forceinline__ void stp(uint16_t* p, int i, float v) { p[i] = f2bf(v); }

template <int kAct>
__device__ __forceinline__ float act_fwd(float z) {
  if constexpr (kAct == 1) return fmaxf(z, 0.0f);
  if constexpr (kAct == 2) return fminf(fmaxf(z, 0.0f), 6.0f);
  return z;
}

// d act / dz as PyTorch defines it (threshold_backward / hardtanh_backward).
template <int kAct>
__device__ __forceinline__ float act_grad(float z) {
  if constexpr (kAct == 1) return z > 0.0f ? 1.0f : 0.0f;
  if constexpr (kAct == 2) return (z > 0.0f && z < 6.0f) ? 1.0f : 0.0f;
  return 1.0f;
}

__device__ __forceinline__ void load8(const float* __restrict__ p, float (&o)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

// Per-channel reduction.  Grid (G, ceil(C / chunk)); a workgroup reduces
// `rows_per_block` rows of one channel chunk into partial[blockIdx.x][c].
//   kMode 0: (Σ (x - x₀), Σ (x - x₀)²)         x₀ = row 0 (the shift)
//   kMode 1: (Σ dz, Σ dz · x̂)                   dz = dy · act'(x·s + t)
template <int kMode, int kAct, typename P, int kU = kUnroll>
__global__ void __launch_bounds__(kThreads) bn_reduce_kernel(
    const bf16x8* __restrict__ x, const bf16x8* __restrict__ dy, const P* __restrict__ gamma,
    const P* __restrict__ beta, const float* __restrict__ mean, const float* __restrict__ invstd,
    float2* __restrict__ partial, int64_t M, int C, int chunk, int rows_per_block) {
  __shared__ float2 red[kThreads * 8];
  const int tpr = chunk >> 3;  // threads per row
  const int rpb = kThreads / tpr;
  const int tid = threadIdx.x;
  const int cg = tid % tpr, ro = tid / tpr;
  const int c0 = blockIdx.y * chunk + cg * 8;
  const bool live = ro < rpb && c0 < C;
  const int cvec = C >> 3;
  const int cv = live ? c0 >> 3 : 0;

  float k0[8], k1[8], k2[8], k3[8];
  if constexpr (kMode == 0) {
    const bf16x8 v = x[cv];
#pragma unroll
    for (int j = 0; j < 8; ++j) k0[j] = bf2f(v.v[j]);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = live ? c0 + j : 0;
      const float is = invstd[c];
      const float s = ldp(gamma, c, 1.0f) * is;
      k0[j] = s;
      k1[j] = ldp(beta, c, 0.0f) - mean[c] * s;
      k2[j] = mean[c];
      k3[j] = is;
    }
  }

  float a1[8], a2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a1[j] = a2[j] = 0.0f;

  const int64_t rbase = (int64_t)blockIdx.x * rows_per_block + ro;
  for (int k = 0; k < rows_per_block; k += rpb * kU) {
    bf16x8 v[kU], g[kU];
    float ok[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t r = rbase + k + u * rpb;
      const bool in = live & (r < M);
      ok[u] = in ? 1.0f : 0.0f;
      const int64_t idx = in ? r * cvec + cv : 0;  // clamped: always a valid address
      v[u] = x[idx];
      if constexpr (kMode == 1) g[u] = dy[idx];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xf = bf2f(v[u].v[j]);
        if constexpr (kMode == 0) {
          const float d = (xf - k0[j]) * ok[u];
          a1[j] += d;
          a2[j] = fmaf(d, d, a2[j]);
        } else {
          const float dz = bf2f(g[u].v[j]) * act_grad<kAct>(fmaf(xf, k0[j], k1[j])) * ok[u];
          a1[j] += dz;
          a2[j] = fmaf(dz, (xf - k2[j]) * k3[j], a2[j]);
        }
      }
    }
  }

  if (ro < rpb) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[ro * chunk + cg * 8 + j] = make_float2(a1[j], a2[j]);
  }
  __syncthreads();
  for (int t = tid; t < chunk; t += kThreads) {
    const int c = blockIdx.y * chunk + t;
    if (c >= C) break;
    float s1 = 0.0f, s2 = 0.0f;
    for (int q = 0; q < rpb; ++q) {
      const float2 p = red[q * chunk + t];
      s1 += p.x;
      s2 += p.y;
    }
    partial[(int64_t)blockIdx.x * C + c] = make_float2(s1, s2);
  }
}

// fp64 merge of the G block partials of kFinC channels: kFinG groups of
// partials summed in parallel, then a log2(kFinG)-step tree in LDS (a serial
// merge here made the finalize a 10 µs latency chain).  Valid in grp == 0.
__device__ __forceinline__ void merge_partials(const float2* __restrict__ partial, int64_t G, int C,
                                               int c, int cl, int grp, double& s1, double& s2) {
  __shared__ double r1[kFinG][kFinC], r2[kFinG][kFinC];
  s1 = 0.0;
  s2 = 0.0;
  if (c < C) {
#pragma unroll 8
    for (int64_t g = grp; g < G; g += kFinG) {
      const float2 p = partial[g * C + c];
      s1 += p.x;
      s2 += p.y;
    }
  }
  r1[grp][cl] = s1;
  r2[grp][cl] = s2;
  __syncthreads();
#pragma unroll
  for (int h = kFinG / 2; h > 0; h >>= 1) {
    if (grp < h) {
      r1[grp][cl] = s1 = s1 + r1[grp + h][cl];
      r2[grp][cl] = s2 = s2 + r2[grp + h][cl];
    }
    __syncthreads();
  }
}

template <typename P>
__global__ void __launch_bounds__(kFinC * kFinG) bn_fwd_finalize_kernel(
    const float2* __restrict__ partial, int64_t G, const uint16_t* __restrict__ x,
    const P* __restrict__ gamma, const P* __restrict__ beta, P* __restrict__ run_mean,
    P* __restrict__ run_var, float* __restrict__ mean, float* __restrict__ invstd,
    float* __restrict__ coef, int64_t M, int C, float eps, float momentum) {
  const int cl = threadIdx.x % kFinC, grp = threadIdx.x / kFinC;
  const int c = blockIdx.x * kFinC + cl;
  double s1, s2;
  merge_partials(partial, G, C, c, cl, grp, s1, s2);
  if (grp != 0 || c >= C) return;
  const double n = (double)M;
  const double m1 = s1 / n;
  double var = s2 / n - m1 * m1;
  if (var < 0.0) var = 0.0;
  const double mu = (x ? (double)bf2f(x[c]) : 0.0) + m1;  // x: the reduction's shift row (null: unshifted sums)
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  mean[c] = (float)mu;
  invstd[c] = is;
  const float s = ldp(gamma, c, 1.0f) * is;
  coef[c] = s;
  coef[C + c] = ldp(beta, c, 0.0f) - (float)mu * s;
  if (run_mean) {
    const float unbiased = (float)(M > 1 ? var * n / (n - 1.0) : var);
    stp(run_mean, c, (1.0f - momentum) * ldp(run_mean, c, 0.0f) + momentum * (float)mu);
    stp(run_var, c, (1.0f - momentum) * ldp(run_var, c, 0.0f) + momentum * unbiased);
  }
}

// dβ = Σ dz, dγ = Σ dz·x̂; dx = s·(dz - dβ/M - x̂·dγ/M) folded to s·dz + cc·x + b.
template <typename P>
__global__ void __launch_bounds__(kFinC * kFinG) bn_bwd_finalize_kernel(
    const float2* __restrict__ partial, int64_t G, const P* __restrict__ gamma,
    const P* __restrict__ beta, const float* __restrict__ mean, const float* __restrict__ invstd,
    P* __restrict__ dgamma, P* __restrict__ dbeta, float* __restrict__ coef, int64_t M, int C) {
  const int cl = threadIdx.x % kFinC, grp = threadIdx.x / kFinC;
  const int c = blockIdx.x * kFinC + cl;
  double s1, s2;
  merge_partials(partial, G, C, c, cl, grp, s1, s2);
  if (grp != 0 || c >= C) return;
  const float db = (float)s1, dg = (float)s2;
  if (dgamma) stp(dgamma, c, dg);
  if (dbeta) stp(dbeta, c, db);
  const float is = invstd[c], mu = mean[c];
  const float s = ldp(gamma, c, 1.0f) * is;
  const float inv_m = (float)(1.0 / (double)M);
  const float cc = -s * is * dg * inv_m;
  coef[c] = s;
  coef[C + c] = ldp(beta, c, 0.0f) - mu * s;
  coef[2 * C + c] = cc;
  coef[3 * C + c] = -s * db * inv_m - mu * cc;
}

#define VGPU_BN_GRID_LOOP(i, ci, nvec, cvec)                                       \
  const uint64_t stride_ = (uint64_t)gridDim.x * kThreads;                         \
  const uint32_t cstep_ = (uint32_t)(stride_ % (cvec));                            \
  uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;                      \
  uint32_t ci = (uint32_t)(i % (cvec));                                            \
  for (; i < (nvec); i += stride_, ci = (ci + cstep_ >= (cvec)) ? ci + cstep_ - (cvec) : ci + cstep_)

template <int kAct>
__global__ void __launch_bounds__(kThreads) bn_apply_kernel(const bf16x8* __restrict__ x,
                                                            bf16x8* __restrict__ y,
                                                            const float* __restrict__ coef,
                                                            uint64_t nvec, uint32_t cvec) {
  const float* sc = coef;
  const float* sh = coef + cvec * 8;
  VGPU_BN_GRID_LOOP(i, ci, nvec, cvec) {
    const bf16x8 v = x[i];
    float s[8], t[8];
    load8(sc + ci * 8, s);
    load8(sh + ci * 8, t);
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o.v[k] = f2bf(act_fwd<kAct>(fmaf(bf2f(v.v[k]), s[k], t[k])));
    y[i] = o;
  }
}

// kAdd: dx += add (a second gradient of x, e.g. the identity shortcut's),
// summed in fp32 before the one bf16 rounding — replaces an autograd add pass.
template <int kAct, bool kAdd>
__global__ void __launch_bounds__(kThreads) bn_bwd_apply_kernel(const bf16x8* __restrict__ dy,
                                                                const bf16x8* __restrict__ x,
                                                                bf16x8* __restrict__ dx,
                                                                const float* __restrict__ coef,
                                                                const bf16x8* __restrict__ add,
                                                                uint64_t nvec, uint32_t cvec) {
  const uint32_t C = cvec * 8;
  VGPU_BN_GRID_LOOP(i, ci, nvec, cvec) {
    const bf16x8 v = x[i];
    const bf16x8 g = dy[i];
    bf16x8 r;
    if constexpr (kAdd) r = add[i];
    float s[8], t[8], cc[8], b[8];
    load8(coef + ci * 8, s);
    load8(coef + C + ci * 8, t);
    load8(coef + 2 * C + ci * 8, cc);
    load8(coef + 3 * C + ci * 8, b);
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xf = bf2f(v.v[k]);
      const float dz = bf2f(g.v[k]) * act_grad<kAct>(fmaf(xf, s[k], t[k]));
      float d = fmaf(s[k], dz, fmaf(cc[k], xf, b[k]));
      if constexpr (kAdd) d += bf2f(r.v[k]);
      o.v[k] = f2bf(d);
    }
    dx[i] = o;
  }
}

// ---- finalize + apply in one launch for small layers ------------------------------
// With the statistics from the conv epilogues (G = ceil(M / 64) pairs per
// channel), a small layer's finalize is a ~5 µs launch of its own for a few µs
// of apply: ResNet-V2-152 b=10 runs 300 of them per step, 14 % of its GPU time
// (profiles/r4/train/bnfuse/).  Here every workgroup of the apply owns a
// 64-channel chunk and a row range, merges that chunk's G pairs itself (fp64,
// the same sums the finalize forms) and applies; row range 0 also writes the
// saved statistics / running stats (forward) or dγ, dβ (backward).  Used when
// G <= kFuseMaxG, so the redundant merges stay a fraction of the apply's bytes.
constexpr int kFuseMaxG = 160;
constexpr int kFuseC = 64;
constexpr int kFuseT = 1024;               // 16 lanes per channel: ≤ 10 pair loads each at G = 160
constexpr int kFuseQ = kFuseT / kFuseC;

__device__ __forceinline__ void merge_chunk(const float2* __restrict__ partial, int64_t G, int C, int c0,
                                            double (&r1)[kFuseQ][kFuseC], double (&r2)[kFuseQ][kFuseC]) {
  const int cl = threadIdx.x & (kFuseC - 1), q = threadIdx.x >> 6;
  double s1 = 0.0, s2 = 0.0;
#pragma unroll 4
  for (int64_t g = q; g < G; g += kFuseQ) {
    const float2 p = partial[g * C + c0 + cl];
    s1 += p.x;
    s2 += p.y;
  }
  r1[q][cl] = s1;
  r2[q][cl] = s2;
  __syncthreads();
}

// shift: the reduction's shift row (x row 0; the plain path's bn_reduce_kernel
// sums x - x0), null for the conv epilogues' unshifted sums.  coef (s, t at
// [0, C) and [C, 2C)), mean and invstd outputs are each nullable.
template <int kAct, typename P>
__global__ void __launch_bounds__(kFuseT) bn_fwd_fused_kernel(
    const float2* __restrict__ partial, int64_t G, const bf16x8* __restrict__ x, bf16x8* __restrict__ y,
    const P* __restrict__ gamma, const P* __restrict__ beta, P* __restrict__ run_mean, P* __restrict__ run_var,
    float* __restrict__ coef, float* __restrict__ mean_out, float* __restrict__ invstd_out,
    const uint16_t* __restrict__ shift, int64_t M, int C, float eps, float momentum, int64_t rows_per,
    const bf16x8* __restrict__ add = nullptr) {
  __shared__ double r1[kFuseQ][kFuseC], r2[kFuseQ][kFuseC];
  __shared__ float sS[kFuseC], sT[kFuseC];
  const int c0 = blockIdx.x * kFuseC;
  merge_chunk(partial, G, C, c0, r1, r2);
  if (threadIdx.x < kFuseC) {
    const int c = c0 + threadIdx.x;
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int q = 0; q < kFuseQ; ++q) {
      s1 += r1[q][threadIdx.x];
      s2 += r2[q][threadIdx.x];
    }
    const double n = (double)M, m1 = s1 / n;
    double var = s2 / n - m1 * m1;
    if (var < 0.0) var = 0.0;
    const double mu = (shift ? (double)bf2f(shift[c]) : 0.0) + m1;
    const float is = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = ldp(gamma, c, 1.0f) * is, sh = ldp(beta, c, 0.0f) - (float)mu * sc;
    sS[threadIdx.x] = sc;
    sT[threadIdx.x] = sh;
    if (blockIdx.y == 0) {
      if (coef) {
        coef[c] = sc;
        coef[C + c] = sh;
      }
      if (mean_out) mean_out[c] = (float)mu;
      if (invstd_out) invstd_out[c] = is;
      if (run_mean) {
        const float unbiased = (float)(M > 1 ? var * n / (n - 1.0) : var);
        stp(run_mean, c, (1.0f - momentum) * ldp(run_mean, c, 0.0f) + momentum * (float)mu);
        stp(run_var, c, (1.0f - momentum) * ldp(run_var, c, 0.0f) + momentum * unbiased);
      }
    }
  }
  __syncthreads();
  const int cg = threadIdx.x & 7, ro = threadIdx.x >> 3;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = sS[cg * 8 + j];
    sh[j] = sT[cg * 8 + j];
  }
  const int cvec = C >> 3, cv = (c0 >> 3) + cg;
  const int64_t r_end = (int64_t)(blockIdx.y + 1) * rows_per < M ? (int64_t)(blockIdx.y + 1) * rows_per : M;
  for (int64_t r = (int64_t)blockIdx.y * rows_per + ro; r < r_end; r += kFuseT / 8) {
    const bf16x8 v = x[r * cvec + cv];
    bf16x8 o;
    if (add) {
      const bf16x8 a = add[r * cvec + cv];
#pragma unroll
      for (int k = 0; k < 8; ++k) o.v[k] = f2bf(act_fwd<kAct>(fmaf(bf2f(v.v[k]), sc[k], sh[k])) + bf2f(a.v[k]));
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) o.v[k] = f2bf(act_fwd<kAct>(fmaf(bf2f(v.v[k]), sc[k], sh[k])));
    }
    y[r * cvec + cv] = o;
  }
}

// kAct == 0: dz already carries act' (the data-gradient epilogue applied it);
// else dz = dy·act'(x·s + t) here (the plain path's reduction partials).
// dx = s·dz + cc·x + b (+ add).
template <int kAct, bool kAdd, typename P>
__global__ void __launch_bounds__(kFuseT) bn_bwd_fused_kernel(
    const float2* __restrict__ partial, int64_t G, const bf16x8* __restrict__ dz, const bf16x8* __restrict__ x,
    bf16x8* __restrict__ dx, const bf16x8* __restrict__ add, const P* __restrict__ gamma, const P* __restrict__ beta,
    const float* __restrict__ mean, const float* __restrict__ invstd, P* __restrict__ dgamma, P* __restrict__ dbeta,
    int64_t M, int C, int64_t rows_per) {
  __shared__ double r1[kFuseQ][kFuseC], r2[kFuseQ][kFuseC];
  __shared__ float sS[kFuseC], sC[kFuseC], sB[kFuseC], sT[kFuseC];
  const int c0 = blockIdx.x * kFuseC;
  merge_chunk(partial, G, C, c0, r1, r2);
  if (threadIdx.x < kFuseC) {
    const int c = c0 + threadIdx.x;
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int q = 0; q < kFuseQ; ++q) {
      s1 += r1[q][threadIdx.x];
      s2 += r2[q][threadIdx.x];
    }
    const float db = (float)s1, dg = (float)s2;
    if (blockIdx.y == 0) {
      if (dgamma) stp(dgamma, c, dg);
      if (dbeta) stp(dbeta, c, db);
    }
    const float is = invstd[c], mu = mean[c];
    const float sc = ldp(gamma, c, 1.0f) * is;
    const float inv_m = (float)(1.0 / (double)M);
    const float cc = -sc * is * dg * inv_m;
    sS[threadIdx.x] = sc;
    sC[threadIdx.x] = cc;
    sB[threadIdx.x] = -sc * db * inv_m - mu * cc;
    sT[threadIdx.x] = ldp(beta, c, 0.0f) - mu * sc;
  }
  __syncthreads();
  const int cg = threadIdx.x & 7, ro = threadIdx.x >> 3;
  float sc[8], cc[8], bb[8], tt[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = sS[cg * 8 + j];
    cc[j] = sC[cg * 8 + j];
    bb[j] = sB[cg * 8 + j];
    tt[j] = sT[cg * 8 + j];
  }
  const int cvec = C >> 3, cv = (c0 >> 3) + cg;
  const int64_t r_end = (int64_t)(blockIdx.y + 1) * rows_per < M ? (int64_t)(blockIdx.y + 1) * rows_per : M;
  for (int64_t r = (int64_t)blockIdx.y * rows_per + ro; r < r_end; r += kFuseT / 8) {
    const int64_t i = r * cvec + cv;
    const bf16x8 v = x[i], g = dz[i];
    bf16x8 rr;
    if constexpr (kAdd) rr = add[i];
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xf = bf2f(v.v[k]);
      float gz = bf2f(g.v[k]);
      if constexpr (kAct != 0) gz *= act_grad<kAct>(fmaf(xf, sc[k], tt[k]));
      float d = fmaf(sc[k], gz, fmaf(cc[k], xf, bb[k]));
      if constexpr (kAdd) d += bf2f(rr.v[k]);
      o.v[k] = f2bf(d);
    }
    dx[i] = o;
  }
}

// ---- one launch per BatchNorm direction for small layers --------------------------
// DeepLab-v3 4.2 (b=1, 384²) runs 46 of its 56 BatchNorms on 24² / 48² maps
// (576 / 2304 rows): there a reduce, a finalize and an apply were three ~4.7 us
// launches for well under a microsecond of memory traffic each, 1/3 of the
// step's dispatches (profiles/r6/train).  Here one 1024-thread workgroup owns a
// 64-channel chunk and ALL its rows: it reduces (shifted sums as
// bn_reduce_kernel, fp32 per thread, 8-row wave shuffles, fp64 across the 16
// waves), finalizes, and applies from the same registers: a thread loads its
// kSmallR rows once, all in flight together (a first version re-read them in
// a row loop: 8.5 / 15.7 us forward / backward at 576 rows, latency-bound,
// profiles/r6/train).  32-channel chunks (4 lanes a row, 64-byte runs): twice
// the workgroups of 64-channel ones, half the rows' latency chain each (the
// 64-channel backward took 10.4 us at 576 rows).  Rows <= kSmallMaxM (768:
// DeepLab's 24² maps).
constexpr int kSC = 32, kSL = kSC / 8;  // channels per workgroup, lanes per row
constexpr int kSmallR = 3;
constexpr int64_t kSmallMaxM = (int64_t)kSmallR * (kFuseT / kSL);  // 768
// The backward holds x and dy: 512 threads (a 256-VGPR budget), 6 rows each.
constexpr int kSmallBT = 512, kSmallBR = 6;
static_assert((int64_t)kSmallBR * (kSmallBT / kSL) == kSmallMaxM, "backward covers the same rows");

__device__ __forceinline__ void wave_rows_reduce(float (&a1)[8], float (&a2)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int o = kSL; o < 64; o <<= 1) {  // lanes cg + kSL·row: xor over the row bits
      a1[j] += __shfl_xor(a1[j], o, 64);
      a2[j] += __shfl_xor(a2[j], o, 64);
    }
}

// add (nullable): y = act(bn(x)) + add, an identity shortcut summed in the
// same pass (MobileNet-V2's project BN + residual; its gradient is dy itself).
template <int kAct, typename P>
__global__ void __launch_bounds__(kFuseT) bn_fwd_small_kernel(
    const bf16x8* __restrict__ x, bf16x8* __restrict__ y, const P* __restrict__ gamma, const P* __restrict__ beta,
    P* __restrict__ run_mean, P* __restrict__ run_var, float* __restrict__ mean, float* __restrict__ invstd,
    float* __restrict__ coef, int64_t M, int C, float eps, float momentum, const bf16x8* __restrict__ add) {
  __shared__ float2 red[kFuseT / 64][kSC];
  __shared__ float sS[kSC], sT[kSC];
  const int cg = threadIdx.x % kSL, ro = threadIdx.x / kSL, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = blockIdx.x * kSC;
  const int cvec = C >> 3, cv = (c0 >> 3) + cg;
  float k0[8], a1[8], a2[8];
  bf16x8 v[kSmallR];
#pragma unroll
  for (int u = 0; u < kSmallR; ++u) {  // rows past M read row 0: shifted, they add 0
    const int64_t r = ro + u * (kFuseT / kSL);
    v[u] = x[(r < M ? r : 0) * cvec + cv];
  }
  const bf16x8 v0 = x[cv];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k0[j] = bf2f(v0.v[j]);
    a1[j] = a2[j] = 0.0f;
  }
#pragma unroll
  for (int u = 0; u < kSmallR; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = bf2f(v[u].v[j]) - k0[j];
      a1[j] += d;
      a2[j] = fmaf(d, d, a2[j]);
    }
  wave_rows_reduce(a1, a2);
  if (lane < kSL)
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wave][lane * 8 + j] = make_float2(a1[j], a2[j]);
  __syncthreads();
  if (threadIdx.x < kSC) {
    const int c = c0 + threadIdx.x;
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int w = 0; w < kFuseT / 64; ++w) {
      s1 += red[w][threadIdx.x].x;
      s2 += red[w][threadIdx.x].y;
    }
    const double n = (double)M, m1 = s1 / n;
    double var = s2 / n - m1 * m1;
    if (var < 0.0) var = 0.0;
    const double mu = (double)bf2f(reinterpret_cast<const uint16_t*>(x)[c]) + m1;
    const float is = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = ldp(gamma, c, 1.0f) * is, sh = ldp(beta, c, 0.0f) - (float)mu * sc;
    sS[threadIdx.x] = sc;
    sT[threadIdx.x] = sh;
    mean[c] = (float)mu;
    invstd[c] = is;
    if (coef) {
      coef[c] = sc;
      coef[C + c] = sh;
    }
    if (run_mean) {
      const float unbiased = (float)(M > 1 ? var * n / (n - 1.0) : var);
      stp(run_mean, c, (1.0f - momentum) * ldp(run_mean, c, 0.0f) + momentum * (float)mu);
      stp(run_var, c, (1.0f - momentum) * ldp(run_var, c, 0.0f) + momentum * unbiased);
    }
  }
  __syncthreads();
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = sS[cg * 8 + j];
    sh[j] = sT[cg * 8 + j];
  }
#pragma unroll
  for (int u = 0; u < kSmallR; ++u) {
    const int64_t r = ro + u * (kFuseT / kSL);
    if (r >= M) break;
    bf16x8 o;
    if (add) {
      const bf16x8 a = add[r * cvec + cv];
#pragma unroll
      for (int k = 0; k < 8; ++k) o.v[k] = f2bf(act_fwd<kAct>(fmaf(bf2f(v[u].v[k]), sc[k], sh[k])) + bf2f(a.v[k]));
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) o.v[k] = f2bf(act_fwd<kAct>(fmaf(bf2f(v[u].v[k]), sc[k], sh[k])));
    }
    y[r * cvec + cv] = o;
  }
}

// Σ dz, Σ dz·x̂ (dz = dy·act'(x·s + t)), dγ / dβ, then dx = s·dz + cc·x + b (+ add):
// bn_reduce_kernel<1> + bn_bwd_finalize_kernel + bn_bwd_apply_kernel in one launch.
template <int kAct, bool kAdd, typename P>
__global__ void __launch_bounds__(kSmallBT) bn_bwd_small_kernel(
    const bf16x8* __restrict__ dy, const bf16x8* __restrict__ x, bf16x8* __restrict__ dx,
    const bf16x8* __restrict__ add, const P* __restrict__ gamma, const P* __restrict__ beta,
    const float* __restrict__ mean, const float* __restrict__ invstd, P* __restrict__ dgamma,
    P* __restrict__ dbeta, int64_t M, int C) {
  __shared__ float2 red[kSmallBT / 64][kSC];
  __shared__ float sC[kSC], sB[kSC];
  const int cg = threadIdx.x % kSL, ro = threadIdx.x / kSL, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = blockIdx.x * kSC;
  const int cvec = C >> 3, cv = (c0 >> 3) + cg;
  float sc[8], sh[8], mu[8], is[8], a1[8], a2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = c0 + cg * 8 + j;
    is[j] = invstd[c];
    mu[j] = mean[c];
    sc[j] = ldp(gamma, c, 1.0f) * is[j];
    sh[j] = ldp(beta, c, 0.0f) - mu[j] * sc[j];
    a1[j] = a2[j] = 0.0f;
  }
  bf16x8 v[kSmallBR], g[kSmallBR];
#pragma unroll
  for (int u = 0; u < kSmallBR; ++u) {
    const int64_t r = ro + u * (kSmallBT / kSL);
    const int64_t i = (r < M ? r : 0) * cvec + cv;
    v[u] = x[i];
    g[u] = dy[i];
  }
#pragma unroll
  for (int u = 0; u < kSmallBR; ++u) {
    const float ok = ro + u * (kSmallBT / kSL) < M ? 1.0f : 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xf = bf2f(v[u].v[j]);
      const float dz = bf2f(g[u].v[j]) * act_grad<kAct>(fmaf(xf, sc[j], sh[j])) * ok;
      a1[j] += dz;
      a2[j] = fmaf(dz, (xf - mu[j]) * is[j], a2[j]);
    }
  }
  wave_rows_reduce(a1, a2);
  if (lane < kSL)
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wave][lane * 8 + j] = make_float2(a1[j], a2[j]);
  __syncthreads();
  if (threadIdx.x < kSC) {
    const int c = c0 + threadIdx.x;
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int w = 0; w < kSmallBT / 64; ++w) {
      s1 += red[w][threadIdx.x].x;
      s2 += red[w][threadIdx.x].y;
    }
    const float db = (float)s1, dg = (float)s2;
    if (dgamma) stp(dgamma, c, dg);
    if (dbeta) stp(dbeta, c, db);
    const float isc = invstd[c];
    const float s_ = ldp(gamma, c, 1.0f) * isc;
    const float inv_m = (float)(1.0 / (double)M);
    const float cc = -s_ * isc * dg * inv_m;
    sC[threadIdx.x] = cc;
    sB[threadIdx.x] = -s_ * db * inv_m - mean[c] * cc;
  }
  __syncthreads();
  float cc[8], bb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    cc[j] = sC[cg * 8 + j];
    bb[j] = sB[cg * 8 + j];
  }
#pragma unroll
  for (int u = 0; u < kSmallBR; ++u) {
    const int64_t r = ro + u * (kSmallBT / kSL);
    if (r >= M) break;
    const int64_t i = r * cvec + cv;
    bf16x8 rr;
    if constexpr (kAdd) rr = add[i];
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xf = bf2f(v[u].v[k]);
      const float dz = bf2f(g[u].v[k]) * act_grad<kAct>(fmaf(xf, sc[k], sh[k]));
      float d = fmaf(sc[k], dz, fmaf(cc[k], xf, bb[k]));
      if constexpr (kAdd) d += bf2f(rr.v[k]);
      o.v[k] = f2bf(d);
    }
    dx[i] = o;
  }
}

// Row ranges per 64-channel chunk: ~one workgroup per CU over the layer, at
// least 128 rows (one pass of the 1024 threads) each.
inline dim3 fused_grid(int64_t M, int C, int64_t& rows_per) {
  const int chunks = C / kFuseC;
  int64_t R = (256 + chunks - 1) / chunks;  // ~one 1024-thread workgroup per CU
  const int64_t rmax = (M + kFuseT / 8 - 1) / (kFuseT / 8);
  if (R > rmax) R = rmax;
  if (R < 1) R = 1;
  rows_per = (M + R - 1) / R;
  R = (M + rows_per - 1) / rows_per;
  return dim3((unsigned)chunks, (unsigned)R);
}

int g_fuse_small = -1;  // VGPU_BN_FUSE_SMALL=0 / vgpu_bn_set_fuse_small: separate finalize launches
inline bool fuse_on();
inline bool fused_ok(int64_t G, int C) { return fuse_on() && G <= kFuseMaxG && C % kFuseC == 0; }

// The plain path (statistics reduced here): kind 0 = reduce / finalize / apply
// (three launches), 1 = reduce + finalize-and-apply (bn_*_fused_kernel over the
// reduction's <= 128 partials, two launches), 2 = one bn_*_small_kernel launch.
inline bool fuse_on() {
  if (g_fuse_small < 0) {
    const char* v = getenv("VGPU_BN_FUSE_SMALL");
    g_fuse_small = (v && v[0] == '0') ? 0 : 1;
  }
  return g_fuse_small == 1;
}

inline int plain_kind(int64_t M, int C) {
  if (!fuse_on() || C % kFuseC) return 0;
  return M <= kSmallMaxM ? 2 : 1;
}

struct Plan {
  int chunk, nchunks, rpb, rows_per_block;
  int64_t G;
};

Plan make_plan(int64_t M, int C) {
  Plan p;
  p.chunk = C <= kMaxChunk ? C : kMaxChunk;
  p.nchunks = (C + p.chunk - 1) / p.chunk;
  p.rpb = kThreads / (p.chunk / 8);
  const int tb = plain_kind(M, C) == 1 ? 128 : g_target_blocks;  // kind 1: G <= 128 <= kFuseMaxG
  int64_t target = tb / p.nchunks;
  if (target < 1) target = 1;
  int64_t iters = (M + p.rpb * target - 1) / (p.rpb * target);
  iters = (iters + g_unroll - 1) / g_unroll * g_unroll;
  p.rows_per_block = (int)(p.rpb * iters);
  p.G = (M + p.rows_per_block - 1) / p.rows_per_block;
  return p;
}

inline unsigned grid_for(uint64_t nvec) {
  uint64_t g = (nvec + kThreads - 1) / kThreads;
  if (g < 1) g = 1;
  if (g > kMaxGrid) g = kMaxGrid;
  return (unsigned)g;
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

inline bool shape_ok(int64_t M, int C) { return M >= 1 && C >= 8 && C % 8 == 0 && M <= (int64_t)1 << 40; }

template <typename P>
int fwd_train(const void* x, void* y, const void* gamma, const void* beta, void* run_mean, void* run_var,
              float* mean, float* invstd, float* ws, int64_t M, int C, float eps, float momentum, int act,
              hipStream_t s, float* coef_out = nullptr, const void* add = nullptr) {
  const int kind = plain_kind(M, C);
  if (add && kind == 0) return -2;  // the three-pass plan has no add: the caller adds
  const auto* addv = static_cast<const bf16x8*>(add);
  const auto* xv = static_cast<const bf16x8*>(x);
  auto* yv = static_cast<bf16x8*>(y);
  const auto* g_ = static_cast<const P*>(gamma);
  const auto* b_ = static_cast<const P*>(beta);
  auto* rm = static_cast<P*>(run_mean);
  auto* rv = static_cast<P*>(run_var);
  if (kind == 2) {
    const dim3 grid((unsigned)(C / kSC));
    switch (act) {
      case 0: hipLaunchKernelGGL((bn_fwd_small_kernel<0, P>), grid, dim3(kFuseT), 0, s, xv, yv, g_, b_, rm, rv, mean, invstd, coef_out, M, C, eps, momentum, addv); break;
      case 1: hipLaunchKernelGGL((bn_fwd_small_kernel<1, P>), grid, dim3(kFuseT), 0, s, xv, yv, g_, b_, rm, rv, mean, invstd, coef_out, M, C, eps, momentum, addv); break;
      case 2: hipLaunchKernelGGL((bn_fwd_small_kernel<2, P>), grid, dim3(kFuseT), 0, s, xv, yv, g_, b_, rm, rv, mean, invstd, coef_out, M, C, eps, momentum, addv); break;
      default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
  }
  const Plan p = make_plan(M, C);
  auto* partial = reinterpret_cast<float2*>(ws);
  float* coef = coef_out ? coef_out : ws + 2 * p.G * C;  // s, t
  if (g_unroll == 8)
    hipLaunchKernelGGL((bn_reduce_kernel<0, 0, P, 8>), dim3((unsigned)p.G, p.nchunks), dim3(kThreads), 0, s, xv,
                       nullptr, nullptr, nullptr, nullptr, nullptr, partial, M, C, p.chunk, p.rows_per_block);
  else
    hipLaunchKernelGGL((bn_reduce_kernel<0, 0, P>), dim3((unsigned)p.G, p.nchunks), dim3(kThreads), 0, s, xv,
                       nullptr, nullptr, nullptr, nullptr, nullptr, partial, M, C, p.chunk, p.rows_per_block);
  if (kind == 1) {
    int64_t rows_per;
    const dim3 grid = fused_grid(M, C, rows_per);
    const auto* xs = static_cast<const uint16_t*>(x);
    switch (act) {
      case 0: hipLaunchKernelGGL((bn_fwd_fused_kernel<0, P>), grid, dim3(kFuseT), 0, s, partial, p.G, xv, yv, g_, b_, rm, rv, coef, mean, invstd, xs, M, C, eps, momentum, rows_per, addv); break;
      case 1: hipLaunchKernelGGL((bn_fwd_fused_kernel<1, P>), grid, dim3(kFuseT), 0, s, partial, p.G, xv, yv, g_, b_, rm, rv, coef, mean, invstd, xs, M, C, eps, momentum, rows_per, addv); break;
      case 2: hipLaunchKernelGGL((bn_fwd_fused_kernel<2, P>), grid, dim3(kFuseT), 0, s, partial, p.G, xv, yv, g_, b_, rm, rv, coef, mean, invstd, xs, M, C, eps, momentum, rows_per, addv); break;
      default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL((bn_fwd_finalize_kernel<P>), dim3((C + kFinC - 1) / kFinC), dim3(kFinC * kFinG), 0, s,
                     partial, p.G, static_cast<const uint16_t*>(x), g_, b_, rm, rv, mean, invstd, coef, M, C, eps,
                     momentum);
  const uint64_t nvec = (uint64_t)M * (C / 8);
  switch (act) {
    case 0: hipLaunchKernelGGL(bn_apply_kernel<0>, dim3(grid_for(nvec)), dim3(kThreads), 0, s, xv, yv, coef, nvec, C / 8); break;
    case 1: hipLaunchKernelGGL(bn_apply_kernel<1>, dim3(grid_for(nvec)), dim3(kThreads), 0, s, xv, yv, coef, nvec, C / 8); break;
    case 2: hipLaunchKernelGGL(bn_apply_kernel<2>, dim3(grid_for(nvec)), dim3(kThreads), 0, s, xv, yv, coef, nvec, C / 8); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

template <int kAct, typename P>
void bwd_launch(const bf16x8* dyv, const bf16x8* xv, bf16x8* dxv, const P* gamma, const P* beta,
                const float* mean, const float* invstd, P* dgamma, P* dbeta, float* ws, int64_t M, int C,
                const bf16x8* addv, hipStream_t s) {
  const int kind = plain_kind(M, C);
  if (kind == 2) {
    const dim3 grid((unsigned)(C / kSC));
    if (addv)
      hipLaunchKernelGGL((bn_bwd_small_kernel<kAct, true, P>), grid, dim3(kSmallBT), 0, s, dyv, xv, dxv, addv, gamma,
                         beta, mean, invstd, dgamma, dbeta, M, C);
    else
      hipLaunchKernelGGL((bn_bwd_small_kernel<kAct, false, P>), grid, dim3(kSmallBT), 0, s, dyv, xv, dxv, addv, gamma,
                         beta, mean, invstd, dgamma, dbeta, M, C);
    return;
  }
  const Plan p = make_plan(M, C);
  auto* partial = reinterpret_cast<float2*>(ws);
  float* coef = ws + 2 * p.G * C;
  if (g_unroll == 8)
    hipLaunchKernelGGL((bn_reduce_kernel<1, kAct, P, 8>), dim3((unsigned)p.G, p.nchunks), dim3(kThreads), 0, s,
                       xv, dyv, gamma, beta, mean, invstd, partial, M, C, p.chunk, p.rows_per_block);
  else
    hipLaunchKernelGGL((bn_reduce_kernel<1, kAct, P>), dim3((unsigned)p.G, p.nchunks), dim3(kThreads), 0, s,
                       xv, dyv, gamma, beta, mean, invstd, partial, M, C, p.chunk, p.rows_per_block);
  if (kind == 1) {
    int64_t rows_per;
    const dim3 grid = fused_grid(M, C, rows_per);
    if (addv)
      hipLaunchKernelGGL((bn_bwd_fused_kernel<kAct, true, P>), grid, dim3(kFuseT), 0, s, partial, p.G, dyv, xv, dxv,
                         addv, gamma, beta, mean, invstd, dgamma, dbeta, M, C, rows_per);
    else
      hipLaunchKernelGGL((bn_bwd_fused_kernel<kAct, false, P>), grid, dim3(kFuseT), 0, s, partial, p.G, dyv, xv,
                         dxv, addv, gamma, beta, mean, invstd, dgamma, dbeta, M, C, rows_per);
    return;
  }
  hipLaunchKernelGGL((bn_bwd_finalize_kernel<P>), dim3((C + kFinC - 1) / kFinC), dim3(kFinC * kFinG), 0, s,
                     partial, p.G, gamma, beta, mean, invstd, dgamma, dbeta, coef, M, C);
  const uint64_t nvec = (uint64_t)M * (C / 8);
  if (addv)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<kAct, true>), dim3(grid_for(nvec)), dim3(kThreads), 0, s, dyv, xv,
                       dxv, coef, addv, nvec, C / 8);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<kAct, false>), dim3(grid_for(nvec)), dim3(kThreads), 0, s, dyv, xv,
                       dxv, coef, addv, nvec, C / 8);
}

template <typename P>
int bwd(const void* dy, const void* x, void* dx, const void* gamma, const void* beta, const float* mean,
        const float* invstd, void* dgamma, void* dbeta, float* ws, int64_t M, int C, int act, const void* add,
        hipStream_t s) {
  const auto* addv = static_cast<const bf16x8*>(add);
  const auto* dyv = static_cast<const bf16x8*>(dy);
  const auto* xv = static_cast<const bf16x8*>(x);
  auto* dxv = static_cast<bf16x8*>(dx);
  const auto* g = static_cast<const P*>(gamma);
  const auto* b = static_cast<const P*>(beta);
  auto* dg = static_cast<P*>(dgamma);
  auto* db = static_cast<P*>(dbeta);
  switch (act) {
    case 0: bwd_launch<0, P>(dyv, xv, dxv, g, b, mean, invstd, dg, db, ws, M, C, addv, s); break;
    case 1: bwd_launch<1, P>(dyv, xv, dxv, g, b, mean, invstd, dg, db, ws, M, C, addv, s); break;
    case 2: bwd_launch<2, P>(dyv, xv, dxv, g, b, mean, invstd, dg, db, ws, M, C, addv, s); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace

// fp32 workspace elements vgpu_bn_act_fwd_train / vgpu_bn_act_bwd need for
// M = N·H·W rows of C channels (block partials + folded coefficients).
VGPU_API int64_t vgpu_bn_workspace(int64_t M, int C) {
  if (!shape_ok(M, C)) return -1;
  return 2 * make_plan(M, C).G * C + 4 * (int64_t)C;
}

// y = act(batchnorm_train(x)); saves mean / invstd (fp32 [C]); updates the
// running stats (unbiased variance, PyTorch momentum convention) when given.
// gamma / beta / running stats: fp32, or bf16 when param_bf16; any may be null
// (affine=False, track_running_stats=False).  act: 0 none, 1 relu, 2 relu6.
VGPU_API int vgpu_bn_act_fwd_train(const void* x, void* y, const void* gamma, const void* beta, void* run_mean,
                                   void* run_var, float* mean, float* invstd, float* ws, int64_t M, int C,
                                   float eps, float momentum, int act, int param_bf16, void* stream) {
  if (!shape_ok(M, C) || !aligned16(x) || !aligned16(y) || !aligned16(ws) || !mean || !invstd ||
      (!run_mean) != (!run_var))
    return (int)hipErrorInvalidValue;
  auto s = (hipStream_t)stream;
  if (param_bf16)
    return fwd_train<uint16_t>(x, y, gamma, beta, run_mean, run_var, mean, invstd, ws, M, C, eps, momentum, act, s);
  return fwd_train<float>(x, y, gamma, beta, run_mean, run_var, mean, invstd, ws, M, C, eps, momentum, act, s);
}

// y = act(batchnorm_train(x)) + add (add: bf16 like y, same layout).  -2
// when this shape's plan has no add form (the three-pass path: C % 64 != 0 or
// VGPU_BN_FUSE_SMALL=0); nothing was launched then.
VGPU_API int vgpu_bn_act_fwd_train_add(const void* x, void* y, const void* gamma, const void* beta, void* run_mean,
                                       void* run_var, float* mean, float* invstd, float* ws, int64_t M, int C,
                                       float eps, float momentum, int act, int param_bf16, const void* add,
                                       void* stream) {
  if (!shape_ok(M, C) || !aligned16(x) || !aligned16(y) || !aligned16(ws) || !mean || !invstd ||
      (!run_mean) != (!run_var) || !add || !aligned16(add))
    return (int)hipErrorInvalidValue;
  auto s = (hipStream_t)stream;
  if (param_bf16)
    return fwd_train<uint16_t>(x, y, gamma, beta, run_mean, run_var, mean, invstd, ws, M, C, eps, momentum, act, s,
                               nullptr, add);
  return fwd_train<float>(x, y, gamma, beta, run_mean, run_var, mean, invstd, ws, M, C, eps, momentum, act, s, nullptr,
                          add);
}

// dx, dgamma, dbeta of y = act(batchnorm_train(x)) given dy and the saved
// mean / invstd.  dgamma / dbeta may be null.
// `add` (nullable, bf16 like dx): a second gradient of x summed into dx.
VGPU_API int vgpu_bn_act_bwd_add(const void* dy, const void* x, void* dx, const void* gamma, const void* beta,
                                 const float* mean, const float* invstd, void* dgamma, void* dbeta, float* ws,
                                 int64_t M, int C, int act, int param_bf16, const void* add, void* stream) {
  if (!shape_ok(M, C) || !aligned16(dy) || !aligned16(x) || !aligned16(dx) || !aligned16(ws) || !mean ||
      !invstd || (add && !aligned16(add)))
    return (int)hipErrorInvalidValue;
  auto s = (hipStream_t)stream;
  if (param_bf16) return bwd<uint16_t>(dy, x, dx, gamma, beta, mean, invstd, dgamma, dbeta, ws, M, C, act, add, s);
  return bwd<float>(dy, x, dx, gamma, beta, mean, invstd, dgamma, dbeta, ws, M, C, act, add, s);
}

VGPU_API int vgpu_bn_act_bwd(const void* dy, const void* x, void* dx, const void* gamma, const void* beta,
                             const float* mean, const float* invstd, void* dgamma, void* dbeta, float* ws,
                             int64_t M, int C, int act, int param_bf16, void* stream) {
  return vgpu_bn_act_bwd_add(dy, x, dx, gamma, beta, mean, invstd, dgamma, dbeta, ws, M, C, act, param_bf16,
                             nullptr, stream);
}

// A/B of the reduction's shape (vgpu.bench.bnab): workgroups targeted over the
// chip and rows in flight per thread (4 or 8).  Call before sizing workspaces.
// ---- statistics from the producing / consuming convolution's epilogue ------------------
// (native/kernels/conv_gemm.hip vgpu_conv2d_nhwc_bn): `partial` holds G = ceil(M / 64)
// fp32 pairs per channel, [G][C], so no reduction pass over the activation runs here.

// Forward from (Σ x, Σ x²) pairs: finalize (mean / invstd, running stats) + apply.
// coef: fp32 [4][C] out = s, t, mean, invstd (what the backward's fused epilogue reads).
VGPU_API int vgpu_bn_act_fwd_partials(const float* partial, int64_t G, const void* x, void* y, const void* gamma,
                                      const void* beta, void* run_mean, void* run_var, float* coef, int64_t M,
                                      int C, float eps, float momentum, int act, int param_bf16, void* stream) {
  if (!shape_ok(M, C) || !partial || G != (M + 63) / 64 || !aligned16(x) || !aligned16(y) || !aligned16(coef) ||
      (!run_mean) != (!run_var) || act < 0 || act > 2)
    return (int)hipErrorInvalidValue;
  auto s = (hipStream_t)stream;
  const auto* pp = reinterpret_cast<const float2*>(partial);
  float* mean = coef + 2 * C;
  float* invstd = coef + 3 * C;
  if (fused_ok(G, C)) {
    int64_t rows_per;
    const dim3 grid = fused_grid(M, C, rows_per);
    const auto* xv = static_cast<const bf16x8*>(x);
    auto* yv = static_cast<bf16x8*>(y);
#define VGPU_BN_FWD_FUSED(A, P_)                                                                                   \
  hipLaunchKernelGGL((bn_fwd_fused_kernel<A, P_>), grid, dim3(kFuseT), 0, s, pp, G, xv, yv,                      \
                     static_cast<const P_*>(gamma), static_cast<const P_*>(beta), static_cast<P_*>(run_mean),      \
                     static_cast<P_*>(run_var), coef, mean, invstd, nullptr, M, C, eps, momentum, rows_per)
    if (param_bf16) {
      if (act == 0) VGPU_BN_FWD_FUSED(0, uint16_t); else if (act == 1) VGPU_BN_FWD_FUSED(1, uint16_t); else VGPU_BN_FWD_FUSED(2, uint16_t);
    } else {
      if (act == 0) VGPU_BN_FWD_FUSED(0, float); else if (act == 1) VGPU_BN_FWD_FUSED(1, float); else VGPU_BN_FWD_FUSED(2, float);
    }
#undef VGPU_BN_FWD_FUSED
    return (int)hipGetLastError();
  }
  const dim3 fg((C + kFinC - 1) / kFinC), fb(kFinC * kFinG);
  if (param_bf16)
    hipLaunchKernelGGL((bn_fwd_finalize_kernel<uint16_t>), fg, fb, 0, s, pp, G, nullptr,
                       static_cast<const uint16_t*>(gamma), static_cast<const uint16_t*>(beta),
                       static_cast<uint16_t*>(run_mean), static_cast<uint16_t*>(run_var), mean, invstd, coef, M, C,
                       eps, momentum);
  else
    hipLaunchKernelGGL((bn_fwd_finalize_kernel<float>), fg, fb, 0, s, pp, G, nullptr,
                       static_cast<const float*>(gamma), static_cast<const float*>(beta),
                       static_cast<float*>(run_mean), static_cast<float*>(run_var), mean, invstd, coef, M, C, eps,
                       momentum);
  const uint64_t nvec = (uint64_t)M * (C / 8);
  const auto* xv = static_cast<const bf16x8*>(x);
  auto* yv = static_cast<bf16x8*>(y);
  switch (act) {
    case 0: hipLaunchKernelGGL(bn_apply_kernel<0>, dim3(grid_for(nvec)), dim3(kThreads), 0, s, xv, yv, coef, nvec, C / 8); break;
    case 1: hipLaunchKernelGGL(bn_apply_kernel<1>, dim3(grid_for(nvec)), dim3(kThreads), 0, s, xv, yv, coef, nvec, C / 8); break;
    default: hipLaunchKernelGGL(bn_apply_kernel<2>, dim3(grid_for(nvec)), dim3(kThreads), 0, s, xv, yv, coef, nvec, C / 8); break;
  }
  return (int)hipGetLastError();
}

// The unfused forward (reduction pass) that also leaves s, t, mean, invstd in
// coef [4][C] (mean / invstd are coef + 2C / + 3C); ws as vgpu_bn_act_fwd_train.
VGPU_API int vgpu_bn_act_fwd_train_coef(const void* x, void* y, const void* gamma, const void* beta, void* run_mean,
                                        void* run_var, float* coef, float* ws, int64_t M, int C, float eps,
                                        float momentum, int act, int param_bf16, void* stream) {
  if (!shape_ok(M, C) || !coef || !aligned16(coef) || !aligned16(x) || !aligned16(y) || !aligned16(ws) ||
      (!run_mean) != (!run_var))
    return (int)hipErrorInvalidValue;
  auto s = (hipStream_t)stream;
  if (param_bf16)
    return fwd_train<uint16_t>(x, y, gamma, beta, run_mean, run_var, coef + 2 * C, coef + 3 * C, ws, M, C, eps,
                               momentum, act, s, coef);
  return fwd_train<float>(x, y, gamma, beta, run_mean, run_var, coef + 2 * C, coef + 3 * C, ws, M, C, eps, momentum,
                          act, s, coef);
}

// Backward from (Σ dz, Σ dz·x̂) pairs, dz = dy·act'(·) already applied by the
// data-gradient epilogue: finalize (dγ, dβ, folded coefficients) + dx = s·dz + cc·x + b
// (+ add).  ws: 4·C fp32.
VGPU_API int vgpu_bn_bwd_partials(const float* partial, int64_t G, const void* dz, const void* x, void* dx,
                                  const void* gamma, const void* beta, const float* mean, const float* invstd,
                                  void* dgamma, void* dbeta, float* ws, int64_t M, int C, int param_bf16,
                                  const void* add, void* stream) {
  if (!shape_ok(M, C) || !partial || G != (M + 63) / 64 || !aligned16(dz) || !aligned16(x) || !aligned16(dx) ||
      !aligned16(ws) || !mean || !invstd || (add && !aligned16(add)))
    return (int)hipErrorInvalidValue;
  auto s = (hipStream_t)stream;
  const auto* pp = reinterpret_cast<const float2*>(partial);
  if (fused_ok(G, C)) {
    int64_t rows_per;
    const dim3 grid = fused_grid(M, C, rows_per);
    const auto* dzv = static_cast<const bf16x8*>(dz);
    const auto* xv = static_cast<const bf16x8*>(x);
    auto* dxv = static_cast<bf16x8*>(dx);
    const auto* addv = static_cast<const bf16x8*>(add);
#define VGPU_BN_BWD_FUSED(K, P_)                                                                                   \
  hipLaunchKernelGGL((bn_bwd_fused_kernel<0, K, P_>), grid, dim3(kFuseT), 0, s, pp, G, dzv, xv, dxv, addv,       \
                     static_cast<const P_*>(gamma), static_cast<const P_*>(beta), mean, invstd,                     \
                     static_cast<P_*>(dgamma), static_cast<P_*>(dbeta), M, C, rows_per)
    if (param_bf16) {
      if (addv) VGPU_BN_BWD_FUSED(true, uint16_t); else VGPU_BN_BWD_FUSED(false, uint16_t);
    } else {
      if (addv) VGPU_BN_BWD_FUSED(true, float); else VGPU_BN_BWD_FUSED(false, float);
    }
#undef VGPU_BN_BWD_FUSED
    return (int)hipGetLastError();
  }
  const dim3 fg((C + kFinC - 1) / kFinC), fb(kFinC * kFinG);
  if (param_bf16)
    hipLaunchKernelGGL((bn_bwd_finalize_kernel<uint16_t>), fg, fb, 0, s, pp, G,
                       static_cast<const uint16_t*>(gamma), static_cast<const uint16_t*>(beta), mean, invstd,
                       static_cast<uint16_t*>(dgamma), static_cast<uint16_t*>(dbeta), ws, M, C);
  else
    hipLaunchKernelGGL((bn_bwd_finalize_kernel<float>), fg, fb, 0, s, pp, G, static_cast<const float*>(gamma),
                       static_cast<const float*>(beta), mean, invstd, static_cast<float*>(dgamma),
                       static_cast<float*>(dbeta), ws, M, C);
  const uint64_t nvec = (uint64_t)M * (C / 8);
  const auto* dzv = static_cast<const bf16x8*>(dz);
  const auto* xv = static_cast<const bf16x8*>(x);
  auto* dxv = static_cast<bf16x8*>(dx);
  const auto* addv = static_cast<const bf16x8*>(add);
  if (addv)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<0, true>), dim3(grid_for(nvec)), dim3(kThreads), 0, s, dzv, xv, dxv, ws,
                       addv, nvec, C / 8);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<0, false>), dim3(grid_for(nvec)), dim3(kThreads), 0, s, dzv, xv, dxv, ws,
                       addv, nvec, C / 8);
  return (int)hipGetLastError();
}

// A/B and tests: 1 = finalize + apply in one launch for small layers (default), 0 = never, -1 = env.
VGPU_API void vgpu_bn_set_fuse_small(int on) { g_fuse_small = on < 0 ? -1 : (on ? 1 : 0); }

VGPU_API void vgpu_bn_set_tuning(int target_blocks, int unroll) {
  g_target_blocks = target_blocks > 0 ? target_blocks : kTargetBlocks;
  g_unroll = unroll == 8 ? 8 : kUnroll;
}
