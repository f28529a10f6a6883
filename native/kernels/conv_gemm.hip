// Implicit-GEMM NHWC bf16 convolution on gfx950 MFMA with fused prologue and
// epilogue — the hot op of the ai-benchmark CNN workloads (ResNet-V2-50/152).
//
// Why a hand-written conv: on MI355X a pre-activation bottleneck is HBM-bound,
// not MFMA-bound (stage 1 at b=50 346²: 12 GFLOP per 1x1 conv against ~240 MB of
// activation traffic).  MIOpen convolutions cannot take a prologue or a
// residual, so a bottleneck costs 7 passes over the 4×-wide activation.  Here
//
//   y = act( conv(pro(x), w) + bias[co] + residual )       pro(x) = relu(x*s[c] + t[c])
//
// is one kernel: the block-entry BN+ReLU is applied while the input tile is
// staged into LDS (so the pre-activation is never written), conv bias + ReLU
// (BN folded into the weights) and the residual add are applied while the
// output tile leaves.  Per bottleneck the wide activation is read twice and
// written once instead of read 4× and written 3×.
//
// GEMM view: M = N*OH*OW output pixels, N = Cout, K = KS*KS*C with k ordered
// (kh, kw, c) — exactly PyTorch's channels_last weight [Cout][KS][KS][C].  A
// 64-wide K tile is one filter tap × 64 input channels, i.e. 128 contiguous
// bytes of one input pixel (or zeros for padding), so the implicit im2col is a
// per-row base pointer + tap offset.  Requires C % 64 == 0, Cout % 64 == 0.
//
// Tiling for CDNA4: 256 threads = 4 wave64s in 2×2, workgroup tile BM=128 ×
// BN∈{64,128}, BK=64, mfma_f32_16x16x32_bf16 (lane l holds A[l&15][8(l>>4)..+7]
// and B[8(l>>4)..+7][l&15]).  Two LDS stages with register prefetch: the global
// loads of tile t+1 are in flight while tile t is multiplied.  LDS rows are
// 128 B with a 16-B-slot XOR swizzle (slot ^ row&7) so every ds_read_b128 lane
// group hits 16 distinct slots (conflict-free).  The epilogue stages the fp32
// accumulator tile through LDS (row pad 4 floats: conflict-free ds_write_b32)
// so bias/residual/store are 16-B coalesced per lane.  Workgroups are numbered
// XCD-aware (bijective remap) so the N-tiles sharing an A panel run on one
// XCD's L2.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define VGPU_API extern "C" __attribute__((visibility("default")))

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
// Native 16-B vector (HIP's u32x4 is a class; copies of it go through memcpy
// and defeat register promotion of the staging arrays).
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

constexpr int kThreads = 256;
constexpr int BK = 64;

struct ConvArgs {
  const uint16_t* x;     // [N][H][W][C]
  const uint16_t* w;     // [Cout][KS][KS][C]
  uint16_t* y;           // [N][OH][OW][Cout]
  const uint16_t* res;   // [N][OH][OW][Cout] or nullptr
  const float* bias;     // [Cout] or nullptr
  const float* pscale;   // [C] prologue scale (PRO only)
  const float* pshift;   // [C] prologue shift
  int N, H, W, C, Cout, OH, OW, stride, pad;
  int M, K, ktiles, cblocks, nM, nN, nwg, act;
  uint32_t x_bytes, y_bytes;  // buffer-resource extents (< 2^31: the host splits the batch)
  int nmajor;                 // conv_halo_kernel: workgroups of one XCD share an N tile
  // Training BatchNorm statistics from the epilogue (vgpu_conv2d_nhwc_bn; glds / halo only).
  // stats: per 64-row group g and output channel c, stats[g·Cout + c] = (Σ v, Σ v·q) over
  // the group's stored (bf16) values v: q = v (forward: the next BN's Σx, Σx²), or with
  // bnx, q = (x - mean)·invstd and v = dy·act'(x·s + t) replacing dy (backward of the
  // BN whose output this conv's data gradient is; bncoef = s, t, mean, invstd [4][Cout]).
  float2* stats;
  const uint16_t* bnx;
  const float* bncoef;
  int bnact;  // 1 relu, 2 relu6, 0 none
  // Backward statistics only: res_stride 2 = the residual is the compact data
  // gradient of a 1x1 / stride-2 projection shortcut, [N][res_h][res_w][Cout],
  // which lands on the even (h, w) pixels of this conv's OH x OW output (zero elsewhere).
  int res_stride, res_h, res_w;
  uint32_t res_bytes;
  int bias_bf16;  // bias is bf16 [Cout] (a model's own parameter, no per-step cast)
  // Split-K (conv_glds_kernel<..., SPLIT>): blockIdx.y = split, K steps
  // [split·kper, +kper), fp32 partial tiles ws[split][M][Cout]; splitk_reduce_kernel
  // sums them in split order and applies bias / residual / activation.
  float* ws;
  int kper, splits;
  // Split-K data gradient into a ReLU layer (splitk_reduce_kernel): the output
  // is masked by gmask > 0 (the ReLU's own output) and per-block column sums of
  // the stored bf16 values go to gpart[block][Cout] -- that layer's bias-gradient
  // partials, so its separate ReLU-backward pass disappears (VGG-16 training).
  const uint16_t* gmask;
  float* gpart;
  // ... and when that layer is followed by a k×k / stride-k max pool (this conv's
  // x is the pool's output): the gradient is scattered through the pool's
  // argmax bytes pidx [M][Cout] into gfull [N][OH·k][OW·k][Cout], masked by
  // gmask (the ReLU output, full resolution) -- y is not written.
  const uint8_t* pidx;
  uint16_t* gfull;
  int pk;
};

// d act / d z as PyTorch defines it (threshold_backward / hardtanh_backward).
__device__ __forceinline__ float bn_act_grad(int act, float z) {
  if (act == 1) return z > 0.0f ? 1.0f : 0.0f;
  if (act == 2) return (z > 0.0f && z < 6.0f) ? 1.0f : 0.0f;
  return 1.0f;
}

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
// Keep `v` in a VGPR as it is here (no rematerialisation, no hoisting past this point).
__device__ __forceinline__ void pin_vgpr(uint32_t& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ void unpack8(const u32x4 v, float (&f)[8]) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
// One v_cvt_pk_bf16_f32 per pair (RNE, the same rounding as two scalar
// conversions); the scalar form costs two conversions + shift + or.
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}
__device__ __forceinline__ u32x4 pack8(const float (&f)[8]) {
  return u32x4{pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7])};
}

__device__ __forceinline__ void load8f(const float* p, float (&o)[8]) {
  const float4 b0 = *reinterpret_cast<const float4*>(p);
  const float4 b1 = *reinterpret_cast<const float4*>(p + 4);
  o[0] = b0.x; o[1] = b0.y; o[2] = b0.z; o[3] = b0.w;
  o[4] = b1.x; o[5] = b1.y; o[6] = b1.z; o[7] = b1.w;
}

__device__ __forceinline__ void load_bias8(const ConvArgs& a, int col, float (&bb)[8]) {
  if (a.bias_bf16) {
    unpack8(*reinterpret_cast<const u32x4*>(reinterpret_cast<const uint16_t*>(a.bias) + col), bb);
  } else {
    const float4 b0 = *reinterpret_cast<const float4*>(a.bias + col);
    const float4 b1 = *reinterpret_cast<const float4*>(a.bias + col + 4);
    bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w;
    bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
  }
}

__device__ __forceinline__ int swz(int row, int slot) { return row * 128 + (((slot ^ (row & 7))) << 4); }

__device__ __forceinline__ void tile_origin(const ConvArgs& a, int tile, int bm, int bn, int& m0,
                                            int& n0) {
  // XCD-aware bijective numbering: tiles that run on one XCD (tile % 8 — the grid
  // stride is a multiple of 8) get consecutive ids, so the N-tiles sharing an A
  // panel meet in that XCD's L2.
  const int xcd = tile & 7, q = a.nwg >> 3, r8 = a.nwg & 7;
  const int id = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (tile >> 3);
  const int mi = id / a.nN;
  m0 = mi * bm;
  n0 = (id - mi * a.nN) * bn;
}

constexpr uint32_t kOOB = 0x80000000u;  // buffer offset past num_records: loads return 0

// Persistent: workgroup b processes tiles b, b+G, b+2G, ... as one flattened
// sequence of K steps, so the global loads of the next step — including the
// first step of the next tile — are in flight while the current step is
// multiplied and the current tile's epilogue runs.
//
// Every global load in the loop is unconditional: activations and the residual
// go through buffer loads whose out-of-range offset (kOOB) returns zeros, which
// gives the conv zero padding and the M tail for free and keeps hipcc from
// branching around loads (a branch around a load makes it wait vmcnt(0) and
// de-pipelines the loop).  The residual of a tile is fetched in its last K step,
// issued before that step's A/B prefetch so the epilogue waits only for it.
template <int KS, int BM, int BN, bool PRO, bool RES>
__global__ void __launch_bounds__(kThreads, 2) conv_gemm_kernel(const ConvArgs a) {
  constexpr int AR = BM * 8 / kThreads;  // 16-B A chunks per thread per K step
  constexpr int BR = BN * 8 / kThreads;
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int CS = BN + 4;  // epilogue fp32 row stride (pad: conflict-free ds_write_b32)
  constexpr int PIPE = 2 * STAGE, EPI = BM * CS * 4;
  constexpr int CPR = BN / 8, RSTEP = kThreads / CPR, RROWS = BM / RSTEP;
  __shared__ __attribute__((aligned(16))) char smem[PIPE > EPI ? PIPE : EPI];

  const int G = gridDim.x;
  int tile = blockIdx.x;
  if (tile >= a.nwg) return;

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int slot = t & 7, r0 = t >> 3;
  const int fr = lane & 15, fk = lane >> 4;
  const int chunk = t % CPR, rfirst = t / CPR;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.x), 0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(RES ? a.res : a.x), 0, RES ? a.y_bytes : 0u, 0x00020000);

  int m0, n0;  // tile whose A/B are being loaded
  tile_origin(a, tile, BM, BN, m0, n0);
  int em0 = m0, en0 = n0;  // tile owned by the accumulators (epilogue)

  int abase[AR], aih[AR], aiw[AR];  // byte offset of the window origin, origin row/col
  bool aok[AR];
#define VGPU_SETUP_ROWS()                                                                    \
  _Pragma("unroll") for (int i = 0; i < AR; ++i) {                                           \
    const int m = m0 + r0 + 32 * i;                                                         \
    aok[i] = m < a.M;                                                                       \
    const int mm = aok[i] ? m : 0;                                                          \
    const int ow = mm % a.OW, t2 = mm / a.OW, oh = t2 % a.OH, n = t2 / a.OH;               \
    aih[i] = oh * a.stride - a.pad;                                                         \
    aiw[i] = ow * a.stride - a.pad;                                                         \
    abase[i] = ((n * a.H + aih[i]) * a.W + aiw[i]) * a.C * 2;                               \
  }

  // Two register sets (A/B chunks + validity + K step): the loads of step s+2
  // are issued while step s is multiplied and step s+1 waits in the other set.
  u32x4 ra0[AR], rb0[BR], ra1[AR], rb1[BR], res[RROWS];
  bool rv0[AR], rv1[AR];
  int kt0 = 0, kt1 = 0;
  // Global → registers for K step ktl of the tile at (m0, n0): implicit im2col
  // (zero padding via out-of-range buffer offsets) for A, a weight panel for B.
#define VGPU_LOAD_TILE(kt_, RA, RB, RV)                                                      \
  {                                                                                          \
    const int ktl = (kt_);                                                                   \
    const int tap = ktl / a.cblocks, cb = ktl - tap * a.cblocks;                             \
    const int kh = tap / KS, kw = tap - kh * KS;                                             \
    const int toff = ((kh * a.W + kw) * a.C + cb * BK + slot * 8) * 2;                       \
    _Pragma("unroll") for (int i = 0; i < AR; ++i) {                                         \
      bool v = aok[i];                                                                       \
      if (KS != 1 || a.pad != 0) {                                                           \
        const int ih = aih[i] + kh, iw = aiw[i] + kw;                                        \
        v = v && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;               \
      }                                                                                      \
      RV[i] = v;                                                                             \
      RA[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, v ? (uint32_t)(abase[i] + toff) : kOOB, 0, 0); \
    }                                                                                        \
    const uint16_t* wp = a.w + (int64_t)(n0 + r0) * a.K + (int64_t)ktl * BK + slot * 8;      \
    _Pragma("unroll") for (int i = 0; i < BR; ++i)                                           \
      RB[i] = *reinterpret_cast<const u32x4*>(wp + (int64_t)(32 * i) * a.K);                 \
  }
  // Residual rows of the epilogue tile; real loads only when `last` (else kOOB: no traffic).
#define VGPU_LOAD_RES(last_)                                                                 \
  _Pragma("unroll") for (int i = 0; i < RROWS; ++i) {                                        \
    const int m = em0 + rfirst + RSTEP * i;                                                 \
    const bool v = (last_) && m < a.M;                                                      \
    res[i] = __builtin_amdgcn_raw_buffer_load_b128(                                         \
        rr, v ? (uint32_t)(((int64_t)m * a.Cout + en0 + chunk * 8) * 2) : kOOB, 0, 0);      \
  }
  // Registers → LDS stage st_, applying the prologue to real (non-padding) pixels.
#define VGPU_STORE_TILE(kt_, st_, RA, RB, RV)                                                \
  {                                                                                          \
    char* sA = smem + (st_) * STAGE;                                                         \
    char* sB = sA + A_BYTES;                                                                 \
    if constexpr (PRO) {                                                                     \
      const int c = ((kt_) % a.cblocks) * BK + slot * 8;                                     \
      const float4 s0 = *reinterpret_cast<const float4*>(a.pscale + c);                     \
      const float4 s1 = *reinterpret_cast<const float4*>(a.pscale + c + 4);                  \
      const float4 h0 = *reinterpret_cast<const float4*>(a.pshift + c);                     \
      const float4 h1 = *reinterpret_cast<const float4*>(a.pshift + c + 4);                  \
      const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};                  \
      const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};                  \
      _Pragma("unroll") for (int i = 0; i < AR; ++i) {                                       \
        float e[8];                                                                          \
        unpack8(RA[i], e);                                                                   \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                      \
          const float f = fmaxf(e[j] * sc[j] + sh[j], 0.0f);                                 \
          e[j] = RV[i] ? f : 0.0f;                                                           \
        }                                                                                    \
        RA[i] = pack8(e);                                                                    \
      }                                                                                      \
    }                                                                                        \
    _Pragma("unroll") for (int i = 0; i < AR; ++i)                                           \
      *reinterpret_cast<u32x4*>(sA + swz(r0 + 32 * i, slot)) = RA[i];                        \
    _Pragma("unroll") for (int i = 0; i < BR; ++i)                                           \
      *reinterpret_cast<u32x4*>(sB + swz(r0 + 32 * i, slot)) = RB[i];                        \
  }
  // Load cursor: the next (tile, K step) to fetch; entering a tile sets up its rows.
  int ltile = tile, lkt = 0;
#define VGPU_ADVANCE_LOAD()                                                                  \
  {                                                                                          \
    if (++lkt == a.ktiles) {                                                                 \
      lkt = 0;                                                                               \
      ltile += G;                                                                            \
      if (ltile < a.nwg) {                                                                   \
        tile_origin(a, ltile, BM, BN, m0, n0);                                               \
        VGPU_SETUP_ROWS()                                                                    \
      }                                                                                      \
    }                                                                                        \
  }

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  VGPU_SETUP_ROWS()
  VGPU_LOAD_TILE(0, ra0, rb0, rv0)
  VGPU_STORE_TILE(0, 0, ra0, rb0, rv0)
  VGPU_ADVANCE_LOAD()
  kt1 = lkt;
  VGPU_LOAD_TILE(ltile < a.nwg ? lkt : 0, ra1, rb1, rv1)
  VGPU_ADVANCE_LOAD()
  __syncthreads();

  int ckt = 0, st = 0;  // compute cursor: K step of `tile` staged in LDS stage st
  // One step: prefetch step s+2 into set F, multiply step s, epilogue at a tile
  // end, then stage step s+1 (set I) for the next iteration.
#define VGPU_STEP(RAF, RBF, RVF, KTF, RAI, RBI, RVI, KTI)                                     \
  {                                                                                          \
    const bool last = ckt + 1 == a.ktiles;                                                   \
    if constexpr (RES) VGPU_LOAD_RES(last)                                                   \
    KTF = lkt;                                                                               \
    VGPU_LOAD_TILE(ltile < a.nwg ? lkt : 0, RAF, RBF, RVF)                                   \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    {                                                                                        \
      const char* sA = smem + st * STAGE;                                                    \
      const char* sB = sA + A_BYTES;                                                         \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk) {                                     \
        bf16x8_t af[TM], bfr[TN];                                                            \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                       \
          af[i] = *reinterpret_cast<const bf16x8_t*>(sA + swz(wm * WTM + i * 16 + fr, kk * 4 + fk)); \
        _Pragma("unroll") for (int j = 0; j < TN; ++j)                                       \
          bfr[j] = *reinterpret_cast<const bf16x8_t*>(sB + swz(wn * WTN + j * 16 + fr, kk * 4 + fk)); \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                       \
          _Pragma("unroll") for (int j = 0; j < TN; ++j)                                     \
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0); \
      }                                                                                      \
    }                                                                                        \
    if (last) VGPU_EPILOGUE()                                                                \
    if (++ckt == a.ktiles) {                                                                 \
      ckt = 0;                                                                               \
      tile += G;                                                                             \
      if (tile >= a.nwg) break;                                                              \
      tile_origin(a, tile, BM, BN, em0, en0);                                                \
    }                                                                                        \
    st ^= 1;                                                                                 \
    VGPU_STORE_TILE(KTI, st, RAI, RBI, RVI)                                                  \
    __syncthreads();                                                                         \
    VGPU_ADVANCE_LOAD()                                                                      \
  }
  // Accumulators → LDS (fp32) → 16-B coalesced bias + residual + act + store.
#define VGPU_EPILOGUE()                                                                      \
  {                                                                                          \
    __syncthreads();                                                                         \
    float* sC = reinterpret_cast<float*>(smem);                                              \
    _Pragma("unroll") for (int i = 0; i < TM; ++i)                                           \
      _Pragma("unroll") for (int j = 0; j < TN; ++j) {                                       \
        _Pragma("unroll") for (int e = 0; e < 4; ++e)                                        \
          sC[(wm * WTM + i * 16 + fk * 4 + e) * CS + wn * WTN + j * 16 + fr] = acc[i][j][e]; \
        acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};                                             \
      }                                                                                      \
    __syncthreads();                                                                         \
    const int col = en0 + chunk * 8;                                                         \
    float bb[8];                                                                             \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) bb[j] = 0.0f;                              \
    if (a.bias) load_bias8(a, col, bb);                                                      \
    _Pragma("unroll") for (int i = 0; i < RROWS; ++i) {                                      \
      const int r = rfirst + RSTEP * i, m = em0 + r;                                         \
      const float4 c0 = *reinterpret_cast<const float4*>(sC + r * CS + chunk * 8);           \
      const float4 c1 = *reinterpret_cast<const float4*>(sC + r * CS + chunk * 8 + 4);       \
      float v[8] = {c0.x + bb[0], c0.y + bb[1], c0.z + bb[2], c0.w + bb[3],                  \
                    c1.x + bb[4], c1.y + bb[5], c1.z + bb[6], c1.w + bb[7]};                 \
      if constexpr (RES) {                                                                   \
        float re[8];                                                                         \
        unpack8(res[i], re);                                                                 \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) v[j] += re[j];                         \
      }                                                                                      \
      if (a.act) {                                                                           \
        const float hi_ = a.act == 2 ? 6.0f : INFINITY;                                      \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) v[j] = fminf(fmaxf(v[j], 0.0f), hi_);  \
      }                                                                                      \
      if (m < a.M) *reinterpret_cast<u32x4*>(a.y + (int64_t)m * a.Cout + col) = pack8(v);    \
    }                                                                                        \
    __syncthreads(); /* staging reads done before the pipeline reuses LDS */                 \
  }

  for (;;) {
    VGPU_STEP(ra0, rb0, rv0, kt0, ra1, rb1, rv1, kt1)
    VGPU_STEP(ra1, rb1, rv1, kt1, ra0, rb0, rv0, kt0)
  }
}

#undef VGPU_SETUP_ROWS
#undef VGPU_LOAD_RES
#undef VGPU_LOAD_TILE
#undef VGPU_STORE_TILE
#undef VGPU_ADVANCE_LOAD
#undef VGPU_STEP
#undef VGPU_EPILOGUE

// ---- LDS-DMA variant (no prologue): A and B tiles go HBM → LDS with
// buffer_load_dword×4 … lds, bypassing the VGPR → ds_write_b128 path.
//
// Why: with register staging a 128×128×64 step writes 32 KB into LDS through
// ds_write_b128 (≈79 B/clk/CU) and reads 64 KB back (256 B/clk/CU): ≈670 LDS
// cycles against 512 MFMA cycles per block-step, i.e. LDS-bound at 2 blocks/CU.
// The DMA writes at the LDS array rate, so the same step costs ≈384 LDS cycles.
//
// The LDS image is the same XOR-swizzled [row][128 B] layout as the register
// path; a DMA lands lane-linearly (wave base + 16·lane), so each lane fetches
// the LOGICAL chunk (lane&7) ^ (row&7) of its row — the swizzle is applied to
// the global source address.  Zero padding / M tail: out-of-range buffer
// offsets load zeros into LDS.  Two stages, one DMA step in flight: wait for
// the current stage with a counted vmcnt (the next stage stays in flight),
// raw s_barrier (a __syncthreads() would drain the DMA with vmcnt(0)).
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int vmcnt_imm(int n) {  // s_waitcnt vmcnt(n), expcnt/lgkmcnt untouched (gfx9 encoding)
  return (n & 15) | (((n >> 4) & 3) << 14) | (7 << 4) | (15 << 8);
}
constexpr int kLgkm0 = 15 | (3 << 14) | (7 << 4);  // s_waitcnt lgkmcnt(0) only
constexpr int lgkm_imm(int n) { return kLgkm0 | ((n & 15) << 8); }  // s_waitcnt lgkmcnt(n) only

// One 64-wide K step of a wave's TM x TN grid of 16x16 sub-tiles from a
// swizzled LDS stage (rows of 128 B): fragment reads software-pipelined — the
// second 32-wide half's ds_reads are issued behind the wait for the first half
// and land while the first half multiplies.  (With LDS DMA in flight hipcc only
// emits full lgkmcnt drains, so the overlap comes from issue order.)
// SWAP: acc += B·A (transposed output tile, conv23's first GEMM).
template <int TM, int TN, bool SWAP = false>
__device__ __forceinline__ void mma_k64(const char* sA, const char* sB, int arow, int brow, int fr, int fk,
                                        f32x4_t (&acc)[TM][TN]) {
  bf16x8_t af[2][TM], bfr[2][TN];
  auto rd = [&](int kk) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
      af[kk][i] = *reinterpret_cast<const bf16x8_t*>(sA + swz(arow + i * 16 + fr, kk * 4 + fk));
#pragma unroll
    for (int j = 0; j < TN; ++j)
      bfr[kk][j] = *reinterpret_cast<const bf16x8_t*>(sB + swz(brow + j * 16 + fr, kk * 4 + fk));
  };
  auto mm = [&](int kk) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = SWAP ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[kk][j], af[kk][i], acc[i][j], 0, 0, 0)
                         : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
  };
  rd(0);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  __builtin_amdgcn_sched_barrier(0);
  rd(1);
  __builtin_amdgcn_sched_barrier(0);
  mm(0);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  __builtin_amdgcn_sched_barrier(0);
  mm(1);
}

// Epilogue, one row half at a time: accumulators → LDS (fp32) → 16-B
// coalesced bias + residual + act + store.  The residual loads of a half
// overlap its accumulator staging.  Needs (BM/2)·(BN+4)·4 bytes of LDS and a
// block-wide barrier behind the last read of the pipeline stages.
// NT: threads of the workgroup (conv23 also runs 512-thread tiles).
template <int BM, int BN, int NT = kThreads>
struct EpiShape {
  static constexpr int HROWS = BM / 2, CPR = BN / 8, RSTEP = NT / CPR, RROWS = HROWS / RSTEP;
};

// Residual rows this thread adds in the epilogue (both halves), issued early —
// before the first DMA of the K loop — so their latency hides behind the loop.
template <int BM, int BN, bool STRIDED = false, int NT = kThreads>
__device__ __forceinline__ void load_residual(const ConvArgs& a, int m0, int n0,
                                              u32x4 (&res)[2][EpiShape<BM, BN, NT>::RROWS]) {
  using E = EpiShape<BM, BN, NT>;
  const int t = threadIdx.x, chunk = t % E::CPR, rfirst = t / E::CPR;
  const bool strided = STRIDED && a.res_stride == 2;
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.res), 0, strided ? a.res_bytes : a.y_bytes, 0x00020000);
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < E::RROWS; ++i) {
      const int m = m0 + h * E::HROWS + rfirst + E::RSTEP * i;
      uint32_t off = m < a.M ? (uint32_t)(((int64_t)m * a.Cout + n0 + chunk * 8) * 2) : kOOB;
      if (strided && m < a.M) {
        const int ow = m % a.OW, t2 = m / a.OW, oh = t2 % a.OH, n = t2 / a.OH;
        off = ((oh | ow) & 1) ? kOOB
                              : (uint32_t)(((((int64_t)n * a.res_h + (oh >> 1)) * a.res_w + (ow >> 1)) * a.Cout +
                                            n0 + chunk * 8) * 2);
      }
      res[h][i] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
    }
}

// ST (BatchNorm statistics, ConvArgs::stats): 0 none, 1 forward (of the stored
// values), 2 backward (masked by the BN's activation derivative; ConvArgs::bnx).
// NT threads = (NT / 128) x 2 waves; each row half is staged by the wave rows
// that own it.
template <int BM, int BN, bool RES, int ST = 0, int NT = kThreads>
__device__ __forceinline__ void epilogue_halves(const ConvArgs& a,
                                                f32x4_t (&acc)[BM / (NT / 128) / 16][BN / 32],
                                                int m0, int n0, char* smem,
                                                const u32x4 (&res)[2][EpiShape<BM, BN, NT>::RROWS]) {
  static_assert(ST == 0 || NT == kThreads, "statistics: 256-thread tiles");
  constexpr int WGM = NT / 128, WPH = WGM / 2;  // wave rows, wave rows per half
  constexpr int WTM = BM / WGM, WTN = BN / 2, TM = WTM / 16, TN = WTN / 16;
  constexpr int CS = BN + 4, HROWS = BM / 2;
  constexpr int CPR = BN / 8, RSTEP = NT / CPR, RROWS = HROWS / RSTEP;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1, fr = lane & 15, fk = lane >> 4;
  const int chunk = t % CPR, rfirst = t / CPR;
  const int col = n0 + chunk * 8;
  float bb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bb[j] = 0.0f;
  if (a.bias) load_bias8(a, col, bb);
  float* sC = reinterpret_cast<float*>(smem);
  // BatchNorm statistics (a.stats, uniform): per-thread sums over its rows, merged
  // per 64-row group through LDS past the staging area (the pipeline stages are free).
  constexpr bool st = ST != 0, bwd = ST == 2;  // bwd + RES: dy = acc + res (a second gradient of the BN output)
  float s1[8], s2[8], bs[8], bt[8], bmu[8], bis[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = bs[j] = bt[j] = bmu[j] = bis[j] = 0.0f;
  u32x4 xb[2][RROWS];
  if constexpr (bwd) {
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t*>(a.bnx), 0, a.y_bytes, 0x00020000);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < RROWS; ++i) {
        const int m = m0 + h * HROWS + rfirst + RSTEP * i;
        xb[h][i] = __builtin_amdgcn_raw_buffer_load_b128(
            xr, m < a.M ? (uint32_t)(((int64_t)m * a.Cout + col) * 2) : kOOB, 0, 0);
      }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bs[j] = a.bncoef[col + j];
      bt[j] = a.bncoef[a.Cout + col + j];
      bmu[j] = a.bncoef[2 * a.Cout + col + j];
      bis[j] = a.bncoef[3 * a.Cout + col + j];
    }
  }
  float2* sS = reinterpret_cast<float2*>(smem + HROWS * CS * 4);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (wm / WPH == h) {
      const int r0 = (wm % WPH) * WTM;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            sC[(r0 + i * 16 + fk * 4 + e) * CS + wn * WTN + j * 16 + fr] = acc[i][j][e];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RROWS; ++i) {
      const int r = rfirst + RSTEP * i, m = m0 + h * HROWS + r;
      const float4 c0 = *reinterpret_cast<const float4*>(sC + r * CS + chunk * 8);
      const float4 c1 = *reinterpret_cast<const float4*>(sC + r * CS + chunk * 8 + 4);
      float v[8] = {c0.x + bb[0], c0.y + bb[1], c0.z + bb[2], c0.w + bb[3],
                    c1.x + bb[4], c1.y + bb[5], c1.z + bb[6], c1.w + bb[7]};
      if constexpr (RES) {
        float re[8];
        unpack8(res[h][i], re);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += re[j];
      }
      if (a.act) {  // 1 ReLU, 2 ReLU6
        const float hi = a.act == 2 ? 6.0f : INFINITY;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fminf(fmaxf(v[j], 0.0f), hi);
      }
      float xf[8];
      if constexpr (bwd) {
        unpack8(xb[h][i], xf);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= bn_act_grad(a.bnact, fmaf(xf[j], bs[j], bt[j]));
      }
      const u32x4 o = pack8(v);
      if (m < a.M) *reinterpret_cast<u32x4*>(a.y + (int64_t)m * a.Cout + col) = o;
      if constexpr (st) {
        float q[8];
        unpack8(o, q);  // the stored (bf16) values
        const float ok = m < a.M ? 1.0f : 0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = q[j] * ok;
          s1[j] += d;
          s2[j] = fmaf(d, bwd ? (xf[j] - bmu[j]) * bis[j] : d, s2[j]);
        }
      }
    }
    // 64-row group complete: BM 128 after each half, BM 64 after both.
    if (st && ((h + 1) * HROWS) % 64 == 0) {  // h is unrolled: folds
      const int g = (m0 + (h + 1) * HROWS - 64) / 64;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sS[rfirst * BN + chunk * 8 + j] = make_float2(s1[j], s2[j]);
        s1[j] = s2[j] = 0.0f;
      }
      __syncthreads();
      if (t < BN && g * 64 < a.M) {
        float2 acc2 = make_float2(0.0f, 0.0f);
#pragma unroll
        for (int q = 0; q < RSTEP; ++q) {
          const float2 p = sS[q * BN + t];
          acc2.x += p.x;
          acc2.y += p.y;
        }
        a.stats[(int64_t)g * a.Cout + n0 + t] = acc2;
      }
    }
    if (h == 0) __syncthreads();  // half 0 read out (and its group merged) before half 1 is staged
  }
}

// CSM = 16: a narrow-input conv (the ResNet stem after space-to-depth: C = 16,
// 4x4 taps) — a 64-wide K step then spans 64/C taps, so each lane derives its
// own tap from its chunk.
// Two LDS stages, one DMA step in flight: the second block per CU covers the
// DMA latency (a 3-stage ring measured slower on every ResNet-50 shape,
// profiles/conv_stages_r1.md).  Prologue convs take conv_pro_kernel (an
// in-register prologue on the DMA'd A fragments measured VALU-bound and slower).
template <int KS, int BM, int BN, bool RES, int CSM = 0, int ST = 0, bool SPLIT = false>
__global__ void __launch_bounds__(kThreads, 2) conv_glds_kernel(const ConvArgs a) {
  static_assert(CSM == 0 || (64 % CSM == 0 && CSM % 8 == 0), "narrow-C variant");
  static_assert(!SPLIT || (!RES && ST == 0 && CSM == 0), "split-K: the reduce kernel does the epilogue");
  constexpr int AR = BM / 32, BR = BN / 32;  // DMA instructions per thread per K step
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int CS = BN + 4;
  constexpr int PIPE = 2 * STAGE;
  constexpr int HROWS = BM / 2, EPI = HROWS * CS * 4;  // epilogue staged in two row halves
  constexpr int BODY = PIPE > EPI ? PIPE : EPI;
  static_assert(ST == 0 || EPI + (kThreads / (BN / 8)) * BN * 8 <= BODY, "statistics merge area fits");
  __shared__ __attribute__((aligned(16))) char smem[BODY];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fk = lane >> 4;
  const int lrow = t >> 3, lchunk = (t & 7) ^ (lrow & 7);
  int m0, n0;
  tile_origin(a, blockIdx.x, BM, BN, m0, n0);

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.x), 0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.w), 0, (uint32_t)((int64_t)a.Cout * a.K * 2), 0x00020000);

  int abase[AR], aih[AR], aiw[AR];
  bool aok[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + lrow + 32 * i;
    aok[i] = m < a.M;
    const int mm = aok[i] ? m : 0;
    const int ow = mm % a.OW, t2 = mm / a.OW, oh = t2 % a.OH, n = t2 / a.OH;
    aih[i] = oh * a.stride - a.pad;
    aiw[i] = ow * a.stride - a.pad;
    abase[i] = ((n * a.H + aih[i]) * a.W + aiw[i]) * a.C * 2;
  }
  const uint32_t boff = (uint32_t)(((n0 + lrow) * a.K + lchunk * 8) * 2);

  auto issue = [&](int kt, int st) {
    char* sA = smem + st * STAGE;
    char* sB = sA + A_BYTES;
    int kh, kw, toff;
    if constexpr (CSM != 0) {  // per-lane tap: k = kt*64 + lchunk*8 = tap*CSM + c
      const int k = kt * BK + lchunk * 8, tap = k / CSM, c = k % CSM;
      kh = tap / KS;
      kw = tap % KS;
      toff = ((kh * a.W + kw) * CSM + c) * 2;
    } else {
      const int tap = kt / a.cblocks, cb = kt - tap * a.cblocks;
      kh = tap / KS;
      kw = tap - kh * KS;
      toff = ((kh * a.W + kw) * a.C + cb * BK + lchunk * 8) * 2;
    }
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      // Bitwise (not short-circuit) validity: no exec-mask branch around the load.
      const int ih = aih[i] + kh, iw = aiw[i] + kw;
      const bool v = aok[i] & ((unsigned)ih < (unsigned)a.H) & ((unsigned)iw < (unsigned)a.W);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xr, (lds_void_t*)(sA + (32 * i + wave * 8) * 128), 16,
          v ? (uint32_t)(abase[i] + toff) : kOOB, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wr, (lds_void_t*)(sB + (32 * i + wave * 8) * 128), 16,
          boff + (uint32_t)((32 * i * a.K + kt * BK) * 2), 0, 0, 0);
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // Short K loops (stage-1 1x1 convs: one K step) fetch the residual up front,
  // so its latency overlaps the A/B DMA; longer loops fetch it after the loop
  // (measured: early fetch costs 5-20 % on K ≥ 4 steps).
  u32x4 res[2][EpiShape<BM, BN>::RROWS];
  const bool early_res = RES && a.ktiles <= 1;
  if constexpr (RES) {
    if (early_res) load_residual<BM, BN, ST == 2>(a, m0, n0, res);
  }
  int kbeg = 0, nk = a.ktiles;
  if constexpr (SPLIT) {
    kbeg = blockIdx.y * a.kper;
    nk = min(a.kper, a.ktiles - kbeg);
  }
  issue(kbeg, 0);
  for (int it = 0; it < nk; ++it) {
    const int st = it & 1;
    if (it + 1 < nk) {
      issue(kbeg + it + 1, st ^ 1);
      __builtin_amdgcn_s_waitcnt(vmcnt_imm(AR + BR));
    } else {
      __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
    }
    __builtin_amdgcn_s_barrier();
    const char* sA = smem + st * STAGE;
    const char* sB = sA + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8_t*>(sA + swz(wm * WTM + i * 16 + fr, kk * 4 + fk));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(sB + swz(wn * WTN + j * 16 + fr, kk * 4 + fk));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    // Stage st fully read (this wave's ds_reads retired) before any wave refills it.
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_s_barrier();
  }
  if constexpr (SPLIT) {
    // fp32 partial tile: lane holds rows 4·fk + e, column fr of each 16x16 sub-tile
    float* out = a.ws + (int64_t)blockIdx.y * a.M * a.Cout;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * WTM + i * 16 + fk * 4 + e;
        if (m < a.M) {
#pragma unroll
          for (int j = 0; j < TN; ++j) out[(int64_t)m * a.Cout + n0 + wn * WTN + j * 16 + fr] = acc[i][j][e];
        }
      }
    return;
  }
  if constexpr (RES) {
    if (!early_res) load_residual<BM, BN, ST == 2>(a, m0, n0, res);
  }
  epilogue_halves<BM, BN, RES, ST>(a, acc, m0, n0, smem, res);
}

// Split-K epilogue: y = act(Σ_split ws[split] + bias (+ residual)) in bf16, the
// splits summed in order (deterministic).  One thread = 8 channels of one row;
// a block covers 256 / (Cout / 8) whole rows.  With gmask: y ·= [gmask > 0] and
// the block's column sums of the stored values go to gpart[block].
__global__ void __launch_bounds__(kThreads) splitk_reduce_kernel(const ConvArgs a) {
  __shared__ float red[kThreads][9];
  const int cv = a.Cout >> 3;
  const int64_t idx = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const bool valid = idx < (int64_t)a.M * cv;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (valid) {
    const int m = (int)(idx / cv), col = (int)(idx - (int64_t)m * cv) * 8;
    const int64_t plane = (int64_t)a.M * a.Cout, off = (int64_t)m * a.Cout + col;
    load8f(a.ws + off, v);
    for (int sp = 1; sp < a.splits; ++sp) {
      float p[8];
      load8f(a.ws + sp * plane + off, p);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += p[j];
    }
    if (a.bias) {
      float bb[8];
      load_bias8(a, col, bb);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += bb[j];
    }
    if (a.res) {
      float re[8];
      unpack8(*reinterpret_cast<const u32x4*>(a.res + off), re);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += re[j];
    }
    if (a.act) {
      const float hi = a.act == 2 ? 6.0f : INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fminf(fmaxf(v[j], 0.0f), hi);
    }
    if (a.gfull) {
      // scatter through the pool: window tap t of pooled pixel m gets v where
      // the argmax byte says t and the ReLU output there is positive
      const uint2 tt = *reinterpret_cast<const uint2*>(a.pidx + off);
      const int ow = m % a.OW, t2 = m / a.OW, oh = t2 % a.OH, n = t2 / a.OH;
      const int FW = a.OW * a.pk, FH = a.OH * a.pk;
      float sum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const u32x4 vb = pack8(v);  // the pool gradient as the unfused path stores it (bf16)
      float vr[8];
      unpack8(vb, vr);
      for (int dh = 0; dh < a.pk; ++dh)
        for (int dw = 0; dw < a.pk; ++dw) {
          const uint32_t tap = dh * a.pk + dw;
          const int64_t fo = (((int64_t)n * FH + oh * a.pk + dh) * FW + ow * a.pk + dw) * a.Cout + col;
          float mk[8], g[8];
          unpack8(*reinterpret_cast<const u32x4*>(a.gmask + fo), mk);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const uint32_t tj = ((j < 4 ? tt.x : tt.y) >> (8 * (j & 3))) & 0xffu;
            g[j] = (tj == tap && mk[j] > 0.0f) ? vr[j] : 0.0f;
            sum[j] += g[j];
          }
          *reinterpret_cast<u32x4*>(a.gfull + fo) = pack8(g);
        }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = sum[j];
    } else {
      if (a.gmask) {
        float mk[8];
        unpack8(*reinterpret_cast<const u32x4*>(a.gmask + off), mk);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = mk[j] > 0.0f ? v[j] : 0.0f;
      }
      const u32x4 o = pack8(v);
      *reinterpret_cast<u32x4*>(a.y + off) = o;
      unpack8(o, v);  // the partial sums add the stored (rounded) values
    }
  }
  if (!a.gpart) return;  // kernel-uniform
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x][j] = valid ? v[j] : 0.0f;
  __syncthreads();
  if ((int)threadIdx.x < cv) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < kThreads / cv; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += red[r * cv + threadIdx.x][j];
    float* out = a.gpart + (int64_t)blockIdx.x * a.Cout + threadIdx.x * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = acc[j];
  }
}

// ---- 256x256 tile for large 1x1 / stride-1 convs without a prologue ----------
// A plain GEMM y[M][Cout] = x[M][C] · W[Cout][C]ᵀ (+bias, +residual, act) whose
// two operands are both K-contiguous.  The 128x128 kernels above spend two
// workgroup barriers and 64 KB of LDS fragment reads per 2.1 MFLOP K step
// (≈800 TFLOP/s on 65536x1024x1024, profiles/gemm_ceiling_r1.md).  Here one
// workgroup of 8 waves (2 M x 4 N, wave tile 128x64) owns a 256x256 output
// tile: a K step is 8.4 MFLOP — 64 MFMAs per wave — against the same two
// barriers, and each wave reads 24 KB of fragments for 4x the work of a
// 64x64 wave tile (LDS traffic per FLOP -33 %).  Two 64 KB LDS stages are
// filled by LDS-DMA one K step ahead (one workgroup per CU: 128 KB of 160).
// The epilogue goes through a per-wave LDS slab in four 32-row quarters so
// every store is a 16-B bf16x8 and the bias is loaded once per lane.
constexpr int kBigThreads = 512;
int conv_cus();


// K steps of 32 (BK32) in an NS-deep ring of 32 KB LDS stages (NS = 4: 128 KB),
// so the DMA of step k+NS-1 is issued while step k is multiplied: three steps
// (1.5 64-deep steps) of lead instead of one, and the wait before the single
// barrier per step is a counted vmcnt that leaves NS-2 steps in flight across
// it.  Fragments are double-buffered in registers: the MFMAs of step k are
// split around the barrier that publishes step k+1, and the reads of step k+1
// are issued behind that barrier under the second half of step k's MFMAs.
//
// LDS image: rows of 64 B (32 bf16), 16-B slots; logical slot f of row r sits
// in physical slot f ^ g((r>>2)&3), g = {0,2,3,1}: the four 16-lane groups of
// a ds_read_b128 (lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) then hit
// 16 distinct bank quads — conflict-free.  The DMA lands lane-linearly (16
// rows per wave instruction), so each lane fetches the logical slot that its
// physical slot holds.
__device__ __forceinline__ int swz_g(int q) { return (q >> 1) | (((q ^ (q >> 1)) & 1) << 1); }
__device__ __forceinline__ int swz32(int row, int slot) {
  return row * 64 + ((slot ^ swz_g((row >> 2) & 3)) << 4);
}

template <bool RES, int NS = 4>
__global__ void __launch_bounds__(kBigThreads, 1) conv_big_kernel(const ConvArgs a) {
  constexpr int BM = 256, BN = 256;
  constexpr int A_BYTES = BM * 64, B_BYTES = BN * 64, STAGE = A_BYTES + B_BYTES;  // 32 KB
  constexpr int TM = 8, TN = 4;              // 16x16 sub-tiles per wave: 128 x 64
  constexpr int CS = 64 + 4;                  // epilogue slab row stride (floats)
  constexpr int SLAB = 16 * CS * 4;           // 16 rows of one wave's 64 columns
  static_assert(8 * SLAB <= NS * STAGE, "epilogue slabs fit in the pipeline stages");
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fk = lane >> 4;
  int m0, n0;
  tile_origin(a, blockIdx.x, BM, BN, m0, n0);

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.x), 0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.w), 0, (uint32_t)((int64_t)a.Cout * a.K * 2), 0x00020000);
  // DMA: wave instruction i (0,1) fills rows 32*wave + 16*i + (lane>>2) of the A and B images.
  const int drow = lane >> 2, dslot = (lane & 3) ^ swz_g((lane >> 4) & 3);
  uint32_t aoff[2], boff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 32 * wave + 16 * i + drow, m = m0 + r;
    aoff[i] = m < a.M ? (uint32_t)(((int64_t)m * a.K + dslot * 8) * 2) : kOOB;
    boff[i] = (uint32_t)(((int64_t)(n0 + r) * a.K + dslot * 8) * 2);
  }
  const int ks = a.K / 32;
  auto issue = [&](int kt) {
    const int kc = kt < ks ? kt : ks - 1;  // past the end: refetch the last step into a stage nobody reads again
    char* sA = smem + (kt % NS) * STAGE;
    char* sB = sA + A_BYTES;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void_t*)(sA + (32 * wave + 16 * i) * 64), 16,
                                               aoff[i] == kOOB ? kOOB : aoff[i] + (uint32_t)kc * 64, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void_t*)(sB + (32 * wave + 16 * i) * 64), 16,
                                               boff[i] + (uint32_t)kc * 64, 0, 0, 0);
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // One rolling set of A fragments (rows 0-3 of step k+1 replace rows 0-3 of
  // step k once the first MFMA half has used them) and two B sets.
  bf16x8_t af[TM], bfr[2][TN];
  const int arow = wm * 128 + fr, brow = wn * 64 + fr;
  auto read_a = [&](int kt, int i0, int i1) {
    const char* sA = smem + (kt % NS) * STAGE;
#pragma unroll
    for (int i = i0; i < i1; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(sA + swz32(arow + i * 16, fk));
  };
  auto read_b = [&](int kt, bf16x8_t (&b)[TN]) {
    const char* sB = smem + (kt % NS) * STAGE + A_BYTES;
#pragma unroll
    for (int j = 0; j < TN; ++j) b[j] = *reinterpret_cast<const bf16x8_t*>(sB + swz32(brow + j * 16, fk));
  };
  auto mfma_rows = [&](const bf16x8_t (&b)[TN], int i0, int i1) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = i0; i < i1; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], b[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // One K step: A rows 4-7 of step kt load under the first MFMA half; the
  // barrier publishing step kt+1 sits between the halves; step kt+1's A rows
  // 0-3 and B load under the second half.
  auto kstep = [&](int kt, bf16x8_t (&bc)[TN], bf16x8_t (&bn)[TN]) {
    issue(kt + NS - 1);  // into the stage of step kt-1, read out before the last barrier
    read_a(kt, TM / 2, TM);
    mfma_rows(bc, 0, TM / 2);
    __builtin_amdgcn_s_waitcnt(vmcnt_imm((NS - 2) * 4));  // step kt+1 landed
    __builtin_amdgcn_s_waitcnt(kLgkm0);                   // every read of step kt retired
    __builtin_amdgcn_s_barrier();
    if (kt + 1 < ks) {
      read_a(kt + 1, 0, TM / 2);
      read_b(kt + 1, bn);
    }
    mfma_rows(bc, TM / 2, TM);
  };

#pragma unroll
  for (int s = 0; s < NS - 1; ++s) issue(s);
  __builtin_amdgcn_s_waitcnt(vmcnt_imm((NS - 2) * 4));  // step 0 landed (this thread's DMAs)
  __builtin_amdgcn_s_barrier();
  read_a(0, 0, TM / 2);
  read_b(0, bfr[0]);
  int kt = 0;
  for (; kt + 1 < ks; kt += 2) {
    kstep(kt, bfr[0], bfr[1]);
    kstep(kt + 1, bfr[1], bfr[0]);
  }
  if (kt < ks) kstep(kt, bfr[0], bfr[1]);
  __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));  // refetches past the end
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  __builtin_amdgcn_s_barrier();

  // Epilogue: per wave, eight 16-row passes through its own slab.
  float* sC = reinterpret_cast<float*>(smem + wave * SLAB);
  const int ecol = (lane & 7) * 8, erow = lane >> 3;
  const int col = n0 + wn * 64 + ecol;
  float bb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bb[j] = 0.0f;
  if (a.bias) load_bias8(a, col, bb);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.res), 0, a.y_bytes, 0x00020000);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    u32x4 res[2];
    if constexpr (RES) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int m = m0 + wm * 128 + i * 16 + erow + 8 * r;
        res[r] = __builtin_amdgcn_raw_buffer_load_b128(
            rr, m < a.M ? (uint32_t)(((int64_t)m * a.Cout + col) * 2) : kOOB, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) sC[(fk * 4 + e) * CS + j * 16 + fr] = acc[i][j][e];
    __builtin_amdgcn_s_waitcnt(kLgkm0);  // one wave owns the slab: no workgroup barrier
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int row = erow + 8 * r, m = m0 + wm * 128 + i * 16 + row;
      const float4 c0 = *reinterpret_cast<const float4*>(sC + row * CS + ecol);
      const float4 c1 = *reinterpret_cast<const float4*>(sC + row * CS + ecol + 4);
      float v[8] = {c0.x + bb[0], c0.y + bb[1], c0.z + bb[2], c0.w + bb[3],
                    c1.x + bb[4], c1.y + bb[5], c1.z + bb[6], c1.w + bb[7]};
      if constexpr (RES) {
        float re[8];
        unpack8(res[r], re);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += re[j];
      }
      if (a.act) {  // 1 ReLU, 2 ReLU6
        const float hi = a.act == 2 ? 6.0f : INFINITY;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fminf(fmaxf(v[j], 0.0f), hi);
      }
      if (m < a.M) *reinterpret_cast<u32x4*>(a.y + (int64_t)m * a.Cout + col) = pack8(v);
    }
    __builtin_amdgcn_s_waitcnt(kLgkm0);  // slab read out before the next pass overwrites it
  }
}

template <bool RES>
hipError_t launch_big(ConvArgs a, hipStream_t s) {
  a.nM = (a.M + 255) / 256;
  a.nN = a.Cout / 256;
  a.nwg = a.nM * a.nN;
  hipLaunchKernelGGL((conv_big_kernel<RES, 4>), dim3(a.nwg), dim3(kBigThreads), 0, s, a);
  return hipGetLastError();
}

// ---- 3x3 / stride-1 convs from a halo tile in LDS ----------------------------
// The LDS-DMA kernel above re-gathers every A row from L2 once per filter tap:
// per 64-channel block a 128-row tile moves 9 × 16 KB of A into the CU, and a
// stage-3/4 layer runs at the per-CU L2→LDS rate (≈70 GB/s; s4 conv2 50 µs ≈
// 1.77 MB per workgroup pair / 70 GB/s).  Here a workgroup owns BM consecutive
// output pixels (m order) and, per 64-channel block, DMAs the input rows those
// pixels touch — their 3x3 neighbourhood, a contiguous pixel range of the NHWC
// input since the rows are whole image rows — into LDS once; all 9 taps read
// their A fragments from that halo image.  A traffic per channel block falls
// from 9·BM·128 B to (rows spanned + 2)·W·128 B (stage 3, BM 256: 295 KB →
// 42 KB), so the weights dominate what a CU takes in and the tile can grow to
// 256 × 128 (8 waves of 64 × 64) at one workgroup per CU.
//
// A fragment addresses are per lane and per tap (pixel → halo row + swizzled
// slot), computed once per tile: 9 × TM registers.  Padding taps and M-tail
// rows point at a zero row — the last row of the halo image, beyond every
// tile's pixel range (the host guarantees the bound), which the DMA fills
// with zeros from out-of-range offsets.  Consecutive pixels map to
// consecutive halo rows for every tap, so the slot ^ (row & 7) swizzle stays
// conflict-free for ds_read_b128 at any row offset.
//
// Pipeline (K order: channel block major, tap minor; K step = tap·cblocks + cb):
// the weight panel of step s+1 is DMA'd while step s multiplies; the halo of
// block cb+1 is DMA'd at tap 0 of block cb behind that panel, into the other
// halo stage, and must land by tap 2.  Past the end the DMAs are dummies
// (out-of-range source → zeros) into stages nobody reads again, so every
// thread issues the same DMA count and the counted vmcnt waits stay exact.
// NMAJOR: workgroups of one XCD share an N tile (weight panels stay in that
// XCD's L2 when the whole filter does not fit, e.g. stage 4: 4.7 MB).
// The wave's 64 x 64 tile is 2 x 2 v_mfma_f32_32x32x16_bf16: half the MFMA
// issues of 4 x 4 16x16x32 for the same operand bytes and 18 instead of 36
// A-address registers (the 16x16 form lost on every halo layer,
// profiles/r4/kernels/convknob_m32.log, and was removed in round 5).
// ST = 1: forward BatchNorm statistics of the stored values (ConvArgs::stats), one
// 64-row group per wave, merged through the wave's own slab.
template <int BM, int BN, int HPMAX, int ST = 0>
__global__ void __launch_bounds__(BM * BN / 64, 2) conv_halo_kernel(const ConvArgs a) {
  static_assert(ST == 0 || ST == 1 || ST == 2, "halo: statistics mode");
  constexpr int T = BM * BN / 64, WN = BN / 64;
  constexpr int TM = 2, TN = 2;                       // wave tile 64 x 64 in 32x32 MFMAs
  constexpr int RPI = T / 8;                          // LDS rows (128 B) per DMA instruction
  constexpr int HI = HPMAX / RPI, BR = BN / RPI;      // DMA instructions per thread: halo, panel
  constexpr int HSTAGE = HPMAX * 128, BSTAGE = BN * 128;
  constexpr int CS = 64 + 4, SLAB = 16 * CS * 4;      // epilogue: per-wave 16-row slab (fp32)
  constexpr int BODY = 2 * HSTAGE + 2 * BSTAGE;
  static_assert(HPMAX % RPI == 0 && BN % RPI == 0, "DMA shape");
  static_assert((T / 64) * SLAB <= BODY, "epilogue slabs fit in the pipeline stages");
  __shared__ __attribute__((aligned(16))) char smem[BODY];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 15, fk = lane >> 4;
  // LDS images: 16-B chunk c of row r sits in slot c ^ f(r).  The 32x32 reads
  // (32 consecutive rows, one k-chunk per 32-lane half) put two rows on one
  // bank group in every ds_read_b128 lane group with f = r & 7 (4 extra LDS
  // cycles per read: SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS = 4.1 in
  // profiles/r4/kernels/pmc_flagship_r4.md), and none with f = (r & 7) ^ bit 3.
  // DMA rows are i·RPI + lrow with RPI a multiple of 16, so f of the LDS row is f(lrow).
  const int lrow = t >> 3;
  const int lchunk = (t & 7) ^ (lrow & 7) ^ ((lrow >> 3) & 1);
  auto swzh = [](int row, int slot) {  // swz() with this kernel's f
    return row * 128 + ((slot ^ (row & 7) ^ ((row >> 3) & 1)) << 4);
  };
  static_assert((T / 8) % 16 == 0, "rows per DMA instruction keep bit 3 of the row");
  int m0, n0;
  if (a.nmajor) {
    const int xcd = blockIdx.x & 7, q = a.nwg >> 3, r8 = a.nwg & 7;
    const int id = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (blockIdx.x >> 3);
    const int ni = id / a.nM;
    m0 = (id - ni * a.nM) * BM;
    n0 = ni * BN;
  } else {
    tile_origin(a, blockIdx.x, BM, BN, m0, n0);
  }
  const int W = a.W, H = a.H;
  const int rows_total = a.N * H;
  const int r0 = m0 / W, mlast = (m0 + BM < a.M ? m0 + BM : a.M) - 1, r1 = mlast / W;
  const int g_lo = r0 > 0 ? r0 - 1 : 0, g_hi = r1 + 1 < rows_total ? r1 + 1 : rows_total - 1;
  const int hp = (g_hi - g_lo + 1) * W;  // halo pixels of this tile (< HPMAX)
  const int pix0 = g_lo * W;

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.x), 0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.w), 0, (uint32_t)((int64_t)a.Cout * a.K * 2), 0x00020000);

  // Halo DMA sources (channel block 0); block cb adds cb·128 B.  A literal
  // array bound: a lambda capturing a local array of value-dependent size
  // fails substitution in the host pass, which then emits no launch stub.
  static_assert(HI <= 6, "halo DMA registers");
  uint32_t hsrc[6];
#pragma unroll
  for (int i = 0; i < HI; ++i) {
    const int h = i * RPI + lrow;
    hsrc[i] = h < hp ? (uint32_t)(((pix0 + h) * a.C + lchunk * 8) * 2) : kOOB;
  }
  const uint32_t boff = (uint32_t)(((n0 + lrow) * a.K + lchunk * 8) * 2);
  auto issue_h = [&](int cb, int hs) {  // cb == cblocks: dummy (zeros into the idle stage)
    char* sH = smem + hs * HSTAGE;
    const bool live = cb < a.cblocks;
#pragma unroll
    for (int i = 0; i < HI; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xr, (lds_void_t*)(sH + (i * RPI + wave * 8) * 128), 16,
          (live && hsrc[i] != kOOB) ? hsrc[i] + (uint32_t)(cb * 128) : kOOB, 0, 0, 0);
  };
  auto issue_b = [&](int kt, int bs) {  // kt < 0: dummy
    char* sB = smem + 2 * HSTAGE + bs * BSTAGE;
#pragma unroll
    for (int i = 0; i < BR; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wr, (lds_void_t*)(sB + (i * RPI + wave * 8) * 128), 16,
          kt >= 0 ? boff + (uint32_t)((i * RPI * a.K + kt * BK) * 2) : kOOB, 0, 0, 0);
  };

  // Per-lane, per-tap A fragment addresses: the byte offset in a halo stage of
  // the lane's k-step-0 chunk, one register per (tap, row tile); pinned per
  // channel block so hipcc cannot hoist derived addresses out of the loop.
  constexpr int ZROW = HPMAX - 1;
  static_assert(HSTAGE <= 65536, "16-bit halo addresses");
  uint32_t aaddr[9][TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * 64 + i * 32 + (lane & 31);
    const bool mok = m < a.M;
    const int row = (mok ? m : m0) / W;
    const int ow = (mok ? m : m0) - row * W, oh = row % H;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int ih = oh + kh - 1, iw = ow + kw - 1;
        const bool v = mok & ((unsigned)ih < (unsigned)H) & ((unsigned)iw < (unsigned)W);
        const int h = v ? (row + kh - 1 - g_lo) * W + iw : ZROW;
        // k-step ks (16 channels) of lane half kb reads chunk 2·ks + kb: the
        // address of ks = that of ks 0 XOR (ks << 5)
        aaddr[kh * 3 + kw][i] = (uint32_t)swzh(h, lane >> 5);
      }
  }

  f32x16_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16_t{};

  // 32x32x16: four 16-channel k-steps per tap; operands of step ks+1 are read
  // while step ks multiplies (lgkmcnt(4): the newer 4 reads may stay in flight).
  auto compute32 = [&](int tap, const char* sH, const char* sB) {
    bf16x8_t af[2][TM], bfr[2][TN];
    auto rd = [&](int ks, int buf) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[buf][i] = *reinterpret_cast<const bf16x8_t*>(sH + (aaddr[tap][i] ^ (uint32_t)(ks << 5)));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[buf][j] = *reinterpret_cast<const bf16x8_t*>(sB + swzh(wn * 64 + j * 32 + (lane & 31), ks * 2 + (lane >> 5)));
    };
    rd(0, 0);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int cur = ks & 1;
      __builtin_amdgcn_sched_barrier(0);
      if (ks < 3) {
        rd(ks + 1, cur ^ 1);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(lgkm_imm(TM + TN));
      } else {
        __builtin_amdgcn_s_waitcnt(kLgkm0);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[cur][i], bfr[cur][j], acc[i][j], 0, 0, 0);
    }
  };

  const int nb = a.cblocks;
  issue_h(0, 0);
  issue_b(0, 0);
  __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
  __builtin_amdgcn_s_barrier();
  int bs = 0;
  for (int cb = 0; cb < nb; ++cb) {
    const int hs = cb & 1;
    const char* sH = smem + hs * HSTAGE;
#pragma unroll
    for (int tp = 0; tp < 9; ++tp)
#pragma unroll
      for (int i = 0; i < TM; ++i) pin_vgpr(aaddr[tp][i]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      // next step's panel: (tap+1, cb), or (0, cb+1) after the last tap; a dummy past the end
      const int kn = tap < 8 ? (tap + 1) * nb + cb : (cb + 1 < nb ? cb + 1 : -1);
      issue_b(kn, bs ^ 1);
      if (tap == 0) {
        issue_h(cb + 1, hs ^ 1);
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(BR + HI));
      } else if (tap == 1) {
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(BR + HI));
      } else {
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(BR));
      }
      __builtin_amdgcn_s_barrier();
      compute32(tap, sH, smem + 2 * HSTAGE + bs * BSTAGE);
      __builtin_amdgcn_s_waitcnt(kLgkm0);
      __builtin_amdgcn_s_barrier();
      bs ^= 1;
    }
  }
  __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));  // trailing dummy DMAs, before the slabs reuse LDS
  __builtin_amdgcn_s_barrier();

  // Epilogue: per wave, four 16-row passes through its own slab (no workgroup barrier).
  float* sC = reinterpret_cast<float*>(smem + wave * SLAB);
  const int ecol = (lane & 7) * 8, erow = lane >> 3;
  const int col = n0 + wn * 64 + ecol;
  float bb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bb[j] = 0.0f;
  if (a.bias) load_bias8(a, col, bb);
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.0f;
  // ST = 2 (a data gradient feeding a BN backward): the BN's x and coefficients
  // (vgpu_conv2d_nhwc_bn), x read per pass beside the accumulator staging.
  float ks_[8], kt_[8], kmu[8], kis[8];
  const __amdgpu_buffer_rsrc_t xr2 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(ST == 2 ? a.bnx : a.y), 0, ST == 2 ? a.y_bytes : 0u, 0x00020000);
  if constexpr (ST == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ks_[j] = a.bncoef[col + j];
      kt_[j] = a.bncoef[a.Cout + col + j];
      kmu[j] = a.bncoef[2 * a.Cout + col + j];
      kis[j] = a.bncoef[3 * a.Cout + col + j];
    }
  }
  // Pass p = half (p & 1) of row tile p >> 1; lane l holds rows
  // 8b + 4(l >> 5) + e (b = 0..3) of column l & 31.
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    u32x4 xb[2];
    if constexpr (ST == 2) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int m = m0 + wm * 64 + p * 16 + erow + 8 * r;
        xb[r] = __builtin_amdgcn_raw_buffer_load_b128(
            xr2, m < a.M ? (uint32_t)(((int64_t)m * a.Cout + col) * 2) : kOOB, 0, 0);
      }
    }
    {
      const int i = p >> 1, hb = (p & 1) * 2;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            sC[(8 * b + 4 * (lane >> 5) + e) * CS + j * 32 + (lane & 31)] = acc[i][j][4 * (hb + b) + e];
    }
    __builtin_amdgcn_s_waitcnt(kLgkm0);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int row = erow + 8 * r, m = m0 + wm * 64 + p * 16 + row;
      const float4 c0 = *reinterpret_cast<const float4*>(sC + row * CS + ecol);
      const float4 c1 = *reinterpret_cast<const float4*>(sC + row * CS + ecol + 4);
      float v[8] = {c0.x + bb[0], c0.y + bb[1], c0.z + bb[2], c0.w + bb[3],
                    c1.x + bb[4], c1.y + bb[5], c1.z + bb[6], c1.w + bb[7]};
      if (a.act) {  // 1 ReLU, 2 ReLU6
        const float hi = a.act == 2 ? 6.0f : INFINITY;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fminf(fmaxf(v[j], 0.0f), hi);
      }
      float xf[8];
      if constexpr (ST == 2) {
        unpack8(xb[r], xf);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= bn_act_grad(a.bnact, fmaf(xf[j], ks_[j], kt_[j]));
      }
      const u32x4 o = pack8(v);
      if (m < a.M) *reinterpret_cast<u32x4*>(a.y + (int64_t)m * a.Cout + col) = o;
      if constexpr (ST != 0) {
        float q[8];
        unpack8(o, q);
        const float ok = m < a.M ? 1.0f : 0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = q[j] * ok;
          s1[j] += d;
          s2[j] = fmaf(d, ST == 2 ? (xf[j] - kmu[j]) * kis[j] : d, s2[j]);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(kLgkm0);
  }
  if constexpr (ST != 0) {
    // lanes of one column chunk (lane & 7) hold erow = lane >> 3: merge the 8 rows
    float2* sS = reinterpret_cast<float2*>(sC);
#pragma unroll
    for (int j = 0; j < 8; ++j) sS[erow * 64 + ecol + j] = make_float2(s1[j], s2[j]);
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    const int g = (m0 + wm * 64) / 64;
    if (g * 64 < a.M) {
      float2 r = make_float2(0.0f, 0.0f);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float2 p = sS[q * 64 + lane];
        r.x += p.x;
        r.y += p.y;
      }
      a.stats[(int64_t)g * a.Cout + n0 + wn * 64 + lane] = r;
    }
  }
}

int g_forced_halo = -1;  // vgpu_conv_set_halo: -1 = env VGPU_CONV_HALO, 0 = off, 1 = on, 2 / 3 = on with BM 256 / 128

bool halo_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* v = getenv("VGPU_CONV_HALO");
    on = (v && (v[0] == '0' || v[0] == 'n' || v[0] == 'f')) ? 0 : 1;
  }
  return on == 1;
}

unsigned long long g_halo_launches = 0;  // vgpu_conv_halo_launches (tests: the halo path ran)

template <int BM, int BN, int HPMAX>
hipError_t launch_halo(ConvArgs a, hipStream_t s) {
  ++g_halo_launches;
  a.nM = (a.M + BM - 1) / BM;
  a.nN = a.Cout / BN;
  a.nwg = a.nM * a.nN;
  // N-major placement when the filter outgrows an XCD's L2 share (4 MiB).
  a.nmajor = (int64_t)a.Cout * a.K * 2 > ((int64_t)5 << 19) ? 1 : 0;
  if (a.stats && a.bnx)
    hipLaunchKernelGGL((conv_halo_kernel<BM, BN, HPMAX, 2>), dim3(a.nwg), dim3(BM * BN / 64), 0, s, a);
  else if (a.stats)
    hipLaunchKernelGGL((conv_halo_kernel<BM, BN, HPMAX, 1>), dim3(a.nwg), dim3(BM * BN / 64), 0, s, a);
  else
    hipLaunchKernelGGL((conv_halo_kernel<BM, BN, HPMAX>), dim3(a.nwg), dim3(BM * BN / 64), 0, s, a);
  return hipGetLastError();
}

// Halo pixels a BM-pixel tile of a W-wide image can need: rows spanned + 2.
inline int halo_pixels(int bm, int w) { return ((bm - 1) / w + 4) * w; }

// 3x3 / stride 1 / pad 1, no prologue / residual, Cout % 128 == 0.  Returns
// hipErrorNotSupported when no halo instantiation fits (the caller falls back).
hipError_t dispatch_halo(const ConvArgs& a, hipStream_t s) {
  if (a.Cout % 128) return hipErrorNotSupported;
  const int64_t tiles256 = (int64_t)((a.M + 255) / 256) * (a.Cout / 128);
  const bool big = g_forced_halo == 2 || (g_forced_halo != 3 && tiles256 * 5 >= (int64_t)conv_cus() * 3);
  if (big && halo_pixels(256, a.W) <= 383) return launch_halo<256, 128, 384>(a, s);
  if (g_forced_halo != 2 && halo_pixels(128, a.W) <= 191) return launch_halo<128, 128, 192>(a, s);
  return hipErrorNotSupported;
}

int g_forced_big = -1;  // vgpu_conv_set_big: -1 = env VGPU_CONV_BIG / heuristic, 0 = off, 1 = whenever eligible

int g_forced_bm = 0;  // vgpu_conv_set_tile_m (A/B benchmarking); 0 = heuristic

template <int KS, int BM, int BN, bool RES, int CSM = 0, int ST = 0>
hipError_t launch_glds(ConvArgs a, hipStream_t s) {
  a.nM = (a.M + BM - 1) / BM;
  a.nN = a.Cout / BN;
  a.nwg = a.nM * a.nN;
  hipLaunchKernelGGL((conv_glds_kernel<KS, BM, BN, RES, CSM, ST>), dim3(a.nwg), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

template <int KS, int BM>
hipError_t dispatch_glds(const ConvArgs& a, bool res, hipStream_t s) {
  if (a.stats) {  // training BatchNorm statistics in the epilogue (backward: no residual)
    const bool bwd = a.bnx != nullptr;
    if (a.Cout % 128 == 0)
      return bwd ? (res ? launch_glds<KS, BM, 128, true, 0, 2>(a, s) : launch_glds<KS, BM, 128, false, 0, 2>(a, s))
                 : (res ? launch_glds<KS, BM, 128, true, 0, 1>(a, s) : launch_glds<KS, BM, 128, false, 0, 1>(a, s));
    return bwd ? (res ? launch_glds<KS, BM, 64, true, 0, 2>(a, s) : launch_glds<KS, BM, 64, false, 0, 2>(a, s))
               : (res ? launch_glds<KS, BM, 64, true, 0, 1>(a, s) : launch_glds<KS, BM, 64, false, 0, 1>(a, s));
  }
  if (a.Cout % 128 == 0)
    return res ? launch_glds<KS, BM, 128, true>(a, s) : launch_glds<KS, BM, 128, false>(a, s);
  return res ? launch_glds<KS, BM, 64, true>(a, s) : launch_glds<KS, BM, 64, false>(a, s);
}

// ---- Prologue convs (block-entry BN+ReLU on the input): A through registers,
// B through LDS-DMA.
//
// The prologue must touch every A element once, so A keeps the register path
// (global → VGPR → affine+ReLU → ds_write, zero padding re-applied after the
// prologue).  The weights need no transform and go HBM → LDS by DMA, which
// halves the ds_write_b128 traffic that bounds the all-register kernel.
// Pipeline: see the K loop (A two steps ahead in registers, B one step ahead
// by DMA).
template <int KS, int BM, int BN, bool RES>
__global__ void __launch_bounds__(kThreads, 2) conv_pro_kernel(const ConvArgs a) {
  constexpr int AR = BM / 32, BR = BN / 32;
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int PIPE = 2 * STAGE, EPI = (BM / 2) * (BN + 4) * 4;
  constexpr int BODY = PIPE > EPI ? PIPE : EPI;
  // BN scale/shift of the input channels.  64-row tiles: they travel with the
  // K step's A rows, loaded into registers with them two steps ahead — an LDS
  // copy of all C channels costs 16 KB and with it the third workgroup per CU.
  // 128-row tiles (two workgroups per CU either way): one LDS copy, read per
  // step (the register form measured 2-7 % slower there: 58 more VGPRs).
  // Never ordinary global loads in the loop: beside the DMA they make hipcc
  // drain vmcnt(0).
  constexpr bool PREG = BM == 64;
  constexpr int PR = PREG ? 4 : 0;  // 16-B parameter loads per K step: 8 scales, 8 shifts
  __shared__ __attribute__((aligned(16))) char smem[BODY + (PREG ? 0 : 2048 * 2 * 4)];
  float* sPar = reinterpret_cast<float*>(smem + BODY);

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fk = lane >> 4;
  const int slot = t & 7, r0 = t >> 3;
  const int lchunk = slot ^ (r0 & 7);  // DMA source chunk (swizzle on the source)
  int m0, n0;
  tile_origin(a, blockIdx.x, BM, BN, m0, n0);

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.x), 0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.w), 0, (uint32_t)((int64_t)a.Cout * a.K * 2), 0x00020000);

  int abase[AR], aih[AR], aiw[AR];
  bool aok[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + r0 + 32 * i;
    aok[i] = m < a.M;
    const int mm = aok[i] ? m : 0;
    const int ow = mm % a.OW, t2 = mm / a.OW, oh = t2 % a.OH, n = t2 / a.OH;
    aih[i] = oh * a.stride - a.pad;
    aiw[i] = ow * a.stride - a.pad;
    abase[i] = ((n * a.H + aih[i]) * a.W + aiw[i]) * a.C * 2;
  }
  const uint32_t boff = (uint32_t)(((n0 + r0) * a.K + lchunk * 8) * 2);
  const __amdgpu_buffer_rsrc_t psr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.pscale), 0, (uint32_t)(a.C * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t ptr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.pshift), 0, (uint32_t)(a.C * 4), 0x00020000);
  if constexpr (!PREG) {
    for (int c = t * 4; c < a.C; c += kThreads * 4) {
      *reinterpret_cast<float4*>(sPar + c) = *reinterpret_cast<const float4*>(a.pscale + c);
      *reinterpret_cast<float4*>(sPar + a.C + c) = *reinterpret_cast<const float4*>(a.pshift + c);
    }
    __syncthreads();
  }

  auto issue_b = [&](int kt, int st) {
    char* sB = smem + st * STAGE + A_BYTES;
#pragma unroll
    for (int i = 0; i < BR; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wr, (lds_void_t*)(sB + (32 * i + wave * 8) * 128), 16,
          boff + (uint32_t)((32 * i * a.K + kt * BK) * 2), 0, 0, 0);
  };
  auto load_a = [&](int kt, u32x4 (&ra)[AR], bool (&rv)[AR], u32x4 (&rp)[PR ? PR : 1]) {
    // 1x1: K = C, so the tap is 0 and the K step is the channel block.
    const int tap = KS == 1 ? 0 : kt / a.cblocks, cb = kt - tap * a.cblocks;
    const int kh = tap / KS, kw = tap - kh * KS;
    const int toff = ((kh * a.W + kw) * a.C + cb * BK + slot * 8) * 2;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      // Bitwise (not short-circuit) validity: no exec-mask branch around the load.
      const int ih = aih[i] + kh, iw = aiw[i] + kw;
      const bool v = aok[i] & ((unsigned)ih < (unsigned)a.H) & ((unsigned)iw < (unsigned)a.W);
      rv[i] = v;
      ra[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, v ? (uint32_t)(abase[i] + toff) : kOOB, 0, 0);
    }
    if constexpr (PREG) {
      const uint32_t po = (uint32_t)((cb * BK + slot * 8) * 4);
      rp[0] = __builtin_amdgcn_raw_buffer_load_b128(psr, po, 0, 0);
      rp[1] = __builtin_amdgcn_raw_buffer_load_b128(psr, po + 16, 0, 0);
      rp[2] = __builtin_amdgcn_raw_buffer_load_b128(ptr, po, 0, 0);
      rp[3] = __builtin_amdgcn_raw_buffer_load_b128(ptr, po + 16, 0, 0);
    }
  };
  auto store_a = [&](int kt, int st, u32x4 (&ra)[AR], const bool (&rv)[AR], u32x4 (&rp)[PR ? PR : 1]) {
    char* sA = smem + st * STAGE;
    // Pin the staged registers here: without it hipcc hoists this step's
    // unpacking into the previous step, ahead of that step's barrier, and
    // waits for the loads a step early.
#pragma unroll
    for (int i = 0; i < AR; ++i) asm volatile("" : "+v"(ra[i]));
    float sc[8], sh[8];
    if constexpr (PREG) {
#pragma unroll
      for (int i = 0; i < PR; ++i) asm volatile("" : "+v"(rp[i]));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sc[j] = __uint_as_float(rp[0][j]);
        sc[4 + j] = __uint_as_float(rp[1][j]);
        sh[j] = __uint_as_float(rp[2][j]);
        sh[4 + j] = __uint_as_float(rp[3][j]);
      }
    } else {
      const int c = (KS == 1 ? kt : kt % a.cblocks) * BK + slot * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sc[j] = sPar[c + j];
        sh[j] = sPar[a.C + c + j];
      }
    }
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      float e[8];
      unpack8(ra[i], e);
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = fmaxf(e[j] * sc[j] + sh[j], 0.0f);
      u32x4 p = pack8(e);
      // Zero padding stays zero after the prologue.  A 1x1 conv has no
      // padding, and an M-tail row only feeds its own (never stored) output
      // row, so it skips the select.
      if constexpr (KS != 1) p = rv[i] ? p : u32x4{0u, 0u, 0u, 0u};
      *reinterpret_cast<u32x4*>(sA + swz(r0 + 32 * i, slot)) = p;
    }
  };
  auto compute = [&](int st, f32x4_t (&acc)[TM][TN]) {
    const char* sA = smem + st * STAGE;
    const char* sB = sA + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8_t*>(sA + swz(wm * WTM + i * 16 + fr, kk * 4 + fk));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(sB + swz(wn * WTN + j * 16 + fr, kk * 4 + fk));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  u32x4 ra0[AR], ra1[AR], rp0[PR ? PR : 1], rp1[PR ? PR : 1];
  bool rv0[AR], rv1[AR];
  const int nk = a.ktiles;
  u32x4 res[2][EpiShape<BM, BN>::RROWS];
  // Per K step kt (stage st = kt & 1 holds A(kt), B(kt)):
  //   prologue + ds_write of A(kt+1) into stage st^1 (registers X, loaded two
  //   steps ago, with its channels' BN scale/shift) · DMA B(kt+1) into st^1 ·
  //   load A(kt+3) into X · MFMA on st · vmcnt(AR + PR): retires B(kt+1) and
  //   A(kt+2) (set Y, loaded one step ago), leaves A(kt+3) in flight · barrier.
  // Every ds_write of a step precedes its DMA: hipcc makes a ds_write wait for
  // all LDS-DMA in flight, which would serialise the pipeline.  The loads of
  // A(kt+3) are issued behind the DMA, so the step's own wait does not retire
  // them: they get two steps of lead.
  load_a(0, ra0, rv0, rp0);
  load_a(nk > 1 ? 1 : 0, ra1, rv1, rp1);
  store_a(0, 0, ra0, rv0, rp0);
  issue_b(0, 0);
  load_a(nk > 2 ? 2 : nk - 1, ra0, rv0, rp0);
  __builtin_amdgcn_s_waitcnt(vmcnt_imm(AR + PR));
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  __builtin_amdgcn_s_barrier();
  // Unrolled by two so the register sets stay static: step kt stores set X
  // and refills it with A(kt+3).
  // Branch-free body: past the last K step the loads re-fetch the last tile into
  // the idle stage (never read) — a branch around a load would make hipcc wait
  // vmcnt(0) there and de-pipeline the loop.
  auto step = [&](int kt, u32x4 (&rx)[AR], bool (&vx)[AR], u32x4 (&px)[PR ? PR : 1]) {
    const int st = kt & 1;
    const int k1 = kt + 1 < nk ? kt + 1 : nk - 1, k3 = kt + 3 < nk ? kt + 3 : nk - 1;
    // sched_barriers keep hipcc's scheduler from reordering the phases (it
    // would hoist the A loads above the ds_writes — so the step's wait retires
    // them — and sink the MFMAs below the wait).
    store_a(k1, st ^ 1, rx, vx, px);
    __builtin_amdgcn_sched_barrier(0);
    issue_b(k1, st ^ 1);
    __builtin_amdgcn_sched_barrier(0);
    load_a(k3, rx, vx, px);
    __builtin_amdgcn_sched_barrier(0);
    compute(st, acc);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(vmcnt_imm(AR + PR));
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_s_barrier();
  };
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(kt, ra1, rv1, rp1);
    step(kt + 1, ra0, rv0, rp0);
  }
  if (kt < nk) step(kt, ra1, rv1, rp1);
  __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));  // the trailing dummy loads, before LDS reuse
  __syncthreads();
  if constexpr (RES) load_residual<BM, BN>(a, m0, n0, res);
  epilogue_halves<BM, BN, RES>(a, acc, m0, n0, smem, res);
}

template <int KS, int BM, int BN, bool RES>
hipError_t launch_pro(ConvArgs a, hipStream_t s) {
  a.nM = (a.M + BM - 1) / BM;
  a.nN = a.Cout / BN;
  a.nwg = a.nM * a.nN;
  hipLaunchKernelGGL((conv_pro_kernel<KS, BM, BN, RES>), dim3(a.nwg), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

template <int KS, int BM>
hipError_t dispatch_pro(const ConvArgs& a, bool res, hipStream_t s) {
  if (a.Cout % 128 == 0)
    return res ? launch_pro<KS, BM, 128, true>(a, s) : launch_pro<KS, BM, 128, false>(a, s);
  return res ? launch_pro<KS, BM, 64, true>(a, s) : launch_pro<KS, BM, 64, false>(a, s);
}

// conv23's conv3-chunk epilogue, one row half at a time: fp32 accumulators →
// LDS staging → + residual → bf16 y.  The stores are unconditional buffer
// stores (rows past M go to an out-of-range offset and are dropped), so every
// thread issues exactly 2·RROWS of them: the kernel's counted vmcnt waits rely
// on that count.  Barriers are raw (lgkmcnt only), so an LDS-DMA issued before
// the epilogue's last LDS write (`mid`) stays in flight across the rest of it
// (a __syncthreads() would drain it).
// NEXT: also p = relu(bf16(y) * s[c] + t[c]) (the next block-entry BN+ReLU,
// rounded to bf16 exactly as conv_pro's prologue stages it) for this thread's
// rows, into registers; s/t are read from LDS (sPs/sPt), never from global
// memory, for the same reason.
template <int BM, int BN, bool NEXT, int NT = kThreads, typename Mid>
__device__ __forceinline__ void tail_epilogue(const ConvArgs& a, f32x4_t (&acc)[BM / (NT / 128) / 16][BN / 32],
                                              int m0, int n0, char* smem,
                                              const u32x4 (&res)[2][EpiShape<BM, BN, NT>::RROWS],
                                              const float* sPs, const float* sPt,
                                              u32x4 (&pv)[2][EpiShape<BM, BN, NT>::RROWS], Mid mid) {
  constexpr int WGM = NT / 128, WPH = WGM / 2;
  constexpr int WTM = BM / WGM, WTN = BN / 2, TM = WTM / 16, TN = WTN / 16;
  constexpr int CS = BN + 4, HROWS = BM / 2;
  using E = EpiShape<BM, BN, NT>;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1, fr = lane & 15, fk = lane >> 4;
  const int chunk = t % E::CPR, rfirst = t / E::CPR;
  const int col = n0 + chunk * 8;
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(a.y, 0, a.y_bytes, 0x00020000);
  float sc[8], sh[8];
  if constexpr (NEXT) {
    const float4 s0 = *reinterpret_cast<const float4*>(sPs + col);
    const float4 s1 = *reinterpret_cast<const float4*>(sPs + col + 4);
    const float4 h0 = *reinterpret_cast<const float4*>(sPt + col);
    const float4 h1 = *reinterpret_cast<const float4*>(sPt + col + 4);
    sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w; sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
    sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w; sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
  }
  float* sC = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (wm / WPH == h) {
      const int r0 = (wm % WPH) * WTM;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            sC[(r0 + i * 16 + fk * 4 + e) * CS + wn * WTN + j * 16 + fr] = acc[i][j][e];
    }
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_s_barrier();
    // This half's staged rows + residual, all read before `mid`: an LDS-DMA
    // issued by `mid` (past the epilogue's last LDS access — hipcc drains every
    // in-flight LDS-DMA at the next ds_read/ds_write) overlaps the stores.
    float v[E::RROWS][8];
#pragma unroll
    for (int i = 0; i < E::RROWS; ++i) {
      const int r = rfirst + E::RSTEP * i;
      const float4 c0 = *reinterpret_cast<const float4*>(sC + r * CS + chunk * 8);
      const float4 c1 = *reinterpret_cast<const float4*>(sC + r * CS + chunk * 8 + 4);
      float re[8];
      unpack8(res[h][i], re);
      v[i][0] = c0.x + re[0]; v[i][1] = c0.y + re[1]; v[i][2] = c0.z + re[2]; v[i][3] = c0.w + re[3];
      v[i][4] = c1.x + re[4]; v[i][5] = c1.y + re[5]; v[i][6] = c1.z + re[6]; v[i][7] = c1.w + re[7];
    }
    if (h == 1) {
      __builtin_amdgcn_s_waitcnt(kLgkm0);
      __builtin_amdgcn_s_barrier();  // every wave's staging reads done
      __builtin_amdgcn_sched_barrier(0);
      mid();
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < E::RROWS; ++i) {
      const int r = rfirst + E::RSTEP * i, m = m0 + h * HROWS + r;
      const u32x4 yv = pack8(v[i]);
      __builtin_amdgcn_raw_buffer_store_b128(yv, yr, m < a.M ? (uint32_t)(((int64_t)m * a.Cout + col) * 2) : kOOB,
                                             0, 0);
      if constexpr (NEXT) {
        float q[8];
        unpack8(yv, q);
#pragma unroll
        for (int j = 0; j < 8; ++j) q[j] = fmaxf(q[j] * sc[j] + sh[j], 0.0f);
        pv[h][i] = pack8(q);
      }
    }
    if (h == 0) {
      __builtin_amdgcn_s_waitcnt(kLgkm0);
      __builtin_amdgcn_s_barrier();  // half 0 read out before half 1 is staged
    }
  }
}

// ---- Fused bottleneck tail: conv2 (3x3, W→W, bias+ReLU) → conv3 (1x1, W→4W)
// + residual, one kernel per row tile.
//
// The conv2 output tile (BM rows × all W channels) never leaves the CU: its
// bias+ReLU'd bf16 values are written straight into LDS in the swizzled A-tile
// layout and become conv3's A operand; conv3 then sweeps its 4W outputs in
// 128-wide chunks whose weight panels are DMA'd into the (now idle) conv2
// pipeline stages.  Per bottleneck this removes the write and the re-read of
// the conv2 activation and one kernel boundary (stage 1 at b=50, 346²: 96 MB
// of HBM traffic per block).  Numerics equal the unfused pair (the conv2
// output is rounded to bf16 exactly where the unfused kernel stores it).
//
// Phase 1 is the LDS-DMA conv loop with the transposed MFMA (mfma(B, A)) so a
// lane holds 4 consecutive conv2 channels of one row: one 8-byte ds_write per
// 16×16 subtile lands them in the conv3 A image.
// NEXT: also the NEXT block's conv1 (1x1, 4W→W, BN+ReLU prologue, bias+ReLU
// epilogue; ConvArgs c) on the conv3 output while it is on chip: after each
// 128-channel conv3 chunk, its BN+ReLU'd bf16 values become a K chunk of conv1's
// A operand (an image in the epilogue staging area) and the matching 128-row K
// chunk of conv1's weights is DMA'd into the conv3 panel slot, so h1 of the next
// block accumulates in registers across the chunks.  Saves the next block's
// re-read of the 4W-wide activation (stage 1 at b=50: 194 MB per block).
// Numerics equal conv23 + conv_pro (same bf16 roundings, same K order).
// NT: the workgroup runs (NT / 128) x 2 waves of 32 x 64 (or 64 x 64) sub-tiles.
// Round 5 measured NT = 512 with 128-row stage-2 tiles -- half the weight-panel
// L2 traffic per row (profiles/r5/kernels/pmc_l2_r5.md) -- and a 3-stage vs a
// 2-stage conv2 ring: the ring won 0.5 %, the wide tile lost 0.5 % (one
// workgroup per CU); the tails are latency-, not L2-bandwidth-bound.
template <int BM, int W, bool NEXT = false, int NS1 = 3, int NT = kThreads>
__global__ void __launch_bounds__(NT, 512 / NT) conv23_kernel(const ConvArgs a, const ConvArgs b,
                                                              const ConvArgs c) {
  constexpr int KCH = W / 64;                // conv3 K chunks (64 channels each)
  constexpr int RPI = NT / 8;                // LDS rows per DMA instruction
  constexpr int WGM = NT / 128;              // wave rows (x 2 wave columns)
  constexpr int AR = BM / RPI, BR = W / RPI; // phase-1 DMA instructions per thread per step
  constexpr int WTM = BM / WGM, WTN = W / 2;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_BYTES = BM * 128, B_BYTES = W * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int BN2 = 128, TN2 = 4;           // conv3 output chunk; 64 columns per wave
  constexpr int B2_BYTES = BN2 * 128 * KCH;
  constexpr int EPI = (BM / 2) * (BN2 + 4) * 4;
  constexpr int A2_BYTES = BM * 128 * KCH;
  // Phase 1's NS1-stage DMA ring and phase 2's [conv3 panel | epilogue staging |
  // conv3 A image] share one region: the A image is written only after the
  // last phase-1 step, so a 3-deep ring still leaves two workgroups per CU.
  constexpr int P1 = NS1 * STAGE, P2 = B2_BYTES + EPI + A2_BYTES;
  constexpr int P = P1 > P2 ? P1 : P2;
  // conv2 bias [W] and (NEXT) conv1's prologue scale/shift [4W] each live in
  // LDS: a global load in phase 2 would make hipcc drain the in-flight DMA.
  constexpr int PAR = (W + (NEXT ? 8 * W : 0)) * 4;
  static_assert(P + PAR <= 160 * 1024, "conv23: LDS");
  static_assert(NT == 512 || 2 * (P + PAR) <= 160 * 1024, "conv23: two workgroups per CU");
  __shared__ __attribute__((aligned(16))) char smem[P + PAR];
  char* sA2 = smem + B2_BYTES + EPI;
  float* sPar = reinterpret_cast<float*>(smem + P);

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fk = lane >> 4;
  const int lrow = t >> 3, lchunk = (t & 7) ^ (lrow & 7);
  int m0, n0;
  tile_origin(a, blockIdx.x, BM, W, m0, n0);  // n0 == 0: one tile spans all of conv2's W outputs

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.x), 0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.w), 0, (uint32_t)((int64_t)a.Cout * a.K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t w3r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(b.w), 0, (uint32_t)((int64_t)b.Cout * b.K * 2), 0x00020000);

  int abase[AR], aih[AR], aiw[AR];
  bool aok[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + lrow + RPI * i;
    aok[i] = m < a.M;
    const int mm = aok[i] ? m : 0;
    const int ow = mm % a.OW, t2 = mm / a.OW, oh = t2 % a.OH, n = t2 / a.OH;
    aih[i] = oh * a.stride - a.pad;
    aiw[i] = ow * a.stride - a.pad;
    abase[i] = ((n * a.H + aih[i]) * a.W + aiw[i]) * a.C * 2;
  }
  const uint32_t boff = (uint32_t)((lrow * a.K + lchunk * 8) * 2);
  for (int i = t * 4; i < W; i += NT * 4)
    *reinterpret_cast<float4*>(sPar + i) = *reinterpret_cast<const float4*>(a.bias + i);
  if constexpr (NEXT) {
    for (int i = t * 4; i < 4 * W; i += NT * 4) {
      *reinterpret_cast<float4*>(sPar + W + i) = *reinterpret_cast<const float4*>(c.pscale + i);
      *reinterpret_cast<float4*>(sPar + 5 * W + i) = *reinterpret_cast<const float4*>(c.pshift + i);
    }
  }
  __syncthreads();

  auto issue = [&](int kt, int st) {
    char* sA = smem + st * STAGE;
    char* sB = sA + A_BYTES;
    const int tap = kt / a.cblocks, cb = kt - tap * a.cblocks;
    const int kh = tap / 3, kw = tap - kh * 3;
    const int toff = ((kh * a.W + kw) * a.C + cb * BK + lchunk * 8) * 2;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int ih = aih[i] + kh, iw = aiw[i] + kw;
      const bool v = aok[i] & ((unsigned)ih < (unsigned)a.H) & ((unsigned)iw < (unsigned)a.W);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xr, (lds_void_t*)(sA + (RPI * i + wave * 8) * 128), 16,
          v ? (uint32_t)(abase[i] + toff) : kOOB, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wr, (lds_void_t*)(sB + (RPI * i + wave * 8) * 128), 16,
          boff + (uint32_t)((RPI * i * a.K + kt * BK) * 2), 0, 0, 0);
  };

  // ---- phase 1: conv2 --------------------------------------------------------------
  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  {
    // Two steps in flight behind the MMA, one barrier per step: step kt's wait
    // + barrier also proves every wave finished step kt-1's reads of the stage
    // that issue(kt+2) refills.
    static_assert(NS1 == 3, "conv23: 3-stage phase 1");
    issue(0, 0);
    if (a.ktiles > 1) issue(1, 1);
    int st = 0;
    for (int kt = 0; kt < a.ktiles; ++kt) {
      if (kt + 1 < a.ktiles)
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(AR + BR));
      else
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
      __builtin_amdgcn_s_waitcnt(kLgkm0);
      __builtin_amdgcn_s_barrier();
      if (kt + 2 < a.ktiles) issue(kt + 2, st == 0 ? 2 : st - 1);
      const char* sA = smem + st * STAGE;
      mma_k64<TM, TN, true>(sA, sA + A_BYTES, wm * WTM, wn * WTN, fr, fk, acc);
      st = st == 2 ? 0 : st + 1;
    }
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_s_barrier();  // the stages are read out before the A image overwrites them
  }

  // ---- phase 2: conv3 over 128-wide output chunks --------------------------------
  // Per chunk ch the weight panel w3(ch) and the residual res(ch) are issued
  // one step ahead (behind the previous chunk's work), so the chunk starts on a
  // counted vmcnt that leaves the residual — and, without NEXT, the previous
  // chunk's y stores — in flight:
  //   wait w3(ch) · conv3 MMA · vmcnt(0) (res landed) · barrier ·
  //   NEXT: load w1(ch) to registers ‖ epilogue + p · A3 image · w1 → LDS ·
  //         conv1 MMA · issue w3/res(ch+1)
  //   else: epilogue, with the DMA of w3(ch+1) issued behind its last LDS
  //         write · issue res(ch+1)
  // VMEM ops complete in issue order (loads, stores and LDS-DMA alike), so a
  // counted wait retires everything older than its window; the epilogue's
  // stores are unconditional, so their count is exact.  w1 goes through
  // registers because hipcc drains every in-flight LDS-DMA at the next
  // ds_write, and the epilogue and the A3 image are all ds_writes.
  using E2 = EpiShape<BM, 128, NT>;
  constexpr int R = 2 * E2::RROWS;  // residual loads = y stores per thread per chunk
  constexpr int WTM2 = BM / WGM, TM2 = WTM2 / 16;
  char* sB2 = smem;
  char* sE = smem + B2_BYTES;
  const int nchunks = b.Cout / BN2;
  auto issue_w3 = [&](int ch) {
#pragma unroll
    for (int kc = 0; kc < KCH; ++kc)
#pragma unroll
      for (int i = 0; i < BN2 / RPI; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            w3r, (lds_void_t*)(sB2 + kc * (BN2 * 128) + (RPI * i + wave * 8) * 128), 16,
            (uint32_t)(((ch * BN2 + lrow + RPI * i) * b.K + kc * 64 + lchunk * 8) * 2), 0, 0, 0);
  };
  u32x4 res[2][E2::RROWS];
  // res(0) flies while the conv2 tile is turned into conv3's A image; w3(0)
  // goes into the (free) phase-1 stages after that image's ds_writes, which
  // would otherwise drain it.
  load_residual<BM, BN2, false, NT>(b, m0, 0, res);

  // conv2 bias + ReLU → bf16 → conv3's A image: lane (fr, fk) of subtile (i, j)
  // holds row i*16+fr (+wave offset), channels j*16+fk*4 .. +3.
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cc0 = wn * WTN + j * 16 + fk * 4;
    const float4 bb = *reinterpret_cast<const float4*>(sPar + cc0);
    const int panel = cc0 >> 6, cc = cc0 & 63;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = wm * WTM + i * 16 + fr;
      const float v0 = fmaxf(acc[i][j][0] + bb.x, 0.f), v1 = fmaxf(acc[i][j][1] + bb.y, 0.f);
      const float v2 = fmaxf(acc[i][j][2] + bb.z, 0.f), v3 = fmaxf(acc[i][j][3] + bb.w, 0.f);
      *reinterpret_cast<uint2*>(sA2 + panel * (BM * 128) + swz(r, cc >> 3) + (cc & 7) * 2) =
          uint2{pack2(v0, v1), pack2(v2, v3)};
    }
  }

  issue_w3(0);

  // phase 3 (NEXT): conv1 of the next block, W outputs per row, K = 4W
  constexpr int TM3 = BM / WGM / 16, TN3 = W / 32;
  f32x4_t acc3[TM3][TN3];
  if constexpr (NEXT) {
#pragma unroll
    for (int i = 0; i < TM3; ++i)
#pragma unroll
      for (int j = 0; j < TN3; ++j) acc3[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  const __amdgpu_buffer_rsrc_t w1r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(NEXT ? c.w : b.w), 0, NEXT ? (uint32_t)((int64_t)c.Cout * c.K * 2) : 0u,
      0x00020000);
  for (int ch = 0; ch < nchunks; ++ch) {
    const int c0 = ch * BN2;
    // w3(ch) landed; res(ch) may fly, and without NEXT the previous chunk's
    // second-half stores (issued after w3(ch), behind the epilogue's last ds_write)
    if (ch == 0)
      __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));  // res(0) was issued before w3(0)
    else if (NEXT)
      __builtin_amdgcn_s_waitcnt(vmcnt_imm(R));
    else
      __builtin_amdgcn_s_waitcnt(vmcnt_imm(R + R / 2));
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_s_barrier();  // B2 visible; A2 written (first chunk); previous staging read out
    f32x4_t acc2[TM2][TN2];
#pragma unroll
    for (int i = 0; i < TM2; ++i)
#pragma unroll
      for (int j = 0; j < TN2; ++j) acc2[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KCH; ++kc)
      mma_k64<TM2, TN2>(sA2 + kc * (BM * 128), sB2 + kc * (BN2 * 128), wm * WTM2, wn * 64, fr, fk, acc2);
    // res(ch) landed before any DMA is issued behind it (hipcc would otherwise
    // drain that DMA at the residual's first use); B2 read out by every wave
    // before the next DMA overwrites it.
    __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_s_barrier();
    u32x4 pv[2][E2::RROWS];
    if constexpr (!NEXT) {
      const bool more = ch + 1 < nchunks;
      tail_epilogue<BM, BN2, false, NT>(b, acc2, m0, c0, sE, res, sPar, sPar, pv, [&] {
        if (more) issue_w3(ch + 1);
      });
      if (more) load_residual<BM, BN2, false, NT>(b, m0, c0 + BN2, res);
    } else {
      // conv1's weight K chunk [W rows][c0 .. c0+127] (two 64-wide K panels of
      // W rows), in flight in registers behind the epilogue.
      u32x4 w1v[2][W / RPI];
#pragma unroll
      for (int kc = 0; kc < 2; ++kc)
#pragma unroll
        for (int i = 0; i < W / RPI; ++i)
          w1v[kc][i] = __builtin_amdgcn_raw_buffer_load_b128(
              w1r, (uint32_t)(((lrow + RPI * i) * c.K + c0 + kc * 64 + (t & 7) * 8) * 2), 0, 0);
      tail_epilogue<BM, BN2, true, NT>(b, acc2, m0, c0, sE, res, sPar + W, sPar + 5 * W, pv, [] {});
      // A3 image (BM rows x 128 channels = two 64-wide swizzled panels) in the
      // staging area, which the epilogue has finished reading.
      {
        const int chunk = t % E2::CPR, rfirst = t / E2::CPR;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < E2::RROWS; ++i) {
            const int r = h * E2::HROWS + rfirst + E2::RSTEP * i;
            *reinterpret_cast<u32x4*>(sE + (chunk >> 3) * (BM * 128) + swz(r, chunk & 7)) = pv[h][i];
          }
      }
#pragma unroll
      for (int kc = 0; kc < 2; ++kc)
#pragma unroll
        for (int i = 0; i < W / RPI; ++i)
          *reinterpret_cast<u32x4*>(sB2 + kc * (W * 128) + swz(lrow + RPI * i, t & 7)) = w1v[kc][i];
      __builtin_amdgcn_s_waitcnt(kLgkm0);
      __builtin_amdgcn_s_barrier();  // A3 written, conv1 weight chunk visible
#pragma unroll
      for (int kc = 0; kc < 2; ++kc)
        mma_k64<TM3, TN3>(sE + kc * (BM * 128), sB2 + kc * (W * 128), wm * (BM / WGM), wn * (W / 2), fr, fk,
                          acc3);
      __builtin_amdgcn_s_waitcnt(kLgkm0);
      __builtin_amdgcn_s_barrier();  // A3 / weight chunk read before the next chunk reuses them
      if (ch + 1 < nchunks) {
        issue_w3(ch + 1);
        load_residual<BM, BN2, false, NT>(b, m0, c0 + BN2, res);
      }
    }
  }
  if constexpr (NEXT) {
    u32x4 none[2][EpiShape<BM, W, NT>::RROWS];
    epilogue_halves<BM, W, false, 0, NT>(c, acc3, m0, 0, smem, none);
  }
}

// CUs this process can occupy on the current device — the grid-fill term of
// the tile choice.  A vGPU pod owns an XCD-balanced CU mask of
// VGPU_DEVICE_CU_LIMIT_<i> % of the device (the enforcement library's env
// contract), so a 50 % pod has 128 CUs to fill, not 256.  VGPU_CONV_CUS
// overrides (A/B).  Cached per device.
int conv_cus() {
  static int forced = -1;
  static int cached[16] = {};
  if (forced < 0) {
    const char* v = getenv("VGPU_CONV_CUS");
    forced = v ? atoi(v) : 0;
  }
  if (forced > 0) return forced;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
  if (cached[dev]) return cached[dev];
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  const char* masked = getenv("VGPU_REPORT_MASKED_CUS");  // the runtime already reports the mask
  char name[40];
  snprintf(name, sizeof name, "VGPU_DEVICE_CU_LIMIT_%d", dev);
  const char* lim = getenv(name);
  const int pct = lim ? atoi(lim) : 0;
  const int phys = cus;
  if (!(masked && masked[0] == '1') && pct > 0 && pct < 100) cus = (cus * pct + 99) / 100;
  // A temporal-pool member that runs with at most k-1 others at a time
  // (VGPU_POOL_CONCURRENCY = k, the device plugin's --pool-concurrency) has
  // 1/k of the GPU while it runs, whatever its long-run share.
  const char* pc = getenv("VGPU_POOL_CONCURRENCY");
  const char* share = getenv("VGPU_CU_SHARE");
  const int k = pc ? atoi(pc) : 0;
  if (k > 0 && share && !strcmp(share, "temporal") && phys / k > cus) cus = phys / k;
  cached[dev] = cus > 0 ? cus : 1;
  return cached[dev];
}

// A/B knob: 128-row tiles for non-prologue 1x1 convs too (VGPU_CONV_1X1_BIG=1).
bool conv_1x1_big() {
  static int on = -1;
  if (on < 0) {
    const char* v = getenv("VGPU_CONV_1X1_BIG");
    on = (v && v[0] == '1') ? 1 : 0;
  }
  return on == 1;
}

template <int KS, int BM, int BN, bool PRO, bool RES>
hipError_t launch(ConvArgs a, hipStream_t s) {
  static int occ = 0;  // resident workgroups per CU (LDS / VGPR bound); one value per instantiation
  if (occ == 0) {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, conv_gemm_kernel<KS, BM, BN, PRO, RES>,
                                                     kThreads, 0) != hipSuccess || o < 1)
      o = 1;
    occ = o;
  }
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  a.nM = (a.M + BM - 1) / BM;
  a.nN = a.Cout / BN;
  a.nwg = a.nM * a.nN;
  int grid = cus * occ;
  grid = grid < 8 ? 8 : grid & ~7;  // multiple of 8: a workgroup keeps its XCD's tiles
  if (a.nwg <= grid) grid = a.nwg;
  hipLaunchKernelGGL((conv_gemm_kernel<KS, BM, BN, PRO, RES>), dim3(grid), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

template <int KS, int BM, int BN>
hipError_t dispatch_pr(const ConvArgs& a, bool pro, bool res, hipStream_t s) {
  if (pro) return res ? launch<KS, BM, BN, true, true>(a, s) : launch<KS, BM, BN, true, false>(a, s);
  return res ? launch<KS, BM, BN, false, true>(a, s) : launch<KS, BM, BN, false, false>(a, s);
}

template <int KS, int BM>
hipError_t dispatch_bn(const ConvArgs& a, bool pro, bool res, hipStream_t s) {
  if (a.Cout % 128 == 0) return dispatch_pr<KS, BM, 128>(a, pro, res, s);
  return dispatch_pr<KS, BM, 64>(a, pro, res, s);
}

// ---- NHWC k x k max pool and fused BN+ReLU+global-average pool ----------------
// One block per output row (grid OH x N): 32-bit index math only (the earlier
// flat-index version spent its time in 64-bit div/mod — it ran ALU-bound, twice
// as slow on half the CUs); K = 3 unrolls the window so all 9 16-B loads of an
// interior output are in flight together.  Row/column reuse is caught by L1/L2.
template <int K>
__global__ void __launch_bounds__(kThreads) maxpool_kernel(const u32x4* __restrict__ x,
                                                          u32x4* __restrict__ y, int H, int W,
                                                          int cv, int OH, int OW, int k, int stride,
                                                          int pad) {
  const int oh = blockIdx.x, n = blockIdx.y;
  if (K) k = K;
  const u32x4* __restrict__ xn = x + (int64_t)n * H * W * cv;
  u32x4* __restrict__ yr = y + ((int64_t)n * OH + oh) * OW * cv;
  const int h0 = oh * stride - pad;
  const int hlo = h0 > 0 ? h0 : 0, hhi = h0 + k < H ? h0 + k : H;
  const int row = OW * cv;
  for (int i = threadIdx.x; i < row; i += kThreads) {
    const int ow = (int)((unsigned)i / (unsigned)cv), c = i - ow * cv;
    const int w0 = ow * stride - pad;
    float m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
    if (K && hlo == h0 && hhi == h0 + K && w0 >= 0 && w0 + K <= W) {
      u32x4 v[K ? K * K : 1];
#pragma unroll
      for (int dh = 0; dh < K; ++dh)
#pragma unroll
        for (int dw = 0; dw < K; ++dw) v[dh * K + dw] = xn[((h0 + dh) * W + w0 + dw) * cv + c];
#pragma unroll
      for (int t = 0; t < K * K; ++t) {
        float e[8];
        unpack8(v[t], e);
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], e[j]);
      }
    } else {
      const int wlo = w0 > 0 ? w0 : 0, whi = w0 + k < W ? w0 + k : W;
      for (int ih = hlo; ih < hhi; ++ih)
        for (int iw = wlo; iw < whi; ++iw) {
          float e[8];
          unpack8(xn[(ih * W + iw) * cv + c], e);
#pragma unroll
          for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], e[j]);
        }
    }
    yr[i] = pack8(m);
  }
}

// out[n][c] = mean_hw relu(x[n,h,w,c]*s[c] + t[c]); grid (N, ceil(cv/64)), 4 waves split pixels.
__global__ void __launch_bounds__(kThreads) ssr_mean_kernel(const u32x4* __restrict__ x,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            u32x4* __restrict__ y, int HW, int cv) {
  __shared__ float part[4][64][8];
  const int n = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + lane;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c < cv) {
    float sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = scale[c * 8 + j]; sh[j] = shift[c * 8 + j]; }
    for (int p = wave; p < HW; p += 4) {
      float e[8];
      unpack8(x[((int64_t)n * HW + p) * cv + c], e);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += fmaxf(e[j] * sc[j] + sh[j], 0.0f);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[wave][lane][j] = acc[j];
  __syncthreads();
  if (wave == 0 && c < cv) {
    const float inv = 1.0f / (float)HW;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      o[j] = (part[0][lane][j] + part[1][lane][j] + part[2][lane][j] + part[3][lane][j]) * inv;
    y[(int64_t)n * cv + c] = pack8(o);
  }
}

// ---- ResNet stem space-to-depth: x [N][H][W][3] → X [N][HS][WS][16] ------------
// X[n][i][j][b*6 + b'*3 + c] = x[n][2i+b-pad][2j+b'-pad][c] (zero outside; channels
// 12..15 zero), so the 7x7/s2 stem becomes a 4x4/s1 conv with C = 16 (16-B
// aligned taps for the LDS-DMA conv).  Grid (ceil(HS*WS/256), N): one thread per
// X pixel of image blockIdx.y, 32-bit index math (one 32-bit divide per pixel),
// 2 x 16-B stores.  (An LDS-staged row version measured slower: 174-pixel blocks
// with a barrier do too little work each.)
__global__ void __launch_bounds__(kThreads) s2d_stem_kernel(const uint16_t* __restrict__ x,
                                                            u32x4* __restrict__ X, int H, int W,
                                                            int HS, int WS, int pad) {
  const int n = blockIdx.y;
  const int p = blockIdx.x * kThreads + threadIdx.x;
  if (p >= HS * WS) return;
  const int i = (int)((unsigned)p / (unsigned)WS), j = p - i * WS;
  const uint16_t* __restrict__ xn = x + (int64_t)n * H * W * 3;
  uint32_t v[12];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int r = 2 * i + b - pad;
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2) {
      const int c0 = 2 * j + b2 - pad;
      const bool ok = (unsigned)r < (unsigned)H && (unsigned)c0 < (unsigned)W;
      const uint16_t* src = xn + (ok ? (r * W + c0) * 3 : 0);
#pragma unroll
      for (int c = 0; c < 3; ++c) v[b * 6 + b2 * 3 + c] = ok ? (uint32_t)src[c] : 0u;
    }
  }
  u32x4 lo, hi;
  lo.x = v[0] | (v[1] << 16); lo.y = v[2] | (v[3] << 16);
  lo.z = v[4] | (v[5] << 16); lo.w = v[6] | (v[7] << 16);
  hi.x = v[8] | (v[9] << 16); hi.y = v[10] | (v[11] << 16);
  hi.z = 0; hi.w = 0;
  u32x4* __restrict__ Xp = X + ((int64_t)n * HS * WS + p) * 2;
  Xp[0] = lo;
  Xp[1] = hi;
}

// ---- ResNet stem conv + 3x3/s2 max pool in one persistent kernel ----------
// The stem conv (4x4/s1 over the space-to-depth input, C = 16, 64 outputs)
// writes a 4x-wide activation (b=50 at 346²: 191 MB) that the max pool reads
// straight back.  Here one task = one pooled output row (n, i): the stem rows
// 2i-1 .. 2i+1 are computed from a 6-row input slab in LDS and rounded to bf16
// into LDS row buffers (exactly what the unfused conv stores), then
// max-pooled from there, so only the input slab and the pooled row touch HBM.
// The 32 KB filter is loaded once per workgroup; the next task's slab is
// fetched into registers while the current task computes.
// The three stem rows are 3 x 11 pixel subtiles of 16; subtile s goes to wave
// s % 8, which computes all 64 channels of it (4 B fragments shared by up to 5
// A fragments per K step).  mfma(B, A) (transposed tile) so a lane holds 4
// consecutive channels of one pixel.  K order (kh, kw, c) and the MFMA
// sequence match the unfused stem conv, so the result is bit-identical to
// conv + maxpool (tests/test_gpu_conv.py).
constexpr int kSPThreads = 512;
constexpr int kSPMaxOW = 176;   // 11 pixel subtiles of 16
constexpr int kSPMaxWS = 180;

__global__ void __launch_bounds__(kSPThreads, 1) stem_pool_kernel(const uint16_t* __restrict__ X,
                                                                  const uint16_t* __restrict__ w,
                                                                  uint16_t* __restrict__ y, int HS, int WS,
                                                                  int OH, int OW, int PH, int PW, int tasks) {
  constexpr int SW_BYTES = 4 * 64 * 128;         // [kh][cout][128 B] swizzled
  constexpr int SR_BYTES = 3 * kSPMaxOW * 128;   // three bf16 stem rows [row][pixel][64 ch] swizzled
  constexpr int SX_BYTES = 6 * kSPMaxWS * 32 + 512;  // 6 input rows [px][16 ch] + over-read pad
  constexpr int XR = (6 * kSPMaxWS * 2 + kSPThreads - 1) / kSPThreads;  // slab chunks per thread
  constexpr int NS = 5;                          // subtiles per wave (33 over 8 waves)
  __shared__ __attribute__((aligned(16))) char smem[SW_BYTES + SR_BYTES + SX_BYTES];
  char* sW = smem;
  char* sR = smem + SW_BYTES;
  char* sX = sR + SR_BYTES;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int MT = (OW + 15) >> 4;
  const int rowc = WS * 2, nchunk = 6 * rowc;  // 16-B chunks per slab row / per slab

  // filter → LDS once: chunk k = (cout, kh, slot)
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = t + kSPThreads * u, co = k >> 5, c16 = k & 31;
    *reinterpret_cast<u32x4*>(sW + (c16 >> 3) * 8192 + swz(co, c16 & 7)) =
        *reinterpret_cast<const u32x4*>(w + co * 256 + c16 * 8);
  }
  auto load_slab = [&](int task, u32x4 (&xr)[XR]) {
    const int n = task / PH, r0 = 2 * (task - n * PH) - 1;
#pragma unroll
    for (int u = 0; u < XR; ++u) {
      const int k = t + kSPThreads * u, q = k / rowc, rem = k - q * rowc, row = r0 + q;
      const bool ok = k < nchunk && row >= 0 && row < HS;
      xr[u] = ok ? *reinterpret_cast<const u32x4*>(X + ((int64_t)(n * HS + row) * WS) * 16 + rem * 8)
                 : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto store_slab = [&](const u32x4 (&xr)[XR]) {
#pragma unroll
    for (int u = 0; u < XR; ++u) {
      const int k = t + kSPThreads * u;
      if (k < nchunk) *reinterpret_cast<u32x4*>(sX + k * 16) = xr[u];
    }
  };
  u32x4 xr[XR];
  int task = blockIdx.x;
  if (task < tasks) {
    load_slab(task, xr);
    store_slab(xr);
  }
  __syncthreads();
  for (; task < tasks; task += gridDim.x) {
    const int n = task / PH, pi = task - n * PH, r0 = 2 * pi - 1;
    const int next = task + gridDim.x;
    if (next < tasks) load_slab(next, xr);  // lands behind this task's compute
    // this wave's subtiles s = wave + 8u: stem row rl = s / MT, pixels (s % MT)*16 ..
    f32x4_t acc[NS][4];
#pragma unroll
    for (int u = 0; u < NS; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[u][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 4; ++kh)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8_t bfr[4], af[NS];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8_t*>(sW + kh * 8192 + swz(j * 16 + fr, kk * 4 + fk));
#pragma unroll
        for (int u = 0; u < NS; ++u) {
          const int sidx = wave + 8 * u, rl = sidx / MT, m = sidx - rl * MT;
          if (sidx < 3 * MT)  // wave-uniform; past the three rows there is nothing to read
            af[u] = *reinterpret_cast<const bf16x8_t*>(
                sX + (((rl + kh) * WS + m * 16 + fr) * 32) + (kk * 4 + fk) * 16);
        }
#pragma unroll
        for (int u = 0; u < NS; ++u)
          if (wave + 8 * u < 3 * MT)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[u], acc[u][j], 0, 0, 0);
      }
    // bf16 stem rows → LDS: lane holds pixel m*16+fr, channels j*16+fk*4 .. +3
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int sidx = wave + 8 * u, rl = sidx / MT, m = sidx - rl * MT;
      if (rl >= 3) continue;
      const int p = m * 16 + fr;
      char* row = sR + rl * (kSPMaxOW * 128) + p * 128;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int slot = j * 2 + (fk >> 1);
        *reinterpret_cast<uint2*>(row + ((slot ^ (p & 7)) << 4) + (fk & 1) * 8) =
            uint2{pack2(acc[u][j][0], acc[u][j][1]), pack2(acc[u][j][2], acc[u][j][3])};
      }
    }
    __syncthreads();
    // 3x3/s2 window (rows of the task that exist, columns 2j-1 .. 2j+1)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int it = t + kSPThreads * k, j = it >> 3, q = it & 7;
      if (j >= PW) continue;
      float pm[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) pm[e] = -INFINITY;
#pragma unroll
      for (int rl = 0; rl < 3; ++rl) {
        if (r0 + rl < 0 || r0 + rl >= OH) continue;
#pragma unroll
        for (int dc = -1; dc <= 1; ++dc) {
          const int c = 2 * j + dc;
          if (c < 0 || c >= OW) continue;
          float e[8];
          unpack8(*reinterpret_cast<const u32x4*>(sR + rl * (kSPMaxOW * 128) + c * 128 + ((q ^ (c & 7)) << 4)), e);
#pragma unroll
          for (int u = 0; u < 8; ++u) pm[u] = fmaxf(pm[u], e[u]);
        }
      }
      *reinterpret_cast<u32x4*>(y + ((int64_t)(n * PH + pi) * PW + j) * 64 + q * 8) = pack8(pm);
    }
    if (next < tasks) {
      __syncthreads();  // every wave done with the slab and the row buffers
      store_slab(xr);
      __syncthreads();
    }
  }
}

}  // namespace

VGPU_API int vgpu_stem_space_to_depth(const void* x, void* X, int N, int H, int W, int pad, int HS,
                                      int WS, hipStream_t s) {
  if (N < 1 || N > 65535 || H < 1 || W < 1 || HS < 1 || WS < 1 || pad < 0) return -1;
  if ((int64_t)H * W * 3 >= ((int64_t)1 << 31) || (int64_t)HS * WS >= ((int64_t)1 << 31) - kThreads)
    return -1;  // per-image offsets are 32-bit in the kernel
  const int blocks = (HS * WS + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(s2d_stem_kernel, dim3(blocks, N), dim3(kThreads), 0, s,
                     static_cast<const uint16_t*>(x), static_cast<u32x4*>(X), H, W, HS, WS, pad);
  return (int)hipGetLastError();
}

// Benchmark knob: force 64- or 128-row tiles (0 = heuristic).
VGPU_API void vgpu_conv_set_tile_m(int bm) { g_forced_bm = bm; }
VGPU_API void vgpu_conv_set_big(int mode) { g_forced_big = mode; }  // -1 env/heuristic, 0 off, 1 when eligible
VGPU_API void vgpu_conv_set_halo(int mode) { g_forced_halo = mode; }  // -1 env, 0 off, 1 on, 2/3 BM 256/128
VGPU_API unsigned long long vgpu_conv_halo_launches() { return g_halo_launches; }

// Fused conv2 (3x3, pad 1, stride s, C = W → W, bias + ReLU) + conv3 (1x1,
// W → 4W) + residual; with w1n, also the next block's conv1 (1x1, 4W → W,
// prologue relu(y*ps + pt), bias b1n + ReLU) into h1n.  W ∈ {64, 128}.
static int conv23_impl(const void* x, const void* w2, const float* b2, const void* w3, const void* res,
                       void* y, const void* w1n, const float* b1n, const float* psn, const float* ptn,
                       void* h1n, int N, int H, int W, int C, int stride, hipStream_t s) {
  if ((C != 64 && C != 128) || stride < 1 || N < 1 || !b2 || !res) return -1;
  const bool next = w1n != nullptr;
  if (next && (!b1n || !psn || !ptn || !h1n)) return -1;
  ConvArgs a{};
  a.x = static_cast<const uint16_t*>(x);
  a.w = static_cast<const uint16_t*>(w2);
  a.bias = b2;
  a.N = N; a.H = H; a.W = W; a.C = C; a.Cout = C; a.stride = stride; a.pad = 1;
  a.OH = (H + 2 - 3) / stride + 1;
  a.OW = (W + 2 - 3) / stride + 1;
  if (a.OH < 1 || a.OW < 1) return -1;
  a.K = 9 * C;
  a.cblocks = C / 64;
  a.ktiles = a.K / 64;
  a.act = 1;
  ConvArgs b{};
  b.w = static_cast<const uint16_t*>(w3);
  b.y = static_cast<uint16_t*>(y);
  b.res = static_cast<const uint16_t*>(res);
  b.Cout = 4 * C;
  b.K = C;
  ConvArgs cn{};
  if (next) {
    cn.w = static_cast<const uint16_t*>(w1n);
    cn.y = static_cast<uint16_t*>(h1n);
    cn.bias = b1n;
    cn.pscale = psn;
    cn.pshift = ptn;
    cn.Cout = C;
    cn.K = 4 * C;
    cn.act = 1;
  }
  const int64_t xi = (int64_t)H * W * C * 2, yi = (int64_t)a.OH * a.OW * b.Cout * 2;
  const int64_t hi = (int64_t)a.OH * a.OW * C * 2;
  const int64_t lim = ((int64_t)1 << 31) - 1;
  const int64_t per = lim / (xi > yi ? xi : yi);
  if (per < 1) return -1;
  for (int n0 = 0; n0 < N; n0 += (int)per) {
    const int nb = (int)((N - n0) < per ? (N - n0) : per);
    ConvArgs c = a, d = b, e = cn;
    c.N = nb;
    c.x = a.x + (int64_t)n0 * (xi / 2);
    c.x_bytes = (uint32_t)(nb * xi);
    c.M = nb * a.OH * a.OW;
    d.M = c.M;
    d.y = b.y + (int64_t)n0 * (yi / 2);
    d.res = b.res + (int64_t)n0 * (yi / 2);
    d.y_bytes = (uint32_t)(nb * yi);
    if (next) {
      e.M = c.M;
      e.y = cn.y + (int64_t)n0 * (hi / 2);
      e.y_bytes = (uint32_t)(nb * hi);
    }
    const int bm = C == 64 ? 128 : 64;
    c.nM = (c.M + bm - 1) / bm; c.nN = 1; c.nwg = c.nM;
    if (C == 64) {
      if (next)
        hipLaunchKernelGGL((conv23_kernel<128, 64, true>), dim3(c.nwg), dim3(kThreads), 0, s, c, d, e);
      else
        hipLaunchKernelGGL((conv23_kernel<128, 64>), dim3(c.nwg), dim3(kThreads), 0, s, c, d, e);
    } else {
      if (next)
        hipLaunchKernelGGL((conv23_kernel<64, 128, true>), dim3(c.nwg), dim3(kThreads), 0, s, c, d, e);
      else
        hipLaunchKernelGGL((conv23_kernel<64, 128>), dim3(c.nwg), dim3(kThreads), 0, s, c, d, e);
    }
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) return (int)err;
  }
  return 0;
}

VGPU_API int vgpu_conv23_nhwc(const void* x, const void* w2, const float* b2, const void* w3,
                              const void* res, void* y, int N, int H, int W, int C, int stride,
                              hipStream_t s) {
  return conv23_impl(x, w2, b2, w3, res, y, nullptr, nullptr, nullptr, nullptr, nullptr, N, H, W, C, stride, s);
}

// conv23 + the next (identity-shortcut) block's conv1 in one kernel: y is the
// next block's input x (still stored: it is that block's residual), h1n its
// conv1 output.  Same constraints as vgpu_conv23_nhwc; b1n/psn/ptn fp32.
VGPU_API int vgpu_conv231_nhwc(const void* x, const void* w2, const float* b2, const void* w3,
                               const void* res, void* y, const void* w1n, const float* b1n,
                               const float* psn, const float* ptn, void* h1n, int N, int H, int W,
                               int C, int stride, hipStream_t s) {
  if (!w1n) return -1;
  return conv23_impl(x, w2, b2, w3, res, y, w1n, b1n, psn, ptn, h1n, N, H, W, C, stride, s);
}

namespace {
int conv2d_impl(const void* x, const void* w, void* y, const void* res, const float* bias, const float* pscale,
                const float* pshift, int N, int H, int W, int C, int Cout, int KS, int stride, int pad, int act,
                float* stats, const void* bnx, const float* bncoef, int bnact, int res_stride, hipStream_t s,
                float* ws = nullptr, int64_t ws_bytes = 0, const void* gmask = nullptr, float* gpart = nullptr,
                const void* pidx = nullptr, void* gfull = nullptr, int pk = 0);

int g_forced_split = -1;  // vgpu_conv_set_splitk: -1 heuristic, 0 off, n > 1 that many splits when eligible

// Split-K for convs whose output tiles cannot fill the CUs this process owns:
// the 28² / 14² layers of VGG-16 at batch 2 are 16-100 workgroups of 64x128 on
// 256 CUs (36-41 us each, ~8 % of MFMA peak; profiles/r5/train).  The K steps
// are cut into `splits` ranges so ~2 workgroups per CU run, each writing an
// fp32 partial tile, and splitk_reduce_kernel applies the epilogue.  Returns
// the split count (1 = no split) and the K steps per split.
int splitk_plan(int64_t M, int C, int Cout, int KS, bool pro, bool narrow, int& kper) {
  const int ktiles = KS * KS * C / 64;
  kper = ktiles;
  if (pro || narrow || C % 64 || (KS != 1 && KS != 3) || g_forced_split == 0) return 1;
  // a kernel forced by an A/B or test setter runs as asked unless splits are forced too
  if (g_forced_split < 0 && (g_forced_halo >= 0 || g_forced_big == 1 || g_forced_bm != 0)) return 1;
  const int bn = Cout % 128 == 0 ? 128 : 64;
  const int64_t tiles = ((M + 63) / 64) * (Cout / bn);
  // Measured (profiles/r5/train/vgg_small_ab.log, graph replay): 100 and 28
  // tiles gain 1.2-1.8x; 196 tiles (56² at b=2) lose 17 % -- split below half the CUs.
  int64_t sp = g_forced_split > 1 ? g_forced_split : (2 * tiles >= conv_cus() ? 1 : 2 * (int64_t)conv_cus() / tiles);
  if (sp > ktiles / 4) sp = ktiles / 4;
  if (sp < 2) return 1;
  kper = (int)((ktiles + sp - 1) / sp);
  return (ktiles + kper - 1) / kper;
}
}  // namespace

// Returns 0, a hipError_t, or -1 for an unsupported shape (checked before any launch).
VGPU_API int vgpu_conv2d_nhwc(const void* x, const void* w, void* y, const void* res,
                              const float* bias, const float* pscale, const float* pshift, int N,
                              int H, int W, int C, int Cout, int KS, int stride, int pad, int act,
                              hipStream_t s) {
  return conv2d_impl(x, w, y, res, bias, pscale, pshift, N, H, W, C, Cout, KS, stride, pad, act, nullptr,
                     nullptr, nullptr, 0, 1, s);
}

// Workspace (bytes) vgpu_conv2d_nhwc_ws wants for a split-K launch of this
// shape; 0 when the conv runs unsplit.
VGPU_API int64_t vgpu_conv2d_workspace(int N, int H, int W, int C, int Cout, int KS, int stride, int pad,
                                       int has_pro) {
  if (N < 1 || stride < 1 || pad < 0 || KS < 1) return 0;
  const int64_t OH = (H + 2 * pad - KS) / stride + 1, OW = (W + 2 * pad - KS) / stride + 1;
  if (OH < 1 || OW < 1) return 0;
  const int64_t M = (int64_t)N * OH * OW;
  const bool narrow = C == 16 && KS == 4 && stride == 1 && !has_pro;
  int kper;
  const int sp = splitk_plan(M, C, Cout, KS, has_pro != 0, narrow, kper);
  return sp > 1 ? (int64_t)sp * M * Cout * 4 : 0;
}

// vgpu_conv2d_nhwc with a split-K workspace (vgpu_conv2d_workspace bytes).
// act bit 8 (act | 256): the bias is bf16 rather than fp32.
VGPU_API int vgpu_conv2d_nhwc_ws(const void* x, const void* w, void* y, const void* res, const void* bias,
                                 const float* pscale, const float* pshift, int N, int H, int W, int C, int Cout,
                                 int KS, int stride, int pad, int act, void* ws, int64_t ws_bytes, hipStream_t s) {
  return conv2d_impl(x, w, y, res, static_cast<const float*>(bias), pscale, pshift, N, H, W, C, Cout, KS, stride,
                     pad, act, nullptr, nullptr, nullptr, 0, 1, s, static_cast<float*>(ws), ws_bytes);
}

VGPU_API void vgpu_conv_set_splitk(int mode) { g_forced_split = mode; }

// Split-K data gradient into a ReLU layer: y = conv(x, w) · [gmask > 0] and
// gpart[block][Cout] the per-block column sums of y (that layer's bias-gradient
// partials; *blocks_out of them).  Only when this shape runs split-K
// (vgpu_conv2d_workspace > 0): returns -1 otherwise, before any launch.
VGPU_API int vgpu_conv2d_masked_splitk(const void* x, const void* w, void* y, int N, int H, int W, int C, int Cout,
                                       int KS, int pad, const void* gmask, void* gpart, int64_t gpart_bytes,
                                       void* ws, int64_t ws_bytes, int* blocks_out, hipStream_t s) {
  if (!gmask || !gpart || !ws || Cout % 8 || kThreads % (Cout / 8) || KS < 1 || pad < 0) return -1;
  const int64_t OH = H + 2 * pad - KS + 1, OW = W + 2 * pad - KS + 1;
  if (OH < 1 || OW < 1) return -1;
  const int64_t M = (int64_t)N * OH * OW;
  const int64_t blocks = (M * (Cout / 8) + kThreads - 1) / kThreads;
  if (vgpu_conv2d_workspace(N, H, W, C, Cout, KS, 1, pad, 0) <= 0 || gpart_bytes < blocks * Cout * 4) return -1;
  if (blocks_out) *blocks_out = (int)blocks;
  return conv2d_impl(x, w, y, nullptr, nullptr, nullptr, nullptr, N, H, W, C, Cout, KS, 1, pad, 0, nullptr, nullptr,
                     nullptr, 0, 1, s, static_cast<float*>(ws), ws_bytes, gmask, static_cast<float*>(gpart));
}

// The same for a ReLU layer followed by a k×k / stride-k max pool whose output
// this conv's x-gradient is: the split reduce scatters through the pool's
// argmax bytes pidx [N][OH][OW][Cout] into gfull [N][OH·k][OW·k][Cout], masked
// by gmask (the ReLU output at full resolution), and sums gpart; y is not written.
VGPU_API int vgpu_conv2d_masked_pool_splitk(const void* x, const void* w, int N, int H, int W, int C, int Cout,
                                            int KS, int pad, const void* pidx, int pk, const void* gmask, void* gfull,
                                            void* gpart, int64_t gpart_bytes, void* ws, int64_t ws_bytes,
                                            int* blocks_out, hipStream_t s) {
  if (!pidx || !gfull || pk < 1 || pk > 15) return -1;
  const int64_t OH = H + 2 * pad - KS + 1, OW = W + 2 * pad - KS + 1;
  if (OH < 1 || OW < 1 || (int64_t)N * OH * pk * OW * pk * Cout * 2 >= ((int64_t)1 << 31)) return -1;
  if (!gmask || !gpart || !ws || Cout % 8 || kThreads % (Cout / 8) || KS < 1 || pad < 0) return -1;
  const int64_t M = (int64_t)N * OH * OW;
  const int64_t blocks = (M * (Cout / 8) + kThreads - 1) / kThreads;
  if (vgpu_conv2d_workspace(N, H, W, C, Cout, KS, 1, pad, 0) <= 0 || gpart_bytes < blocks * Cout * 4) return -1;
  if (blocks_out) *blocks_out = (int)blocks;
  return conv2d_impl(x, w, nullptr, nullptr, nullptr, nullptr, nullptr, N, H, W, C, Cout, KS, 1, pad, 0, nullptr,
                     nullptr, nullptr, 0, 1, s, static_cast<float*>(ws), ws_bytes, gmask, static_cast<float*>(gpart),
                     pidx, gfull, pk);
}

// Training convolution with the BatchNorm statistics of its output from the
// epilogue (ConvArgs::stats): stats = fp32 pairs [ceil(M / 64)][Cout], M = N·OH·OW.
//   bnx == nullptr: forward — (Σ y, Σ y²) per 64-row group of the stored y.
//   bnx = x of the BN whose output's gradient this conv computes (a data
//   gradient): y = dy·act'(x·s + t) is stored instead of dy, and the pairs are
//   (Σ y, Σ y·(x - mean)·invstd); bncoef = s, t, mean, invstd [4][Cout], bnact
//   its activation (1 relu, 2 relu6, 0 none).  A residual there is a second
//   gradient of the BN output (a projection shortcut's), added before the mask;
//   res_stride 2: that of a 1x1 / stride-2 shortcut in compact form
//   [N][ceil(OH/2)][ceil(OW/2)][Cout] (its even pixels; the others get none).
// The LDS-DMA kernels only (no prologue, C % 64 == 0); returns -1 when the
// shape takes another kernel (the caller runs the unfused path).
VGPU_API int vgpu_conv2d_nhwc_bn(const void* x, const void* w, void* y, const void* res, int N, int H, int W,
                                 int C, int Cout, int KS, int stride, int pad, float* stats, const void* bnx,
                                 const float* bncoef, int bnact, int res_stride, hipStream_t s) {
  if (!stats || (bnx && !bncoef) || bnact < 0 || bnact > 2 || (res_stride != 1 && (res_stride != 2 || !bnx || !res)))
    return -1;
  return conv2d_impl(x, w, y, res, nullptr, nullptr, nullptr, N, H, W, C, Cout, KS, stride, pad, 0, stats, bnx,
                     bncoef, bnact, res_stride, s);
}

namespace {
int conv2d_impl(const void* x, const void* w, void* y, const void* res, const float* bias, const float* pscale,
                const float* pshift, int N, int H, int W, int C, int Cout, int KS, int stride, int pad, int act,
                float* stats, const void* bnx, const float* bncoef, int bnact, int res_stride, hipStream_t s,
                float* ws, int64_t ws_bytes, const void* gmask, float* gpart, const void* pidx, void* gfull,
                int pk) {
  const int bias_bf16 = (act >> 8) & 1;
  act &= 0xff;
  if (act > 2) return -1;
  // C % 64 == 0 with 1x1 / 3x3 filters, or the narrow stem form (C = 16, 4x4,
  // stride 1, no prologue: a 7x7/s2 conv on a space-to-depth input).
  const bool narrow = C == 16 && KS == 4 && stride == 1 && pscale == nullptr;
  if (!narrow && (C % 64 || (KS != 1 && KS != 3))) return -1;
  if (Cout % 64 || stride < 1 || pad < 0 || N < 1) return -1;
  if ((pscale == nullptr) != (pshift == nullptr)) return -1;
  ConvArgs a{};
  a.x = static_cast<const uint16_t*>(x);
  a.w = static_cast<const uint16_t*>(w);
  a.y = static_cast<uint16_t*>(y);
  a.res = static_cast<const uint16_t*>(res);
  a.bias = bias;
  a.pscale = pscale;
  a.pshift = pshift;
  a.N = N; a.H = H; a.W = W; a.C = C; a.Cout = Cout; a.stride = stride; a.pad = pad;
  a.OH = (H + 2 * pad - KS) / stride + 1;
  a.OW = (W + 2 * pad - KS) / stride + 1;
  if (a.OH < 1 || a.OW < 1) return -1;
  a.K = KS * KS * C;
  a.cblocks = C / 64;
  a.ktiles = a.K / 64;
  a.act = act;  // 0 none, 1 ReLU, 2 ReLU6
  a.bias_bf16 = bias_bf16;
  a.stats = reinterpret_cast<float2*>(stats);
  a.bnx = static_cast<const uint16_t*>(bnx);
  a.bncoef = bncoef;
  a.bnact = bnact;
  a.res_stride = res_stride;
  a.res_h = (a.OH + 1) / 2;
  a.res_w = (a.OW + 1) / 2;
  a.res_bytes = 0;
  if (res_stride == 2) {
    const int64_t rb = (int64_t)N * a.res_h * a.res_w * Cout * 2;
    if (rb >= ((int64_t)1 << 31)) return -1;
    a.res_bytes = (uint32_t)rb;
  }
  const bool pro = pscale != nullptr, has_res = res != nullptr;
  if (stats && (narrow || pro)) return -1;
  // Buffer offsets are 32-bit: run the batch in slices whose activations stay < 2 GiB.
  const int64_t xi = (int64_t)H * W * C * 2, yi = (int64_t)a.OH * a.OW * Cout * 2;
  const int64_t lim = ((int64_t)1 << 31) - 1;
  const int64_t per = lim / (xi > yi ? xi : yi);
  if (per < 1 || (stats && per < N)) return -1;  // statistics: one slice (group rows are global)
  const int bn = (Cout % 128 == 0) ? 128 : 64;
  for (int n0 = 0; n0 < N; n0 += (int)per) {
    const int nb = (int)((N - n0) < per ? (N - n0) : per);
    ConvArgs c = a;
    c.N = nb;
    c.x = a.x + (int64_t)n0 * (xi / 2);
    c.y = a.y + (int64_t)n0 * (yi / 2);
    if (has_res) c.res = a.res + (int64_t)n0 * (yi / 2);
    c.x_bytes = (uint32_t)(nb * xi);
    c.y_bytes = (uint32_t)(nb * yi);
    c.M = nb * a.OH * a.OW;
    // Small-M layers use 64-row tiles so the grid still fills the CUs this
    // process owns: 128-row tiles fetch fewer bytes per FLOP, but below ~1.5
    // workgroups per CU the kernel is latency-bound (profiles/conv_cus_r1.md:
    // exclusive 256 CUs and 50 % pods of 128 CUs agree with this threshold).
    const int64_t tiles128 = (int64_t)((c.M + 127) / 128) * (Cout / bn);
    bool small = tiles128 < (int64_t)conv_cus() * 3 / 2;
    // Non-prologue 1x1 convs (conv3 + residual) are DMA/HBM-bound: 64-row tiles
    // (48 KB LDS → 3 blocks per CU) beat 128-row tiles on every ResNet-50 shape
    // (profiles/conv_tiles_r1.md).
    if (!pro && KS == 1) small = !conv_1x1_big();
    if (g_forced_bm == 64) small = true;
    if (g_forced_bm == 128) small = false;
    hipError_t e;
    int kper;
    const int splits = (ws && !stats && per >= N) ? splitk_plan(c.M, C, Cout, KS, pro, narrow, kper) : 1;
    if (gmask && splits <= 1) return -1;  // the masked form exists only as a split-K reduce
    if (splits > 1) {
      if (ws_bytes < (int64_t)splits * c.M * Cout * 4) return -1;
      c.ws = ws;
      c.kper = kper;
      c.splits = splits;
      c.gmask = static_cast<const uint16_t*>(gmask);
      c.gpart = gpart;
      c.pidx = static_cast<const uint8_t*>(pidx);
      c.gfull = static_cast<uint16_t*>(gfull);
      c.pk = pk;
      c.nM = (c.M + 63) / 64;
      c.nN = Cout / bn;
      c.nwg = c.nM * c.nN;
      const dim3 grid(c.nwg, splits);
      if (bn == 128) {
        if (KS == 1) hipLaunchKernelGGL((conv_glds_kernel<1, 64, 128, false, 0, 0, true>), grid, dim3(kThreads), 0, s, c);
        else hipLaunchKernelGGL((conv_glds_kernel<3, 64, 128, false, 0, 0, true>), grid, dim3(kThreads), 0, s, c);
      } else {
        if (KS == 1) hipLaunchKernelGGL((conv_glds_kernel<1, 64, 64, false, 0, 0, true>), grid, dim3(kThreads), 0, s, c);
        else hipLaunchKernelGGL((conv_glds_kernel<3, 64, 64, false, 0, 0, true>), grid, dim3(kThreads), 0, s, c);
      }
      if ((e = hipGetLastError()) != hipSuccess) return (int)e;
      const int64_t threads = (int64_t)c.M * (Cout / 8);
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((threads + kThreads - 1) / kThreads)), dim3(kThreads),
                         0, s, c);
      if ((e = hipGetLastError()) != hipSuccess) return (int)e;
      continue;
    }
    // LDS-DMA kernels for every conv without a prologue; prologue convs stage A
    // through registers (conv_pro_kernel / conv_gemm_kernel).
    const bool glds = !pro;
    // 256x256 tiles: 1x1 / stride 1 / no prologue, Cout % 256 == 0, deep K
    // (≥ 1024: below it these layers are HBM-bound and the 64-row tiles at 3
    // blocks per CU win — the ResNet-50 flagship measured 1 % slower with the
    // big tile on its K = 128-512 conv3 layers), and enough tiles to give every
    // CU this process owns at least one.
    if (g_forced_big < 0) {
      const char* v = getenv("VGPU_CONV_BIG");
      g_forced_big = v ? (v[0] == '1' ? 1 : (v[0] == '0' ? 0 : 2)) : 2;
    }
    const bool big_ok = !narrow && !pro && KS == 1 && stride == 1 && pad == 0 && Cout % 256 == 0 && C >= 128;
    const int64_t tiles256 = (int64_t)((c.M + 255) / 256) * (Cout / 256);
    const bool big = !stats && big_ok && (g_forced_big == 1 ||
                                (g_forced_big == 2 && C >= 1024 && tiles256 >= (int64_t)conv_cus()));
    // 3x3 / stride 1 without prologue or residual: the halo-tile kernel.
    const bool halo = (g_forced_halo < 0 ? halo_enabled() : g_forced_halo > 0) && !narrow && !pro && !has_res &&
                      KS == 3 && stride == 1 && pad == 1;
    if (halo && (e = dispatch_halo(c, s)) != hipErrorNotSupported) {
      // launched (or a launch error)
    } else if (big)
      e = has_res ? launch_big<true>(c, s) : launch_big<false>(c, s);
    else if (narrow)
      e = small ? launch_glds<4, 64, 64, false, 16>(c, s) : launch_glds<4, 128, 64, false, 16>(c, s);
    // Short K (≤ 2 steps) or 64-wide outputs: the persistent register kernel,
    // which overlaps the next tile's loads with this tile's epilogue, wins there.
    // (conv_pro's 1x1 form assumes no padding: it skips the zero-padding select.)
    else if (pro && C <= 2048 && a.ktiles > 2 && Cout > 64 && (KS != 1 || pad == 0))
      e = KS == 1 ? (small ? dispatch_pro<1, 64>(c, has_res, s) : dispatch_pro<1, 128>(c, has_res, s))
                  : (small ? dispatch_pro<3, 64>(c, has_res, s) : dispatch_pro<3, 128>(c, has_res, s));
    else if (glds)
      e = KS == 1 ? (small ? dispatch_glds<1, 64>(c, has_res, s) : dispatch_glds<1, 128>(c, has_res, s))
                  : (small ? dispatch_glds<3, 64>(c, has_res, s) : dispatch_glds<3, 128>(c, has_res, s));
    else if (KS == 1)
      e = small ? dispatch_bn<1, 64>(c, pro, has_res, s) : dispatch_bn<1, 128>(c, pro, has_res, s);
    else
      e = small ? dispatch_bn<3, 64>(c, pro, has_res, s) : dispatch_bn<3, 128>(c, pro, has_res, s);
    if (e == hipErrorNotSupported && stats) return -1;
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}
}  // namespace

// NHWC bf16 max pool (k×k window, stride, symmetric zero-excluded padding), 16 B per lane.
// Fused stem: X [N][HS][WS][16] (space-to-depth input), w [64][4][4][16] →
// y [N][PH][PW][64] = maxpool3x3/s2/p1(conv4x4/s1(X, w)), bf16 NHWC.
VGPU_API int vgpu_stem_pool_nhwc(const void* X, const void* w, void* y, int N, int HS, int WS, hipStream_t s) {
  const int OH = HS - 3, OW = WS - 3;
  if (N < 1 || OH < 1 || OW < 1 || OW > kSPMaxOW || WS > kSPMaxWS) return -1;
  if ((int64_t)N * HS * WS * 16 >= ((int64_t)1 << 31)) return -1;
  const int PH = (OH + 2 - 3) / 2 + 1, PW = (OW + 2 - 3) / 2 + 1;
  if (PW * 8 > 2 * kSPThreads) return -1;
  const int tasks = N * PH;
  // One workgroup per CU of the device (LDS allows one), not conv_cus(): a
  // time-shared pod runs on every CU while it runs, and a masked one just
  // queues the extra workgroups (the task loop takes any grid).
  int dev = 0, grid = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&grid, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || grid < 1)
    grid = 256;
  if (grid > tasks) grid = tasks;
  hipLaunchKernelGGL(stem_pool_kernel, dim3(grid), dim3(kSPThreads), 0, s, static_cast<const uint16_t*>(X),
                     static_cast<const uint16_t*>(w), static_cast<uint16_t*>(y), HS, WS, OH, OW, PH, PW, tasks);
  return (int)hipGetLastError();
}

VGPU_API int vgpu_maxpool_nhwc(const void* x, void* y, int N, int H, int W, int C, int k, int stride,
                               int pad, hipStream_t s) {
  if (C % 8 || k < 1 || stride < 1 || pad < 0 || 2 * pad >= k + 1 || N < 1 || N > 65535) return -1;
  const int OH = (H + 2 * pad - k) / stride + 1, OW = (W + 2 * pad - k) / stride + 1;
  if (OH < 1 || OW < 1) return -1;
  if ((int64_t)H * W * (C / 8) >= ((int64_t)1 << 31) || (int64_t)OW * (C / 8) >= ((int64_t)1 << 31))
    return -1;  // per-image offsets are 32-bit in the kernel
  auto kern = k == 3 ? maxpool_kernel<3> : maxpool_kernel<0>;
  hipLaunchKernelGGL(kern, dim3(OH, N), dim3(kThreads), 0, s, static_cast<const u32x4*>(x),
                     static_cast<u32x4*>(y), H, W, C / 8, OH, OW, k, stride, pad);
  return (int)hipGetLastError();
}

VGPU_API int vgpu_scale_shift_relu_mean_nhwc(const void* x, const float* scale, const float* shift,
                                             void* y, int N, int HW, int C, hipStream_t s) {
  if (C % 8) return -1;
  const int cv = C / 8;
  hipLaunchKernelGGL(ssr_mean_kernel, dim3(N, (cv + 63) / 64), dim3(kThreads), 0, s,
                     static_cast<const u32x4*>(x), scale, shift, static_cast<u32x4*>(y), HW, cv);
  return (int)hipGetLastError();
}
