// Fused LSTM recurrence on gfx950 (ai-benchmark 5.1 / 5.2, LSTM-Sentiment:
// hidden 128, 2 layers, 1024 steps, batch 100 inference / 10 training).
//
// Why: PyTorch-ROCm runs nn.LSTM as MIOpen's per-timestep kernel sequence —
// about 4 000 dispatches of a few microseconds per 2-layer forward.  One pod is then
// bound by dispatch latency, and several pods sharing a GPU contend for the
// command processor instead of for CUs (docs/benchmarks.md, round 2).  Here one
// layer is one GEMM for the input projection of its timesteps (hipBLASLt, outside)
// plus ONE persistent kernel for the recurrence:
//
//   gates_t = Xp_t + h_{t-1} · W_hhᵀ          Xp = X · W_ihᵀ + b_ih + b_hh  (precomputed)
//   c_t = σ(f)·c_{t-1} + σ(i)·tanh(g),  h_t = σ(o)·tanh(c_t)      (gate order i, f, g, o)
//
// A workgroup owns 16 batch rows for the whole sequence.  Its 4 waves own the
// 4 gate blocks (128 columns each); each wave keeps its 128x128 slice of W_hh
// as MFMA B fragments in registers (32 x bf16x8 = 128 VGPRs) for all steps,
// so a timestep is 32 mfma_f32_16x16x32_bf16 per wave on h_{t-1} (16x128 bf16
// in LDS, rows padded to 272 B), the gate activations through LDS (fp32), and
// the cell update with c_t held in registers (8 cells per thread).  The Xp
// values of step t+1 are loaded while step t computes.
//
// Chunks: a call may cover a window [t0, t0 + T) of the
// sequence, starting from a carried state (h0 bf16, c0 fp32) and leaving the
// final state (hT, cT) for the next window.  vgpu.ops.lstm runs the layers as a
// wavefront over windows on two streams — layer 2 on window k while layer 1
// runs window k + 1 — instead of one layer after the other; outputs are strided
// (ys_row, ys_t) so a window's h can be written timestep-major for the next
// layer's projection GEMM.  The backward kernel carries (dh, dc) the same way.
//
// prof (optional, workgroup 0, thread 0): s_memtime cycles spent per step in
// each phase, summed over the window — see vgpu_lstm_profile.
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
constexpr int kPhases = 5;         // profiled phases of a forward step

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
// v_exp_f32 + v_rcp_f32 (1 ulp): an IEEE division here is a ~10-instruction
// div_scale / div_fmas / div_fixup sequence, and a step evaluates 40 of these
// per lane on the recurrence's critical path.  Saturates correctly: exp -> inf
// gives rcp -> 0.
__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) { return 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * x)) - 1.0f; }

struct FwdArgs {
  const uint16_t* xp;    // [T][B][4H] bf16 of this window (biases folded in)
  const uint16_t* whh;   // [4H][H] bf16 (PyTorch weight_hh_l*)
  uint16_t* y;           // h_t at y[row * ys_row + t * ys_t], or nullptr
  int64_t ys_row, ys_t;
  uint16_t* hlast;       // [B][H] bf16: h of the window's last step, or nullptr
  uint16_t* gates_out;   // training: activated gates bf16 [T][B][4H] of this window, or nullptr
  float* cells_out;      // training: c fp32 [T][B][H] of this window
  const uint16_t* h0;    // [B][H] bf16 initial h, nullptr = 0
  const float* c0;       // [B][H] fp32 initial c, nullptr = 0
  float* c_last;         // [B][H] fp32 c of the window's last step, or nullptr
  unsigned long long* prof;
  // wavefront (lstm2_forward_kernel): wait for xp of step t until *wait > t;
  // after step t's y stores, *publish = t + 1 (agent-scope release)
  const int* wait;
  int* publish;
  int* error;
  int B, T;
};

__device__ bool wait_flag(const int* flag, int need, int* error);
constexpr int kPubEvery = 8;  // wavefront hand-offs are published (fence + count) every 8 steps

// A wait that remembers the last count it saw: only a step past it polls L2.
struct Waiter {
  const int* flag;
  int* error;
  int seen;
  __device__ void until(int need) {  // until *flag > need
    if (!flag || need < seen) return;
    wait_flag(flag, need, error);
    seen = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  }
};
// publish after step index `done` (0-based count of finished steps - 1) of `total`?
__device__ __forceinline__ bool pub_step(int done, int total) { return (done + 1) % kPubEvery == 0 || done + 1 == total; }

// Layout of a step (profiles/r6/lstm): wave w owns hidden
// units [32w, 32w+32) of ALL four gates — its 8 MFMA tiles are (gate q, half h)
// = gate columns q·128 + 32w + 16h + 0..15 — and multiplies W·hᵀ (operands
// swapped), so lane (fr, fk) of tile (q, h) holds the pre-activations of batch
// row fr, units 32w + 16h + 4fk + 0..3 for gate q.  A lane therefore has i, f,
// g, o of the same 8 cells: the cell update runs in registers straight after
// the MFMAs (no gate round trip through LDS), h_t goes to the other half of a
// ping-pong LDS buffer (one barrier per step), and the step's Xp is 8
// contiguous bytes per tile.
__device__ void recurrence_body(const FwdArgs& a, int blk, uint16_t* sh) {
  const int t_ = threadIdx.x, lane = t_ & 63, w = t_ >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int b0 = blk * kRows;
  const int B = a.B, T = a.T;
  const bool prof = a.prof && blk == 0 && t_ == 0;
  unsigned long long ph[kPhases] = {0, 0, 0, 0, 0};
  const int row = b0 + fr;              // this lane's batch row
  const bool live = row < B;
  const int xrow = live ? row : 0;      // loads stay unconditional (no branch around them)

  // gate column of tile jn = (gate q = jn >> 1, half h = jn & 1), element i: col(jn) + 4fk + i
  auto col = [&](int jn) { return (jn >> 1) * kH + w * 32 + (jn & 1) * 16; };
  // W_hh rows of this wave's tiles as A fragments: row col(jn) + fr, k = 32kk + 8fk .. +7
  bf16x8_t wf[8][4];
#pragma unroll
  for (int jn = 0; jn < 8; ++jn)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      wf[jn][kk] = *reinterpret_cast<const bf16x8_t*>(a.whh + (size_t)(col(jn) + fr) * kH + kk * 32 + fk * 8);

  // h_{-1}: the carried state (zero without one); c: this lane's 8 cells
  for (int i = t_; i < 2 * kRows * kHStride; i += 256) sh[i] = 0;
  __syncthreads();
  if (a.h0 && t_ < 256) {
    const int r = t_ >> 4, u = (t_ & 15) * 8;
    if (b0 + r < B)
      *reinterpret_cast<u32x4*>(sh + r * kHStride + u) = *reinterpret_cast<const u32x4*>(a.h0 + (size_t)(b0 + r) * kH + u);
  }
  float c[8];  // cells (half h, element i) at c[4h + i]: unit 32w + 16h + 4fk + i
#pragma unroll
  for (int q = 0; q < 8; ++q)
    c[q] = (a.c0 && live) ? a.c0[(size_t)row * kH + w * 32 + (q >> 2) * 16 + fk * 4 + (q & 3)] : 0.0f;

  uint2 xn[8];  // Xp of the next step: tile jn, 4 bf16
  auto load_xp = [&](int t) {
    const uint16_t* p = a.xp + ((size_t)t * B + xrow) * (4 * kH) + fk * 4;
#pragma unroll
    for (int jn = 0; jn < 8; ++jn) xn[jn] = *reinterpret_cast<const uint2*>(p + col(jn));
  };
  Waiter wt{a.wait, a.error, 0};
  wt.until(0);
  load_xp(0);
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    unsigned long long t0 = prof ? __builtin_amdgcn_s_memtime() : 0, t1;
    f32x4_t acc[8];
#pragma unroll
    for (int jn = 0; jn < 8; ++jn)
      acc[jn] = f32x4_t{bf2f((uint16_t)(xn[jn].x & 0xffff)), bf2f((uint16_t)(xn[jn].x >> 16)),
                        bf2f((uint16_t)(xn[jn].y & 0xffff)), bf2f((uint16_t)(xn[jn].y >> 16))};
    if (t + 1 < T) {
      wt.until(t + 1);
      load_xp(t + 1);  // lands while this step computes
    }
    bf16x8_t hf[4];  // B operand: h_{t-1}[batch fr][k = 32kk + 8fk .. +7]
    const uint16_t* hcur = sh + (t & 1) * kRows * kHStride;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      hf[kk] = *reinterpret_cast<const bf16x8_t*>(hcur + fr * kHStride + kk * 32 + fk * 8);
    if (prof) { t1 = __builtin_amdgcn_s_memtime(); ph[0] += t1 - t0; t0 = t1; }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int jn = 0; jn < 8; ++jn)
        acc[jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[jn][kk], hf[kk], acc[jn], 0, 0, 0);
    // activations and the cell update, in registers: tiles 2q + h hold gate q
    float gi[8], gf[8], gg[8], go[8];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gi[4 * h + i] = sigm(acc[0 + h][i]);
        gf[4 * h + i] = sigm(acc[2 + h][i]);
        gg[4 * h + i] = tanh_f(acc[4 + h][i]);
        go[4 * h + i] = sigm(acc[6 + h][i]);
      }
    uint16_t hv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      c[q] = gf[q] * c[q] + gi[q] * gg[q];
      hv[q] = f2bf(go[q] * tanh_f(c[q]));
    }
    if (prof) { t1 = __builtin_amdgcn_s_memtime(); ph[1] += t1 - t0; t0 = t1; }
    uint16_t* hnext = sh + ((t + 1) & 1) * kRows * kHStride;  // ping-pong: step t reads the other buffer
    const uint2 hp[2] = {uint2{(uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16)},
                         uint2{(uint32_t)hv[4] | ((uint32_t)hv[5] << 16), (uint32_t)hv[6] | ((uint32_t)hv[7] << 16)}};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = w * 32 + h * 16 + fk * 4;
      *reinterpret_cast<uint2*>(hnext + fr * kHStride + u) = hp[h];
      if (live) {
        if (a.y) *reinterpret_cast<uint2*>(a.y + row * a.ys_row + t * a.ys_t + u) = hp[h];
        if (a.hlast && t == T - 1) *reinterpret_cast<uint2*>(a.hlast + (size_t)row * kH + u) = hp[h];
        if (a.gates_out) {
          const float* gsrc[4] = {gi, gf, gg, go};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float* v = gsrc[q] + 4 * h;
            *reinterpret_cast<uint2*>(a.gates_out + ((size_t)t * B + row) * (4 * kH) + q * kH + u) =
                uint2{(uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                      (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16)};
          }
          *reinterpret_cast<float4*>(a.cells_out + ((size_t)t * B + row) * kH + u) =
              float4{c[4 * h], c[4 * h + 1], c[4 * h + 2], c[4 * h + 3]};
        }
      }
    }
    const bool pub = a.publish && pub_step(t, T);
    if (pub) __threadfence();  // y up to t visible device-wide before the count moves
    if (prof) { t1 = __builtin_amdgcn_s_memtime(); ph[3] += t1 - t0; t0 = t1; }
    __syncthreads();  // h_t published; every read of h_{t-1} done (its buffer is written at t + 1)
    if (pub && t_ == 0) __hip_atomic_store(a.publish, t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (prof) { t1 = __builtin_amdgcn_s_memtime(); ph[4] += t1 - t0; }
  }
  if (live && a.c_last)
#pragma unroll
    for (int q = 0; q < 8; ++q) a.c_last[(size_t)row * kH + w * 32 + (q >> 2) * 16 + fk * 4 + (q & 3)] = c[q];
  if (prof)
    for (int i = 0; i < kPhases; ++i) a.prof[i] = ph[i];
}

__global__ void __launch_bounds__(256, 1) lstm_recurrence_kernel(const FwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t sh[2 * kRows * kHStride];   // h ping-pong, bf16
  recurrence_body(a, blockIdx.x, sh);
}

// Backward through time of one layer.  dgates_t (pre-activation) from the saved
// activated gates and cells, dh_t = dY_t + dh_next, and
//   dh_next = dgates_t · W_hh          (16 x 512) · (512 x 128) on MFMA
// with wave w owning hidden columns [32w, 32w+32) and its W_hh slice (k = all
// 512 gate rows) as B fragments in registers.  dgates go to global (bf16
// [T][B][4H]) for the weight-gradient GEMMs done outside.
constexpr int kGStride = 4 * kH + 8;  // dgates rows in LDS: 1040 B

struct BwdArgs {
  const uint16_t* gates;  // [T][B][4H] of this window
  const float* cells;     // [T][B][H] of this window; cells[-1] is read when has_prev
  const uint16_t* dy;     // dY_t at dy[row * ds_row + t * ds_t], or nullptr (no output gradient)
  int64_t ds_row, ds_t;
  const uint16_t* whh;
  uint16_t* dgates;       // [T][B][4H] of this window
  float* dh;              // [B][H] fp32 carried dh_next (in/out), or nullptr = zero, not kept
  float* dc;              // [B][H] fp32 carried dc_next (in/out), or nullptr
  // wavefront (lstm2_backward_kernel): wait for dY of step t until *wait >= T - t;
  // after step t's dgates stores, *publish = T - t
  const int* wait;
  int* publish;
  int* error;
  int B, T, has_prev;
};

// Same ownership as the forward: wave w owns hidden units [32w, 32w+32), lane
// (fr, fk) the 8 cells of batch row fr, units 32w + 16h + 4fk + 0..3.  dh_next =
// W_hhᵀ·dgatesᵀ (operands swapped) lands in exactly those lanes, so it never
// leaves registers; dgates_t goes through a ping-pong LDS buffer (the MFMA's
// B operand needs whole rows), one barrier per step.  The saved gates, cells
// and dY of step t-1 are loaded while step t computes.
__device__ void backward_body(const BwdArgs& a, int blk, uint16_t* sdg) {
  const int t_ = threadIdx.x, lane = t_ & 63, w = t_ >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int b0 = blk * kRows;
  const int B = a.B, T = a.T;
  const int row = b0 + fr;
  const bool live = row < B;
  const int xrow = live ? row : 0;
  // A operand: W_hhᵀ rows = hidden units 32w + 16jn + fr, k = gate row 32ks + 8fk .. +7
  bf16x8_t wf[2][16];
#pragma unroll
  for (int jn = 0; jn < 2; ++jn)
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      uint16_t v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = a.whh[(size_t)(ks * 32 + fk * 8 + j) * kH + w * 32 + jn * 16 + fr];
      wf[jn][ks] = __builtin_bit_cast(bf16x8_t, u32x4{(uint32_t)v[0] | ((uint32_t)v[1] << 16),
                                                       (uint32_t)v[2] | ((uint32_t)v[3] << 16),
                                                       (uint32_t)v[4] | ((uint32_t)v[5] << 16),
                                                       (uint32_t)v[6] | ((uint32_t)v[7] << 16)});
    }
  auto unit = [&](int h) { return w * 32 + h * 16 + fk * 4; };
  f32x4_t dh[2], dcn[2];  // carried dh_next / dc_next of this lane's cells (half h)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    dh[h] = (a.dh && live) ? *reinterpret_cast<const f32x4_t*>(a.dh + (size_t)row * kH + unit(h)) : f32x4_t{0, 0, 0, 0};
    dcn[h] = (a.dc && live) ? *reinterpret_cast<const f32x4_t*>(a.dc + (size_t)row * kH + unit(h)) : f32x4_t{0, 0, 0, 0};
  }
  // saved values of one step for this lane's cells (prefetched a step ahead)
  uint2 ng[2][4], ndy[2];
  float4 nc[2], ncp[2];
  Waiter wt{a.wait, a.error, 0};
  auto load_step = [&](int t) {
    wt.until(T - t - 1);
    const bool prev = t > 0 || a.has_prev;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = unit(h);
      const uint16_t* gp = a.gates + ((size_t)t * B + xrow) * (4 * kH) + u;
#pragma unroll
      for (int q = 0; q < 4; ++q) ng[h][q] = *reinterpret_cast<const uint2*>(gp + q * kH);
      nc[h] = *reinterpret_cast<const float4*>(a.cells + ((size_t)t * B + xrow) * kH + u);
      ncp[h] = prev ? *reinterpret_cast<const float4*>(a.cells + ((int64_t)(t - 1) * B + xrow) * kH + u)
                    : float4{0.f, 0.f, 0.f, 0.f};
      ndy[h] = a.dy ? *reinterpret_cast<const uint2*>(a.dy + xrow * a.ds_row + t * a.ds_t + u) : uint2{0u, 0u};
    }
  };
  load_step(T - 1);

  for (int t = T - 1; t >= 0; --t) {
    uint2 cg[2][4], cdy[2];
    float4 cc[2], ccp[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int q = 0; q < 4; ++q) cg[h][q] = ng[h][q];
      cc[h] = nc[h], ccp[h] = ncp[h], cdy[h] = ndy[h];
    }
    if (t > 0) load_step(t - 1);
    uint16_t* buf = sdg + (t & 1) * kRows * kGStride;  // ping-pong
    uint2 dgp[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float dgv[4][4];
      const float cv[4] = {cc[h].x, cc[h].y, cc[h].z, cc[h].w}, cpv[4] = {ccp[h].x, ccp[h].y, ccp[h].z, ccp[h].w};
      const float dyv[4] = {bf2f((uint16_t)(cdy[h].x & 0xffff)), bf2f((uint16_t)(cdy[h].x >> 16)),
                            bf2f((uint16_t)(cdy[h].y & 0xffff)), bf2f((uint16_t)(cdy[h].y >> 16))};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        auto gate = [&](int q) {
          const uint32_t v = (e >> 1) ? cg[h][q].y : cg[h][q].x;
          return bf2f((uint16_t)((e & 1) ? (v >> 16) : (v & 0xffff)));
        };
        const float i = gate(0), f = gate(1), g = gate(2), o = gate(3);
        const float dhv = live ? dyv[e] + dh[h][e] : 0.0f;
        const float tc = tanh_f(cv[e]);
        const float dc = dhv * o * (1.0f - tc * tc) + dcn[h][e];
        dgv[3][e] = dhv * tc * o * (1.0f - o);
        dgv[0][e] = dc * g * i * (1.0f - i);
        dgv[2][e] = dc * i * (1.0f - g * g);
        dgv[1][e] = dc * cpv[e] * f * (1.0f - f);
        dcn[h][e] = live ? dc * f : 0.0f;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        dgp[h][q] = uint2{(uint32_t)f2bf(dgv[q][0]) | ((uint32_t)f2bf(dgv[q][1]) << 16),
                          (uint32_t)f2bf(dgv[q][2]) | ((uint32_t)f2bf(dgv[q][3]) << 16)};
        *reinterpret_cast<uint2*>(buf + fr * kGStride + q * kH + unit(h)) = dgp[h][q];
        if (live) *reinterpret_cast<uint2*>(a.dgates + ((size_t)t * B + row) * (4 * kH) + q * kH + unit(h)) = dgp[h][q];
      }
    }
    const bool pub = a.publish && pub_step(T - 1 - t, T);
    if (pub) __threadfence();  // dgates down to t visible device-wide before the count moves
    __syncthreads();  // dgates_t complete in LDS (its other buffer was last read a step ago)
    if (pub && t_ == 0) __hip_atomic_store(a.publish, T - t, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const bf16x8_t bv = *reinterpret_cast<const bf16x8_t*>(buf + fr * kGStride + ks * 32 + fk * 8);
#pragma unroll
      for (int jn = 0; jn < 2; ++jn) acc[jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[jn][ks], bv, acc[jn], 0, 0, 0);
    }
    dh[0] = acc[0], dh[1] = acc[1];
  }
  // carry (dh_next, dc_next) of the window's first step to the window before it
  if (live)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (a.dh) *reinterpret_cast<f32x4_t*>(a.dh + (size_t)row * kH + unit(h)) = dh[h];
      if (a.dc) *reinterpret_cast<f32x4_t*>(a.dc + (size_t)row * kH + unit(h)) = dcn[h];
    }
}

__global__ void __launch_bounds__(256, 1) lstm_backward_kernel(const BwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t sdg[2 * kRows * kGStride];  // dgates ping-pong, bf16
  backward_body(a, blockIdx.x, sdg);
}

// ---- two layers as one wavefront ------------------------------
// One launch runs both layers of the stack at once, three 4-wave workgroups per
// 16-row block:
//   producer   layer 1's recurrence (forward) / layer 2's backward through time,
//              publishing each step's h1_t (dgates2_t) through L2;
//   projection layer 2's input projection xp2_t = W_ih2·h1_t + b2 (forward) /
//              layer 1's output gradient dy1_t = dgates2_t·W_ih2 (backward), with
//              W_ih2 held in registers as MFMA B fragments;
//   consumer   layer 2's recurrence (forward) / layer 1's backward through time,
//              reading what the projection published.
// Each hand-off is a per-block step counter, released at agent scope after the
// data's stores every kPubEvery steps (the fence and the poll are paid once per
// 8 steps, not per step) and acquired before its loads; the consumer runs a few
// steps behind the producer, so the two layers' 1024 steps overlap instead of running
// back to back and layer 2's input projection is no separate GEMM.
//
// Placement: block b of the grid is (group b/24, slot b%24); slots 0-7, 8-15 and
// 16-23 are the producer, projection and consumer of row block 8·group + slot%8,
// so the three are 8 blocks apart (one XCD and its L2 under round-robin
// dispatch) and every waiting workgroup's producer has the lower block index
// (dispatched first: no wait on a workgroup that is not resident).  A wait gives
// up after 5 s of wall time (error flag), so every wave reaches the end.
constexpr uint64_t kWaitTicks = 500000000ull;  // 5 s of the 100 MHz real-time counter

// Spin until *flag > need (agent-scope acquire); false after the deadline.
__device__ bool wait_flag(const int* flag, int need, int* error) {
  if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) > need) return true;
  // after one timeout every later wait returns at once: the launch drains in ~5 s
  if (error && __hip_atomic_load(error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
  const uint64_t end = __builtin_amdgcn_s_memrealtime() + kWaitTicks;
  while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) <= need) {
    if (__builtin_amdgcn_s_memrealtime() > end) {
      if (error) __hip_atomic_store(error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

// role 0 producer, 1 projection, 2 consumer; false for a block past the last row block
__device__ __forceinline__ bool wave_role(int bid, int nblk, int* r, int* role) {
  const int grp = bid / 24, k = bid % 24;
  *role = k >> 3;
  *r = grp * 8 + (k & 7);
  return *r < nblk;
}

int triple_grid(int nblk) { return 24 * ((nblk + 7) / 8); }

// Forward projection: xp2_t[rows of blk] = W_ih2 · h1_t + b2 for every t, h1_t read
// from y1 ([T][B][H], published up to *wait), xp2 written and counted in *publish.
__device__ void project_fwd_body(const uint16_t* __restrict__ y1, const uint16_t* __restrict__ wih2,
                                 const uint16_t* __restrict__ b2, uint16_t* __restrict__ xp2, const int* wait,
                                 int* publish, int* error, int blk, int B, int T) {
  // wave g owns gate block g; W_ih2·hᵀ (operands swapped): lane (fr, fk) of tile jn
  // holds batch row fr, gate columns 128g + 16jn + 4fk + 0..3 -> 8-byte stores
  const int t_ = threadIdx.x, lane = t_ & 63, g = t_ >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int b0 = blk * kRows;
  bf16x8_t wf[8][4];
#pragma unroll
  for (int jn = 0; jn < 8; ++jn)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      wf[jn][kk] = *reinterpret_cast<const bf16x8_t*>(wih2 + (size_t)(g * kH + jn * 16 + fr) * kH + kk * 32 + fk * 8);
  f32x4_t bias[8];
#pragma unroll
  for (int jn = 0; jn < 8; ++jn) {
    const uint2 bv = *reinterpret_cast<const uint2*>(b2 + g * kH + jn * 16 + fk * 4);
    bias[jn] = f32x4_t{bf2f((uint16_t)(bv.x & 0xffff)), bf2f((uint16_t)(bv.x >> 16)), bf2f((uint16_t)(bv.y & 0xffff)),
                       bf2f((uint16_t)(bv.y >> 16))};
  }
  const int row = b0 + fr;
  const bool live = row < B;
  const int xrow = live ? row : 0;
  bf16x8_t hn[4];
  Waiter wt{wait, error, 0};
  auto load_h = [&](int t) {  // B fragments of h1_t: batch row fr, k = 32kk + 8fk .. +7
    wt.until(t);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      hn[kk] = *reinterpret_cast<const bf16x8_t*>(y1 + ((size_t)t * B + xrow) * kH + kk * 32 + fk * 8);
  };
  load_h(0);
  for (int t = 0; t < T; ++t) {
    const bf16x8_t hf[4] = {hn[0], hn[1], hn[2], hn[3]};
    if (t + 1 < T) load_h(t + 1);
    f32x4_t acc[8];
#pragma unroll
    for (int jn = 0; jn < 8; ++jn) acc[jn] = bias[jn];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int jn = 0; jn < 8; ++jn)
        acc[jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[jn][kk], hf[kk], acc[jn], 0, 0, 0);
    if (live) {
      uint16_t* p = xp2 + ((size_t)t * B + row) * (4 * kH) + g * kH + fk * 4;
#pragma unroll
      for (int jn = 0; jn < 8; ++jn)
        *reinterpret_cast<uint2*>(p + jn * 16) = uint2{(uint32_t)f2bf(acc[jn][0]) | ((uint32_t)f2bf(acc[jn][1]) << 16),
                                                       (uint32_t)f2bf(acc[jn][2]) | ((uint32_t)f2bf(acc[jn][3]) << 16)};
    }
    const bool pub = pub_step(t, T);
    if (pub) __threadfence();
    __syncthreads();
    if (pub && t_ == 0) __hip_atomic_store(publish, t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Backward projection: dy1_t = dgates2_t · W_ih2 ([16 x 512] x [512 x 128]) for
// t = T-1 .. 0, dgates2 published up to *wait (counted from the end), dy1
// ([T][B][H] bf16) counted in *publish.
__device__ void project_bwd_body(const uint16_t* __restrict__ dgates2, const uint16_t* __restrict__ wih2,
                                 uint16_t* __restrict__ dy1, const int* wait, int* publish, int* error, int blk,
                                 int B, int T) {
  // wave q owns hidden units [32q, 32q+32); W_ih2ᵀ·dgatesᵀ (operands swapped): lane
  // (fr, fk) of tile jn holds batch row fr, units 32q + 16jn + 4fk + 0..3
  const int t_ = threadIdx.x, lane = t_ & 63, q = t_ >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int b0 = blk * kRows;
  bf16x8_t wf[2][16];
#pragma unroll
  for (int jn = 0; jn < 2; ++jn)
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      uint16_t v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = wih2[(size_t)(ks * 32 + fk * 8 + j) * kH + q * 32 + jn * 16 + fr];
      wf[jn][ks] = __builtin_bit_cast(bf16x8_t, u32x4{(uint32_t)v[0] | ((uint32_t)v[1] << 16),
                                                       (uint32_t)v[2] | ((uint32_t)v[3] << 16),
                                                       (uint32_t)v[4] | ((uint32_t)v[5] << 16),
                                                       (uint32_t)v[6] | ((uint32_t)v[7] << 16)});
    }
  const int row = b0 + fr;
  const bool live = row < B;
  const int xrow = live ? row : 0;
  bf16x8_t an[16];
  Waiter wt{wait, error, 0};
  auto load_dg = [&](int t) {  // B fragments of dgates2_t: batch row fr, k = 32ks + 8fk .. +7
    wt.until(T - t - 1);
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
      an[ks] = *reinterpret_cast<const bf16x8_t*>(dgates2 + ((size_t)t * B + xrow) * (4 * kH) + ks * 32 + fk * 8);
  };
  load_dg(T - 1);
  for (int t = T - 1; t >= 0; --t) {
    bf16x8_t av[16];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) av[ks] = an[ks];
    if (t > 0) load_dg(t - 1);
    f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
#pragma unroll
      for (int jn = 0; jn < 2; ++jn) acc[jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[jn][ks], av[ks], acc[jn], 0, 0, 0);
    if (live) {
      uint16_t* p = dy1 + ((size_t)t * B + row) * kH + q * 32 + fk * 4;
#pragma unroll
      for (int jn = 0; jn < 2; ++jn)
        *reinterpret_cast<uint2*>(p + jn * 16) = uint2{(uint32_t)f2bf(acc[jn][0]) | ((uint32_t)f2bf(acc[jn][1]) << 16),
                                                       (uint32_t)f2bf(acc[jn][2]) | ((uint32_t)f2bf(acc[jn][3]) << 16)};
    }
    const bool pub = pub_step(T - 1 - t, T);
    if (pub) __threadfence();
    __syncthreads();
    if (pub && t_ == 0) __hip_atomic_store(publish, T - t, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

struct Wave2Args {
  FwdArgs l1, l2;           // the two recurrences (l1.publish / l2.wait set by the host)
  const uint16_t* wih2;
  const uint16_t* b2;       // [4H] bf16: b_ih2 + b_hh2
  uint16_t* xp2;            // [T][B][4H] scratch
  int* flags;               // [2][nblk] counters + error
  int nblk;
};

__global__ void __launch_bounds__(256, 1) lstm2_forward_kernel(const Wave2Args a) {
  __shared__ __attribute__((aligned(16))) uint16_t sh[2 * kRows * kHStride];
  int r, role;
  if (!wave_role(blockIdx.x, a.nblk, &r, &role)) return;  // the whole workgroup
  int* err = a.flags + 2 * a.nblk;
  if (role == 0) {
    FwdArgs l1 = a.l1;
    l1.publish = a.flags + r;
    l1.error = err;
    recurrence_body(l1, r, sh);
  } else if (role == 1) {
    project_fwd_body(a.l1.y, a.wih2, a.b2, a.xp2, a.flags + r, a.flags + a.nblk + r, err, r, a.l1.B, a.l1.T);
  } else {
    FwdArgs l2 = a.l2;
    l2.wait = a.flags + a.nblk + r;
    l2.error = err;
    recurrence_body(l2, r, sh);
  }
}

struct Wave2BwdArgs {
  BwdArgs l2, l1;           // layer 2 runs first (producer), layer 1 consumes dy1
  const uint16_t* wih2;
  uint16_t* dy1;            // [T][B][H] scratch
  int* flags;               // [2][nblk] counters + error
  int nblk;
};

__global__ void __launch_bounds__(256, 1) lstm2_backward_kernel(const Wave2BwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t sdg[2 * kRows * kGStride];
  int r, role;
  if (!wave_role(blockIdx.x, a.nblk, &r, &role)) return;
  int* err = a.flags + 2 * a.nblk;
  if (role == 0) {
    BwdArgs l2 = a.l2;
    l2.publish = a.flags + r;
    l2.error = err;
    backward_body(l2, r, sdg);
  } else if (role == 1) {
    project_bwd_body(a.l2.dgates, a.wih2, a.dy1, a.flags + r, a.flags + a.nblk + r, err, r, a.l2.B, a.l2.T);
  } else {
    BwdArgs l1 = a.l1;
    l1.wait = a.flags + a.nblk + r;
    l1.error = err;
    backward_body(l1, r, sdg);
  }
}

int launch_fwd(const FwdArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(lstm_recurrence_kernel, dim3((a.B + kRows - 1) / kRows), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

}  // namespace

VGPU_API int vgpu_lstm_forward_train(const void* xp, const void* whh, void* y, void* gates, void* cells, int B,
                                     int T, int H, hipStream_t s) {
  if (H != kH || B < 1 || T < 1 || !gates || !cells) return -1;
  FwdArgs a{};
  a.xp = static_cast<const uint16_t*>(xp);
  a.whh = static_cast<const uint16_t*>(whh);
  a.y = static_cast<uint16_t*>(y);
  a.ys_row = (int64_t)T * kH;
  a.ys_t = kH;
  a.gates_out = static_cast<uint16_t*>(gates);
  a.cells_out = static_cast<float*>(cells);
  a.B = B, a.T = T;
  return launch_fwd(a, s);
}

VGPU_API int vgpu_lstm_backward(const void* gates, const void* cells, const void* dy, const void* whh, void* dgates,
                                int B, int T, int H, hipStream_t s) {
  if (H != kH || B < 1 || T < 1) return -1;
  BwdArgs a{};
  a.gates = static_cast<const uint16_t*>(gates);
  a.cells = static_cast<const float*>(cells);
  a.dy = static_cast<const uint16_t*>(dy);
  a.ds_row = (int64_t)T * kH;
  a.ds_t = kH;
  a.whh = static_cast<const uint16_t*>(whh);
  a.dgates = static_cast<uint16_t*>(dgates);
  a.B = B, a.T = T;
  hipLaunchKernelGGL(lstm_backward_kernel, dim3((B + kRows - 1) / kRows), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

// Returns 0, or -1 for an unsupported shape (hidden size must be 128).
VGPU_API int vgpu_lstm_recurrence(const void* xp, const void* whh, void* y, void* hlast, int B, int T, int H,
                                  hipStream_t s) {
  if (H != kH || B < 1 || T < 1) return -1;
  FwdArgs a{};
  a.xp = static_cast<const uint16_t*>(xp);
  a.whh = static_cast<const uint16_t*>(whh);
  a.y = static_cast<uint16_t*>(y);
  a.ys_row = (int64_t)T * kH;
  a.ys_t = kH;
  a.hlast = static_cast<uint16_t*>(hlast);
  a.B = B, a.T = T;
  return launch_fwd(a, s);
}

// One window [t0, t0 + T) of a layer (pointers already offset to the window):
// y strided (ys_row, ys_t elements), state carried through h_state (bf16 [B][H])
// and c_state (fp32 [B][H]) — read at the start unless `first`, written at the
// end.  gates / cells (training) as in vgpu_lstm_forward_train, or null.
VGPU_API int vgpu_lstm_recurrence_window(const void* xp, const void* whh, void* y, int64_t ys_row, int64_t ys_t,
                                         void* h_state, void* c_state, int first, void* gates, void* cells, int B,
                                         int T, int H, void* prof, hipStream_t s) {
  if (H != kH || B < 1 || T < 1 || !h_state || !c_state) return -1;
  FwdArgs a{};
  a.xp = static_cast<const uint16_t*>(xp);
  a.whh = static_cast<const uint16_t*>(whh);
  a.y = static_cast<uint16_t*>(y);
  a.ys_row = ys_row, a.ys_t = ys_t;
  a.hlast = static_cast<uint16_t*>(h_state);
  a.c_last = static_cast<float*>(c_state);
  a.h0 = first ? nullptr : static_cast<const uint16_t*>(h_state);
  a.c0 = first ? nullptr : static_cast<const float*>(c_state);
  a.gates_out = static_cast<uint16_t*>(gates);
  a.cells_out = static_cast<float*>(cells);
  a.prof = static_cast<unsigned long long*>(prof);
  a.B = B, a.T = T;
  return launch_fwd(a, s);
}

// Backward over one window (pointers offset to it), newest window first:
// (dh, dc) fp32 [B][H] carried between windows (zeroed by the caller before
// the last window); has_prev: the window does not start at t = 0 (cells[-1]
// is the previous window's last cell).  dy strided like the forward's y, or null.
VGPU_API int vgpu_lstm_backward_window(const void* gates, const void* cells, const void* dy, int64_t ds_row,
                                       int64_t ds_t, const void* whh, void* dgates, void* dh, void* dc, int has_prev,
                                       int B, int T, int H, hipStream_t s) {
  if (H != kH || B < 1 || T < 1 || !dh || !dc) return -1;
  BwdArgs a{};
  a.gates = static_cast<const uint16_t*>(gates);
  a.cells = static_cast<const float*>(cells);
  a.dy = static_cast<const uint16_t*>(dy);
  a.ds_row = ds_row, a.ds_t = ds_t;
  a.whh = static_cast<const uint16_t*>(whh);
  a.dgates = static_cast<uint16_t*>(dgates);
  a.dh = static_cast<float*>(dh);
  a.dc = static_cast<float*>(dc);
  a.has_prev = has_prev;
  a.B = B, a.T = T;
  hipLaunchKernelGGL(lstm_backward_kernel, dim3((B + kRows - 1) / kRows), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

// Both layers of a 2-layer stack in one wavefront launch (lstm2_forward_kernel).
// xp1 [T][B][4H] (layer-1 projection, biases folded in); b2 = b_ih2 + b_hh2 bf16
// [4H].  Workspace: y1t [T][B][H] bf16 (layer-1 h, timestep-major: the training
// backward uses it too), xp2 [T][B][4H] bf16, flags (2·ceil(B/16) + 1 ints, zeroed
// here).  Inference: hlast [B][H].  Training: y2 [T][B][H], gates1/2 [T][B][4H],
// cells1/2 fp32 [T][B][H] (all non-null).
VGPU_API int vgpu_lstm2_forward(const void* xp1, const void* whh1, const void* wih2, const void* b2, const void* whh2,
                                void* y1t, void* xp2, int* flags, void* hlast, void* y2, void* gates1, void* gates2,
                                void* cells1, void* cells2, int B, int T, int H, hipStream_t s) {
  if (H != kH || B < 1 || T < 1 || !y1t || !xp2 || !flags) return -1;
  const bool train = gates1 && gates2 && cells1 && cells2;
  const int nblk = (B + kRows - 1) / kRows;
  hipError_t e = hipMemsetAsync(flags, 0, sizeof(int) * (2 * nblk + 1), s);
  if (e != hipSuccess) return (int)e;
  Wave2Args a{};
  a.l1.xp = static_cast<const uint16_t*>(xp1);
  a.l1.whh = static_cast<const uint16_t*>(whh1);
  a.l1.y = static_cast<uint16_t*>(y1t);
  a.l1.ys_row = kH, a.l1.ys_t = (int64_t)B * kH;
  a.l1.gates_out = train ? static_cast<uint16_t*>(gates1) : nullptr;
  a.l1.cells_out = train ? static_cast<float*>(cells1) : nullptr;
  a.l1.B = B, a.l1.T = T;
  a.l2.xp = static_cast<const uint16_t*>(xp2);
  a.l2.whh = static_cast<const uint16_t*>(whh2);
  a.l2.y = static_cast<uint16_t*>(y2);
  a.l2.ys_row = kH, a.l2.ys_t = (int64_t)B * kH;
  a.l2.hlast = static_cast<uint16_t*>(hlast);
  a.l2.gates_out = train ? static_cast<uint16_t*>(gates2) : nullptr;
  a.l2.cells_out = train ? static_cast<float*>(cells2) : nullptr;
  a.l2.B = B, a.l2.T = T;
  a.wih2 = static_cast<const uint16_t*>(wih2);
  a.b2 = static_cast<const uint16_t*>(b2);
  a.xp2 = static_cast<uint16_t*>(xp2);
  a.flags = flags;
  a.nblk = nblk;
  hipLaunchKernelGGL(lstm2_forward_kernel, dim3(triple_grid(nblk)), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

// Backward of the 2-layer stack in one wavefront launch (lstm2_backward_kernel):
// dgates1/2 [T][B][4H] bf16 for the weight-gradient GEMMs.  dy2: gradient of the
// layer-2 output [B][T][H], or null.  Workspace: dy1 [T][B][H] bf16, flags
// (2·ceil(B/16) + 1 ints, zeroed here).
VGPU_API int vgpu_lstm2_backward(const void* gates1, const void* cells1, const void* gates2, const void* cells2,
                                 const void* dy2, const void* whh1, const void* whh2, const void* wih2,
                                 void* dgates1, void* dgates2, void* dy1, int* flags, int B, int T, int H,
                                 hipStream_t s) {
  if (H != kH || B < 1 || T < 1 || !dy1 || !flags) return -1;
  const int nblk = (B + kRows - 1) / kRows;
  hipError_t e = hipMemsetAsync(flags, 0, sizeof(int) * (2 * nblk + 1), s);
  if (e != hipSuccess) return (int)e;
  Wave2BwdArgs a{};
  a.l2.gates = static_cast<const uint16_t*>(gates2);
  a.l2.cells = static_cast<const float*>(cells2);
  a.l2.dy = static_cast<const uint16_t*>(dy2);
  a.l2.ds_row = (int64_t)T * kH, a.l2.ds_t = kH;
  a.l2.whh = static_cast<const uint16_t*>(whh2);
  a.l2.dgates = static_cast<uint16_t*>(dgates2);
  a.l2.B = B, a.l2.T = T;
  a.l1.gates = static_cast<const uint16_t*>(gates1);
  a.l1.cells = static_cast<const float*>(cells1);
  a.l1.dy = static_cast<const uint16_t*>(dy1);
  a.l1.ds_row = kH, a.l1.ds_t = (int64_t)B * kH;
  a.l1.whh = static_cast<const uint16_t*>(whh1);
  a.l1.dgates = static_cast<uint16_t*>(dgates1);
  a.l1.B = B, a.l1.T = T;
  a.wih2 = static_cast<const uint16_t*>(wih2);
  a.dy1 = static_cast<uint16_t*>(dy1);
  a.flags = flags;
  a.nblk = nblk;
  hipLaunchKernelGGL(lstm2_backward_kernel, dim3(triple_grid(nblk)), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

// Reads (and clears) the wavefront kernels' error flag: 1 when a wait timed out.
VGPU_API int vgpu_lstm2_flags_error(const int* flags, int B) {
  const int nblk = (B + kRows - 1) / kRows;
  int v = 0;
  if (hipMemcpy(&v, flags + 2 * nblk, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return v;
}
