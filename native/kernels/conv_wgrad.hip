// Convolution weight gradient on gfx950 MFMA (NHWC bf16, training of the
// ai-benchmark CNNs: ResNet-V2-50/152 tests 1.2 / 2.2).
//
//   dW[co][kh][kw][c] = Σ_{n,oh,ow} dy[n][oh][ow][co] · x[n][oh·s−p+kh][ow·s−p+kw][c]
//
// GEMM view: M = Cout, N = KS·KS·C (ordered (kh, kw, c) = the channels_last
// weight layout), K = P = N·OH·OW output pixels.  Both operands have the
// reduction (pixel) index as their OUTER memory dimension — dy is [P][Cout],
// the implicit im2col of x is [P][C] per tap — while the MFMA operand wants 8
// consecutive k per lane.  Tiles are therefore staged in LDS exactly as they
// sit in HBM ([pixel][channel], 16-B coalesced loads) and read back with
// gfx950's transposing `ds_read_b64_tr_b16` (4 pixels × 16 channels per 16-lane
// group, delivered column-major): no shuffles, no second LDS image.
//
// K is huge and M·N small (stage 1 at b=20 346²: 64×576 outputs over 151k
// pixels), so the pixel range is split across workgroups (split-K) until the
// grid covers the chip; each split writes an fp32 partial tile to a workspace
// and a second kernel sums the splits and rounds to bf16 — deterministic, no
// atomics.  Padding taps and the pixel tail load zeros through out-of-range
// buffer offsets (branch-free loads).
//
// Tiling: 256 threads = 4 wave64 in 2×2, workgroup tile BM (co) × BN (c) ∈
// {64,128}², K step 32 pixels = one mfma_f32_16x16x32_bf16 depth (64-pixel
// steps measured slower: the 128² tile then spills or drops to one wave/SIMD); register
// prefetch two steps ahead, double-buffered LDS, one barrier per step.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#define VGPU_API extern "C" __attribute__((visibility("default")))

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) char lds_char;  // 32-bit LDS addressing

constexpr int kThreads = 256;
constexpr int KP = 32;                     // pixels per K step (one MFMA depth)
constexpr uint32_t kOOB = 0x80000000u;     // buffer offset past num_records: loads return 0
typedef __attribute__((address_space(3))) void lds_void_t;
constexpr int vmcnt_imm_w(int n) { return (n & 15) | (((n >> 4) & 3) << 14) | (7 << 4) | (15 << 8); }
constexpr int kLgkm0w = 15 | (3 << 14) | (7 << 4);  // s_waitcnt lgkmcnt(0) only

struct WgradArgs {
  const uint16_t* dy;  // [N][OH][OW][Cout]
  const uint16_t* x;   // [N][H][W][C]
  float* ws;           // [splits][Cout][Ktot] fp32 partials (splits > 1)
  uint16_t* dw;        // [Cout][Ktot] bf16 (written directly when splits == 1)
  int N, H, W, C, Cout, OH, OW, KS, stride, pad;
  int P, Ktot, cblocks, steps, splits;
  int nseg;            // 3x3 tap-fused path: 32-pixel segments per output row
  uint32_t dy_bytes, x_bytes;
};

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

// LDS images of [pixel][channel] tiles are XOR-swizzled by 32-B column group:
// a 32-lane half of a transposed read covers pixel rows {8g+q, 8g+8+q} (q<4)
// at one 32-B column, which in plain 256-B (or 128-B) rows all sit on the same
// 8 banks -- an 8-way (4-way) conflict on every read.  Row r's 16-B chunk ch
// lives at slot ch ^ swz(r): 256-B rows permute the 8 column groups by
// (r&3, r>>3 & 1), 128-B rows the 4 groups of each half row by (r>>1 & 1,
// r>>3 & 1) -- the eight rows a half reads then hit eight distinct bank
// groups.  Rows r and r+4 (the two reads of one operand) share a swizzle.
template <int RS>
__device__ __forceinline__ int swz(int r) {
  if constexpr (RS == 256) return ((((r & 3) << 1) | ((r >> 3) & 1)) << 1);
  else return ((((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1);
}

// Two transposed 4-pixel reads → the 8 k-values (pixels 8g..8g+7) of one
// MFMA operand row (channel base + lane&15).  `tile` is a [KP][RS/2] bf16 image
// stored with swz<RS>.
template <int RS>
__device__ __forceinline__ bf16x8_t tr_operand(const lds_char* tile, int base_ch, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r = 8 * g + q, byte = (base_ch + 4 * p) * 2;
  const lds_char* a0 = tile + r * RS + (((byte >> 4) ^ swz<RS>(r)) << 4) + (byte & 15);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * RS));
  const s16x4 v[2] = {lo, hi};
  return __builtin_bit_cast(bf16x8_t, v);
}

template <int BM, int BN>
__global__ void __launch_bounds__(kThreads, 2) wgrad_kernel(const WgradArgs a) {
  constexpr int RSA = BM * 2, RSB = BN * 2;           // LDS row bytes
  constexpr int A_BYTES = KP * RSA, B_BYTES = KP * RSB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int CPA = BM / 8, CPB = BN / 8;           // 16-B chunks per row
  constexpr int LA = KP * CPA / kThreads, LB = KP * CPB / kThreads;  // loads per thread
  constexpr int WTM = BM / 2, WTN = BN / 2, TM = WTM / 16, TN = WTN / 16;
  static_assert(LA >= 1 && LB >= 1, "tile too small for 256 threads");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fk = lane >> 4;
  const int tap = blockIdx.x / a.cblocks, cb = blockIdx.x - tap * a.cblocks;
  const int kh = tap / a.KS, kw = tap - kh * a.KS;
  const int m0 = blockIdx.y * BM;
  const int split = blockIdx.z;
  const int step0 = split * a.steps;
  const int ohw = a.OH * a.OW;

  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.dy), 0, a.dy_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.x), 0, a.x_bytes, 0x00020000);

  u32x4 ra0[LA], rb0[LB], ra1[LA], rb1[LB];
  auto load = [&](int step, u32x4 (&ra)[LA], u32x4 (&rb)[LB]) {
    const int pbase = (step0 + step) * KP;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = t + i * kThreads, r = idx / CPA, ch = idx - r * CPA;
      const int pix = pbase + r;
      const uint32_t off = pix < a.P ? (uint32_t)(((int64_t)pix * a.Cout + m0 + ch * 8) * 2) : kOOB;
      ra[i] = __builtin_amdgcn_raw_buffer_load_b128(dyr, off, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = t + i * kThreads, r = idx / CPB, ch = idx - r * CPB;
      const int pix = pbase + r;
      const int n = pix / ohw, rem = pix - n * ohw, oh = rem / a.OW, ow = rem - oh * a.OW;
      const int ih = oh * a.stride - a.pad + kh, iw = ow * a.stride - a.pad + kw;
      const bool v = (pix < a.P) & ((unsigned)ih < (unsigned)a.H) & ((unsigned)iw < (unsigned)a.W);
      const uint32_t off =
          v ? (uint32_t)(((((int64_t)n * a.H + ih) * a.W + iw) * a.C + cb * BN + ch * 8) * 2) : kOOB;
      rb[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
    }
  };
  auto store = [&](int st, const u32x4 (&ra)[LA], const u32x4 (&rb)[LB]) {
    char* sA = smem + st * STAGE;
    char* sB = sA + A_BYTES;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = t + i * kThreads, r = idx / CPA, ch = idx - r * CPA;
      *reinterpret_cast<u32x4*>(sA + r * RSA + ((ch ^ swz<RSA>(r)) << 4)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = t + i * kThreads, r = idx / CPB, ch = idx - r * CPB;
      *reinterpret_cast<u32x4*>(sB + r * RSB + ((ch ^ swz<RSB>(r)) << 4)) = rb[i];
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // Two register sets in flight: the loads of step s+2 are issued while step
  // s is multiplied, so each step's global latency is covered by two steps.
  auto mma = [&](int st) {
    const lds_char* sA = (const lds_char*)smem + st * STAGE;
    const lds_char* sB = sA + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < KP / 32; ++kk) {  // 32 pixels per MFMA depth
      bf16x8_t af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = tr_operand<RSA>(sA + kk * 32 * RSA, wm * WTM + i * 16, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = tr_operand<RSB>(sB + kk * 32 * RSB, wn * WTN + j * 16, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  };
  const int nsteps = min(a.steps, (a.P + KP - 1) / KP - step0);
  if (nsteps > 0) load(0, ra0, rb0);
  if (nsteps > 1) load(1, ra1, rb1);
  for (int s = 0; s < nsteps; s += 2) {
    // even step: stage 0, register set 0
    store(0, ra0, rb0);
    __syncthreads();  // stage 0 written; stage 1 (read at s-1) free
    if (s + 2 < nsteps) load(s + 2, ra0, rb0);
    mma(0);
    if (s + 1 >= nsteps) break;
    // odd step: stage 1, register set 1
    store(1, ra1, rb1);
    __syncthreads();
    if (s + 3 < nsteps) load(s + 3, ra1, rb1);
    mma(1);
  }

  // Output row (co) 4·fk+e, column fr: bf16 gradient (one split) or the
  // split's fp32 partial tile.
  const int col0 = tap * a.C + cb * BN + wn * WTN;
  if (a.splits == 1) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = m0 + wm * WTM + i * 16 + fk * 4 + e;
          a.dw[(int64_t)co * a.Ktot + col0 + j * 16 + fr] = f2bf(acc[i][j][e]);
        }
    return;
  }
  float* out = a.ws + (int64_t)split * a.Cout * a.Ktot;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = m0 + wm * WTM + i * 16 + fk * 4 + e;
        out[(int64_t)co * a.Ktot + col0 + j * 16 + fr] = acc[i][j][e];
      }
}

// dW = bf16(Σ_split ws[split]).  A workgroup owns 256 / L float4 columns; its
// L split-lanes each sum every L-th split (4 independent accumulators, so the
// loads stay in flight), then the L partials are added in a fixed tree order
// through LDS — deterministic for a given split count.  L grows with the split
// count (≈ 4 splits per lane): with 16 lanes at 2-8 splits most threads idled
// and the pass ran at 9.6 us for 19 MB (VGG-16 b=2, profiles/r5/train).
// Optional second job of the reduce launch: a bias gradient db[c] = Σ_slab
// part[slab][c] (the per-slab partials of vgpu_relu_bias_grad_partial_nhwc),
// 16 channels per block, 16 threads per channel over the slab residues,
// merged in a fixed order.  Folding it in saves the bias-gradient launch of
// every conv + bias + ReLU layer (VGG-16: 13 per step at ~4.7 us).
struct DbJob {
  const float* part;
  void* db;
  int c, slabs, bf16;
  int stride;  // floats between consecutive entries (2: the .x of float2 BN statistics)
};

__device__ void db_reduce_block(const DbJob& j, int blk) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x % 16, q = threadIdx.x / 16, ch = blk * 16 + cl;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (ch < j.c) {
    int k = q;
    const int st = j.stride > 0 ? j.stride : 1;
    for (; k + 48 < j.slabs; k += 64) {
      a0 += j.part[((int64_t)k * j.c + ch) * st];
      a1 += j.part[((int64_t)(k + 16) * j.c + ch) * st];
      a2 += j.part[((int64_t)(k + 32) * j.c + ch) * st];
      a3 += j.part[((int64_t)(k + 48) * j.c + ch) * st];
    }
    for (; k < j.slabs; k += 16) a0 += j.part[((int64_t)k * j.c + ch) * st];
  }
  red[q][cl] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (q == 0 && ch < j.c) {
    float a = 0.f;
    for (int i = 0; i < 16; ++i) a += red[i][cl];
    if (j.bf16) static_cast<uint16_t*>(j.db)[ch] = f2bf(a);
    else static_cast<float*>(j.db)[ch] = a;
  }
}

template <int L>
__global__ void __launch_bounds__(kThreads) wgrad_reduce_kernel(const float* __restrict__ ws,
                                                                uint16_t* __restrict__ dw,
                                                                int64_t n4, int64_t stride4,
                                                                int splits, const DbJob job, int dw_blocks) {
  if ((int)blockIdx.x >= dw_blocks) {  // block-uniform: the bias-gradient job
    db_reduce_block(job, blockIdx.x - dw_blocks);
    return;
  }
  __shared__ f32x4_t part[L][kThreads / L];
  const int e = threadIdx.x % (kThreads / L), j = threadIdx.x / (kThreads / L);
  const int64_t i = blockIdx.x * (int64_t)(kThreads / L) + e;
  const f32x4_t* w4 = reinterpret_cast<const f32x4_t*>(ws);
  f32x4_t s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0, s3 = s0;
  if (i < n4) {
    int k = j;
    for (; k + 3 * L < splits; k += 4 * L) {
      s0 += w4[i + k * stride4];
      s1 += w4[i + (k + L) * stride4];
      s2 += w4[i + (k + 2 * L) * stride4];
      s3 += w4[i + (k + 3 * L) * stride4];
    }
    for (; k < splits; k += L) s0 += w4[i + k * stride4];
  }
  f32x4_t s = (s0 + s1) + (s2 + s3);
  if constexpr (L > 1) {
    part[j][e] = s;
    __syncthreads();
    for (int h = L / 2; h > 0; h >>= 1) {
      if (j < h) part[j][e] += part[j + h][e];
      __syncthreads();
    }
    s = part[0][e];
  }
  if (j == 0 && i < n4) {
    const uint32_t lo = (uint32_t)f2bf(s[0]) | ((uint32_t)f2bf(s[1]) << 16);
    const uint32_t hi = (uint32_t)f2bf(s[2]) | ((uint32_t)f2bf(s[3]) << 16);
    reinterpret_cast<uint2*>(dw)[i] = make_uint2(lo, hi);
  }
}

template <int L>
hipError_t launch_wgrad_reduce(const float* ws, uint16_t* dw, int64_t n4, int splits, const DbJob& job,
                               hipStream_t s) {
  const int64_t per = kThreads / L;
  const int dw_blocks = n4 > 0 ? (int)((n4 + per - 1) / per) : 0;
  const int db_blocks = job.part ? (job.c + 15) / 16 : 0;
  hipLaunchKernelGGL((wgrad_reduce_kernel<L>), dim3((unsigned)(dw_blocks + db_blocks)), dim3(kThreads), 0, s, ws,
                     dw, n4, n4, splits, job, dw_blocks);
  return hipGetLastError();
}

// 3x3 (pad 1) weight gradient with the nine taps fused: a K step is one
// 32-pixel segment of one output row; the block stages that segment of dy once
// and the x halo the nine taps need (3 input rows × (32·S + 2) columns) once,
// and feeds each tap's B operand from the same halo through per-lane row
// addresses of the transposing read (pixel j of tap (kh, kw) is halo row
// kh·HC + j·S + kw).  Versus nine independent GEMMs: dy is read once instead of
// nine times and x ≈ 3× instead of 9×, and each barrier covers 36 MFMAs per
// wave instead of 4.
template <int STRIDE>
__device__ __forceinline__ bf16x8_t tr_halo(const lds_char* halo, int kh, int kw, int base_ch, int lane) {
  constexpr int HC = 32 * STRIDE + 2, RS = 128;
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const lds_char* a0 = halo + (kh * HC + (8 * g + q) * STRIDE + kw) * RS + (base_ch + 4 * p) * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * STRIDE * RS));
  const s16x4 v[2] = {lo, hi};
  return __builtin_bit_cast(bf16x8_t, v);
}

template <int STRIDE>
__global__ void __launch_bounds__(kThreads, 1) wgrad3_kernel(const WgradArgs a) {
  constexpr int RS = 128;                          // LDS row: 64 bf16 channels
  constexpr int HC = 32 * STRIDE + 2, HROWS = 3 * HC;
  constexpr int LX = (HROWS * 8 + kThreads - 1) / kThreads;
  // halo image padded to LX·256 chunks: every thread's LDS store is in bounds
  // (no branch around it; the pad rows hold zeros and are never read)
  constexpr int DY_BYTES = KP * RS, STAGE = DY_BYTES + LX * kThreads * 16;
  constexpr int TM = 2, TN = 2;                    // 64x64 tile, 2x2 waves of 32x32
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fk = lane >> 4;
  const int cb = blockIdx.x, m0 = blockIdx.y * 64, split = blockIdx.z;
  const int step0 = split * a.steps;
  const int per_img = a.OH * a.nseg;
  const int total = a.N * per_img;

  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.dy), 0, a.dy_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.x), 0, a.x_bytes, 0x00020000);

  u32x4 rd0, rd1, rx0[LX], rx1[LX];
  auto load = [&](int step, u32x4& rd, u32x4 (&rx)[LX]) {
    const int seg = step0 + step;
    const bool vs = seg < total;
    const int n = seg / per_img, rem = seg - n * per_img, oh = rem / a.nseg;
    const int ow0 = (rem - oh * a.nseg) * 32;
    {
      const int r = t >> 3, ch = t & 7, ow = ow0 + r;
      const bool ok = vs & (ow < a.OW);
      rd = __builtin_amdgcn_raw_buffer_load_b128(
          dyr, ok ? (uint32_t)(((((int64_t)n * a.OH + oh) * a.OW + ow) * a.Cout + m0 + ch * 8) * 2) : kOOB,
          0, 0);
    }
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int idx = t + i * kThreads, hr = idx >> 3, ch = idx & 7;
      const int kh = hr / HC, col = hr - kh * HC;
      const int ih = oh * STRIDE - a.pad + kh, iw = ow0 * STRIDE - a.pad + col;
      const bool ok = vs & (idx < HROWS * 8) & ((unsigned)ih < (unsigned)a.H) & ((unsigned)iw < (unsigned)a.W);
      rx[i] = __builtin_amdgcn_raw_buffer_load_b128(
          xr, ok ? (uint32_t)(((((int64_t)n * a.H + ih) * a.W + iw) * a.C + cb * 64 + ch * 8) * 2) : kOOB,
          0, 0);
    }
  };
  auto store = [&](int st, const u32x4& rd, const u32x4 (&rx)[LX]) {
    char* sD = smem + st * STAGE;
    char* sX = sD + DY_BYTES;
    *reinterpret_cast<u32x4*>(sD + (t >> 3) * RS + (((t & 7) ^ swz<RS>(t >> 3)) << 4)) = rd;
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int idx = t + i * kThreads;
      *reinterpret_cast<u32x4*>(sX + (idx >> 3) * RS + (idx & 7) * 16) = rx[i];
    }
  };

  f32x4_t acc[9][TM][TN];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[k][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto mma = [&](int st) {
    const lds_char* sD = (const lds_char*)smem + st * STAGE;
    const lds_char* sX = sD + DY_BYTES;
    bf16x8_t af[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = tr_operand<RS>(sD, wm * 32 + i * 16, lane);
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        bf16x8_t bf[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) bf[j] = tr_halo<STRIDE>(sX, kh, kw, wn * 32 + j * 16, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[kh * 3 + kw][i][j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[kh * 3 + kw][i][j], 0, 0, 0);
        // keep one tap's operands live at a time (unbounded hoisting of the 36
        // transposed reads spills the 144 accumulator registers)
        __builtin_amdgcn_sched_barrier(0);
      }
  };

  const int nsteps = min(a.steps, total - step0);
  if (nsteps > 0) load(0, rd0, rx0);
  if (nsteps > 1) load(1, rd1, rx1);
  for (int s = 0; s < nsteps; s += 2) {
    store(0, rd0, rx0);
    __syncthreads();
    if (s + 2 < nsteps) load(s + 2, rd0, rx0);
    mma(0);
    if (s + 1 >= nsteps) break;
    store(1, rd1, rx1);
    __syncthreads();
    if (s + 3 < nsteps) load(s + 3, rd1, rx1);
    mma(1);
  }

  // One uniform branch, then straight-line stores.
  const int64_t lane_off = (int64_t)(m0 + wm * 32 + fk * 4) * a.Ktot + cb * 64 + wn * 32 + fr;
  if (a.splits == 1) {
    uint16_t* out = a.dw + lane_off;
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            out[(i * 16 + e) * a.Ktot + k * a.C + j * 16] = f2bf(acc[k][i][j][e]);
  } else {
    float* out = a.ws + (int64_t)split * a.Cout * a.Ktot + lane_off;
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            out[(i * 16 + e) * a.Ktot + k * a.C + j * 16] = acc[k][i][j][e];
  }
}

template <int BM, int BN>
hipError_t launch_wgrad(const WgradArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((wgrad_kernel<BM, BN>), dim3(a.Ktot / BN, a.Cout / BM, a.splits), dim3(kThreads),
                     0, s, a);
  return hipGetLastError();
}

}  // namespace

namespace {
int g_wgrad3 = -1;  // VGPU_CONV_WGRAD3=0 disables the tap-fused 3x3 path (A/B)
// The tap-fused 3x3 kernel wins on long pixel reductions (ResNet stage 1:
// 44.6-47.4 us vs 55.8-57.7 per tap); from stage 2 on the per-tap GEMMs on the
// swizzled images are faster (43.3 vs 54.5 at 38k pixels, 44.1 vs 54.6 at 9.7k;
// profiles/r4/train/convtrain_wgrad_*.log).
bool wgrad3_eligible(int KS, int stride, int pad, int64_t P) {
  if (g_wgrad3 < 0) {
    const char* v = getenv("VGPU_CONV_WGRAD3");
    g_wgrad3 = (v && v[0] == '0') ? 0 : 1;
  }
  return g_wgrad3 == 1 && KS == 3 && pad == 1 && (stride == 1 || stride == 2) && P >= 65536;
}

double g_launch_us = -1.0;
double launch_us() {
  if (g_launch_us < 0.0) {
    const char* v = getenv("VGPU_WGRAD_LAUNCH_US");
    g_launch_us = v ? atof(v) : 4.0;
    if (g_launch_us < 0.0) g_launch_us = 0.0;
  }
  return g_launch_us;
}

// Split-K factor for a shape; -1 = unsupported.
int64_t wgrad_splits(int N, int H, int W, int C, int Cout, int KS, int stride, int pad) {
  const int OH = (H + 2 * pad - KS) / stride + 1, OW = (W + 2 * pad - KS) / stride + 1;
  if (OH < 1 || OW < 1 || C % 64 || Cout % 64) return -1;
  const int64_t P = (int64_t)N * OH * OW;
  const bool fused3 = wgrad3_eligible(KS, stride, pad, P);
  const int bm = fused3 ? 64 : Cout % 128 == 0 ? 128 : 64, bn = fused3 ? 64 : C % 128 == 0 ? 128 : 64;
  const int64_t tiles = fused3 ? (int64_t)(C / 64) * (Cout / 64) : (int64_t)(KS * KS * C / bn) * (Cout / bm);
  const int64_t steps_total = fused3 ? (int64_t)N * OH * ((OW + 31) / 32) : (P + KP - 1) / KP;
  // Split count from a small cost model (µs): the K loop of a split is
  // latency-bound (t_step per step plus ≈ 3 µs fixed), splits run
  // `slots` at a time (resident workgroups: 4 waves each, occupancy per tile
  // shape from the kernel's resource usage), and every split costs a partial
  // tile written and re-read in fp32 at ≈ 4 TB/s.  Few output tiles over many
  // pixels (stage 1) want hundreds of splits; big tiles over few pixels
  // (stage 4) want 1-2, or the workspace traffic dominates.
  const int occ = fused3 ? 1 : (bm == 128 && bn == 128) ? 2 : (bm == 128 || bn == 128) ? 4 : 7;
  const double slots = occ * 256.0, tile_bytes = (double)Cout * KS * KS * C * 4;
  // µs per K step: latency plus the step's bytes (KP·(BM+BN)·2) at a CU's fill
  // rate; the fused 3x3 step carries nine taps' MFMAs
  const double t_step = fused3 ? 0.8 + 0.4 * stride : 0.4 + KP * (bm + bn) * 2 / 16384.0 * 0.6;
  int64_t splits = 1;
  double best = 1e30;
  for (int64_t sp = 1; sp <= 1024 && sp <= (steps_total + 3) / 4; sp *= 2) {
    const double waves = (double)((tiles * sp + (int64_t)slots - 1) / (int64_t)slots);
    // (+ the reduce's own launch when split: a dispatch inside a replayed
    // graph costs ~4.7 us however small, profiles/r6/train; VGPU_WGRAD_LAUNCH_US)
    const double est = waves * (t_step * (double)((steps_total + sp - 1) / sp) + 3.0) +
                       (sp > 1 ? 2.0 * sp * tile_bytes / 4.0e6 + launch_us() : tile_bytes / 8.0e6);
    if (est < best) { best = est; splits = sp; }
  }
  return splits;
}
}  // namespace

// Workspace bytes vgpu_conv_wgrad_nhwc needs for this shape (fp32 partial
// tiles; 0 when one split writes the bf16 gradient directly).
VGPU_API int64_t vgpu_conv_wgrad_workspace(int N, int H, int W, int C, int Cout, int KS, int stride,
                                           int pad) {
  const int64_t sp = wgrad_splits(N, H, W, C, Cout, KS, stride, pad);
  if (sp < 0) return -1;
  return sp == 1 ? 0 : sp * Cout * (int64_t)KS * KS * C * 4;
}

// dw [Cout][KS][KS][C] bf16 = weight gradient of y = conv(x, w; stride, pad),
// dy [N][OH][OW][Cout] and x [N][H][W][C] bf16 NHWC.  `ws` must hold
// vgpu_conv_wgrad_workspace(...) bytes.  Returns 0, a hipError_t, or -1 for an
// unsupported shape (checked before any launch).
namespace {
int wgrad_impl(const void* dy, const void* x, void* dw, void* ws, int64_t ws_bytes, int N, int H, int W, int C,
               int Cout, int KS, int stride, int pad, const DbJob& job, hipStream_t s);
}  // namespace

VGPU_API int vgpu_conv_wgrad_nhwc(const void* dy, const void* x, void* dw, void* ws, int64_t ws_bytes,
                                  int N, int H, int W, int C, int Cout, int KS, int stride, int pad,
                                  hipStream_t s) {
  return wgrad_impl(dy, x, dw, ws, ws_bytes, N, H, W, C, Cout, KS, stride, pad, DbJob{}, s);
}

// The same, and db[c] (fp32, or bf16 when db_bf16) = Σ_slab dbpart[slab][c]
// in the reduce launch (a launch of its own when the weight gradient needs no
// reduce).  dbpart: vgpu_relu_bias_grad_partial_nhwc's partials.
VGPU_API int vgpu_conv_wgrad_db_nhwc(const void* dy, const void* x, void* dw, void* ws, int64_t ws_bytes, int N,
                                     int H, int W, int C, int Cout, int KS, int stride, int pad, const float* dbpart,
                                     int slabs, int dbc, void* db, int db_bf16, int db_stride, hipStream_t s) {
  if (!dbpart || !db || slabs < 1 || dbc < 1 || db_stride < 1) return -1;
  return wgrad_impl(dy, x, dw, ws, ws_bytes, N, H, W, C, Cout, KS, stride, pad,
                    DbJob{dbpart, db, dbc, slabs, db_bf16, db_stride}, s);
}

// db alone (the layer's weight gradient ran elsewhere).
VGPU_API int vgpu_bias_grad_reduce(const float* dbpart, int slabs, int dbc, void* db, int db_bf16, int db_stride,
                                   hipStream_t s) {
  if (!dbpart || !db || slabs < 1 || dbc < 1 || db_stride < 1) return -1;
  return (int)launch_wgrad_reduce<1>(nullptr, nullptr, 0, 0, DbJob{dbpart, db, dbc, slabs, db_bf16, db_stride}, s);
}

namespace {
int wgrad_impl(const void* dy, const void* x, void* dw, void* ws, int64_t ws_bytes, int N, int H, int W, int C,
               int Cout, int KS, int stride, int pad, const DbJob& job, hipStream_t s) {
  if (C % 64 || Cout % 64 || KS < 1 || stride < 1 || pad < 0 || N < 1) return -1;
  WgradArgs a{};
  a.dy = static_cast<const uint16_t*>(dy);
  a.x = static_cast<const uint16_t*>(x);
  a.ws = static_cast<float*>(ws);
  a.N = N; a.H = H; a.W = W; a.C = C; a.Cout = Cout; a.KS = KS; a.stride = stride; a.pad = pad;
  a.OH = (H + 2 * pad - KS) / stride + 1;
  a.OW = (W + 2 * pad - KS) / stride + 1;
  if (a.OH < 1 || a.OW < 1) return -1;
  const int64_t P = (int64_t)N * a.OH * a.OW;
  const int64_t dyb = P * Cout * 2, xb = (int64_t)N * H * W * C * 2;
  if (P >= ((int64_t)1 << 31) || dyb >= ((int64_t)1 << 31) || xb >= ((int64_t)1 << 31)) return -1;
  a.P = (int)P;
  a.dy_bytes = (uint32_t)dyb;
  a.x_bytes = (uint32_t)xb;
  a.Ktot = KS * KS * C;
  const int bm = Cout % 128 == 0 ? 128 : 64, bn = C % 128 == 0 ? 128 : 64;
  a.cblocks = C / bn;
  const int64_t sp = wgrad_splits(N, H, W, C, Cout, KS, stride, pad);
  if (sp < 1 || ws_bytes < (sp == 1 ? 0 : sp * Cout * (int64_t)a.Ktot * 4)) return -1;
  a.splits = (int)sp;
  a.dw = static_cast<uint16_t*>(dw);
  hipError_t e;
  if (wgrad3_eligible(KS, stride, pad, P)) {
    a.nseg = (a.OW + 31) / 32;
    const int64_t steps_total = (int64_t)N * a.OH * a.nseg;
    a.steps = (int)((steps_total + a.splits - 1) / a.splits);
    const dim3 grid(C / 64, Cout / 64, a.splits);
    if (stride == 1) hipLaunchKernelGGL((wgrad3_kernel<1>), grid, dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((wgrad3_kernel<2>), grid, dim3(kThreads), 0, s, a);
    e = hipGetLastError();
  } else {
    const int64_t steps_total = (P + KP - 1) / KP;
    a.steps = (int)((steps_total + a.splits - 1) / a.splits);
    if (bm == 128 && bn == 128) e = launch_wgrad<128, 128>(a, s);
    else if (bm == 128) e = launch_wgrad<128, 64>(a, s);
    else if (bn == 128) e = launch_wgrad<64, 128>(a, s);
    else e = launch_wgrad<64, 64>(a, s);
  }
  if (e != hipSuccess) return (int)e;
  if (a.splits == 1)  // the K loop wrote bf16 directly; the bias job (if any) alone
    return job.part ? (int)launch_wgrad_reduce<1>(nullptr, nullptr, 0, 0, job, s) : 0;
  const int64_t n4 = (int64_t)Cout * a.Ktot / 4;
  const float* wsf = static_cast<const float*>(ws);
  uint16_t* dwp = static_cast<uint16_t*>(dw);
  const int nsp = a.splits;
  if (nsp >= 64) e = launch_wgrad_reduce<16>(wsf, dwp, n4, nsp, job, s);
  else if (nsp >= 32) e = launch_wgrad_reduce<8>(wsf, dwp, n4, nsp, job, s);
  else if (nsp >= 16) e = launch_wgrad_reduce<4>(wsf, dwp, n4, nsp, job, s);
  else if (nsp >= 8) e = launch_wgrad_reduce<2>(wsf, dwp, n4, nsp, job, s);
  else e = launch_wgrad_reduce<1>(wsf, dwp, n4, nsp, job, s);
  return (int)e;
}
}  // namespace

