// Depthwise 3x3 convolution for NHWC bf16 activations (MobileNet-V2 / DeepLab-v3
// training): forward, data gradient and weight gradient, any
// stride and dilation, padding = dilation ("same" for k = 3).
//
// A depthwise conv is 9 multiply-adds per output element: no GEMM, nothing
// for the MFMA, HBM / L2-bound.  Every kernel gives a thread 8 consecutive
// channels of one pixel (one 16-byte load per tap: a 64-lane wavefront reads
// 1 KiB contiguous runs of a pixel's channels) and keeps the weights as fp32
// [9][C] (the host op transposes the [C,1,3,3] filter once per step).
//   * forward: one thread per (output pixel, 8 channels), 9 taps gathered;
//   * data gradient: one thread per (input pixel, 8 channels) gathers the
//     output pixels whose window holds it (stride-divisible taps only) -- no
//     atomics, no zero-fill;
//   * weight gradient: a block takes a slab of output pixels (8 per thread
//     for any C), its threads' 9 x 8 fp32 sums are merged in LDS into one
//     partial row per slab, and a second kernel sums the slabs in a fixed
//     order, 16 threads per element (deterministic).  (A first version gave
//     each thread its own slab: 64k partial rows whose one-thread-per-element
//     reduce cost 59 µs a layer, profiles/r5/train/prof_4_2_after.md.)
// fp32 accumulation, one bf16 rounding per output (forward / data gradient).
//
// Weights: fp32 [9][C] (the inference path's BN-folded filter), or the
// module's own bf16 [C][9] ([C,1,3,3] as stored) -- a thread's 8 channels x 9
// taps are then one contiguous 144-byte run, nine 16-byte loads; the weight
// gradient is written in that layout too.  (Converting the filter to fp32
// [9][C] and back per layer and step was 4 launches per depthwise layer, 68 a
// DeepLab step: profiles/r6/train.)
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

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  typedef __attribute__((ext_vector_type(2))) float f2;
  typedef __attribute__((ext_vector_type(2))) __bf16 b2;
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{lo, hi}, b2));
}

__device__ __forceinline__ u32x4 pack8(const float (&v)[8]) {
  return u32x4{pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7])};
}

__device__ __forceinline__ void load_w8(const float* __restrict__ w, int C, int tap, int c8, float (&f)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(w + (int64_t)tap * C + c8);
  const float4 b = *reinterpret_cast<const float4*>(w + (int64_t)tap * C + c8 + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
  f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// A thread's 8 channels x 9 taps of a bf16 [C][9] filter (w + c8 * 9: 144-B
// aligned, since c8 is a multiple of 8).
struct W72 {
  u32x4 q[9];
  __device__ __forceinline__ void load(const uint16_t* __restrict__ w, int c8) {
    const u32x4* p = reinterpret_cast<const u32x4*>(w + (int64_t)c8 * 9);
#pragma unroll
    for (int i = 0; i < 9; ++i) q[i] = p[i];
  }
  // channel j, tap k (compile-time after unrolling)
  __device__ __forceinline__ float at(int j, int k) const {
    const int e = j * 9 + k;
    const u32x4 v = q[e >> 3];
    const int wd = (e & 7) >> 1;
    const uint32_t u = wd == 0 ? v.x : (wd == 1 ? v.y : (wd == 2 ? v.z : v.w));
    return __uint_as_float((e & 1) ? (u & 0xffff0000u) : (u << 16));
  }
};

template <bool kC9>
__device__ __forceinline__ void tap_w8(const void* __restrict__ w, const W72& wc, int C, int tap, int c8,
                                       float (&f)[8]) {
  if constexpr (kC9) {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = wc.at(j, tap);
  } else {
    load_w8(static_cast<const float*>(w), C, tap, c8, f);
  }
}

struct Shape {
  int N, H, W, C, OH, OW, stride, dil;
};

// bias (fp32 [C], optional) and act (0 none, 1 ReLU, 2 ReLU6): a folded
// BatchNorm + activation in inference (vgpu.models.vision DeepLab fusion).
template <bool kC9>
__global__ void __launch_bounds__(kThreads) dw_fwd_kernel(const u32x4* __restrict__ x, const void* __restrict__ w,
                                                          const float* __restrict__ bias, int act,
                                                          u32x4* __restrict__ y, const Shape s, int64_t total) {
  const int cv = s.C / 8;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total; i += (int64_t)gridDim.x * kThreads) {
    const int cg = (int)(i % cv);
    int64_t r = i / cv;
    const int ow = (int)(r % s.OW);
    r /= s.OW;
    const int oh = (int)(r % s.OH);
    const int n = (int)(r / s.OH);
    const int h0 = oh * s.stride - s.dil, w0 = ow * s.stride - s.dil;
    const u32x4* xn = x + (int64_t)n * s.H * s.W * cv + cg;
    W72 wc;
    if constexpr (kC9) wc.load(static_cast<const uint16_t*>(w), cg * 8);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = h0 + kh * s.dil;
      if ((unsigned)ih >= (unsigned)s.H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = w0 + kw * s.dil;
        if ((unsigned)iw >= (unsigned)s.W) continue;
        float xv[8], wv[8];
        unpack8(xn[((int64_t)ih * s.W + iw) * cv], xv);
        tap_w8<kC9>(w, wc, s.C, kh * 3 + kw, cg * 8, wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(xv[j], wv[j], acc[j]);
      }
    }
    if (bias) {
      const float4 b0 = *reinterpret_cast<const float4*>(bias + cg * 8);
      const float4 b1 = *reinterpret_cast<const float4*>(bias + cg * 8 + 4);
      acc[0] += b0.x; acc[1] += b0.y; acc[2] += b0.z; acc[3] += b0.w;
      acc[4] += b1.x; acc[5] += b1.y; acc[6] += b1.z; acc[7] += b1.w;
    }
    if (act) {
      const float hi = act == 2 ? 6.0f : INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fminf(fmaxf(acc[j], 0.0f), hi);
    }
    y[i] = pack8(acc);
  }
}

template <bool kC9>
__global__ void __launch_bounds__(kThreads) dw_dgrad_kernel(const u32x4* __restrict__ dy, const void* __restrict__ w,
                                                            u32x4* __restrict__ dx, const Shape s, int64_t total) {
  const int cv = s.C / 8;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total; i += (int64_t)gridDim.x * kThreads) {
    const int cg = (int)(i % cv);
    int64_t r = i / cv;
    const int iw = (int)(r % s.W);
    r /= s.W;
    const int ih = (int)(r % s.H);
    const int n = (int)(r / s.H);
    const u32x4* dyn = dy + (int64_t)n * s.OH * s.OW * cv + cg;
    W72 wc;
    if constexpr (kC9) wc.load(static_cast<const uint16_t*>(w), cg * 8);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      // ih = oh·stride - dil + kh·dil
      const int th = ih + s.dil - kh * s.dil;
      if (th < 0 || th % s.stride) continue;
      const int oh = th / s.stride;
      if (oh >= s.OH) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int tw = iw + s.dil - kw * s.dil;
        if (tw < 0 || tw % s.stride) continue;
        const int ow = tw / s.stride;
        if (ow >= s.OW) continue;
        float gv[8], wv[8];
        unpack8(dyn[((int64_t)oh * s.OW + ow) * cv], gv);
        tap_w8<kC9>(w, wc, s.C, kh * 3 + kw, cg * 8, wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(gv[j], wv[j], acc[j]);
      }
    }
    dx[i] = pack8(acc);
  }
}

// Block = one slab of pb output pixels (pb = k · (256 / cv), k <= kWgPix): thread t owns
// channel group t % cv and pixels p0 + t / cv + k · (256 / cv), two pixels'
// loads in flight.  Its 9 x 8 sums are merged across the block one tap at a
// time with every thread taking part: P = 256 / C threads per channel each
// fold a strided share of the sub-rows, then C threads fold the P shares
// (fixed order).  The first version had only C / 8 threads walk all sub-rows
// for each tap at 8 pixels per thread: 30 us per DeepLab layer, 10 % of its
// training step (profiles/r5/train/deeplab_step_kernels.md).
constexpr int kWgPix = 8;
__global__ void __launch_bounds__(kThreads) dw_wgrad_kernel(const u32x4* __restrict__ dy, const u32x4* __restrict__ x,
                                                            float* __restrict__ part, const Shape s, int pb) {
  __shared__ float red[kThreads * 8];  // [sub][C] for one tap (nsub · C = 256 · 8 floats)
  __shared__ float red2[kThreads];
  const int cv = s.C / 8, nsub = kThreads / cv;
  const int t = threadIdx.x, cg = t % cv, sub = t / cv;
  const int64_t P = (int64_t)s.N * s.OH * s.OW;
  const int64_t p0 = (int64_t)blockIdx.x * pb, p1 = p0 + pb < P ? p0 + pb : P;
  float acc[9][8];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  auto pixel = [&](int64_t p) {
    const int ow = (int)(p % s.OW);
    const int64_t r = p / s.OW;
    const int oh = (int)(r % s.OH);
    const int n = (int)(r / s.OH);
    float g[8];
    unpack8(dy[p * cv + cg], g);
    const int h0 = oh * s.stride - s.dil, w0 = ow * s.stride - s.dil;
    const u32x4* xn = x + (int64_t)n * s.H * s.W * cv + cg;
    u32x4 xv[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int ih = h0 + (k / 3) * s.dil, iw = w0 + (k % 3) * s.dil;
      const bool ok = (unsigned)ih < (unsigned)s.H && (unsigned)iw < (unsigned)s.W;
      xv[k] = ok ? xn[((int64_t)ih * s.W + iw) * cv] : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      float xf[8];
      unpack8(xv[k], xf);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[k][j] = fmaf(g[j], xf[j], acc[k][j]);
    }
  };
  if (sub < nsub)
    for (int64_t p = p0 + sub; p < p1; p += nsub) pixel(p);
  const int C = s.C;
  const int PP = kThreads / C > 0 ? kThreads / C : 1;  // threads per channel in the first fold
  float* out = part + (int64_t)blockIdx.x * 9 * C;
#pragma unroll 1
  for (int k = 0; k < 9; ++k) {
    if (sub < nsub) {
#pragma unroll
      for (int j = 0; j < 8; ++j) red[sub * C + cg * 8 + j] = acc[k][j];
    }
    __syncthreads();
    // fold 1: thread (e, q) sums sub-rows q, q + PP, ... of element e
    for (int e0 = 0; e0 < C; e0 += kThreads / PP) {
      const int e = e0 + t % (kThreads / PP), q = t / (kThreads / PP);
      float a = 0.f;
      if (e < C && q < PP)
        for (int r = q; r < nsub; r += PP) a += red[r * C + e];
      if (e < C && q < PP) red2[q * (kThreads / PP) + (e - e0)] = a;
      __syncthreads();
      // fold 2: the PP shares of each element in order
      if (t < kThreads / PP && e0 + t < C) {
        float b = 0.f;
        for (int q2 = 0; q2 < PP; ++q2) b += red2[q2 * (kThreads / PP) + t];
        out[(int64_t)k * C + e0 + t] = b;
      }
      __syncthreads();
    }
  }
}

// dw[i] = Σ_slab part[slab][i] for i < 9C: 16 threads per element (slab
// residues mod 16, four accumulators each), merged in a fixed order.
// c9: write bf16 [C][9] (the module's weight layout) instead of fp32 [9][C].
__global__ void __launch_bounds__(kThreads) dw_wgrad_reduce_kernel(const float* __restrict__ part,
                                                                   void* __restrict__ dw, int n9c, int slabs,
                                                                   int c9) {
  __shared__ float red[16][17];
  const int el = threadIdx.x % 16, q = threadIdx.x / 16, i = blockIdx.x * 16 + el;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (i < n9c) {
    int k = q;
    for (; k + 48 < slabs; k += 64) {
      a0 += part[(int64_t)k * n9c + i];
      a1 += part[(int64_t)(k + 16) * n9c + i];
      a2 += part[(int64_t)(k + 32) * n9c + i];
      a3 += part[(int64_t)(k + 48) * n9c + i];
    }
    for (; k < slabs; k += 16) a0 += part[(int64_t)k * n9c + i];
  }
  red[q][el] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (q == 0 && i < n9c) {
    float a = 0.f;
    for (int r = 0; r < 16; ++r) a += red[r][el];
    if (c9) {
      const int C = n9c / 9, k = i / C, c = i - k * C;
      __bf16 b = (__bf16)a;
      static_cast<uint16_t*>(dw)[c * 9 + k] = __builtin_bit_cast(uint16_t, b);
    } else {
      static_cast<float*>(dw)[i] = a;
    }
  }
}

// Weight gradient, round 6: a workgroup owns ONE channel group (8 channels)
// and a slab of 256·ppt output pixels, a thread one pixel in 256 of the slab
// (ppt of them, all nine taps' loads in flight per pixel); the 72 sums fold
// across the wave by shuffles and across the 4 waves in LDS, in a fixed order.
// With one slab the block writes the gradient itself -- no partial rows, no
// reduce launch.  (A mapping with 8 channel groups x 32 pixel lanes per
// workgroup coalesced the loads but cut the threads 8x: 25 us at 24², worse.)  (The kernel above gave a 24² DeepLab layer
// 2-pixel slabs: 288 partial rows of 9·C floats and 18-42 us per layer, plus a
// ~5 us reduce: 430 us a 4.2 step, profiles/r6/train.)
__global__ void __launch_bounds__(kThreads) dw_wgrad2_kernel(const u32x4* __restrict__ dy,
                                                             const u32x4* __restrict__ x, float* __restrict__ part,
                                                             void* __restrict__ out, int out_fmt, const Shape s,
                                                             int ppt) {
  __shared__ float tr[72][kThreads + 1];  // +1: a thread's 72 stores hit 72 banks apart
  __shared__ float red[4][72];
  const int cv = s.C / 8, cg = blockIdx.x, t = threadIdx.x;
  const int64_t P = (int64_t)s.N * s.OH * s.OW;
  const int64_t p0 = (int64_t)blockIdx.y * kThreads * ppt;
  float acc[9][8];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  // pixel i + 1's ten loads are issued before pixel i's FMAs (32-bit index
  // math: the host keeps P < 2^31)
  const int Pi = (int)P;
  auto load = [&](int i, u32x4& gv, u32x4 (&xv)[9]) {
    const int p = (int)p0 + i * kThreads + t;
    const bool in = p < Pi;
    const int pp = in ? p : 0;
    const int ow = pp % s.OW, r = pp / s.OW;
    const int oh = r % s.OH, n = r / s.OH;
    const int h0 = oh * s.stride - s.dil, w0 = ow * s.stride - s.dil;
    const u32x4* xn = x + (int64_t)n * s.H * s.W * cv + cg;
    gv = in ? dy[(int64_t)pp * cv + cg] : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int ih = h0 + (k / 3) * s.dil, iw = w0 + (k % 3) * s.dil;
      const bool ok = in && (unsigned)ih < (unsigned)s.H && (unsigned)iw < (unsigned)s.W;
      xv[k] = ok ? xn[((int64_t)ih * s.W + iw) * cv] : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto fma9 = [&](const u32x4& gv, const u32x4 (&xv)[9]) {
    float g[8];
    unpack8(gv, g);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      float xf[8];
      unpack8(xv[k], xf);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[k][j] = fmaf(g[j], xf[j], acc[k][j]);
    }
  };
  int n_pix = (int)((P - p0 + kThreads - 1) / kThreads);  // iterations with any live lane
  if (n_pix > ppt) n_pix = ppt;
  u32x4 ga, gb, xa[9], xb[9];
  if (n_pix > 0) load(0, ga, xa);
  for (int i = 0; i < n_pix; i += 2) {
    if (i + 1 < n_pix) load(i + 1, gb, xb);
    fma9(ga, xa);  // out-of-range pixels loaded zeros: they add nothing
    if (i + 1 >= n_pix) break;
    if (i + 2 < n_pix) load(i + 2, ga, xa);
    fma9(gb, xb);
  }
  // 72 sums x 256 threads through LDS: every thread stores its row, then 288
  // threads-tasks each add a 64-thread column run, then 72 threads merge the 4
  // runs in order.  (Wave shuffles took 432 cross-lane ops a thread: ~22 us
  // per call whatever the layer size.)
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) tr[k * 8 + j][t] = acc[k][j];
  __syncthreads();
  for (int task = t; task < 72 * 4; task += kThreads) {
    const int q = task / 72, o = task - q * 72;  // a wave's lanes: consecutive rows, distinct banks
    const float* row = &tr[o][q * 64];
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll 4
    for (int i = 0; i < 64; i += 4) {
      a0 += row[i];
      a1 += row[i + 1];
      a2 += row[i + 2];
      a3 += row[i + 3];
    }
    red[q][o] = (a0 + a1) + (a2 + a3);
  }
  __syncthreads();
  if (t < 72) {
    const float v = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
    const int k = t >> 3, c = cg * 8 + (t & 7);
    if (part) {
      part[(int64_t)blockIdx.y * 9 * s.C + (int64_t)k * s.C + c] = v;
    } else if (out_fmt) {
      __bf16 b = (__bf16)v;
      static_cast<uint16_t*>(out)[c * 9 + k] = __builtin_bit_cast(uint16_t, b);
    } else {
      static_cast<float*>(out)[k * s.C + c] = v;
    }
  }
}

// (pixels per thread, slabs) of dw_wgrad2_kernel.  Its lanes read a pixel's
// 16 bytes each (uncoalesced, 10 loads in flight per pixel), so the layer's
// loads in flight scale with its thread count: up to 3 pixels a thread in one
// slab (DeepLab's 24² layers, ~10 us), else slabs of 4 pixels a thread plus
// the reduce launch (a 48² layer in one slab of 24 workgroups took 20-29 us).
void wgrad2_plan(const Shape& s, int& ppt, int& slabs) {
  const int64_t P = (int64_t)s.N * s.OH * s.OW;
  if (P <= 3 * kThreads) {
    ppt = (int)((P + kThreads - 1) / kThreads);
    slabs = 1;
    return;
  }
  ppt = 4;
  int64_t sl = (P + kThreads * 4 - 1) / (kThreads * 4);
  while (sl * (s.C / 8) > 2048 && ppt < 64) {  // bound the partial rows
    ppt *= 2;
    sl = (P + (int64_t)kThreads * ppt - 1) / ((int64_t)kThreads * ppt);
  }
  slabs = (int)sl;
}

bool make_shape(Shape& s, int N, int H, int W, int C, int stride, int dil) {
  if (N < 1 || H < 1 || W < 1 || C < 8 || C % 8 || stride < 1 || dil < 1) return false;
  s = Shape{N, H, W, C, (H - 1) / stride + 1, (W - 1) / stride + 1, stride, dil};
  return true;
}

int grid_for(int64_t total) {
  const int64_t b = (total + kThreads - 1) / kThreads;
  return (int)(b < 65536 ? (b > 0 ? b : 1) : 65536);
}

// Pixels per weight-gradient block: up to kWgPix per thread, fewer when that
// would leave the grid under 512 blocks (DeepLab's 48x48 / 24x24 layers ran 30-80
// slabs -- 30-80 of 256 CUs, ~48 us per layer, profiles/r5/train/prof_4_2_after.md).
int wgrad_pb(const Shape& s) {
  const int nsub = kThreads / (s.C / 8);
  const int64_t P = (int64_t)s.N * s.OH * s.OW;
  int64_t k = P / (512ll * nsub);
  k = k < 1 ? 1 : (k > kWgPix ? kWgPix : k);
  return (int)k * nsub;
}

int wgrad_slabs(const Shape& s) {
  const int64_t P = (int64_t)s.N * s.OH * s.OW;
  const int pb = wgrad_pb(s);
  return (int)((P + pb - 1) / pb);
}

}  // namespace

// w: fp32 [9][C] (wfmt 0) or bf16 [C][9] (wfmt 1, 16-B aligned).
VGPU_API int vgpu_dwconv3_fwd_nhwc(const void* x, const void* w, int wfmt, const float* bias, int act, void* y,
                                   int N, int H, int W, int C, int stride, int dil, hipStream_t st) {
  Shape s;
  if (!make_shape(s, N, H, W, C, stride, dil) || act < 0 || act > 2 || wfmt < 0 || wfmt > 1 ||
      (wfmt == 1 && ((uintptr_t)w & 15u)))
    return -1;
  const int64_t total = (int64_t)N * s.OH * s.OW * (C / 8);
  if (wfmt)
    hipLaunchKernelGGL(dw_fwd_kernel<true>, dim3(grid_for(total)), dim3(kThreads), 0, st, (const u32x4*)x, w, bias,
                       act, (u32x4*)y, s, total);
  else
    hipLaunchKernelGGL(dw_fwd_kernel<false>, dim3(grid_for(total)), dim3(kThreads), 0, st, (const u32x4*)x, w, bias,
                       act, (u32x4*)y, s, total);
  return (int)hipGetLastError();
}

VGPU_API int vgpu_dwconv3_dgrad_nhwc(const void* dy, const void* w, int wfmt, void* dx, int N, int H, int W, int C,
                                     int stride, int dil, hipStream_t st) {
  Shape s;
  if (!make_shape(s, N, H, W, C, stride, dil) || wfmt < 0 || wfmt > 1 || (wfmt == 1 && ((uintptr_t)w & 15u)))
    return -1;
  const int64_t total = (int64_t)N * H * W * (C / 8);
  if (wfmt)
    hipLaunchKernelGGL(dw_dgrad_kernel<true>, dim3(grid_for(total)), dim3(kThreads), 0, st, (const u32x4*)dy, w,
                       (u32x4*)dx, s, total);
  else
    hipLaunchKernelGGL(dw_dgrad_kernel<false>, dim3(grid_for(total)), dim3(kThreads), 0, st, (const u32x4*)dy, w,
                       (u32x4*)dx, s, total);
  return (int)hipGetLastError();
}

static int g_wgrad_v1 = -1;  // VGPU_DW_WGRAD=1: the round-5 slab kernel (A/B)
static bool wgrad_v1() {
  if (g_wgrad_v1 < 0) {
    const char* v = getenv("VGPU_DW_WGRAD");
    g_wgrad_v1 = (v && v[0] == '1') ? 1 : 0;
  }
  return g_wgrad_v1 == 1;
}

VGPU_API int64_t vgpu_dwconv3_wgrad_workspace(int N, int H, int W, int C, int stride, int dil) {
  Shape s;
  if (!make_shape(s, N, H, W, C, stride, dil) || C / 8 > kThreads) return -1;
  if (!wgrad_v1()) {
    int ppt, slabs;
    wgrad2_plan(s, ppt, slabs);
    return slabs == 1 ? 0 : (int64_t)slabs * 9 * C * 4;
  }
  return (int64_t)wgrad_slabs(s) * 9 * C * 4;
}

// dw: fp32 [9][C] (dfmt 0) or bf16 [C][9] (dfmt 1).  ws: vgpu_dwconv3_wgrad_workspace bytes.
VGPU_API int vgpu_dwconv3_wgrad_nhwc(const void* dy, const void* x, void* dw, int dfmt, void* ws, int64_t ws_bytes,
                                     int N, int H, int W, int C, int stride, int dil, hipStream_t st) {
  Shape s;
  if (!make_shape(s, N, H, W, C, stride, dil) || C / 8 > kThreads || dfmt < 0 || dfmt > 1) return -1;
  if (!wgrad_v1()) {
    int ppt, sl;
    wgrad2_plan(s, ppt, sl);
    if (sl > 1 && ws_bytes < (int64_t)sl * 9 * C * 4) return -2;
    if ((int64_t)N * s.OH * s.OW + (int64_t)kThreads * ppt >= ((int64_t)1 << 31)) return -1;
    hipLaunchKernelGGL(dw_wgrad2_kernel, dim3(C / 8, sl), dim3(kThreads), 0, st, (const u32x4*)dy,
                       (const u32x4*)x, sl > 1 ? (float*)ws : nullptr, dw, dfmt, s, ppt);
    if (sl > 1) {
      const int n9c = 9 * C;
      hipLaunchKernelGGL(dw_wgrad_reduce_kernel, dim3((n9c + 15) / 16), dim3(kThreads), 0, st, (const float*)ws, dw,
                         n9c, sl, dfmt);
    }
    return (int)hipGetLastError();
  }
  const int slabs = wgrad_slabs(s);
  if (ws_bytes < (int64_t)slabs * 9 * C * 4) return -2;
  hipLaunchKernelGGL(dw_wgrad_kernel, dim3(slabs), dim3(kThreads), 0, st, (const u32x4*)dy, (const u32x4*)x,
                     (float*)ws, s, wgrad_pb(s));
  const int n9c = 9 * C;
  hipLaunchKernelGGL(dw_wgrad_reduce_kernel, dim3((n9c + 15) / 16), dim3(kThreads), 0, st, (const float*)ws, dw,
                     n9c, slabs, dfmt);
  return (int)hipGetLastError();
}
