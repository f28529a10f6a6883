// Data-gradient filters for a whole network in one launch (training).
//
// The data gradient of a stride-1 convolution is a convolution of dy with the
// filter transposed (Cout <-> C) and flipped (kh, kw -> KS-1-kh, KS-1-kw):
//
//   w'[c][kh][kw][co] = w[co][KS-1-kh][KS-1-kw][c]     (both channels_last)
//
// ResNet-V2-50 training built it per layer with transpose + flip + contiguous:
// ~100 small copy kernels per step, 380 us of a 9 ms step
// (profiles/r4/train/rocprof_train_1.2_steady_r4.txt).  Here one launch moves
// every layer's filter: the workgroups of all descriptors form one grid, a
// workgroup transposes one 64(co) x 64(c) tile of one tap through LDS (16-B
// loads along c, 16-B stores along co).  The descriptor table lives in device
// memory and is built once, so the launch can be captured in a hipGraph.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VGPU_API extern "C" __attribute__((visibility("default")))

namespace {

struct WtDesc {
  const uint16_t* src;  // [Cout][KS][KS][C]
  uint16_t* dst;        // [C][KS][KS][Cout]
  int cout, c, ks;
  int tile0;            // first tile of this descriptor in the grid
};

constexpr int kT = 64;  // tile edge (channels); C and Cout are multiples of 64

__global__ void __launch_bounds__(256) wt_flip_kernel(const WtDesc* __restrict__ descs, int ndesc) {
  __shared__ uint16_t tile[kT][kT + 8];  // +8 bf16 per row: 16-B aligned rows, no 2-way column conflicts
  const int b = blockIdx.x;
  int lo = 0, hi = ndesc - 1;  // last descriptor whose tile0 <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].tile0 <= b) lo = mid;
    else hi = mid - 1;
  }
  const WtDesc d = descs[lo];
  const int taps = d.ks * d.ks, nco = d.cout / kT, nc = d.c / kT;
  int r = b - d.tile0;
  const int tap = r % taps;
  r /= taps;
  const int ci = r % nc, coi = r / nc;
  if (coi >= nco) return;  // never: the host sizes the grid exactly
  const int kh = tap / d.ks, kw = tap - kh * d.ks;
  const int t = threadIdx.x;
  // load: 64 co rows x 64 c (8 x 16 B per row); 512 chunks, 2 per thread
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = t + k * 256, row = idx >> 3, ch = idx & 7;
    const int64_t off = ((int64_t)(coi * kT + row) * taps + tap) * d.c + ci * kT + ch * 8;
    const uint4 v = *reinterpret_cast<const uint4*>(d.src + off);
    *reinterpret_cast<uint4*>(&tile[row][ch * 8]) = v;
  }
  __syncthreads();
  // store: 64 c rows x 64 co, at the flipped tap
  const int ftap = (d.ks - 1 - kh) * d.ks + (d.ks - 1 - kw);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = t + k * 256, row = idx >> 3, ch = idx & 7;  // row = c within the tile, ch = co chunk
    uint16_t v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = tile[ch * 8 + e][row];
    const int64_t off = ((int64_t)(ci * kT + row) * taps + ftap) * d.cout + coi * kT + ch * 8;
    *reinterpret_cast<uint4*>(d.dst + off) = *reinterpret_cast<const uint4*>(v);
  }
}

}  // namespace

// Tiles one descriptor contributes (the host builds tile0 prefixes from it).
VGPU_API int vgpu_wt_flip_tiles(int cout, int c, int ks) {
  if (cout <= 0 || c <= 0 || ks <= 0 || cout % kT || c % kT) return -1;
  return ks * ks * (cout / kT) * (c / kT);
}

// descs: device array of `ndesc` records {src, dst, cout, c, ks, tile0}
// (32 bytes each: two pointers, four int32), tile0 ascending; `tiles` = the total.
VGPU_API int vgpu_wt_flip_batched(const void* descs, int ndesc, int tiles, void* stream) {
  if (!descs || ndesc <= 0 || tiles <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(wt_flip_kernel, dim3(tiles), dim3(256), 0, (hipStream_t)stream,
                     static_cast<const WtDesc*>(descs), ndesc);
  return (int)hipGetLastError();
}

VGPU_API int vgpu_wt_desc_size() { return (int)sizeof(WtDesc); }
