// A tiny gfx950 code object for the module-charging probe
// (vgpu/bench/probes.py arrays: hipModuleLoadData of this image must be
// charged to the container's module class by the enforcement library).
#include <hip/hip_runtime.h>

extern "C" __global__ void vgpu_module_probe(float* out, float v) {
  out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}
