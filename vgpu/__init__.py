"""vgpu — MI355X-native Kubernetes vGPU stack.

Layers (top → bottom):
  vgpu.scheduler     mutating webhook + scheduler extender (filter / bind / metrics)
  vgpu.device        vendor device policy (resource parsing, type/NUMA/xGMI checks, CU masks)
  vgpu.deviceplugin  kubelet device plugin (ListAndWatch / Allocate / registration)
  vgpu.monitor       node monitor (shared-region reader, priority feedback, metrics)
  native/            libvgpu.so in-container enforcement (HBM cap, CU masks, dispatch limiter)
  vgpu.ops           hand-written gfx950 kernels (census/busy, page copy, fill/verify) + pager
  vgpu.models        ai-benchmark-equivalent workloads + Llama-3 for virtual device memory
"""
__version__ = "0.1.0"
