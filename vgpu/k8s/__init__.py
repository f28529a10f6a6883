"""vgpu.k8s."""
