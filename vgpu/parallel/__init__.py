"""vgpu.parallel."""
