"""vgpu.scheduler."""
