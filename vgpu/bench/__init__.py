"""vgpu.bench."""
