"""vgpu.ops."""
