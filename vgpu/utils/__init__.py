"""vgpu.utils."""
