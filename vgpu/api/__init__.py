"""vgpu.api."""
