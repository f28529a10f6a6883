"""vgpu.device."""
