"""vgpu.monitor."""
