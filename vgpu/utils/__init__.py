"""vgpu.utils: small shared helpers (GPU timing for the kernel benchmarks)."""
