"""vgpu.parallel: multi-GPU data-parallel training over RCCL (ddp.py) — the
scaling harness of SURVEY.md §2.9; the headline bench scales by running
independent vGPU pods per GPU (bench.py)."""
