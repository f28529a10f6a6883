"""Cap holes closed in round 3, on a real MI355X:
stream-ordered pools (PyTorch's hipMallocAsync backend) and graph alloc nodes
never let physical VRAM use pass the container's cap."""
import pytest

from test_gpu_shim import probe

pytestmark = pytest.mark.gpu


def test_hipmallocasync_backend_never_exceeds_the_cap(gpu_build):
    cap_mib = 8192
    res = probe(["asynccap", cap_mib, 1024], {"VGPU_DEVICE_MEMORY_LIMIT_0": f"{cap_mib}m",
                                             "PYTORCH_HIP_ALLOC_CONF": "backend:hipMallocAsync",
                                             "PYTORCH_CUDA_ALLOC_CONF": "backend:hipMallocAsync"}, timeout=900)
    assert "error" not in res, res
    assert res["backend"] == "cudaMallocAsync", res
    cap = cap_mib << 20
    # amdgpu's own VRAM counter, this process's whole footprint (context included)
    assert res["peak_over_baseline"] <= cap * 1.01, res
    assert res["max_live_reached"] >= 0.75 * cap, res  # the cap is reachable
    assert res["ooms"] >= 6 and res["graphs_replayed"] >= 1, res
