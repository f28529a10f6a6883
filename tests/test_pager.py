"""HostPager residency logic (CPU) and the paged Llama runner (GPU)."""
import pytest
import torch

from vgpu.ops.pager import HostPager


def test_lru_eviction_and_writeback_cpu():
    p = HostPager(budget_bytes=3 * 400, device="cpu")
    for i in range(5):
        p.register(f"c{i}", torch.full((100,), float(i)))
    p.prefetch(["c0", "c1", "c2"])
    assert list(p.resident) == ["c0", "c1", "c2"] and p.used == 1200
    t = p.get("c0", write=True)
    t += 10  # modify a resident chunk
    p.prefetch(["c3"])  # evicts LRU = c1 (c0 was touched)
    assert "c1" not in p.resident and "c0" in p.resident
    p.prefetch(["c4"])  # evicts c2
    p.prefetch(["c1"])  # evicts c0 → dirty write-back
    assert torch.all(p.host["c0"] == 10.0)
    assert p.stats.evictions == 3 and p.stats.swap_out_bytes == 400
    assert p.stats.swap_in_bytes == 6 * 400


def test_pinned_chunks_are_not_evicted_cpu():
    p = HostPager(budget_bytes=2 * 400, device="cpu")
    for i in range(3):
        p.register(f"c{i}", torch.zeros(100))
    p.get("c0")
    p.pin("c0")
    p.prefetch(["c1"])
    p.prefetch(["c2"])
    assert "c0" in p.resident and "c1" not in p.resident
    p.pin("c2")
    with pytest.raises(MemoryError):
        p.prefetch(["c1"])


def test_chunk_larger_than_budget_cpu():
    p = HostPager(budget_bytes=100, device="cpu")
    p.register("big", torch.zeros(1000))
    with pytest.raises(MemoryError):
        p.get("big")


def test_streamed_llama_matches_resident_cpu():
    from vgpu.models.llama import Llama, LlamaConfig
    from vgpu.models.streamed import StreamedLlama
    torch.manual_seed(0)
    cfg = LlamaConfig.tiny()
    m = Llama(cfg).eval()
    tokens = torch.randint(0, cfg.vocab, (1, 8))
    with torch.inference_mode():
        ref = m(tokens)
    layer_bytes = sum(p.numel() * 4 for p in m.layers[0].parameters())
    sm = StreamedLlama(m, budget_bytes=layer_bytes, device="cpu", lookahead=0)
    torch.testing.assert_close(sm(tokens), ref)
    assert sm.pager.stats.evictions == cfg.layers - 1


def test_streamed_llama_pins_prefix_cpu():
    """Cyclic layer scans thrash LRU; the runner pins a prefix and streams the rest."""
    from vgpu.models.llama import Llama, LlamaConfig
    from vgpu.models.streamed import StreamedLlama
    torch.manual_seed(0)
    cfg = LlamaConfig.tiny()
    cfg.layers = 6
    m = Llama(cfg).eval()
    tokens = torch.randint(0, cfg.vocab, (1, 4))
    with torch.inference_mode():
        ref = m(tokens)
    lb = sum(p.numel() * 4 for p in m.layers[0].parameters())
    sm = StreamedLlama(m, budget_bytes=4 * lb, device="cpu", lookahead=1)
    assert sm.n_resident() == 2
    for _ in range(3):
        torch.testing.assert_close(sm(tokens), ref)
    # token 1 loads all 6 layers, tokens 2-3 stream only the 4 non-resident ones
    assert sm.pager.stats.swap_in_bytes == (6 + 4 + 4) * lb
    sm.policy = "lru"
    s0 = sm.pager.stats.swap_in_bytes
    sm(tokens)
    assert sm.pager.stats.swap_in_bytes - s0 >= 4 * lb


@pytest.mark.gpu
def test_streamed_llama_matches_resident(gpu_build):
    from vgpu.models.llama import Llama, LlamaConfig
    from vgpu.models.streamed import StreamedLlama
    torch.manual_seed(0)
    cfg = LlamaConfig.tiny()
    cfg.layers = 6
    m = Llama(cfg).to(torch.bfloat16)
    ref_model = Llama(cfg).to(torch.bfloat16)
    ref_model.load_state_dict(m.state_dict())
    ref_model = ref_model.cuda().eval()
    tokens = torch.randint(0, cfg.vocab, (2, 16), device="cuda")
    with torch.inference_mode():
        ref = ref_model(tokens).float()
    layer_bytes = sum(p.numel() * 2 for p in m.layers[0].parameters())
    sm = StreamedLlama(m.eval(), budget_bytes=3 * layer_bytes, lookahead=2)
    got = sm(tokens).float()
    torch.cuda.synchronize()
    torch.testing.assert_close(got, ref, atol=2e-2, rtol=2e-2)
    st = sm.pager.stats
    assert st.misses == 6 and st.evictions >= 3 and st.swap_in_bytes == 6 * layer_bytes
    # second token: budget holds 3 layers, so some hits
    got2 = sm(tokens).float()
    torch.testing.assert_close(got2, ref, atol=2e-2, rtol=2e-2)
