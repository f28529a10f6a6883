"""Data-parallel training harness (vgpu/parallel/ddp.py) on CPU over gloo with
world_size 2: the flat-buffer bucketed all-reduce gives every rank the
average gradient, replicas stay identical, and the torchrun entry point prints
the aggregate throughput line."""
import json
import os
import socket
import subprocess
import sys

import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank: int, world: int, port: int, out):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    import copy
    import torch.distributed as dist
    from vgpu.parallel import ddp as D
    _, _, device = D.setup("gloo")
    torch.manual_seed(0)
    _, model = D.build_model("1.2", device, shrink=True)
    ref = copy.deepcopy(model)
    grads = D.GradBuckets(model.parameters(), bucket_mb=1)  # several buckets: exercises the hooks' order
    assert len(grads.buckets) > 1
    g = torch.Generator().manual_seed(rank)
    x = torch.randn(2, 3, 32, 32, generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (2,), generator=g)
    for _ in range(2):  # a second step: begin() re-arms the buckets and zeroes the flat buffer
        grads.begin()
        torch.nn.functional.cross_entropy(model(x), y).backward()
        grads.finish()
    ddp_grad = torch.cat([p.grad.flatten() for p in model.parameters()])
    torch.nn.functional.cross_entropy(ref(x), y).backward()
    local = torch.cat([p.grad.flatten() for p in ref.parameters()])
    allg = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(allg, local)
    mean = torch.stack(allg).mean(0)
    others = [torch.empty_like(ddp_grad) for _ in range(world)]
    dist.all_gather(others, ddp_grad)
    out[rank] = (float((ddp_grad - mean).abs().max()), float((others[0] - others[1]).abs().max()),
                 float(mean.abs().max()))
    dist.destroy_process_group()


def test_ddp_grads_are_rank_average_and_replicas_agree():
    world, port = 2, _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    for rank in range(world):
        err, spread, scale = res[rank]
        assert scale > 0
        assert err <= 1e-5 * max(1.0, scale), res
        assert spread == 0.0, res


def _unused_worker(rank: int, world: int, port: int, out):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    import torch.distributed as dist
    from vgpu.parallel import ddp as D
    D.setup("gloo")
    torch.manual_seed(0)
    used = torch.nn.Linear(8, 4)
    aux = torch.nn.Linear(8, 4)  # an aux head this step never touches
    grads = D.GradBuckets(list(used.parameters()) + list(aux.parameters()), bucket_mb=1)
    x = torch.randn(3, 8, generator=torch.Generator().manual_seed(rank))
    grads.begin()
    used(x).square().sum().backward()
    grads.finish()
    g = torch.cat([p.grad.flatten() for p in used.parameters()])
    allg = [torch.empty_like(g) for _ in range(world)]
    dist.all_gather(allg, g)
    out[rank] = (float((allg[0] - allg[1]).abs().max()), float(aux.weight.grad.abs().max()), len(grads.buckets))
    dist.destroy_process_group()


def test_ddp_unused_parameter_bucket_still_reduced():
    """a bucket holding a parameter with no gradient this
    step was never all-reduced, and the replicas silently diverged.  finish()
    now reduces every bucket whose hooks did not all fire."""
    world, port = 2, _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_unused_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    for rank in range(world):
        spread, aux_grad, nb = res[rank]
        assert nb == 1  # used and unused parameters share the bucket
        assert spread == 0.0, res
        assert aux_grad == 0.0


def test_ddp_entry_point_under_torchrun():
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={port}", "-m", "vgpu.parallel.ddp",
                        "--shrink", "--backend", "gloo", "--steps", "2", "--warmup", "1",
                        "--batch", "2", "--size", "32"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["world"] == 2 and res["backend"] == "gloo" and res["value"] > 0
    assert res["weights_in_sync"]
