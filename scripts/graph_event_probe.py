"""Does a HIP event recorded after hipGraphLaunch wait for the graph's kernels?
(The GPU-time limiter's markers rely on it; round 2 saw them complete early
under rocprofv3 --kernel-trace, profiles/temporal_r2.md.)  Run plain and under
rocprofv3; prints, per launch form, how long after the record the event
reported completion against the kernel's own duration."""
import json
import time
import torch
from vgpu.ops import kernels as K

torch.cuda.init()
s = torch.cuda.Stream()
busy_iters = 20000


def work():
    K.busy(4096, busy_iters)


with torch.cuda.stream(s):
    work()
torch.cuda.synchronize()
t0 = time.perf_counter()
with torch.cuda.stream(s):
    work()
torch.cuda.synchronize()
eager_ms = (time.perf_counter() - t0) * 1e3

g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    work()
torch.cuda.synchronize()


def probe(launch):
    torch.cuda.synchronize()
    ev = torch.cuda.Event()
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        launch()
        ev.record(s)
    first = ev.query()
    while not ev.query():
        pass
    t_ev = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) * 1e3
    return {"query_right_after": bool(first), "event_done_ms": round(t_ev, 3), "stream_done_ms": round(t_all, 3)}


out = {"kernel_ms_eager": round(eager_ms, 3)}
out["eager"] = probe(work)
out["graph"] = probe(g.replay)
print(json.dumps(out), flush=True)
