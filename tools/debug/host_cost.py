"""Host-side cost of each piece of one GraphedPipeline / eager pipeline step (SSG B=32 N=1024):
the wall time the Python thread spends issuing, with the GPU kept busy (not synchronised)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import cases  # noqa: E402
from pn2 import heads as H, shard  # noqa: E402
from pn2.pipeline import GraphedPipeline, PipelinedForward  # noqa: E402

DEV = torch.device("cuda", 0)
torch.manual_seed(8)
model = H.ClsSSG().eval()
cases.randomize_bn(model, 8)
model = model.to(DEV)
B, N = 32, 1024
x = cases.cloud("uniform3", B, N, 90).permute(0, 2, 1).contiguous().to(DEV)
gp = GraphedPipeline(model, geometry_cus=int(os.environ.get("GEO_CUS", "0")), tail=True)
gp.run([x] * 3)
torch.cuda.synchronize()
sl = gp._slots[0]


def t_host(fn, n=50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6


for name, fn in [
    ("draw_start (cpu randint)", lambda: shard.draw_start(B, N)),
    ("start upload copy_", lambda: sl.starts[0][0].copy_(shard.draw_start(B, N), non_blocking=True)),
    ("pre-drawn upload", lambda: sl.start_buf.copy_(gp._pinned[gp._pinned_cur][0], non_blocking=True)),
    ("x copy_ (d2d)", lambda: sl.x.copy_(x, non_blocking=True)),
    ("fps graph replay", lambda: sl.fps.replay()),
    ("sa graph replay", lambda: sl.sa.replay()),
    ("head graph replay", lambda: sl.head.replay()),
    ("record+wait event", lambda: torch.cuda.current_stream().wait_event(torch.cuda.current_stream().record_event())),
    ("clone outputs", lambda: [t.clone() for t in sl.out if isinstance(t, torch.Tensor)]),
    ("eager model(x)", lambda: model(x)),
]:
    with torch.no_grad():
        h, w = t_host(fn, 20 if "eager" in name else 50)
    print("%-28s host %8.1f us/call   wall %8.1f us/call" % (name, h, w))

for k in (10, 40, 100):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gp.run([x] * k)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("GraphedPipeline.run(%d): host %.1f us/batch, wall %.1f us/batch" % (k, (t1 - t0) / k * 1e6, (t2 - t0) / k * 1e6))
pf = PipelinedForward(model, geometry_cus=32)
pf.run([x] * 3)
for k in (10, 40, 100):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pf.run([x] * k)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("PipelinedForward.run(%d): host %.1f us/batch, wall %.1f us/batch" % (k, (t1 - t0) / k * 1e6, (t2 - t0) / k * 1e6))
print("graph nodes: fps %s sa %s head %s" % tuple(
    getattr(g, "debug_dump", None) and "?" for g in (sl.fps, sl.sa, sl.head)))
