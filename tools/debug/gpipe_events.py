"""Untraced per-stream timeline of the GraphedPipeline loop (SSG B=32 N=1024): the run() loop
re-stated with timing events at every stage boundary; prints per-batch times relative to the
first batch's compute start."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import cases  # noqa: E402
from pn2 import heads as H, shard  # noqa: E402
from pn2.pipeline import GraphedPipeline, _streams, _clone  # noqa: E402

DEV = torch.device("cuda", 0)
torch.manual_seed(8)
model = H.ClsSSG().eval()
cases.randomize_bn(model, 8)
model = model.to(DEV)
B, N = 32, 1024
x = cases.cloud("uniform3", B, N, 90).permute(0, 2, 1).contiguous().to(DEV)
tail_on = "--no-tail" not in sys.argv
gp = GraphedPipeline(model, geometry_cus=int(os.environ.get("GEO", "32")), tail=tail_on)
gp.run([x] * 3)
torch.cuda.synchronize()
geo, main, tail = _streams(0, gp.geometry_cus)
K = 12
batches = [x] * K


def ev(stream):
    e = torch.cuda.Event(enable_timing=True)
    e.record(stream)
    return e


marks = [dict() for _ in range(K)]
ev_fps, ev_sa, ev_head = [None, None], [None, None], [None, None]


def issue_fps(j):
    s = j % 2
    sl = gp._slots[s]
    with torch.cuda.stream(geo):
        if ev_sa[s] is not None:
            geo.wait_event(ev_sa[s])
        marks[j]["geo0"] = ev(geo)
        sl.x.copy_(batches[j], non_blocking=True)
        for t, b, n in sl.starts:
            t.copy_(shard.draw_start(b, n), non_blocking=True)
        marks[j]["fps0"] = ev(geo)
        sl.fps.replay()
        ev_fps[s] = ev(geo)
        marks[j]["fps1"] = ev_fps[s]


torch.cuda.synchronize()
with torch.no_grad():
    issue_fps(0)
    for i in range(K):
        s = i % 2
        sl = gp._slots[s]
        if i + 1 < K:
            issue_fps(i + 1)
        with torch.cuda.stream(main):
            main.wait_event(ev_fps[s])
            if ev_head[s] is not None:
                main.wait_event(ev_head[s])
            marks[i]["sa0"] = ev(main)
            sl.sa.replay()
            ev_sa[s] = ev(main)
            marks[i]["sa1"] = ev_sa[s]
        ts = tail if sl.head is not None else main
        with torch.cuda.stream(ts):
            if sl.head is not None:
                ts.wait_event(ev_sa[s])
            marks[i]["hd0"] = ev(ts)
            if sl.head is not None:
                sl.head.replay()
            out = _clone(sl.out)
            ev_head[s] = ev(ts)
            marks[i]["hd1"] = ev_head[s]
torch.cuda.synchronize()
t0 = marks[0]["sa0"]
print("batch  geo0    fps0    fps1  |  sa0     sa1   |  hd0     hd1   (us from batch 0 sa0)")
for i, m in enumerate(marks):
    r = {k: t0.elapsed_time(e) * 1e3 for k, e in m.items()}
    print("%3d  %7.1f %7.1f %7.1f | %7.1f %7.1f | %7.1f %7.1f   sa %5.1f fps %5.1f head %5.1f" % (
        i, r.get("geo0", 0), r.get("fps0", 0), r.get("fps1", 0), r["sa0"], r["sa1"], r["hd0"],
        r["hd1"], r["sa1"] - r["sa0"], r.get("fps1", 0) - r.get("fps0", 0), r["hd1"] - r["hd0"]))
