"""Untraced per-stream timeline of GraphedPipeline.run (SSG B=32 N=1024, the bench's launch;
CONFIG=pose: MultiHead(rotation_ssg, translation_ssg) B=8 N=2048 one-hot):
GPU events and host issue times the pipeline records at every stage boundary when
``GraphedPipeline.trace`` is a list.  Prints per-batch times relative to the first batch's
compute start, and host issue times (ms of perf_counter) beside them."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import cases  # noqa: E402
from pn2 import heads as H  # noqa: E402
from pn2.pipeline import GraphedPipeline, MultiHead  # noqa: E402

DEV = torch.device("cuda", 0)
torch.manual_seed(8)
if os.environ.get("CONFIG", "ssg") == "pose":
    model = MultiHead([H.RotationSSG().eval(), H.TranslationSSG().eval()], [1])
    B, N, kind = 8, 2048, "onehot10"
else:
    model = H.ClsSSG().eval()
    B, N, kind = 32, 1024, "uniform3"
cases.randomize_bn(model, 8)
model = model.to(DEV)
x = cases.cloud(kind, B, N, 90).permute(0, 2, 1).contiguous().to(DEV)
gp = GraphedPipeline(model, nslots=int(os.environ.get("SLOTS", "8")),
                     geometry_streams=int(os.environ.get("GEOS", "1")),
                     geometry_batches=int(os.environ.get("GB", "2")),
                     compute_streams=int(os.environ["CS"]) if "CS" in os.environ else None)
ex = [(torch.zeros(B, 3, device=DEV),)] if os.environ.get("CONFIG", "ssg") == "pose" else None
gp.run([x] * 3, None if ex is None else ex * 3)
torch.cuda.synchronize()
K = int(os.environ.get("K", "16"))
gp.trace = []
t_start, t_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
if os.environ.get("FROM_START"):  # a timed run as the bench times it: K batches from idle
    t_start.record()
    import time
    h_start = time.perf_counter()
    gp.run([x] * K, None if ex is None else ex * K)
    t_end.record()
    print("host: geo0 issued %.1f us, sa0 issued %.1f us after run() was called" % (
        (gp.trace[0]["geo0"][1] - h_start) * 1e6, (gp.trace[0]["sa0"][1] - h_start) * 1e6))
    torch.cuda.synchronize()
    tr = gp.trace
    print("whole run %.1f us for %d batches (%.0f clouds/s)" % (
        t_start.elapsed_time(t_end) * 1e3, K, K * B / (t_start.elapsed_time(t_end) * 1e-3)))
    for i, m in enumerate(tr):
        print("%3d " % i + " ".join("%s %7.1f" % (k, t_start.elapsed_time(m[k][0]) * 1e3)
                                    for k in ("geo0", "geo1", "sa0", "sa1", "hd0", "hd1") if k in m))
    sys.exit(0)
gp.run([x] * (K + 1), None if ex is None else ex * (K + 1))
torch.cuda.synchronize()
tr = gp.trace[1:]
names = ("geo0", "geo1", "sa0", "sa1", "hd0", "hd1")
e0, h0 = tr[0]["sa0"]
print("batch " + " ".join("%8s" % n for n in names) + "  | host issue (us, same origin)   geo  sa  head")
for i, m in enumerate(tr):
    g = {k: e0.elapsed_time(m[k][0]) * 1e3 for k in names if k in m}
    h = {k: (m[k][1] - h0) * 1e6 for k in names if k in m}
    print("%3d  " % i + " ".join("%8.1f" % g.get(k, float("nan")) for k in names) + "  | " +
          " ".join("%8.1f" % h.get(k, float("nan")) for k in ("geo0", "sa0", "hd0")) +
          "   %5.1f %5.1f %5.1f" % (g.get("geo1", float("nan")) - g.get("geo0", float("nan")),
                                   g["sa1"] - g["sa0"], g["hd1"] - g["hd0"]))
per = [(e0.elapsed_time(tr[i + 1]["sa0"][0]) - e0.elapsed_time(tr[i]["sa0"][0])) * 1e3
       for i in range(len(tr) - 1)]
print("period sa0->sa0: median %.1f us" % sorted(per)[len(per) // 2])
