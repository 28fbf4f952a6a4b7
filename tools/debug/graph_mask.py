"""Does a HIP graph replayed on a CU-masked stream keep the mask?  One partition per process
(GEO env: geometry CUs): the SA stage of a GraphedPipeline slot (MFMA-bound) timed eagerly and
replayed, on the geometry stream (GEO CUs) and on the compute stream (the rest).  With the mask
honoured the geometry-stream times scale like 1/GEO."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import cases  # noqa: E402
from pn2 import heads as H, geometry  # noqa: E402
from pn2.pipeline import GraphedPipeline, _streams  # noqa: E402

GEO = int(os.environ.get("GEO", "32"))
DEV = torch.device("cuda", 0)
torch.manual_seed(8)
model = H.ClsSSG().eval()
cases.randomize_bn(model, 8)
model = model.to(DEV)
x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
gp = GraphedPipeline(model, geometry_cus=GEO, tail=False)
gp.run([x] * 3)
sl = gp._slots[0]
geo, main, tail = _streams(0, GEO)


def timeit(stream, fn, n=10):
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        fn()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(n):
            fn()
        b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def eager_fwd():
    with geometry.provide(dict(sl.entries)):
        model(sl.x)


with torch.no_grad():
    r = {}
    for name, st in (("geo", geo), ("main", main), ("default", torch.cuda.default_stream())):
        r[name] = (timeit(st, eager_fwd), timeit(st, lambda: sl.sa.replay()),
                   timeit(st, lambda: sl.fps.replay()))
print("GEO=%d  " % GEO + "  ".join("%s: fwd eager %.0f graph %.0f, fps graph %.0f" % ((k,) + v)
                                   for k, v in r.items()))
