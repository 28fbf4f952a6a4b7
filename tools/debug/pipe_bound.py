"""Which stream bounds GraphedPipeline?  SSG B=32 N=1024 (CONFIG=pose: the pose MultiHead),
K batches through the graphed pipeline, then the same with one stage's replays turned into
no-ops (diagnostic only -- results are garbage):
  full        the real pipeline
  no_geo      fps graphs not replayed (the compute + tail streams alone)
  no_sa       sa graphs not replayed (geometry + tail)
  no_head     head graphs not replayed (geometry + compute)
Prints clouds/s of each."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import cases  # noqa: E402
from pn2 import heads as H  # noqa: E402
from pn2.pipeline import GraphedPipeline, MultiHead  # noqa: E402

DEV = torch.device("cuda", 0)
torch.manual_seed(8)
pose = os.environ.get("CONFIG", "ssg") == "pose"
if pose:
    model = MultiHead([H.RotationSSG().eval(), H.TranslationSSG().eval()], [1])
    B, N, kind = int(os.environ.get("B", "8")), 2048, "onehot10"
else:
    model = H.ClsSSG().eval()
    B, N, kind = 32, 1024, "uniform3"
cases.randomize_bn(model, 8)
model = model.to(DEV)
x = cases.cloud(kind, B, N, 90).permute(0, 2, 1).contiguous().to(DEV)
ex = [(torch.zeros(B, 3, device=DEV),)] if pose else None
gp = GraphedPipeline(model, nslots=int(os.environ.get("SLOTS", "8")),
                     geometry_streams=int(os.environ.get("GEOS", "1")),
                     geometry_batches=int(os.environ.get("GB", "2")),
                     compute_streams=int(os.environ["CS"]) if "CS" in os.environ else None)
K = 100
gp.run([x] * 3, None if ex is None else ex * 3)
torch.cuda.synchronize()


def rate():
    best = 0
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gp.run([x] * K, None if ex is None else ex * K)
        torch.cuda.synchronize()
        best = max(best, B * K / (time.perf_counter() - t0))
    return best


print("full     %.0f clouds/s" % rate())
for stage in ("fps", "sa", "head"):
    # fps graphs belong to the group slots, sa / head graphs to their batch slots
    objs = list(gp._slots) if stage == "fps" else [h for grp in gp._slots for h in grp.halves]
    saved = [getattr(o, stage) for o in objs]
    if saved[0] is None:
        continue

    class Nop:
        def replay(self):
            pass
    for o in objs:
        setattr(o, stage, Nop())
    print("no_%-5s %.0f clouds/s" % (stage, rate()))
    for o, g in zip(objs, saved):
        setattr(o, stage, g)
