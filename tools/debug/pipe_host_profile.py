"""Host-side cProfile of one GraphedPipeline.run (SSG B=32 N=1024, K batches): where the issue
loop's host time goes (graph replays, copies, event records, draws)."""
import cProfile
import os
import pstats
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import cases  # noqa: E402
from pn2 import heads as H  # noqa: E402
from pn2.pipeline import GraphedPipeline  # noqa: E402

DEV = torch.device("cuda", 0)
torch.manual_seed(8)
model = H.ClsSSG().eval()
cases.randomize_bn(model, 8)
model = model.to(DEV)
x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
gp = GraphedPipeline(model)
gp.run([x] * 5)
torch.cuda.synchronize()
K = int(os.environ.get("K", "100"))
pr = cProfile.Profile()
pr.enable()
gp.run([x] * K)
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
