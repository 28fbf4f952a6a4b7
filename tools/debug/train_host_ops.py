"""Host-side cost of one v1 (pointnet_cls B=32) train step on the fused path: torch profiler,
CPU time per op, to see where the eager step's host time goes."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pointnet-like-pose-estimation_amd"), os.path.join(ROOT, "tests", "golden")]
import cases  # noqa: E402
from pn2.heads_v1 import PointNetCls  # noqa: E402
from pn2.pointnet_utils import feature_transform_reguliarzer  # noqa: E402

B = 32
x = cases.cloud("uniform3", B, 1024, 5).permute(0, 2, 1).contiguous().cuda()
y = (torch.arange(B) % 7).cuda()
model = PointNetCls().cuda().train()
opt = torch.optim.SGD(model.parameters(), lr=1e-3, momentum=0.9)


def step():
    opt.zero_grad(set_to_none=True)
    logp, aux, _ = model(x)
    (torch.nn.functional.nll_loss(logp, y) + 0.001 * feature_transform_reguliarzer(aux)).backward()
    opt.step()


for _ in range(5):
    step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU]) as prof:
    for _ in range(5):
        step()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=30))
