"""Training step (train mode, forward + backward + SGD step) of pointnet2_cls_ssg (MODEL=ssg,
default; B=32 N=1024) or PointNet-v1 pointnet_cls (MODEL=v1, loss + 0.001 x the feature-transform
regulariser as the reference's get_loss): the fused batch-statistics kernels (pn2/train.py) vs
the reference's torch formulation on the same GPU (PN2 kernels for FPS / ball query in both).
Prints ms/step and clouds/s per path."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pointnet-like-pose-estimation_amd"), os.path.join(ROOT, "tests", "golden")]
import cases  # noqa: E402
from pn2 import heads as H, train  # noqa: E402
from pn2.heads_v1 import PointNetCls  # noqa: E402
from pn2.pointnet_utils import feature_transform_reguliarzer  # noqa: E402

MODEL = os.environ.get("MODEL", "ssg")
B, N = int(os.environ.get("B", "32")), 1024
x = cases.cloud("uniform3", B, N, 5).permute(0, 2, 1).contiguous().cuda()
y = (torch.arange(B) % 7).cuda()
res = {}
for path in os.environ.get("PATHS", "fused,torch").split(","):
    torch.manual_seed(0)
    model = (H.ClsSSG() if MODEL == "ssg" else PointNetCls()).cuda().train()
    opt = torch.optim.SGD(model.parameters(), lr=1e-3, momentum=0.9)
    orig = train.eligible
    if path == "torch":
        train.eligible = lambda *a: False
    try:
        def step():
            opt.zero_grad(set_to_none=True)
            logp, aux, _ = model(x)
            loss = torch.nn.functional.nll_loss(logp, y)
            if MODEL != "ssg":
                loss = loss + 0.001 * feature_transform_reguliarzer(aux)
            loss.backward()
            opt.step()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        K = 20
        t0 = time.perf_counter()
        for _ in range(K):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / K * 1e3
    finally:
        train.eligible = orig
    res[path] = ms
    print(json.dumps({"model": MODEL, "path": path, "B": B, "N": N, "ms_per_step": round(ms, 3),
                      "clouds_per_s": round(B / ms * 1e3, 1)}))
if len(res) == 2:
    print(json.dumps({"speedup_fused_over_torch": round(res["torch"] / res["fused"], 2)}))
