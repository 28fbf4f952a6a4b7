"""Training step with and without HIP-graph capture (torch.cuda.graph around zero_grad +
forward + backward + SGD step), fused pn2.train path vs torch's formulation: separates GPU time
from host launch overhead.  MODEL=ssg|v1, B (default 32)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "pointnet-like-pose-estimation_amd"), os.path.join(ROOT, "tests", "golden")]
import cases  # noqa: E402
from pn2 import heads as H, train  # noqa: E402
from pn2.heads_v1 import PointNetCls  # noqa: E402
from pn2.pointnet_utils import feature_transform_reguliarzer  # noqa: E402

MODEL = os.environ.get("MODEL", "v1")
B, N = int(os.environ.get("B", "32")), 1024
x = cases.cloud("uniform3", B, N, 5).permute(0, 2, 1).contiguous().cuda()
y = (torch.arange(B) % 7).cuda()
for path in ("fused", "torch"):
    for graphed in (False, True):
        torch.manual_seed(0)
        model = (H.ClsSSG() if MODEL == "ssg" else PointNetCls()).cuda().train()
        opt = torch.optim.SGD(model.parameters(), lr=1e-3, momentum=0.9)
        orig = train.eligible
        if path == "torch":
            train.eligible = lambda *a: False
        try:
            def step():
                opt.zero_grad(set_to_none=False)
                logp, aux, _ = model(x)
                loss = torch.nn.functional.nll_loss(logp, y)
                if MODEL != "ssg":
                    loss = loss + 0.001 * feature_transform_reguliarzer(aux)
                loss.backward()
                opt.step()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(3):
                    step()
            torch.cuda.current_stream().wait_stream(s)
            run = step
            if graphed:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    step()
                run = g.replay
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            K = 30
            t0 = time.perf_counter()
            for _ in range(K):
                run()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / K * 1e3
        except Exception as e:  # capture may refuse a path
            ms = float("nan")
            print("capture failed:", path, repr(e)[:200])
        finally:
            train.eligible = orig
        print(json.dumps({"model": MODEL, "path": path, "graphed": graphed, "B": B,
                          "ms_per_step": round(ms, 3)}))
