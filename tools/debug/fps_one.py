"""One FPS shape, a few launches (for rocprofv3 counter passes):
    python tools/debug/fps_one.py <B> <N> <S> <fps_cull>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import cases  # noqa: E402
import pn2  # noqa: E402,F401
from pn2 import tuning  # noqa: E402

B, N, S, cull = (int(v) for v in sys.argv[1:5])
x = cases.as_layout(cases.cloud("uniform3", B, N, 5), "strided")
xd = x.permute(0, 2, 1).contiguous().cuda().permute(0, 2, 1)
sd = torch.randint(0, N, (B,), generator=torch.Generator().manual_seed(1)).cuda()
with tuning.override(fps_cull=cull):
    for _ in range(3):
        torch.ops.pn2.fps(xd, S, sd)
torch.cuda.synchronize()
