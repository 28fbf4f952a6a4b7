"""Run one ball-query shape REPS times (for rocprofv3 counter passes):
    python tools/debug/bq_one.py [shape] [reps]      shape: ssg_sa1 | ssg_sa2 | stress_sa1 | pose_sa1
PN2_BQ_CPW selects the centroids-per-wave variant."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import cases  # noqa: E402
import pn2  # noqa: E402,F401
from pn2 import ops  # noqa: E402

SHAPES = {"ssg_sa1": (32, 1024, 3, 512, 0.2, 32, "uniform3"), "ssg_sa2": (32, 512, 3, 128, 0.4, 64, "uniform3"),
          "stress_sa1": (128, 16384, 3, 512, 0.2, 32, "uniform3"), "pose_sa1": (64, 2048, 10, 512, 0.2, 32, "onehot10")}
name = sys.argv[1] if len(sys.argv) > 1 else "ssg_sa1"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
B, N, C, S, r, K, kind = SHAPES[name]
x = cases.cloud(kind, B, N, 5).cuda()
start = torch.randint(0, N, (B,), generator=torch.Generator().manual_seed(1)).cuda()
_, _, cpk, ppk = ops.fps_direct(x, S, start)
for _ in range(reps):
    ops.ball_query_direct(ppk, cpk, C, r, K, True)
torch.cuda.synchronize()
print("ok", name, reps)
