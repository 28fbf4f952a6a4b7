"""Debug dump of the grid ball query's per-workgroup grid (tuning bq_grid_stop = 9)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402,F401
import cases  # noqa: E402
from pn2 import ops, tuning  # noqa: E402

DEV = torch.device("cuda", 0)
B = 32
p = cases.cloud("uniform3", B, 1024, 90).to(DEV)
_, _, c1, p1 = torch.ops.pn2.fps(p, 512, torch.zeros(B, dtype=torch.long, device=DEV))
with tuning.override(bq_grid=2, bq_grid_stop=9):
    _, cnt = ops.ball_query_direct(p1, c1, 3, 0.2, 32, True)
d = cnt.cpu().numpy().reshape(-1)[:64].reshape(4, 16)
for r in d:
    f = r.view(np.float32)
    print("G", r[:3], "nfin", r[3], "lo", f[4:7], "inv", f[7:10], "ssqmax", f[10], "hix", f[11], "h", f[12],
          "cstart", r[13:16])
print("first records", p1[0, :3].cpu().numpy())
