"""Ball query per-launch time at SSG's shapes, scan kernel vs grid kernel (tuning bq_grid,
bq_grid_waves): HIP events around 50 back-to-back launches.  python tools/debug/bq_grid_time.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402,F401  (its sys.path setup)
import cases  # noqa: E402
from pn2 import ops, tuning  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    B = 32
    p = cases.cloud("uniform3", B, 1024, 90).to(DEV)
    _, _, c1, p1 = torch.ops.pn2.fps(p, 512, torch.zeros(B, dtype=torch.long, device=DEV))
    x2 = c1[..., :3].contiguous()
    _, _, c2, p2 = torch.ops.pn2.fps(x2, 128, torch.zeros(B, dtype=torch.long, device=DEV))
    shapes = {"sa1 N1024 S512 r0.2 K32": (p1, c1, 0.2, 32), "sa2 N512 S128 r0.4 K64": (p2, c2, 0.4, 64)}
    variants = [("scan", dict(bq_grid=0)), ("grid auto", dict(bq_grid=2)),
                ("grid wv2", dict(bq_grid=2, bq_grid_waves=2)), ("grid wv4", dict(bq_grid=2, bq_grid_waves=4)),
                ("stop1 box", dict(bq_grid=2, bq_grid_stop=1)), ("stop2 scatter", dict(bq_grid=2, bq_grid_stop=2)),
                ("stop3 query", dict(bq_grid=2, bq_grid_stop=3))]
    only = sys.argv[1:]  # variant names to run (default all)
    for name, (pp, cp, r, K) in shapes.items():
        for vn, kw in variants:
            if only and vn not in only:
                continue
            with tuning.override(**kw):
                for _ in range(5):
                    ops.ball_query_direct(pp, cp, 3, r, K, True)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    ops.ball_query_direct(pp, cp, 3, r, K, True)
                e1.record()
                torch.cuda.synchronize()
                print("%-24s %-10s %7.2f us/launch" % (name, vn, e0.elapsed_time(e1) / 50 * 1e3))


if __name__ == "__main__":
    main()
