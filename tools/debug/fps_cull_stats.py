"""Culled FPS diagnostics: active-chunk fractions (a -DPN2_FPS_STATS build) and the loop's
fixed cost (a -DPN2_FPS_FLOOR build, wrong indices) per BASELINE geometry.
    bash tools/debug/build_var.sh fpsstats fps.hip -DPN2_FPS_STATS
    bash tools/debug/build_var.sh fpsfloor fps.hip -DPN2_FPS_FLOOR
    PN2_TUNING=lib=pn2/var/fpsstats.so python tools/debug/fps_cull_stats.py stats
    PN2_TUNING=lib=pn2/var/fpsfloor.so python tools/debug/fps_cull_stats.py time"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import cases  # noqa: E402
import pn2  # noqa: E402
from pn2 import _lib, tuning  # noqa: E402

SHAPES = [("ssg_sa1", 32, 1024, 512), ("ssg_sa2", 32, 512, 128), ("msg_sa1", 32, 4096, 512),
          ("stress_sa1", 128, 16384, 512)]
mode = sys.argv[1] if len(sys.argv) > 1 else "stats"
L = _lib.load()
dev = torch.device("cuda")
for name, B, N, S in SHAPES:
    x = cases.as_layout(cases.cloud("uniform3", B, N, 5), "strided")
    xd = x.permute(0, 2, 1).contiguous().to(dev).permute(0, 2, 1)
    sd = torch.randint(0, N, (B,), generator=torch.Generator().manual_seed(1)).to(dev)
    for cull in ([1] if mode == "stats" else [0, 1]):
        with tuning.override(fps_cull=cull):
            torch.ops.pn2.fps(xd, S, sd)
            torch.cuda.synchronize()
            if mode == "stats":
                st = (ctypes.c_ulonglong * 4)()
                L.pn2_debug_fps_stats(st, 1)
                torch.ops.pn2.fps(xd, S, sd)
                L.pn2_debug_fps_stats(st, 1)
                print("%-10s active chunks %.3f  active wave-iterations %.3f" % (
                    name, st[0] / max(st[1], 1), st[2] / max(st[3], 1)), flush=True)
            else:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    torch.ops.pn2.fps(xd, S, sd)
                e1.record()
                torch.cuda.synchronize()
                print("%-10s cull=%d %.3f us/iter" % (name, cull, e0.elapsed_time(e1) * 1e3 / 5 / S), flush=True)
