"""Per-iteration timeline of the culled FPS kernel (a -DPN2_FPS_STAMPS build), cloud 0 of the
STRESS shape: per iteration the slowest wave's phases (s_memtime cycles).
    bash tools/debug/build_var.sh fpsstamps fps.hip -DPN2_FPS_STAMPS
    PN2_TUNING=lib=pointnet-like-pose-estimation_amd/pn2/var/fpsstamps.so python tools/debug/fps_stamps.py [B N S cull]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import cases  # noqa: E402
import pn2  # noqa: E402,F401
from pn2 import _lib, tuning  # noqa: E402

B, N, S, cull = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (128, 16384, 512, 1)))
x = cases.as_layout(cases.cloud("uniform3", B, N, 5), "strided")
xd = x.permute(0, 2, 1).contiguous().cuda().permute(0, 2, 1)
sd = torch.randint(0, N, (B,), generator=torch.Generator().manual_seed(1)).cuda()
with tuning.override(fps_cull=cull):
    torch.ops.pn2.fps(xd, S, sd)
    torch.cuda.synchronize()
    torch.ops.pn2.fps(xd, S, sd)
    torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (128 * 16 * 4))()
_lib.load().pn2_debug_fps_stamps(buf, None) if False else _lib.load().pn2_debug_fps_stamps(buf)
a = np.frombuffer(buf, dtype=np.uint64).reshape(128, 16, 4).astype(np.int64)
nw = int((a[1, :, 0] != 0).sum())
a = a[:, :nw]
print("waves", nw)
for it in list(range(1, 12)) + list(range(60, 64)) + list(range(120, 127)):
    t0 = a[it, :, 0].min()
    d = a[it] - t0
    nxt = a[it + 1, :, 0].min() - t0
    # per wave: test, update, barrier-exit
    print("it %3d  iter %5d | test max %4d | update max %5d med %5d | at barrier exit max %5d" % (
        it, nxt, (a[it, :, 1] - a[it, :, 0]).max(), (a[it, :, 2] - a[it, :, 1]).max(),
        int(np.median(a[it, :, 2] - a[it, :, 1])), d[:, 3].max()))
per = np.diff(a[1:127, :, 0].min(1))
print("median iteration cycles %d" % np.median(per))
upd = (a[1:127, :, 2] - a[1:127, :, 1])
print("update phase: median over (it, wave) %d, median of per-iteration max %d" % (np.median(upd), np.median(upd.max(1))))
print("top-of-loop to pre-barrier (slowest wave) median %d; barrier wait after the last wave arrives median %d" % (
    np.median((a[1:127, :, 2] - a[1:127, :, 0]).max(1)), np.median(a[1:127, :, 3].min(1) - a[1:127, :, 2].max(1))))
