"""Per-workgroup timeline of the dense layer kernel (diagnostic build,
tools/debug/build_dense_stamps.sh): PN2_DEBUG_LIB=.../pn2/var/dstamps.so python tools/debug/dense_stamps.py
Runs one eager SSG B=32 N=1024 forward after warm-up; the last dense launch of it is sa3's
512 -> 1024 layer (group_all, pooled over the 128 points of a cloud); SEL selects another launch (below); CONFIG=pose: translation_ssg's
sa2 512 -> 1024 layer at B=64 (GRID=1024 wide tiles, NST=8); B=<n> the SSG batch (B=128: the
pipeline's four-batch group), DENSE_LDS=0 the register-staged kernel the pipeline runs.  Prints the spread of
workgroup start times, percentiles of the prologue (entry -> stage 0 landed), of each stage
(barrier to barrier), of the epilogue, and of the workgroup lifetime."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import cases  # noqa: E402
import varlib  # noqa: E402
varlib.setup()
from pn2 import _lib  # noqa: E402
from pn2 import heads as H  # noqa: E402

DEV = torch.device("cuda", 0)
fn = _lib.load().pn2_debug_dense_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
# SEL=<mode * 1000 + output tiles>: stamp only those launches (SEL=1008: sa3's first layer)
assert _lib.load().pn2_debug_dense_select(int(os.environ.get("SEL", "-1"))) == 0
NW, NS = 4096, 18
torch.manual_seed(8)
pose = os.environ.get("CONFIG", "ssg") == "pose"  # translation_ssg B=64 N=2048: group_all over 32768 rows
model = H.TranslationSSG().eval() if pose else H.ClsSSG().eval()
cases.randomize_bn(model, 8)
model = model.to(DEV)
if pose:
    x = cases.cloud("onehot10", 64, 2048, 90).permute(0, 2, 1).contiguous().to(DEV)
    args = (x, torch.zeros(64, 3, device=DEV))
else:
    args = (cases.cloud("uniform3", int(os.environ.get("B", "32")), 1024, 90).permute(0, 2, 1).contiguous().to(DEV),)
from pn2 import tuning  # noqa: E402
ov = {"dense_lds": int(os.environ["DENSE_LDS"])} if "DENSE_LDS" in os.environ else {}
with torch.no_grad(), tuning.override(**ov):
    for _ in range(5):
        model(*args)
    torch.cuda.synchronize()
    model(*args)
torch.cuda.synchronize()
a = np.zeros(NW * NS, np.uint64)
assert fn(a.ctypes.data, a.size) == 0
st = a.reshape(NW, NS).astype(np.int64)
grid = int(os.environ.get("GRID", "512"))
st = st[:grid]
t0 = st[:, 0].min()
us = lambda v: v / 100.0
nst = int(os.environ.get("NST", "8"))
print("workgroups %d; entry spread p10/p50/p90/max %.2f %.2f %.2f %.2f us; span %.1f us" % (
    grid, *np.percentile(us(st[:, 0] - t0), [10, 50, 90, 100]), us(st[:, 15].max() - t0)))
clk = (st[:, 17] - st[:, 16]) / np.maximum(1, st[:, 15] - st[:, 0]) * 100.0  # MHz
print("in-kernel clock p10/p50/p90 %.0f %.0f %.0f MHz" % tuple(np.percentile(clk, [10, 50, 90])))
rows = [("prologue", st[:, 1] - st[:, 0])]
for c in range(1, nst):
    rows.append(("stage %d" % (c - 1), st[:, 1 + c] - st[:, c]))
rows.append(("stage %d+loop" % (nst - 1), st[:, 14] - st[:, nst]))
rows.append(("epilogue", st[:, 15] - st[:, 14]))
rows.append(("life", st[:, 15] - st[:, 0]))
for name, v in rows:
    print("   %-14s p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us" % (name, *np.percentile(us(v), [10, 50, 90, 100])))
for i in range(10):
    t = t0 + (st[:, 15].max() - t0) * (i + 0.5) / 10
    print("   t=%6.1f us live %4d" % (us(t - t0), int(((st[:, 0] <= t) & (st[:, 15] > t)).sum())))
