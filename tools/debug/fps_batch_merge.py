import os, sys, torch
sys.path[:0]=["/root/repo/pointnet-like-pose-estimation_amd","/root/repo/tests/golden"]
import cases
from pn2 import ops
x8 = cases.cloud("onehot10", 8, 2048, 3).cuda()
x16 = torch.cat([x8, x8]).contiguous()
def t(x, reps=20):
    B, N, C = x.shape
    st = torch.randint(0, N, (B,)).cuda()
    for _ in range(3): ops.fps_direct(x, 512, st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(reps): ops.fps_direct(x, 512, st)
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
print("B=8: %.1f us  B=16: %.1f us" % (t(x8), t(x16)))
