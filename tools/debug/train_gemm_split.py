"""Training forward GEMM Y = X W^T + b at the SSG layer shapes: the library fp32 GEMM (addmm) vs
pn2's split-bf16 dense kernel (rows source, unpooled, PN2_LAYER_NO_RELU, alpha = 1, beta = b),
weights packed per call (they change every step).  HIP-event time per call and the max error of
each against float64."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
from pn2 import _lib, ops  # noqa: E402


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        out = fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3, out


for M, cin, cout in ((524288, 3, 64), (524288, 64, 64), (524288, 64, 128), (262144, 131, 128),
                     (262144, 128, 128), (262144, 128, 256), (4096, 259, 256), (4096, 256, 512),
                     (4096, 512, 1024)):
    torch.manual_seed(0)
    X = torch.randn(M, cin, device="cuda")
    W = torch.randn(cout, cin, 1, 1, device="cuda") / cin ** 0.5
    b = torch.randn(cout, device="cuda")

    def lib():
        return torch.addmm(b, X, W.reshape(cout, cin).t())

    def split():
        wt, al, be = ops.pack_layer_direct(W, b, None, None, None, None, 0.0, 0)
        sp = ops.pack_layer_split_direct(W, 0, True)
        out = torch.empty(M, cout, device="cuda")
        ops.sa_mlp_max_direct(out, _lib.SRC_ROWS, None, None, None, None, [wt], [al], [be], [cin], [sp],
                              "fp32", [_lib.LAYER_NO_RELU], rows=X.view(1, M, cin), pool=False)
        return out
    t_lib, y_lib = timed(lib)
    t_sp, y_sp = timed(split)
    ref = torch.addmm(b.double(), X.double(), W.reshape(cout, cin).t().double())
    sc = float(ref.abs().max())
    print("M=%d %d->%d  lib %.1f us (err %.1e)  split %.1f us (err %.1e)" % (
        M, cin, cout, t_lib, float((y_lib.double() - ref).abs().max()) / sc, t_sp,
        float((y_sp.double() - ref).abs().max()) / sc), flush=True)
