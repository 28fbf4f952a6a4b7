"""Small-batch FC layers of the v1 tails (B rows x K -> N): F.linear vs pn2.ops.linear_rows,
GPU time per call from a captured graph of 50 back-to-back calls (host launch cost excluded)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
from pn2 import ops  # noqa: E402


def graph_us(fn, reps=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / (10 * reps) * 1e3, 2)


for B in [int(v) for v in os.environ.get("BS", "8,16,32").split(",")]:
    for K, N in ((1024, 512), (512, 256), (256, 9), (256, 4096)):
        x = torch.randn(B, K, device="cuda")
        W = torch.randn(N, K, device="cuda")
        b = torch.randn(N, device="cuda")
        res = {"linear+relu": graph_us(lambda: torch.nn.functional.linear(x, W, b).relu_()),
               "pn2": graph_us(lambda: ops.linear_rows(x, W, b, True))}
        print(B, K, N, res, flush=True)
