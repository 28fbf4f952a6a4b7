"""Time the heads' FC tail pieces on the GPU (per-launch averages over a loop, HIP events):
fc1 / fc2 / fc3 as pn2_linear_rows_f32 launches and pn2_fc_tail_f32 at several N3 (how much of
the second launch is the last-arriver tail).  python tools/bench_tail.py [B]"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pointnet-like-pose-estimation_amd"))
from pn2 import _lib  # noqa: E402

L = _lib.load()
dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
K, N1, N2 = 1024, 512, 256
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.relu(torch.randn(B, K, generator=g)).to(dev)
W1, b1 = (torch.randn(N1, K, generator=g) / 32).to(dev), torch.randn(N1, generator=g).to(dev)
W2, b2 = (torch.randn(N2, N1, generator=g) / 22).to(dev), torch.randn(N2, generator=g).to(dev)
st = torch.cuda.current_stream().cuda_stream


def timed(fn, n=50, reps=5):
    """Per-launch GPU time: n launches captured in one graph, replayed (no host launch gaps)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        global st
        st = s.cuda_stream
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        gr.capture_begin()
        for _ in range(n):
            fn()
        gr.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (n * reps) * 1e3


def lin(xx, W, b, N, Kk, out, relu=1):
    return lambda: _lib.check(L.pn2_linear_rows_f32(xx.data_ptr(), Kk, B, Kk, W.data_ptr(), b.data_ptr(),
                                                    out.data_ptr(), N, N, relu, ctypes.c_void_p(st)), "lin")


y1 = torch.empty(B, N1, device=dev)
y2 = torch.empty(B, N2, device=dev)
res = {"B": B, "fc1_us": timed(lin(x, W1, b1, N1, K, y1)), "fc2_us": timed(lin(y1, W2, b2, N2, N1, y2))}
for N3 in (1, 4, 40):
    W3, b3 = (torch.randn(N3, N2, generator=g) / 16).to(dev), torch.randn(N3, generator=g).to(dev)
    y3 = torch.empty(B, N3, device=dev)
    res["fc3_%d_us" % N3] = timed(lin(y2, W3, b3, N3, N2, y3, 0))
    ws = torch.empty(int(L.pn2_fc_tail_workspace_bytes(B, N1, N2)) // 4 + 4, device=dev)
    out = torch.empty(B, N3, device=dev)
    am = torch.empty(B, dtype=torch.int64, device=dev)

    def tail():
        _lib.check(L.pn2_fc_tail_f32(x.data_ptr(), K, B, K, W1.data_ptr(), b1.data_ptr(), N1, W2.data_ptr(),
                                     b2.data_ptr(), N2, W3.data_ptr(), b3.data_ptr(), N3, 1, out.data_ptr(), N3,
                                     am.data_ptr(), ws.data_ptr(), ws.numel() * 4, ctypes.c_void_p(st)), "tail")
    res["tail_%d_us" % N3] = timed(tail)
print(json.dumps({k: round(v, 2) if isinstance(v, float) else v for k, v in res.items()}))
