"""D2D copy rates for the pipeline's input staging (one STRESS batch: 128 x 3 x 16384 fp32 =
25 MB; one SSG batch: 32 x 3 x 1024 = 393 KB): torch copy_ (hipMemcpyAsync D2D, rocclr's blit
kernel) vs a pn2_copy_f32 entry point when a build has one.  r05: copy_ alone 8.0 us per STRESS
batch (6.3 TB/s read + write), a plain float4 copy kernel 31.6 us -- the ~70 us the pipelined
STRESS profile shows per copy is contention beside the chains, not the blit kernel (no change
made)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
from pn2 import _lib  # noqa: E402

L = _lib.load()
dev = torch.device("cuda", 0)
for name, shape in [("stress", (128, 3, 16384)), ("ssg", (32, 3, 1024))]:
    src = torch.randn(shape, device=dev)
    dst = torch.empty(4 * shape[0], *shape[1:], device=dev)
    ways = {"copy_": lambda h: dst[h * shape[0]:(h + 1) * shape[0]].copy_(src, non_blocking=True)}
    if hasattr(L, "pn2_copy_f32"):
        def pn2c(h):
            d = dst[h * shape[0]:(h + 1) * shape[0]]
            assert L.pn2_copy_f32(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                  ctypes.c_int64(src.numel()),
                                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
        ways["pn2_copy_f32"] = pn2c
    for w, f in ways.items():
        for _ in range(3):
            f(0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(40):
            f(i % 4)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 40
        print("%-6s %-13s %8.2f us per batch  %7.1f GB/s (read + write)" % (
            name, w, us, 2 * src.numel() * 4 / us / 1e3))
    assert torch.equal(dst[:shape[0]], src)
