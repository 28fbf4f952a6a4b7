"""Per-link cycle breakdown of the FPS serial loop from a diagnostic build:
    bash tools/debug/build_var.sh fpsst fps.hip -DPN2_FPS_STAMPS
    PN2_DEBUG_LIB=pointnet-like-pose-estimation_amd/pn2/var/fpsst.so python tools/debug/fps_stamps.py
Every wave of workgroups 0-3 sums s_memtime deltas per link of the loop (csrc/fps_body.h
PN2_FPS_T; each stamp first waits for the wave's LDS operations, so a link carries the latency
of its own LDS traffic, and the stamps themselves add cycles).  Prints, per shape, the mean over
waves of cycles per iteration for each link, the slowest wave's, and the instrumented launch's
microseconds per iteration."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import varlib  # noqa: E402
if not varlib.setup():
    raise SystemExit("set PN2_DEBUG_LIB to a -DPN2_FPS_STAMPS build (see the docstring)")
import torch  # noqa: E402

import cases  # noqa: E402
import pn2  # noqa: E402,F401
from pn2 import _lib, ops  # noqa: E402

LINKS = ["loop top", "distances + min", "lane + wave max", "owner lane/point", "key atomic",
         "barrier", "key read", "centroid read"]
# (name, B, N, S, waves of the block shape dispatch_fps picks)
SHAPES = [("ssg_sa1", 32, 1024, 512, 8), ("ssg_sa2", 32, 512, 128, 8), ("msg_sa1", 32, 4096, 512, 16)]


def main():
    L = _lib.load()
    fn = L.pn2_debug_fps_stamps
    fn.argtypes = [ctypes.c_void_p]
    out = {}
    for name, B, N, S, nw in SHAPES:
        x = cases.as_layout(cases.cloud("uniform3", B, N, 5), "strided")
        x = x.permute(0, 2, 1).contiguous().cuda().permute(0, 2, 1)
        start = torch.randint(0, N, (B,), generator=torch.Generator().manual_seed(1))
        for _ in range(3):
            ops.fps_direct(x, S, start)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.fps_direct(x, S, start)
        e1.record()
        torch.cuda.synchronize()
        buf = np.zeros(4 * 16 * 8, dtype=np.uint64)
        assert fn(buf.ctypes.data) == 0
        st = buf.reshape(4, 16, 8).astype(np.float64)[:, :nw] / (S - 1)
        mean = st.mean(axis=(0, 1))
        slow = st[np.unravel_index(np.argmax(st.sum(axis=2)), st.shape[:2])]
        us = e0.elapsed_time(e1) * 1e3 / (S - 1)
        row = {"us_per_iter_instrumented": round(us, 3), "cycles_per_iter": round(float(mean.sum()), 1),
               "mean": {k: round(float(v), 1) for k, v in zip(LINKS, mean)},
               "slowest_wave": {k: round(float(v), 1) for k, v in zip(LINKS, slow)}}
        out[name] = row
        print(name, json.dumps(row), flush=True)
    with open(os.path.join(ROOT, "gpurun_out", "fps_stamps.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
