"""Per-workgroup entry / exit times of the FPS launches inside the pipelined SSG run (diagnostic
build with -DPN2_FPS_WGSTAMPS, load with PN2_DEBUG_LIB=...):
    python tools/debug/fps_wg.py [K]
Every geometry group launches FPS sa1 then FPS sa2, 64 workgroups each (2 batches x 32 clouds).
Prints per launch the spread of the workgroups' start times (how long the launch waited for
room on the CUs) and their lifetimes, then the same for an idle-chip run."""
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
from pn2.pipeline import GraphedPipeline  # noqa: E402

DEV = torch.device("cuda", 0)
L = _lib.load()
fn = L.pn2_debug_fps_wg
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]


def read():
    a = np.zeros(65536 * 2, np.uint64)
    c = np.zeros(1, np.uint32)
    assert fn(a.ctypes.data, c.ctypes.data) == 0
    return a.reshape(65536, 2).astype(np.int64), int(c[0])


def report(tag, st, lo, hi, per=64):
    rows = []
    for l0 in range(lo, hi - per + 1, per):
        s = st[l0 % 65536:l0 % 65536 + per]
        starts, life = s[:, 0], s[:, 1] - s[:, 0]
        rows.append(((starts.max() - starts.min()) / 100.0, np.median(life) / 100.0, life.max() / 100.0))
    r = np.array(rows)
    print("%s: %d launches; start spread p50 %.1f p90 %.1f max %.1f us; WG life p50 %.1f max %.1f us" % (
        tag, len(r), np.percentile(r[:, 0], 50), np.percentile(r[:, 0], 90), r[:, 0].max(),
        np.median(r[:, 1]), r[:, 2].max()))
    for k in range(0, len(r), 2):
        print("   launch %2d (sa1) spread %6.1f life p50 %6.1f | sa2 spread %6.1f life p50 %6.1f" % (
            k // 2, r[k, 0], r[k, 1], r[k + 1, 0] if k + 1 < len(r) else -1, r[k + 1, 1] if k + 1 < len(r) else -1))


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    torch.manual_seed(8)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 8)
    model = model.to(DEV)
    x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
    gp = GraphedPipeline(model)
    gp.run([x] * 5)
    torch.cuda.synchronize()
    _, c0 = read()
    gp.run([x] * K)
    torch.cuda.synchronize()
    st, c1 = read()
    report("pipelined K=%d" % K, st, c0, c1)
    # the same geometry graph alone on an idle chip
    g = gp._slots[0]
    _, c2 = read()
    for _ in range(4):
        g.fps.replay()
        torch.cuda.synchronize()
    st, c3 = read()
    report("geometry graph alone", st, c2, c3)


if __name__ == "__main__":
    main()
