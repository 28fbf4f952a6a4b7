"""Per-workgroup timeline of the SA chain kernel (diagnostic build, tools/debug/build_stamps.sh):
PN2_DEBUG_LIB=.../pn2/var/stamps.so python tools/debug/chain_stamps.py
Runs the SSG B=32 N=1024 sa1 and sa2 layers once each (eager, after warm-up) and prints, per
layer: kernel span, workgroups that did work / left early, percentiles of each phase
(setup = entry -> BN staged, layer 0 incl. gather, layer 1, layer 2 + pooling, write-out)
and of the workgroup lifetime, and how many workgroups were live over time."""
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
lib = _lib.load()
fn = lib.pn2_debug_chain_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
NW, NS = 16384, 6


def stamps():
    torch.cuda.synchronize()
    a = np.zeros(NW * NS, np.uint64)
    assert fn(a.ctypes.data, a.size) == 0
    return a.reshape(NW, NS).astype(np.int64)


def report(name, st, grid):
    st = st[:grid]
    s0 = st[:, 0]
    t0 = s0.min()
    us = lambda v: (v - t0) / 100.0  # 100 MHz ticks -> us
    early = st[:, 1] < st[:, 0]  # stamps 1-4 left from an earlier launch: left early
    work = ~early
    print("== %s: %d workgroups, %d did work, %d left early; span %.1f us" % (
        name, grid, work.sum(), early.sum(), us(st[:, 5].max())))
    if work.any():
        w = st[work]
        ph = {"setup": w[:, 1] - w[:, 0], "layer0": w[:, 2] - w[:, 1], "layer1": w[:, 3] - w[:, 2],
              "layer2": w[:, 4] - w[:, 3], "write": w[:, 5] - w[:, 4], "life": w[:, 5] - w[:, 0]}
        for k, v in ph.items():
            p = np.percentile(v / 100.0, [10, 50, 90, 99])
            print("   %-7s p10 %6.2f  p50 %6.2f  p90 %6.2f  p99 %6.2f us" % (k, *p))
    if early.any():
        e = st[early]
        print("   early-exit life p50 %.2f us; first start %.2f, last start %.2f us" % (
            np.percentile((e[:, 5] - e[:, 0]) / 100.0, 50), us(e[:, 0].min()), us(e[:, 0].max())))
    # live workgroups over time (10 bins)
    end = st[:, 5]
    span = end.max() - t0
    for i in range(10):
        t = t0 + span * (i + 0.5) / 10
        print("   t=%6.1f us live %5d (working %5d)" % (
            (t - t0) / 100.0, ((s0 <= t) & (end >= t)).sum(), ((s0 <= t) & (end >= t) & work).sum()))


def main():
    torch.manual_seed(8)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 8)
    model = model.to(DEV)
    x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
    with torch.no_grad():
        for _ in range(3):
            l1p, l1f = model.sa1(x, None)
            l2p, l2f = model.sa2(l1p, l1f)
        torch.cuda.synchronize()
        model.sa1(x, None)
        st1 = stamps()
        report("sa1 (compact, KB0M=1)", st1, 32 * 512 * 32 // 128)
        model.sa2(l1p, l1f)
        st2 = stamps()
        report("sa2 (pre-pass, KB0M=-1)", st2, 32 * 128 * 64 // 128)
        # the compact variant of sa2 (compact: distinct rows only, 8-row units)
        os.environ["PN2_COMPACT"] = "1"
        model.sa2(l1p, l1f)
        model.sa2(l1p, l1f)
        st3 = stamps()
        report("sa2 compact", st3, 32 * 128 * 64 // 128)
        del os.environ["PN2_COMPACT"]


if __name__ == "__main__":
    main()
