"""Can sa1's ball query + chain run beside its FPS without slowing the FPS?  (SSG B=32 N=1024)

Times (HIP events, median of REPS):
  fps_alone            sa1's FPS launch by itself
  chain_alone          sa1's ball query + compact scan + chain (geometry precomputed)
  fps_shared / chain   FPS on a high-priority stream, 3 chain passes on another, both on every CU
  fps_masked / chain   FPS on a stream masked to GEO CUs (GEO/8 per XCD), chains on the others
  chain_masked_alone   the chain passes alone on the complement mask
    python tools/micro/overlap_probe.py   [GEO=32 REPS=10]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import cases  # noqa: E402
from pn2 import _lib, heads, ops, pipeline  # noqa: E402
from pn2.pointnet2_utils import _pack_chain  # noqa: E402

DEV = torch.device("cuda", 0)
GEO = int(os.environ.get("GEO", "32"))
REPS = int(os.environ.get("REPS", "10"))
PASSES = int(os.environ.get("PASSES", "3"))

torch.manual_seed(8)
model = heads.ClsSSG().eval()
cases.randomize_bn(model, 8)
model = model.to(DEV)
x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
pts = x.permute(0, 2, 1)
sa1 = model.sa1
B, N, C = pts.shape
S, K = sa1.point_number, sa1.sample_number
start = torch.randint(0, N, (B,))
wts, als, bes, cins, splits = _pack_chain(sa1.mlp_convs, sa1.mlp_bns, sa1._pack_cache, 0, C, True)
_, newp, cpk, ppk = ops.fps_direct(pts, S, start)
out = torch.empty(B * S, wts[-1].shape[1], device=DEV)
torch.cuda.synchronize()


def fps():
    ops.fps_direct(pts, S, start)


def chain():
    for _ in range(PASSES):
        idx, cnt = ops.ball_query_direct(ppk, cpk, C, sa1.radius, K, True)
        ops.sa_mlp_max_impl(out, _lib.SRC_GROUP_XYZ_FIRST, pts, None, newp, idx, wts, als, bes,
                            cins, splits, "fp32", cnt=cnt)


def timed(pairs):
    """pairs: [(stream, fn)] launched back to back; -> ms per stream (first launch to its end)."""
    res = [[] for _ in pairs]
    for _ in range(REPS):
        torch.cuda.synchronize()
        evs = []
        for st, fn in pairs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                e0.record(st)
                fn()
                e1.record(st)
            evs.append((e0, e1))
        torch.cuda.synchronize()
        for i, (e0, e1) in enumerate(evs):
            res[i].append(e0.elapsed_time(e1) * 1e3)
    return [sorted(r)[len(r) // 2] for r in res]


lo, hi = torch.cuda.Stream.priority_range()
s_hi = torch.cuda.Stream(DEV, priority=min(lo, hi))
s_lo = torch.cuda.Stream(DEV)
ncu = pipeline._cu_count(0)
g_st, _ = pipeline._masked_stream(0, list(range(GEO)), ncu)
c_st, _ = pipeline._masked_stream(0, list(range(GEO, ncu)), ncu)
for _ in range(3):
    timed([(s_hi, fps), (s_lo, chain)])
print("cus %d geo %d passes %d" % (ncu, GEO, PASSES))
print("fps_alone %.1f us" % timed([(s_hi, fps)])[0])
print("chain_alone %.1f us" % timed([(s_lo, chain)])[0])
print("fps_masked_alone %.1f us" % timed([(g_st, fps)])[0])
print("chain_masked_alone %.1f us" % timed([(c_st, chain)])[0])
f, c = timed([(s_hi, fps), (s_lo, chain)])
print("shared: fps %.1f us, chain %.1f us" % (f, c))
f, c = timed([(g_st, fps), (c_st, chain)])
print("masked: fps %.1f us, chain %.1f us" % (f, c))
f, c = timed([(g_st, fps), (s_lo, chain)])
print("fps masked, chain unmasked: fps %.1f us, chain %.1f us" % (f, c))
