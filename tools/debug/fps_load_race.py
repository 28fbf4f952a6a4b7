"""Plain FPS (fps_direct) and the FPS side job while SA chain kernels run on another stream:
REPS launches each against a quiet reference (PN2_DEBUG_LIB: run against another build)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import cases  # noqa: E402
import varlib  # noqa: E402
if os.environ.get("VARPKG"):
    sys.path.insert(0, os.environ["VARPKG"])
else:
    varlib.setup()
import pn2  # noqa: E402
from pn2 import ops, tuning  # noqa: E402
from pn2.pointnet2_utils import _pack_chain  # noqa: E402

DEV = torch.device("cuda", 0)
REPS = int(os.environ.get("REPS", "30"))
torch.manual_seed(4)
sa = pn2.PointNetSetAbstraction(512, 32, 0.2, 3, [64, 64, 128])
cases.randomize_bn(sa, 4)
sa = sa.to(DEV).eval()
B, N = 32, 1024
pts = cases.cloud("uniform3", B, N, 7).permute(0, 2, 1).contiguous().to(DEV).permute(0, 2, 1)
lo, hi = torch.cuda.Stream.priority_range()
s_hi = torch.cuda.Stream(DEV, priority=min(lo, hi))
s_lo = torch.cuda.Stream(DEV)
with torch.no_grad():
    s0 = torch.randint(0, N, (B,), generator=torch.Generator().manual_seed(1))
    _, newp, cpk, ppk = ops.fps_direct(pts, 512, s0)
    idx, cnt = ops.ball_query_direct(ppk, cpk, 3, 0.2, 32, True)
    wts, als, bes, cins, splits = _pack_chain(sa.mlp_convs, sa.mlp_bns, sa._pack_cache, 0, 3, True)
    out = torch.empty(B * 512, 128, device=DEV)
    st = torch.randint(0, 512, (B,), generator=torch.Generator().manual_seed(9))
    for name, p, S, start in (("sa2 plain", newp, 128, st), ("sa1 plain", pts, 512, s0)):
        ref = ops.fps_direct(p, S, start)
        torch.cuda.synchronize()
        for prio in (1, 0):
            with tuning.override(fps_prio=prio):
                for load in (False, True):
                    bad = 0
                    for rep in range(REPS):
                        if load:
                            with torch.cuda.stream(s_lo):
                                for _ in range(3):
                                    ops.sa_mlp_max_impl(out, 0, pts, None, newp, idx, wts, als, bes, cins,
                                                        splits, cnt=cnt)
                        with torch.cuda.stream(s_hi):
                            got = ops.fps_direct(p, S, start)
                        torch.cuda.synchronize()
                        bad += 0 if all(torch.equal(a, b) for a, b in zip(got, ref)) else 1
                    print("%s, fps_prio %d, chain load %s: %d of %d differ" % (name, prio, load, bad, REPS),
                          flush=True)
    ref = ops.fps_direct(newp, 128, st)
    for prio in (1, 0):
        with tuning.override(fps_prio=prio):
            bad = 0
            for rep in range(REPS):
                job, outs = ops.fps_side_job(newp, 128, st)
                ops.sa_mlp_max_impl(out, 0, pts, None, newp, idx, wts, als, bes, cins, splits, cnt=cnt,
                                    fps_side=job)
                torch.cuda.synchronize()
                bad += 0 if torch.equal(outs[0], ref[0]) else 1
            print("side job (FPS only), fps_prio %d: %d of %d differ" % (prio, bad, REPS), flush=True)
