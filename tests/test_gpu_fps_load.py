"""FPS beside other kernels: launched on a high-priority stream while SA chain kernels run on
another stream (the pipelines' geometry streams, concurrent heads on threads), and as the side
job inside a chain launch, FPS gives the quiet result every time.  A cross-wave race in the
iteration's key exchange shows only when the chip is shared (round 6: an FPS variant with extra
LDS traffic in its loop chose a wrong centroid in ~1 of 2000 iterations under load and never
alone; tools/debug/fps_load_race.py).  Reference: pointnet2_utils.py:47-68."""
import pytest
import torch

import cases

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_fps_deterministic_beside_chain_launches():
    import pn2
    from pn2 import ops
    from pn2.pointnet2_utils import _pack_chain
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
        for p, S, start in ((newp, 128, st), (pts, 512, s0)):
            ref = ops.fps_direct(p, S, start)
            torch.cuda.synchronize()
            bad = 0
            for _ in range(15):
                s_lo.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s_lo):
                    for _ in range(3):
                        ops.sa_mlp_max_impl(out, 0, pts, None, newp, idx, wts, als, bes, cins, splits, cnt=cnt)
                with torch.cuda.stream(s_hi):
                    got = ops.fps_direct(p, S, start)
                torch.cuda.synchronize()
                bad += 0 if all(torch.equal(a, b) for a, b in zip(got, ref)) else 1
            assert bad == 0, "%d of 15 FPS launches beside the chains differ (S=%d)" % (bad, S)
        # the side job inside sa1's chain launch (its workgroups beside the chain's)
        ref = ops.fps_direct(newp, 128, st)
        bad = 0
        for _ in range(15):
            job, outs = ops.fps_side_job(newp, 128, st)
            ops.sa_mlp_max_impl(out, 0, pts, None, newp, idx, wts, als, bes, cins, splits, cnt=cnt, fps_side=job)
            assert pn2._lib.load().pn2_sa_mlp_last_fps_side() == 1
            torch.cuda.synchronize()
            bad += 0 if all(torch.equal(a, b) for a, b in zip(outs, ref)) else 1
        assert bad == 0, "%d of 15 side jobs differ" % bad
