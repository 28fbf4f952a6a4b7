"""The next SA layer's FPS as a side job of this layer's MLP launch (pn2_fps_side; the heads'
geometry.fps_ahead): bit-identical to sampling in the next layer's own forward, with the same
CPU generator walk, whether the chain launch takes the job or it runs as its own launch."""
import numpy as np
import pytest
import torch

import cases
import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _plain_forward(model, x):
    """The head's forward without the lookahead: sa1, sa2, sa3 called one after another."""
    from pn2 import heads as H
    B = x.shape[0]
    l1p, l1f = model.sa1(x, None)
    l2p, l2f = model.sa2(l1p, l1f)
    _, l3f = model.sa3(l2p, l2f)
    if isinstance(model, (H.ClsSSG, H.ClsMSG)):
        return model._fc_log_softmax(l3f.reshape(B, 1024))[0], (l1p, l1f, l2p, l2f)
    return model._fc(l3f.reshape(B, 1024)), (l1p, l1f, l2p, l2f)


@pytest.mark.parametrize("head,C,N", [("pointnet2_cls_ssg", 3, 1024), ("pointnet2_cls_msg", 3, 1024),
                                      ("rotation_ssg", 10, 2048), ("rotation_msg", 10, 1024)])
@pytest.mark.parametrize("side", [1, 0])
def test_fps_ahead_matches_plain_forward(head, C, N, side):
    """side = 1: the chain launch runs sa2's FPS; side = 0 (tuning fps_side = 0): the library
    launches it on its own.  Either way every output bit and the generator state equal the
    forward without lookahead."""
    from pn2 import heads as H, tuning
    torch.manual_seed(21)
    model = H.HEADS[head]()
    cases.randomize_bn(model, 21)
    model = model.to(DEV).eval()
    B = 6
    x = cases.cloud("onehot10" if C == 10 else "uniform3", B, N, 22).permute(0, 2, 1).contiguous().to(DEV)
    from pn2 import _lib
    where = []
    hk = model.sa1.register_forward_hook(lambda *a: where.append(_lib.load().pn2_sa_mlp_last_fps_side()))
    with torch.no_grad(), tuning.override(fps_side=side):
        torch.manual_seed(5)
        got = model(x)
    hk.remove()
    # where sa1's MLP call ran sa2's FPS: inside the chain launch (the N = 512 centroid clouds
    # of the SSG heads fit the chain's side-job block) or, with fps_side = 0, as its own launch
    if head in ("pointnet2_cls_ssg", "rotation_ssg"):
        assert where == [1 if side else 0]
    with torch.no_grad(), tuning.override(fps_side=side):
        torch.manual_seed(5)
        got = model(x)
        got = got[0] if isinstance(got, tuple) else got
        rng_got = torch.randint(0, 1 << 30, (3,))
        torch.manual_seed(5)
        want, acts = _plain_forward(model, x)
        rng_want = torch.randint(0, 1 << 30, (3,))
    assert torch.equal(rng_got, rng_want)
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), want.cpu().numpy().view(np.uint32))


def test_fps_side_job_direct():
    """ops.sa_mlp_max_impl(..., fps_side=job) on SSG sa1: the side job's outputs equal fps_direct's
    (and the oracle's indices), the MLP output equals the call without the job; a job the chain
    cannot take (N > 512: its own launch) likewise; a start outside [0, N) raises."""
    import pn2
    from pn2 import ops
    from pn2.pointnet2_utils import _pack_chain
    torch.manual_seed(4)
    sa = pn2.PointNetSetAbstraction(512, 32, 0.2, 3, [64, 64, 128])
    cases.randomize_bn(sa, 4)
    sa = sa.to(DEV).eval()
    B, N = 4, 1024
    pts = cases.cloud("uniform3", B, N, 7).to(DEV)
    with torch.no_grad():
        s0 = torch.randint(0, N, (B,), generator=torch.Generator().manual_seed(1))
        _, newp, cpk, ppk = ops.fps_direct(pts, 512, s0)
        idx, cnt = ops.ball_query_direct(ppk, cpk, 3, 0.2, 32, True)
        wts, als, bes, cins, splits = _pack_chain(sa.mlp_convs, sa.mlp_bns, sa._pack_cache, 0, 3, True)
        ref = torch.empty(B * 512, 128, device=DEV)
        ops.sa_mlp_max_impl(ref, 0, pts, None, newp, idx, wts, als, bes, cins, splits, cnt=cnt)
        for side_pts, S2 in ((newp, 128), (pts, 64)):  # N = 512: chain-borne; N = 1024: own launch
            n2 = side_pts.shape[1]
            st = torch.randint(0, n2, (B,), generator=torch.Generator().manual_seed(n2))
            job, outs = ops.fps_side_job(side_pts, S2, st)
            out = torch.empty_like(ref)
            ops.sa_mlp_max_impl(out, 0, pts, None, newp, idx, wts, als, bes, cins, splits, cnt=cnt, fps_side=job)
            assert pn2._lib.load().pn2_sa_mlp_last_fps_side() == (1 if n2 == 512 else 0)
            want = ops.fps_direct(side_pts, S2, st)
            for a, b in zip(outs, want):
                assert torch.equal(a, b)
            assert torch.equal(out, ref)
            np.testing.assert_array_equal(outs[0][:1].cpu().numpy(),
                                          oracle.farthest_point_sample(side_pts[:1].cpu(), S2, st[:1]))
        job, _ = ops.fps_side_job(newp, 128, torch.tensor([0, 1, 512, 3]))
        with pytest.raises(RuntimeError, match="start"):
            ops.sa_mlp_max_impl(torch.empty_like(ref), 0, pts, None, newp, idx, wts, als, bes, cins, splits,
                                cnt=cnt, fps_side=job)
