"""query_ball_point / SA layers at any sample_number <= N (pointnet2_utils.py:83-89: the
reference sorts each row and slices [:, :, :number], so any number up to N is accepted).

The ball query keeps a row buffer in LDS while 64 rows of K + 1 entries fit in 96 KB (K <= 191
for the public int64 op, K <= 383 for the SA layers' int32 lists); longer rows are written
straight to HBM (ball_query.hip, ROWBUF = false).  Both forms are checked bit-exact against the
oracle, the direct form also at small K through the tuning key bq_rowbuf_kb = 0, and an SA
forward at sample_number 256 / 512 against the oracle's float64 MLP (1e-5 relative)."""
import numpy as np
import pytest
import torch

import cases
import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(got, want, rtol=1e-5):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    atol = rtol * max(float(np.abs(want).max()), 1e-30)
    np.testing.assert_allclose(got, want, rtol=rtol, atol=atol)


@pytest.fixture(scope="module", autouse=True)
def _pn2():
    import pn2  # noqa: F401
    assert torch.cuda.is_available()


def _geometry(kind, B, N, S, seed, C=3):
    p = cases.as_layout(cases.cloud(kind, B, N, seed), "strided")
    start = torch.randint(0, N, (B,), generator=torch.Generator().manual_seed(seed))
    ctr = oracle.index_points(p, oracle.farthest_point_sample(p, S, start))
    d = p.permute(0, 2, 1).contiguous().to(DEV).permute(0, 2, 1)
    return p, d, ctr


@pytest.mark.parametrize("K", [192, 256, 384, 512, 1024])
@pytest.mark.parametrize("radius", [0.3, 0.8, 3.0])
def test_public_query_ball_point_large_k(K, radius):
    """The public int64 op: K from just past the LDS row buffer up to N, balls that hold a few
    points (rows mostly padding), about half the cloud, and all of it (K = N: the row is 0..N-1)."""
    import pn2
    B, N, S = 2, 1024, 96
    p, d, ctr = _geometry("uniform3", B, N, S, 11)
    want = oracle.query_ball_point(radius, K, p, ctr)
    got = pn2.query_ball_point(radius, K, d, torch.from_numpy(ctr).to(DEV))
    assert got.dtype == torch.int64 and got.shape == (B, S, K)
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    if radius == 3.0 and K == N:
        np.testing.assert_array_equal(want[0, 0], np.arange(N))


@pytest.mark.parametrize("K", [192, 256, 384, 512, 2048])
def test_sa_int32_lists_large_k(K):
    """The SA layers' int32 lists with distinct-neighbour counts (pn2_ball_query_i32): LDS rows
    up to K = 383, direct rows past it; a 10-channel pose cloud as well as xyz."""
    from pn2 import ops
    for kind, C, N in (("uniform3", 3, 2048), ("onehot10", 10, 2048)):
        B, S = 2, 80
        p, d, ctr = _geometry(kind, B, N, S, 12 + C)
        idx, newp, cpk, ppk = torch.ops.pn2.fps(d, S, torch.tensor([3, N - 5], device=DEV))
        np.testing.assert_array_equal(newp.cpu().numpy(), oracle.index_points(p, idx.cpu().numpy()))
        ctr = newp.cpu().numpy()
        for radius in (0.25, 1.0):
            want = oracle.query_ball_point(radius, K, p, ctr)
            got, cnt = ops.ball_query_direct(ppk, cpk, C, radius, K, True)
            assert got.dtype == torch.int32
            np.testing.assert_array_equal(got.cpu().numpy(), want.astype(np.int32))
            # the count is the number of distinct hits (capped at K): rows past it repeat the first
            w = want
            distinct = np.minimum(K, 1 + (np.diff(w, axis=-1) > 0).sum(-1))
            np.testing.assert_array_equal(cnt.cpu().numpy(), distinct)


@pytest.mark.parametrize("K", [1, 16, 32, 64, 100, 128])
def test_direct_rows_match_lds_rows(K):
    """Forcing the direct-to-HBM rows at the small K the LDS row buffer normally serves
    (tuning bq_rowbuf_kb = 0) gives the same bits, for both index types."""
    import pn2
    from pn2 import ops, tuning
    B, N, S = 3, 1024, 200
    p, d, ctr = _geometry("dup3", B, N, S, 21)
    dc = torch.from_numpy(ctr).to(DEV)
    idx, newp, cpk, ppk = torch.ops.pn2.fps(d, S, torch.tensor([0, 9, N - 1], device=DEV))
    for radius in (0.05, 0.2, 0.6):
        want = oracle.query_ball_point(radius, K, p, ctr)
        a = pn2.query_ball_point(radius, K, d, dc)
        a32, c32 = ops.ball_query_direct(ppk, cpk, 3, radius, K, True)
        with tuning.override(bq_rowbuf_kb=0):
            b = pn2.query_ball_point(radius, K, d, dc)
            b32, d32 = ops.ball_query_direct(ppk, cpk, 3, radius, K, True)
        np.testing.assert_array_equal(a.cpu().numpy(), want)
        np.testing.assert_array_equal(b.cpu().numpy(), want)
        np.testing.assert_array_equal(b32.cpu().numpy(), a32.cpu().numpy())
        np.testing.assert_array_equal(d32.cpu().numpy(), c32.cpu().numpy())


def test_direct_rows_no_neighbour_pad():
    """A centroid with no point in its ball: the direct rows pad with N as the LDS rows do (the
    reference's out-of-range pad, pointnet2_utils.py:85-89) and raise the device error."""
    import pn2
    pn2.check_device_errors()
    B, N, S, K, r = 2, 1024, 256, 256, 0.01
    pts = cases.cloud("uniform3", B, N, 3) * 1000.0
    ps = pts.permute(0, 2, 1).contiguous().permute(0, 2, 1)
    start = torch.tensor([4, 700])
    ctr = oracle.index_points(ps, oracle.farthest_point_sample(ps, S, start))
    want = oracle.query_ball_point(r, K, ps, ctr)
    assert (want[:, :, 0] == N).sum() > 0
    x = pts.permute(0, 2, 1).contiguous().to(DEV)
    got = pn2.query_ball_point(r, K, x.permute(0, 2, 1), torch.from_numpy(ctr).to(DEV))
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    with pytest.raises(IndexError, match="no point within its radius"):
        pn2.check_device_errors()


def _oracle_layers(convs, bns):
    out = []
    for conv, bn in zip(convs, bns):
        out.append(dict(W=conv.weight.detach().reshape(conv.weight.shape[0], -1).cpu().numpy(),
                        b=conv.bias.detach().cpu().numpy(), gamma=bn.weight.detach().cpu().numpy(),
                        beta=bn.bias.detach().cpu().numpy(), mean=bn.running_mean.cpu().numpy(),
                        var=bn.running_var.cpu().numpy(), eps=bn.eps))
    return out


# (C, D, K, S, N, radius, mlp, msg)
SA_LARGE = [
    (3, 0, 256, 64, 1024, 0.4, [64, 64, 128], False),      # sa1-like, sample_number 256
    (3, 0, 512, 32, 1024, 0.8, [64, 64, 128], False),      # 512: direct int32 rows
    (3, 64, 256, 32, 512, 0.6, [128, 128, 256], False),    # sa2-like with features (pre-pass)
    (3, 13, 256, 32, 1024, 0.5, [32, 32, 64], True),       # MSG row order, unaligned features
    (10, 0, 384, 32, 2048, 0.5, [64, 64, 128], False),     # pose layout, 384
]


@pytest.mark.parametrize("case", range(len(SA_LARGE)))
def test_sa_forward_large_sample_number(case):
    """PointNetSetAbstraction(Msg) with sample_number 256-512 through the fused eval path:
    centroids bit-exact, features within 1e-5 of the oracle's float64 MLP + max."""
    import pn2
    C, D, K, S, N, radius, mlp, msg = SA_LARGE[case]
    B = 2
    pts = cases.cloud("onehot10" if C == 10 else "uniform3", B, N, 700 + case)
    feat = torch.randn(B, N, D, generator=torch.Generator().manual_seed(800 + case)) if D else None
    torch.manual_seed(case)
    if msg:
        sa = pn2.PointNetSetAbstractionMsg(S, [K], [radius], D, [mlp])
        convs, bns = sa.conv_blocks[0], sa.bn_blocks[0]
    else:
        sa = pn2.PointNetSetAbstraction(S, K, radius, C + D, mlp)
        convs, bns = sa.mlp_convs, sa.mlp_bns
    cases.randomize_bn(sa, case)
    sa = sa.to(DEV).eval()
    x = pts.permute(0, 2, 1).contiguous()
    f = feat.permute(0, 2, 1).contiguous() if D else None
    torch.manual_seed(900 + case)
    with torch.no_grad():
        newp, newf = sa(x.to(DEV), None if f is None else f.to(DEV))
    ps = x.permute(0, 2, 1)
    torch.manual_seed(900 + case)
    start = torch.randint(0, N, (B,), dtype=torch.long)
    ctr = oracle.index_points(ps, oracle.farthest_point_sample(ps, S, start))
    np.testing.assert_array_equal(newp.permute(0, 2, 1).cpu().numpy(), ctr)
    idx = oracle.query_ball_point(radius, K, ps, ctr)
    want = oracle.mlp_max(oracle.group(ps, feat, idx, ctr, feature_first=msg), _oracle_layers(convs, bns))
    _close(newf.permute(0, 2, 1).cpu().numpy(), want)
