"""GPU parity of the index-path ops through the C ABI (torch.ops.pn2.*) -- bit-exact against
the reference's goldens and against the pinned CPU oracle on seeded random inputs."""
import numpy as np
import pytest
import torch

import cases
import oracle
from conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"
INDEX = golden_names("index_")


def _points(g):
    return cases.as_layout(torch.from_numpy(g["points"]), str(g["layout"]))


def _to_dev_view(p):
    """Move a [B,N,C] view to the device keeping its storage layout (strided vs contig)."""
    if p.stride(2) == 1:
        return p.contiguous().to(DEV)
    return p.permute(0, 2, 1).contiguous().to(DEV).permute(0, 2, 1)


@pytest.fixture(scope="module", autouse=True)
def _pn2():
    import pn2  # noqa: F401
    assert torch.cuda.is_available()


@pytest.mark.parametrize("name", INDEX)
def test_fps_matches_reference(name):
    g = load_golden("index_%s.npz" % name)
    pts = _to_dev_view(_points(g))
    idx, newp, cpk, ppk = torch.ops.pn2.fps(pts, int(g["S"]), torch.from_numpy(g["start"]).to(DEV))
    np.testing.assert_array_equal(idx.cpu().numpy(), g["fps_idx"])
    np.testing.assert_array_equal(newp.cpu().numpy().view(np.uint32), g["new_points"].view(np.uint32))


@pytest.mark.parametrize("name", INDEX)
def test_ball_query_matches_reference(name):
    import pn2
    g = load_golden("index_%s.npz" % name)
    pts = _to_dev_view(_points(g))
    newp = torch.from_numpy(g["new_points"]).to(DEV)
    i = 0
    while "bq%d_K" % i in g:
        r, K = float(g["bq%d_radius" % i]), int(g["bq%d_K" % i])
        want = g["bq%d_idx" % i]
        if want.size == 0:
            with pytest.raises(IndexError):
                pn2.query_ball_point(r, K, pts, newp)
        else:
            got = pn2.query_ball_point(r, K, pts, newp)
            assert got.dtype == torch.int64
            np.testing.assert_array_equal(got.cpu().numpy(), want)
        i += 1


@pytest.mark.parametrize("name", INDEX)
def test_fused_fps_packing_feeds_ball_query(name):
    """The packed records emitted by the FPS kernel give the same ball query as packing the
    tensors separately (the SA module's path)."""
    g = load_golden("index_%s.npz" % name)
    pts = _to_dev_view(_points(g))
    N, C = pts.shape[1], pts.shape[2]
    idx, newp, cpk, ppk = torch.ops.pn2.fps(pts, int(g["S"]), torch.from_numpy(g["start"]).to(DEV))
    r, K = float(g["bq0_radius"]), int(g["bq0_K"])
    if K > N:
        pytest.skip("K > N")
    got = torch.ops.pn2.ball_query(ppk, cpk, C, r, K)
    np.testing.assert_array_equal(got.cpu().numpy(), g["bq0_idx"])


@pytest.mark.parametrize("name", [n for n in INDEX if "sqdist" in load_golden("index_%s.npz" % n)])
def test_square_distance_bit_exact(name):
    import pn2
    g = load_golden("index_%s.npz" % name)
    got = pn2.square_distance(torch.from_numpy(g["new_points"]).to(DEV), _to_dev_view(_points(g)))
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), g["sqdist"].view(np.uint32))


@pytest.mark.parametrize("C,layout", [(3, "strided"), (3, "contig"), (6, "contig"), (10, "strided"),
                                      (13, "contig"), (16, "strided")])
@pytest.mark.parametrize("N", [1, 2, 6, 20, 48, 63, 65, 300, 600, 1000, 2049, 4096])
def test_fps_and_ball_query_random_vs_oracle(C, layout, N):
    import pn2
    gen = torch.Generator().manual_seed(1000 * C + N)
    B = 3
    p = torch.randn(B, N, C, generator=gen) * 0.5
    p = cases.as_layout(p, layout)
    S = min(N, 300) if N > 4 else 6   # S may exceed N in the reference; covered by goldens too
    start = torch.randint(0, N, (B,), generator=gen)
    want = oracle.farthest_point_sample(p, S, start)
    dp = _to_dev_view(p)
    idx, newp, cpk, ppk = torch.ops.pn2.fps(dp, S, start.to(DEV))
    np.testing.assert_array_equal(idx.cpu().numpy(), want)
    newp_h = oracle.index_points(p, want)
    for r, K in ((0.3, min(N, 16)), (0.8, min(N, 64))):
        exp = oracle.query_ball_point(r, K, p, newp_h)
        got = torch.ops.pn2.ball_query(ppk, cpk, C, r, K)
        np.testing.assert_array_equal(got.cpu().numpy(), exp)
        got2 = pn2.query_ball_point(r, K, dp, newp)
        np.testing.assert_array_equal(got2.cpu().numpy(), exp)


def test_index_points_and_group_exact():
    import pn2
    gen = torch.Generator().manual_seed(5)
    B, N, C, D, S, K = 2, 200, 3, 7, 16, 8
    pts = torch.randn(B, C, N, generator=gen).permute(0, 2, 1)
    feat = torch.randn(B, D, N, generator=gen).permute(0, 2, 1)
    ctr = torch.randn(B, S, C, generator=gen)
    idx = torch.randint(0, N, (B, S, K), generator=gen)
    dp, dfe = _to_dev_view(pts), _to_dev_view(feat)
    got = pn2.index_points(dp, idx.to(DEV))
    np.testing.assert_array_equal(got.cpu().numpy(), oracle.index_points(pts, idx))
    for ff in (False, True):
        got = torch.ops.pn2.group(dp, dfe, ctr.to(DEV), idx.to(DEV), ff)
        np.testing.assert_array_equal(got.cpu().numpy(), oracle.group(pts, feat, idx, ctr, feature_first=ff))
    got = torch.ops.pn2.group(dp, None, ctr.to(DEV), idx.to(DEV), False)
    np.testing.assert_array_equal(got.cpu().numpy(), oracle.group(pts, None, idx, ctr))


def test_sample_and_group_matches_oracle():
    import pn2
    gen = torch.Generator().manual_seed(9)
    B, N, D = 2, 512, 5
    pts = cases.cloud("uniform3", B, N, 9)
    feat = torch.randn(B, N, D, generator=gen)
    torch.manual_seed(77)
    newp, newf, grouped, fps_idx = pn2.sample_and_group(pts.to(DEV), feat.to(DEV), 64, 16, 0.3, returnfps=True)
    torch.manual_seed(77)
    start = torch.randint(0, N, (B,), dtype=torch.long)
    f = oracle.farthest_point_sample(pts, 64, start)
    np.testing.assert_array_equal(fps_idx.cpu().numpy(), f)
    c = oracle.index_points(pts, f)
    idx = oracle.query_ball_point(0.3, 16, pts, c)
    np.testing.assert_array_equal(newf.cpu().numpy(), oracle.group(pts, feat, idx, c))
    np.testing.assert_array_equal(grouped.cpu().numpy(), oracle.index_points(feat, idx))
    np2, nf2 = pn2.sample_and_group_all(pts.to(DEV), feat.to(DEV))
    assert np2.shape == (B, 1, 3) and float(np2.abs().sum()) == 0.0
    np.testing.assert_array_equal(nf2.cpu().numpy()[:, 0], np.concatenate([pts.numpy(), feat.numpy()], -1))


def test_errors_are_loud():
    import pn2
    from pn2._lib import Pn2Error
    pts = torch.rand(1, 8, 3, device=DEV)
    with pytest.raises(IndexError):
        pn2.query_ball_point(0.2, 9, pts, pts[:, :2])
    with pytest.raises(RuntimeError):
        pn2.farthest_point_sample(torch.rand(1, 8, 3), 4)  # CPU tensor: no CPU path
    with pytest.raises(Pn2Error):
        torch.ops.pn2.fps(torch.rand(1, 8, 65, device=DEV), 4, torch.zeros(1, dtype=torch.long, device=DEV))


def test_fps_stress_size_vs_oracle():
    """STRESS config geometry (N=16384) for two clouds, plus a 2048-point one-hot pose cloud."""
    for kind, B, N, S in (("uniform3", 2, 16384, 512), ("onehot10", 2, 2048, 512)):
        p = cases.as_layout(cases.cloud(kind, B, N, 3), "strided")
        start = torch.tensor([5, N - 1])
        want = oracle.farthest_point_sample(p, S, start)
        idx = torch.ops.pn2.fps(_to_dev_view(p), S, start.to(DEV))[0]
        np.testing.assert_array_equal(idx.cpu().numpy(), want)


@pytest.mark.parametrize("kind,layout,N,S", [
    ("uniform3", "strided", 32768, 512),  # streamed kernel, running distances in LDS
    ("uniform3", "contig", 50000, 256),   # streamed, distances in the caller workspace
    ("onehot10", "strided", 20000, 256),  # 10 channels past the resident cap
    ("random13", "contig", 17000, 128),   # the generic-C kernel
    ("randn10", "contig", 18000, 128),    # 10 varying channels: the channel-sum order
    ("dup3", "strided", 20000, 256),      # many exact duplicates: first-index ties
    ("uniform3", "contig", 9000, 8500),   # npoint past the resident 8192
])
def test_fps_streamed_past_resident_caps(kind, layout, N, S):
    """The shapes past the register-resident kernels (N > 16384, npoint > 8192) run the
    streamed FPS: indices bit-exact vs the oracle (pointnet2_utils.py:47-68), the gathered
    centroids and the packed records feed the same ball query."""
    B = 2
    if kind == "random13":
        p = torch.randn(B, N, 13, generator=torch.Generator().manual_seed(N)) * 0.5
    else:
        p = cases.cloud(kind, B, N, 4)
    p = cases.as_layout(p, layout)
    start = torch.tensor([7, N - 2])
    want = oracle.farthest_point_sample(p, S, start)
    dp = _to_dev_view(p)
    idx, newp, cpk, ppk = torch.ops.pn2.fps(dp, S, start.to(DEV))
    np.testing.assert_array_equal(idx.cpu().numpy(), want)
    ctr = oracle.index_points(p, want)
    np.testing.assert_array_equal(newp.cpu().numpy(), ctr)
    C = p.shape[2]
    exp = oracle.query_ball_point(0.2, 16, p, ctr)
    np.testing.assert_array_equal(torch.ops.pn2.ball_query(ppk, cpk, C, 0.2, 16).cpu().numpy(), exp)


def test_no_neighbour_centroids_flagged_not_read_out_of_bounds():
    """Clouds on a millimetre scale: the -2ab + a^2 + b^2 cancellation puts some centroids'
    distance to themselves above a small r^2, so they have no neighbour.  The reference pads
    their rows with index N (pointnet2_utils.py:85-89) and its index_points then raises
    IndexError.  Here query_ball_point returns the same N-padded rows (bit-exact vs the
    oracle), the SA kernels stay inside the cloud (finite outputs), and
    pn2.check_device_errors() raises the reference's IndexError -- once (the word clears)."""
    import pn2
    pn2.check_device_errors()  # nothing pending from earlier tests
    B, N, S, K, r = 2, 1024, 512, 32, 0.01
    pts = cases.cloud("uniform3", B, N, 3) * 1000.0
    torch.manual_seed(0)
    start = torch.randint(0, N, (B,))
    ps = pts.permute(0, 2, 1).contiguous().permute(0, 2, 1)
    ctr = oracle.index_points(ps, oracle.farthest_point_sample(ps, S, start))
    want = oracle.query_ball_point(r, K, ps, ctr)
    assert (want[:, :, 0] == N).sum() > 0  # the case under test exists
    x = pts.permute(0, 2, 1).contiguous().to(DEV)
    got = pn2.query_ball_point(r, K, x.permute(0, 2, 1), torch.from_numpy(ctr).to(DEV))
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    with pytest.raises(IndexError, match="no point within its radius"):
        pn2.check_device_errors()
    pn2.check_device_errors()  # cleared
    torch.manual_seed(1)
    sa = pn2.PointNetSetAbstraction(S, K, r, 3, [64, 64, 128]).to(DEV).eval()
    with torch.no_grad():
        _, f = sa(x, None)
    assert torch.isfinite(f).all()
    with pytest.raises(IndexError):
        pn2.check_device_errors()


def test_index_points_out_of_range_is_nan_and_flagged():
    """torch's index rule: -N <= n < 0 counts from the end; outside [-N, N) the reference raises
    IndexError -- here the element is NaN and check_device_errors() raises it."""
    import pn2
    pn2.check_device_errors()
    pts = torch.randn(2, 16, 3, device=DEV)
    idx = torch.tensor([[0, -1, 5], [15, -16, 3]], device=DEV)
    got = pn2.index_points(pts, idx)
    b = torch.arange(2, device=DEV)[:, None]
    torch.testing.assert_close(got, pts[b, idx], rtol=0, atol=0)
    pn2.check_device_errors()
    bad = torch.tensor([[0, 16, 1], [-17, 2, 3]], device=DEV)
    got = pn2.index_points(pts, bad)
    assert torch.isnan(got[0, 1]).all() and torch.isnan(got[1, 0]).all()
    assert torch.equal(got[0, 0], pts[0, 0])
    with pytest.raises(IndexError, match="out of range"):
        pn2.check_device_errors()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs")
def test_device_error_goes_to_the_launch_streams_device():
    """a model on cuda:1 launched while cuda:0 is the current device raises its
    device error bits into cuda:1's slot (the slot follows the launch stream's device,
    hipStreamGetDevice), and cuda:0's check stays clean."""
    import pn2
    torch.cuda.set_device(0)
    d1 = torch.device("cuda", 1)
    pn2.check_device_errors("cuda:0")
    pn2.check_device_errors(d1)
    pts = torch.randn(2, 16, 3, device=d1)
    got = pn2.index_points(pts, torch.tensor([[0, 16, 1], [-17, 2, 3]], device=d1))
    assert torch.cuda.current_device() == 0
    assert torch.isnan(got[0, 1]).all() and torch.isnan(got[1, 0]).all()
    pn2.check_device_errors("cuda:0")
    with pytest.raises(IndexError, match="out of range"):
        pn2.check_device_errors(d1)


@pytest.mark.parametrize("mid", [256, 512])
@pytest.mark.parametrize("C,N", [(3, 1024), (3, 512), (3, 300), (10, 1024), (6, 777)])
def test_fps_mid_shapes_exact(mid, C, N):
    """Both automatic FPS blocks for 256 < N <= 1024 (tuning fps_mid: 512 x 2, the eager
    default; 256 x 4, the pipelines' geometry) give the oracle's indices."""
    from pn2 import tuning
    gen = torch.Generator().manual_seed(77 + C + N)
    B, S = 4, min(N, 256)
    p = cases.as_layout(torch.randn(B, N, C, generator=gen), "strided")
    start = torch.randint(0, N, (B,), generator=gen)
    want = oracle.farthest_point_sample(p, S, start)
    with tuning.override(fps_mid=mid):
        idx, newp, cpk, ppk = torch.ops.pn2.fps(_to_dev_view(p), S, start.to(DEV))
    np.testing.assert_array_equal(idx.cpu().numpy(), want)


# pn2_fps_host_ws_f32: the start draw in host memory, carried in the launch's arguments
# (256 clouds per launch): the same bits as the device-start entry point, past the per-launch
# cap (B = 300: two launches), on the streamed kernel, and checked on the host.
@pytest.mark.parametrize("B,N,C,S", [(5, 1024, 3, 512), (300, 64, 3, 16), (3, 20000, 3, 8),
                                     (4, 700, 10, 64), (2, 50000, 3, 4)])
def test_fps_host_start_matches_device_start(B, N, C, S):
    from pn2 import ops
    pts = cases.as_layout(cases.cloud("onehot10" if C == 10 else "uniform3", B, N, 31), "strided")
    pd = _to_dev_view(pts)
    start = torch.randint(0, N, (B,), generator=torch.Generator().manual_seed(B + N))
    a = ops.fps_direct(pd, S, start)          # CPU tensor: host entry point
    b = ops.fps_direct(pd, S, start.to(DEV))  # device entry point
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x.cpu().numpy().view(np.uint32 if x.dtype == torch.float32 else np.int64),
                                      y.cpu().numpy().view(np.uint32 if y.dtype == torch.float32 else np.int64))
    want = oracle.farthest_point_sample(pts[:1], S, start[:1])
    np.testing.assert_array_equal(a[0][:1].cpu().numpy(), want)


def test_fps_host_start_out_of_range_raises():
    from pn2 import ops
    pd = torch.rand(2, 64, 3, device=DEV)
    with pytest.raises(RuntimeError, match="start"):
        ops.fps_direct(pd, 8, torch.tensor([3, 64]))


# pn2_ball_query_multi_i32: an MSG layer's radii in one launch == one pn2_ball_query_i32 per
# radius, bit for bit (lists and counts), on LDS row buffers and direct row writes, C = 3 / 10,
# partial 32-point words, early exit (dense radius) and a radius with no neighbours
@pytest.mark.parametrize("C,N,S,radii,ks,rowbuf", [
    (3, 4096, 512, [0.1, 0.2, 0.4], [16, 32, 128], 96),   # MSG sa1
    (3, 512, 128, [0.2, 0.4, 0.8], [32, 64, 128], 96),    # MSG sa2
    (3, 1000, 100, [0.05, 0.3], [8, 40], 96),             # partial words, two radii
    (10, 2048, 256, [0.1, 0.2, 0.4], [16, 32, 64], 96),   # pose channels
    (3, 4096, 512, [0.1, 0.2, 0.4], [16, 32, 128], 0),    # rows straight to HBM
    (3, 700, 64, [1e-6, 0.3, 2.5], [4, 16, 700], 96),     # no neighbours / whole cloud
])
def test_ball_query_multi_matches_single(C, N, S, radii, ks, rowbuf):
    from pn2 import ops, tuning
    B = 3
    pts = cases.cloud("onehot10" if C == 10 else "uniform3", B, N, 41).to(DEV)
    ctr = pts[:, :S].contiguous()
    ppk, cpk = ops.pack_points_direct(pts), ops.pack_points_direct(ctr)
    with tuning.override(bq_rowbuf_kb=rowbuf):
        multi = ops.ball_query_multi_direct(ppk, cpk, C, radii, ks)
        single = [ops.ball_query_direct(ppk, cpk, C, r, k, True) for r, k in zip(radii, ks)]
    from pn2 import _lib
    _lib.device_errors(DEV)  # (the 1e-6 radius may leave centroids without neighbours: flagged)
    for (a, ca), (b, cb) in zip(multi, single):
        assert torch.equal(a, b) and torch.equal(ca, cb)

