"""The grid ball query for xyz clouds (ball_query.hip, ball_query_grid_kernel): bit-exact against
the oracle's query_ball_point (pointnet2_utils.py:70-90) with the grid forced (tuning
bq_grid = 2) and off (0), for both index types, on inputs built to break a cell-culling query:
points at exactly the radius on a lattice, un-normalised and offset clouds, flat and collinear
clouds (zero extent on an axis), duplicates, non-finite points and centroids, radii from a tiny
fraction of the cloud to all of it, and K from 1 to past the LDS row budget."""
import numpy as np
import pytest
import torch

import cases
import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _pn2():
    import pn2  # noqa: F401
    assert torch.cuda.is_available()


def _cloud(kind, B, N, seed):
    g = torch.Generator().manual_seed(seed)
    if kind in ("uniform3", "dup3"):
        return cases.cloud(kind, B, N, seed)
    if kind == "far":  # un-normalised, far from the origin
        return torch.rand(B, N, 3, generator=g) * 700.0 + torch.tensor([1e4, -3e3, 250.0])
    if kind == "lattice":  # spacing 0.1: many pairs at exactly the radius, up to rounding
        i = torch.randint(0, 10, (B, N, 3), generator=g).float()
        return i * 0.1 - 0.5
    if kind == "flat":  # z = 0 everywhere
        p = torch.rand(B, N, 3, generator=g) * 2 - 1
        p[..., 2] = 0.0
        return p
    if kind == "line":  # only x varies
        p = torch.zeros(B, N, 3)
        p[..., 0] = torch.rand(B, N, generator=g) * 2 - 1
        return p
    if kind == "nonfinite":
        p = torch.rand(B, N, 3, generator=g) * 2 - 1
        p[0, 5, 1] = float("nan")
        p[0, 17, 0] = float("inf")
        p[-1, N - 1, 2] = -float("inf")
        p[-1, N // 2] = float("nan")
        return p
    raise ValueError(kind)


def _centroids(p, S, seed, nonfinite=False):
    g = torch.Generator().manual_seed(seed)
    B, N, _ = p.shape
    idx = torch.randint(0, N, (B, S), generator=g)
    ctr = oracle.index_points(p, idx.numpy()).copy()
    if nonfinite:
        ctr[0, 0, 0] = np.nan
        ctr[-1, S - 1, 1] = np.inf
    return ctr


def _check(p, ctr, radius, K, both_types=True):
    import pn2
    from pn2 import ops, tuning
    want = oracle.query_ball_point(radius, K, p, ctr)
    d = p.contiguous().to(DEV)
    dc = torch.from_numpy(np.ascontiguousarray(ctr)).to(DEV)
    C = p.shape[2]
    out = {}
    for mode in (2, 0):
        with tuning.override(bq_grid=mode):
            got = pn2.query_ball_point(radius, K, d, dc)
            np.testing.assert_array_equal(got.cpu().numpy(), want, err_msg="bq_grid=%d int64" % mode)
            if both_types:
                ppk, cpk = ops.pack_points_direct(d), ops.pack_points_direct(dc)
                g32, c32 = ops.ball_query_direct(ppk, cpk, C, radius, K, True)
                np.testing.assert_array_equal(g32.cpu().numpy(), want.astype(np.int32),
                                              err_msg="bq_grid=%d int32" % mode)
                out[mode] = c32.cpu().numpy()
    if both_types:
        np.testing.assert_array_equal(out[2], out[0])
    if (want[..., 0] == p.shape[1]).any():  # rows with no neighbour raised the device error
        with pytest.raises(IndexError, match="no point within its radius"):
            pn2.check_device_errors()
    else:
        pn2.check_device_errors()


@pytest.mark.parametrize("kind", ["uniform3", "dup3", "far", "lattice", "flat", "line"])
@pytest.mark.parametrize("N,S", [(1024, 512), (512, 128), (300, 77), (2048, 200)])
def test_grid_matches_oracle(kind, N, S):
    B = 3
    p = _cloud(kind, B, N, 31 + N)
    ctr = _centroids(p, S, 7 + S)
    ext = float((p.max(1)[0] - p.min(1)[0]).max())
    for frac, K in ((0.005, 8), (0.1, 32), (0.2, 64), (0.4, 16), (1.5, 128)):
        radius = 0.1 if kind == "lattice" and frac == 0.1 else frac * ext
        _check(p, ctr, radius, min(K, N))


@pytest.mark.parametrize("K", [1, 2, 31, 32, 33, 64, 100, 191, 192, 256])
def test_grid_k(K):
    """K from 1 past the grid's LDS row budget (the scan kernel takes over there)."""
    p = _cloud("uniform3", 2, 1024, 5)
    ctr = _centroids(p, 300, 6)
    for radius in (0.2, 0.6):
        _check(p, ctr, radius, K)


def test_grid_nonfinite():
    """NaN / inf points are hits for every centroid (!(NaN > r^2)); a NaN or inf centroid hits
    every point whose distance is NaN or within the radius -- both kernels as the oracle."""
    import pn2
    p = _cloud("nonfinite", 2, 1024, 9)
    ctr = _centroids(p, 256, 10, nonfinite=True)
    for radius in (0.1, 0.3):
        want = oracle.query_ball_point(radius, 32, p, ctr)
        assert (want[0, :, 0] == 5).any()  # the NaN point is every row's first hit in cloud 0
        _check(p, ctr, radius, 32)
    pn2.check_device_errors()


def test_grid_no_neighbour_pad():
    """A centroid with no point within its radius: row padded with N and the device error, as
    the scan kernel (a centroid far outside the cloud's box)."""
    import pn2
    pn2.check_device_errors()
    p = _cloud("uniform3", 2, 1024, 3)
    ctr = _centroids(p, 256, 4)
    ctr[1, 7] = [5.0, 5.0, 5.0]
    want = oracle.query_ball_point(0.2, 32, p, ctr)
    assert want[1, 7, 0] == 1024
    for mode in (2, 0):
        from pn2 import tuning
        with tuning.override(bq_grid=mode):
            got = pn2.query_ball_point(0.2, 32, p.to(DEV), torch.from_numpy(ctr).to(DEV))
            np.testing.assert_array_equal(got.cpu().numpy(), want)
            with pytest.raises(IndexError, match="no point within its radius"):
                pn2.check_device_errors()


def test_grid_sa_forward_default():
    """The SA layers take the grid by default at SSG's shapes: the SSG head's ball queries
    (sa1 N = 1024 r 0.2 K 32, sa2 N = 512 r 0.4 K 64) equal the scan kernel's lists."""
    from pn2 import ops, tuning
    p = cases.cloud("uniform3", 4, 1024, 77)
    d = p.to(DEV)
    idx, newp, cpk, ppk = torch.ops.pn2.fps(d, 512, torch.tensor([1, 2, 3, 4], device=DEV))
    a, ca = ops.ball_query_direct(ppk, cpk, 3, 0.2, 32, True)
    with tuning.override(bq_grid=0):
        b, cb = ops.ball_query_direct(ppk, cpk, 3, 0.2, 32, True)
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    np.testing.assert_array_equal(ca.cpu().numpy(), cb.cpu().numpy())
    np.testing.assert_array_equal(a.cpu().numpy().astype(np.int64),
                                  oracle.query_ball_point(0.2, 32, p, newp.cpu().numpy()))
