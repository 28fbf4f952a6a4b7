"""The culled FPS kernel (fps.hip fps_cull_kernel: spatially sorted ownership, chunks skipped
when a lower bound on their distances proves no running distance can change) against the
oracle (pointnet2_utils.py:47-68) and bit for bit against the index-ordered kernel
(tuning fps_cull = 0): indices, gathered centroids and the packed records the ball query reads.

Clouds that stress the exactness arguments: exact duplicates (first-index ties across lanes,
waves and chunks), every point identical (all distances 0 after the first pick), collinear and
lattice points (degenerate boxes, many equal distances), coordinates of 1e6 (distances past
the 1e10 initial value: chunks skip from the first iteration), and clustered real-scan-like
clouds."""
import numpy as np
import pytest
import torch

import cases
import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (fps_cull shape NT*100 + Q*10 + PPC, N)
SHAPES = [(25612, 512), (25612, 300), (25614, 1024), (25622, 1000), (51212, 1024), (102412, 2048),
          (102422, 4096), (102414, 3000), (102424, 8192), (102442, 8192), (102444, 16384),
          (102444, 9000), (102482, 16384), (25684, 8192), (25684, 5000), (51284, 16384),
          (51362, 16384), (51362, 12000), (51248, 16384)]


def _cloud(kind, B, N, seed):
    g = torch.Generator().manual_seed(seed)
    if kind == "uniform":
        return cases.cloud("uniform3", B, N, seed)
    if kind == "dup":
        return cases.cloud("dup3", B, N, seed)
    if kind == "same":
        return torch.full((B, N, 3), 0.25)
    if kind == "line":
        t = torch.rand(B, N, 1, generator=g)
        return torch.cat([t, 2 * t, torch.zeros_like(t)], 2)
    if kind == "lattice":
        v = torch.randint(0, 6, (B, N, 3), generator=g).float() * 0.25
        return v
    if kind == "huge":
        return cases.cloud("uniform3", B, N, seed) * 1e6
    if kind == "clusters":
        ctr = torch.randn(B, 5, 3, generator=g)
        which = torch.randint(0, 5, (B, N), generator=g)
        return ctr[torch.arange(B)[:, None], which] + 0.02 * torch.randn(B, N, 3, generator=g)
    raise ValueError(kind)


def _run(xd, S, sd, cull):
    from pn2 import tuning
    with tuning.override(fps_cull=cull):
        return [t.cpu() for t in torch.ops.pn2.fps(xd, S, sd)]


@pytest.mark.parametrize("kind", ["uniform", "dup", "same", "line", "lattice", "huge", "clusters"])
@pytest.mark.parametrize("shape,N", SHAPES)
def test_culled_fps_matches_oracle_and_index_ordered(shape, N, kind):
    B = 3
    S = min(512, N)
    x = cases.as_layout(_cloud(kind, B, N, N + len(kind)), "strided" if N % 2 else "contig")
    start = torch.tensor([0, N // 3, N - 1])
    if x.stride(2) == 1:
        xd = x.contiguous().to(DEV)
    else:
        xd = x.permute(0, 2, 1).contiguous().to(DEV).permute(0, 2, 1)
    sd = start.to(DEV)
    got = _run(xd, S, sd, shape)
    ref = _run(xd, S, sd, 0)
    want = oracle.farthest_point_sample(x, S, start)
    np.testing.assert_array_equal(got[0].numpy(), want)
    for a, r in zip(got, ref):
        np.testing.assert_array_equal(a.numpy().view(np.uint8), r.numpy().view(np.uint8))


@pytest.mark.parametrize("N,S", [(1024, 512), (512, 128), (4096, 512), (16384, 512), (257, 256), (2000, 2000)])
def test_culled_fps_default_dispatch(N, S):
    """The default shapes (tuning fps_cull = 1) at the BASELINE geometries, npoint = N included."""
    B = 4
    x = cases.as_layout(cases.cloud("uniform3", B, N, 7 * N), "strided")
    start = torch.randint(0, N, (B,), generator=torch.Generator().manual_seed(N))
    xd = x.permute(0, 2, 1).contiguous().to(DEV).permute(0, 2, 1)
    got = _run(xd, S, start.to(DEV), 1)
    ref = _run(xd, S, start.to(DEV), 0)
    np.testing.assert_array_equal(got[0].numpy(), oracle.farthest_point_sample(x, S, start))
    for a, r in zip(got, ref):
        np.testing.assert_array_equal(a.numpy().view(np.uint8), r.numpy().view(np.uint8))
