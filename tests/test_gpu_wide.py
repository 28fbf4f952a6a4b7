"""Points with more than 16 channels (16 < C <= 64): the streamed FPS with 256-thread
workgroups, the wide ball query, the generic SA MLP path -- against the reference.

  sa_<case>.npz      eval-mode reference SA layers (PointNetSetAbstraction / ...Msg,
                     pointnet2_utils.py:143-224) on N(0,1) points with C = 20..40 channels
  index_r{24,40,64}_*.npz   FPS / ball query / square_distance goldens (test_gpu_ops.py runs them)
Centroids bit-exact; features within the north star's 1e-5 (test_gpu_sa.assert_feat_close).
The channel-sum orders these need past 16 channels are pinned in oracle/pn2_oracle.c."""
import numpy as np
import pytest
import torch

import cases
import oracle
from conftest import golden_names, load_golden

DEV = "cuda"
SA_WIDE = golden_names("sa_")


def _build(name):
    from pn2 import pointnet2_utils as P
    kind, args, B, N, C, D, wseed, fseed = cases.SA_WIDE_CASES[name]
    ctor = P.PointNetSetAbstraction if kind == "ssg" else P.PointNetSetAbstractionMsg
    torch.manual_seed(wseed)
    mod = ctor(*args)
    cases.randomize_bn(mod, wseed + 1)
    return mod.eval(), fseed


def test_sa_wide_cases_have_goldens():
    assert sorted(SA_WIDE) == sorted(cases.SA_WIDE_CASES)


@pytest.mark.parametrize("name", SA_WIDE)
def test_sa_wide_modules_rebuild_reference_weights(name):
    mod, _ = _build(name)
    assert cases.state_hash(mod) == str(load_golden("sa_%s.npz" % name)["state_hash"])


def test_channel_limit_rejected_without_gpu():
    """C = 65 is past every kernel: PN2_EUNSUPPORTED before any device call."""
    from pn2 import _lib
    L = _lib.load()
    rc = L.pn2_fps_f32(1, 1, 8, 65, 8 * 65, 65, 1, 1, 4, 1, None, None, None, None)
    assert rc == -2 and b"unsupported C=65" in L.pn2_last_error()
    rc = L.pn2_ball_query_f32(1, 1, 1, 8, 4, 65, 0.2, 4, 1, None)
    assert rc == -2 and b"unsupported C=65" in L.pn2_last_error()
    rc = L.pn2_square_distance_f32(1, 1, 1, 4, 8, 65, 1, None)
    assert rc == -2 and b"unsupported C=65" in L.pn2_last_error()
    rc = L.pn2_pack_points_f32(1, 1, 8, 65, 8 * 65, 65, 1, 1, None)
    assert rc == -2 and b"unsupported C=65" in L.pn2_last_error()
    # the wide shapes need no FPS workspace while the distances fit the LDS (256 threads)
    assert L.pn2_fps_workspace_bytes(2, 40000, 24, 512) == 0
    assert L.pn2_fps_workspace_bytes(2, 41000, 24, 512) == 2 * 41000 * 4


@pytest.mark.gpu
@pytest.mark.parametrize("name", SA_WIDE)
def test_sa_wide_matches_reference(name):
    from test_gpu_sa import assert_feat_close
    g = load_golden("sa_%s.npz" % name)
    mod, fseed = _build(name)
    mod = mod.to(DEV)
    pts = torch.from_numpy(g["points"]).to(DEV)
    feat = torch.from_numpy(g["feature"]).to(DEV) if "feature" in g else None
    torch.manual_seed(fseed)
    with torch.no_grad():
        new_points, new_feature = mod(pts, feat)
    np.testing.assert_array_equal(new_points.cpu().numpy().view(np.uint32), g["new_points"].view(np.uint32))
    assert_feat_close(new_feature.cpu().numpy(), g["new_feature"])


@pytest.mark.gpu
def test_sa_wide_bf16_precision_fails_loudly():
    """The split-bf16 kernels hold at most 16 point channels: an explicit bf16 request on wider
    points raises instead of silently running fp32."""
    g = load_golden("sa_ssg_c24.npz")
    mod, _ = _build("ssg_c24")
    mod = mod.to(DEV)
    mod.mlp_precision = "bf16"
    with pytest.raises(ValueError, match="split weight images"):
        with torch.no_grad():
            mod(torch.from_numpy(g["points"]).to(DEV), torch.from_numpy(g["feature"]).to(DEV))


@pytest.mark.gpu
@pytest.mark.parametrize("C,layout", [(17, "strided"), (24, "contig"), (33, "strided"), (40, "contig"),
                                      (64, "strided")])
@pytest.mark.parametrize("N", [1, 5, 48, 333, 1000])
def test_wide_fps_ball_query_square_distance_vs_oracle(C, layout, N):
    """Seeded random clouds against the pinned oracle: FPS indices, both ball-query entry points
    (int64 / int32 + counts, one and three radii), square_distance -- bit-exact."""
    import pn2
    from pn2 import ops
    gen = torch.Generator().manual_seed(7 * C + N)
    B = 2
    p = cases.as_layout(torch.randn(B, N, C, generator=gen), layout)
    S = min(N, 96)
    start = torch.randint(0, N, (B,), generator=gen)
    want = oracle.farthest_point_sample(p, S, start)
    dp = p.permute(0, 2, 1).contiguous().to(DEV).permute(0, 2, 1) if layout == "strided" else p.contiguous().to(DEV)
    idx, newp, cpk, ppk = torch.ops.pn2.fps(dp, S, start.to(DEV))
    np.testing.assert_array_equal(idx.cpu().numpy(), want)
    newp_h = oracle.index_points(p, want)
    np.testing.assert_array_equal(newp.cpu().numpy().view(np.uint32), np.asarray(newp_h).view(np.uint32))
    scale = float(np.sqrt(2.0 * C))
    radii = [0.8 * scale, 1.0 * scale, 1.2 * scale]
    Ks = [min(N, 8), min(N, 32), min(N, 64)]
    for r, K in zip(radii, Ks):
        exp = oracle.query_ball_point(r, K, p, newp_h)
        np.testing.assert_array_equal(torch.ops.pn2.ball_query(ppk, cpk, C, r, K).cpu().numpy(), exp)
        np.testing.assert_array_equal(pn2.query_ball_point(r, K, dp, newp).cpu().numpy(), exp)
    multi = ops.ball_query_multi_direct(ppk, cpk, C, radii, Ks)
    for (i32, cnt), r, K in zip(multi, radii, Ks):
        exp = oracle.query_ball_point(r, K, p, newp_h)
        np.testing.assert_array_equal(i32.cpu().numpy(), exp)
        distinct = [len(set(row.tolist()) - {N}) for row in exp.reshape(-1, K)]
        np.testing.assert_array_equal(cnt.cpu().numpy().reshape(-1), distinct)
    sq = pn2.square_distance(newp, dp).cpu().numpy()
    np.testing.assert_array_equal(sq.view(np.uint32), oracle.square_distance(newp_h, p).view(np.uint32))
