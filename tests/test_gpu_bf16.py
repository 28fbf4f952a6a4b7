"""bf16 arithmetic of the grouped MLP + max (pn2_sa_mlp_max_bf16; BASELINE config 5 asks for the
large-N stress run with "features/MLP in bf16").  The reference has no bf16 path, so two bars:

  * exact semantics: against oracle.mlp_max_bf16 (inputs and weights rounded to bf16 per layer,
    exact products, float64 sums).  The GPU sums in fp32 and may round a hidden activation to
    the neighbouring bf16 value where its fp32 sum sits on a rounding boundary, so the bar is
    2e-3 relative + 2e-3 of the output's max magnitude.
  * against the reference's fp32 arithmetic (oracle.mlp_max, float64): 3e-2 of the output's max
    magnitude -- bf16 keeps 8 significant bits per operand.

Indices (FPS, ball query) do not depend on the MLP precision and stay bit-exact (checked at
the stress shape in test_stress_bf16_model)."""
import numpy as np
import pytest
import torch

import cases
import oracle
from test_gpu_mlp import CASES, GROUP_ALL, _oracle_layers

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(got, want, rtol):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    np.testing.assert_allclose(got, want, rtol=rtol, atol=rtol * max(float(np.abs(want).max()), 1e-30))


def _grouped_case(case):
    import pn2
    C, D, K, S, N, mlp, msg, chain_ok = CASES[case]
    B, radius = 2, 0.35
    pts = cases.cloud("onehot10" if C == 10 else "uniform3", B, N, 100 + case)
    feat = torch.randn(B, N, D, generator=torch.Generator().manual_seed(200 + case)) if D else None
    torch.manual_seed(case)
    if msg:
        sa = pn2.PointNetSetAbstractionMsg(S, [K], [radius], D, [mlp])
        convs, bns = sa.conv_blocks[0], sa.bn_blocks[0]
    else:
        sa = pn2.PointNetSetAbstraction(S, K, radius, C + D, mlp)
        convs, bns = sa.mlp_convs, sa.mlp_bns
    cases.randomize_bn(sa, case)
    return sa.to(DEV).eval(), convs, bns, pts, feat, (C, D, K, S, N, msg, chain_ok, B, radius)


@pytest.mark.parametrize("case", range(len(CASES)))
def test_sa_mlp_bf16_vs_oracle(case):
    import pn2
    from pn2 import _lib
    sa, convs, bns, pts, feat, (C, D, K, S, N, msg, chain_ok, B, radius) = _grouped_case(case)
    x = pts.permute(0, 2, 1).contiguous()
    f = feat.permute(0, 2, 1).contiguous().to(DEV) if D else None
    torch.manual_seed(1000 + case)
    if not chain_ok:  # no bf16 kernel for this chain: an error, never a silent fp32 run
        with pytest.raises(_lib.Pn2Error):
            with torch.no_grad(), pn2.mlp_precision("bf16"):
                sa(x.to(DEV), f)
        return
    with torch.no_grad(), pn2.mlp_precision("bf16"):
        newp, newf = sa(x.to(DEV), f)
    torch.cuda.synchronize()
    assert _lib.load().pn2_sa_mlp_last_path() == _lib.PATH_BF16
    ps = x.permute(0, 2, 1)
    torch.manual_seed(1000 + case)
    start = torch.randint(0, N, (B,), dtype=torch.long)
    ctr = oracle.index_points(ps, oracle.farthest_point_sample(ps, S, start))
    np.testing.assert_array_equal(newp.permute(0, 2, 1).cpu().numpy(), ctr)
    grouped = oracle.group(ps, feat, oracle.query_ball_point(radius, K, ps, ctr), ctr, feature_first=msg)
    got = newf.permute(0, 2, 1).cpu().numpy()
    layers = _oracle_layers(convs, bns)
    _close(got, oracle.mlp_max_bf16(grouped, layers), 2e-3)
    _close(got, oracle.mlp_max(grouped, layers), 3e-2)


@pytest.mark.parametrize("case", range(len(GROUP_ALL)))
def test_group_all_bf16_vs_oracle(case):
    import pn2
    from pn2 import _lib
    C, D, N, mlp, _ = GROUP_ALL[case]
    B = 3
    pts = cases.cloud("onehot10" if C == 10 else "uniform3", B, N, 400 + case)
    feat = torch.randn(B, N, D, generator=torch.Generator().manual_seed(500 + case)) if D else None
    torch.manual_seed(case)
    sa = pn2.PointNetSetAbstraction(None, None, None, C + D, mlp, True)
    cases.randomize_bn(sa, case)
    sa.mlp_precision = "bf16"  # the per-module switch
    sa = sa.to(DEV).eval()
    x = pts.permute(0, 2, 1).contiguous().to(DEV)
    f = feat.permute(0, 2, 1).contiguous().to(DEV) if D else None
    with torch.no_grad():
        _, newf = sa(x, f)
    torch.cuda.synchronize()
    assert _lib.load().pn2_sa_mlp_last_path() == _lib.PATH_BF16
    rows = pts.numpy() if feat is None else np.concatenate([pts.numpy(), feat.numpy()], -1)
    layers = _oracle_layers(sa.mlp_convs, sa.mlp_bns)
    got = newf.permute(0, 2, 1).cpu().numpy()
    _close(got, oracle.mlp_max_bf16(rows[:, None], layers), 2e-3)
    _close(got, oracle.mlp_max(rows[:, None], layers), 3e-2)


def test_bf16_deterministic():
    import pn2
    sa, *_ , pts, feat, meta = _grouped_case(1)
    x = pts.permute(0, 2, 1).contiguous().to(DEV)
    f = feat.permute(0, 2, 1).contiguous().to(DEV)
    outs = []
    for _ in range(4):
        torch.manual_seed(3)
        with torch.no_grad(), pn2.mlp_precision("bf16"):
            outs.append(sa(x, f)[1].cpu().numpy())
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])


def test_stress_bf16_model():
    """BASELINE config 5 shape (SSG, N=16384) on 2 clouds: sampled centroids bit-identical to the
    fp32 run (the geometry is precision-independent) and to the oracle's FPS; the global feature
    and logits of the bf16 run within the bf16 bar of the fp32 run."""
    import pn2
    from pn2 import heads
    B, N = 2, 16384
    torch.manual_seed(11)
    model = heads.ClsSSG()
    cases.randomize_bn(model, 11)
    model = model.to(DEV).eval()
    x = cases.cloud("uniform3", B, N, 12).permute(0, 2, 1).contiguous().to(DEV)
    res = {}
    for prec in ("fp32", "bf16"):
        torch.manual_seed(5)
        with torch.no_grad(), pn2.mlp_precision(prec):
            l1p, l1f = model.sa1(x, None)
            l2p, l2f = model.sa2(l1p, l1f)
            _, l3f = model.sa3(l2p, l2f)
        res[prec] = [t.cpu().numpy() for t in (l1p, l2p, l3f)]
    np.testing.assert_array_equal(res["bf16"][0], res["fp32"][0])
    np.testing.assert_array_equal(res["bf16"][1], res["fp32"][1])
    torch.manual_seed(5)
    start = torch.randint(0, N, (B,), dtype=torch.long)
    ps = x.cpu().permute(0, 2, 1)
    want = oracle.index_points(ps, oracle.farthest_point_sample(ps, 512, start))
    np.testing.assert_array_equal(res["fp32"][0].transpose(0, 2, 1), want)
    _close(res["bf16"][2], res["fp32"][2], 3e-2)
