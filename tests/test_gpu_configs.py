"""The BASELINE configs at their real batch sizes against the oracle.

Kernel choices depend on the batch (dense tile widths via dense_minwg, 256 x 128 tiles at >= 512
workgroups, the XCD remap when the workgroup count is a multiple of 8, the compact pool modes,
FPS over a geometry group of 4 batches in the fused pipeline), so the reduced-batch goldens do not
cover the configs' own launches.  Here each config runs at its batch:

  msg     pointnet2_cls_msg  B=32  N=4096     (pointnet2_cls_msg.py:22-38)
  pose    rotation_ssg + translation_ssg  B=64  N=2048, 10 channels  (rotation_ssg.py:24-38,
          translation_ssg.py:28-44)
  stress  pointnet2_cls_ssg  B=128 N=16384, MLP in bf16

and every SA layer is checked on the inputs it received (forward hooks): its centroids bit-exact
for every cloud against the oracle's FPS (pointnet2_utils.py:47-68), its neighbour lists through
the oracle's ball query (pointnet2_utils.py:70-90), and its features against the oracle's
float64 MLP + max (pointnet2_utils.py:163-172, 211-221): fp32 within 1e-5 relative + 1e-5 of the
output's max magnitude; bf16 against the oracle's bf16 emulation within 2e-3 (test_gpu_bf16.py's
bar).  Features are checked for every cloud where the float64 MLP takes seconds (msg, pose) and
for 33 clouds spread over the batch at stress (every 4th and the last; the oracle's bf16
emulation of all 128 takes minutes) -- there every cloud's features are also checked against a
torch restatement of the bf16 arithmetic on the GPU (same bar); indices for every cloud everywhere.  The same batch through pn2.pipeline.GraphedPipeline
(one batch per launch, and four batches fused per launch; graphs on their streams) must give the
eager outputs bit for bit, and so must POSE's per-rank shape (global B=64 over 8 ranks: B=8, with
the batch_shard draws) through both launches, shard by shard.
"""
import itertools

import numpy as np
import pytest
import torch

import cases
import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"

# name: (heads, B, N, cloud kind, precision, clouds whose features are checked (None: all))
CONFIGS = {
    "msg": (["pointnet2_cls_msg"], 32, 4096, "uniform3", "fp32", None),
    "pose": (["rotation_ssg", "translation_ssg"], 64, 2048, "onehot10", "fp32", None),
    "stress": (["pointnet2_cls_ssg"], 128, 16384, "uniform3", "bf16", tuple(range(0, 128, 4)) + (127,)),
}


def _close(got, want, rtol, what):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    atol = rtol * max(float(np.abs(want).max()), 1e-30)
    np.testing.assert_allclose(got, want, rtol=rtol, atol=atol, err_msg=what)


def _layers(convs, bns):
    return [dict(W=c.weight.detach().reshape(c.weight.shape[0], -1).cpu().numpy(),
                 b=c.bias.detach().cpu().numpy(), gamma=n.weight.detach().cpu().numpy(),
                 beta=n.bias.detach().cpu().numpy(), mean=n.running_mean.cpu().numpy(),
                 var=n.running_var.cpu().numpy(), eps=n.eps) for c, n in zip(convs, bns)]


def _build(cfg):
    from pn2 import heads as H
    names, B, N, kind, prec, check = CONFIGS[cfg]
    models = []
    for i, n in enumerate(names):
        models.append(cases.build_head(H.HEADS[n], 1300 + i).to(DEV))
    x = cases.cloud(kind, B, N, 1400).permute(0, 2, 1).contiguous()
    mean = torch.randn(B, 3, generator=torch.Generator().manual_seed(1401))
    return names, models, x, mean, prec, (range(B) if check is None else check)


def _forward(names, models, x, mean, prec):
    import pn2
    outs = []
    with torch.no_grad(), pn2.mlp_precision(prec):
        for n, m in zip(names, models):
            outs.append(m(x, mean) if n.startswith("translation") else m(x))
    return outs


def _record(models):
    """Forward hooks on every SA layer: (module, points in, feature in, points out, feature out)
    as host tensors, first call only."""
    from pn2.pointnet2_utils import PointNetSetAbstraction, PointNetSetAbstractionMsg
    rec, hs = [], []
    seen = set()
    for m in models:
        for mod in m.modules():
            if isinstance(mod, (PointNetSetAbstraction, PointNetSetAbstractionMsg)):
                def hook(mod, inp, out):
                    if id(mod) in seen:
                        return
                    seen.add(id(mod))
                    rec.append((mod, inp[0].cpu(), None if inp[1] is None else inp[1].cpu(),
                                out[0].cpu(), out[1].cpu()))
                hs.append(mod.register_forward_hook(hook))
    return rec, hs


def _draws(names, models, B, N):
    """The FPS start draws one eager pass over the heads takes, in call order."""
    draws = []
    for m in models:
        n = N
        for tag in ("sa1", "sa2", "sa3"):
            sa = getattr(m, tag, None)
            if sa is None or getattr(sa, "group_all", False):
                break
            draws.append(torch.randint(0, n, (B,), dtype=torch.long))
            n = sa.point_number
    return draws


def _mlp(grouped, layers, prec):
    return (oracle.mlp_max_bf16 if prec == "bf16" else oracle.mlp_max)(grouped, layers)


def _torch_mlp_max_bf16(grouped, layers):
    """The bf16 MLP + max restated in torch on the GPU (every clouds' check at STRESS, where the
    oracle's emulation takes minutes): each layer's input and weight rounded to bf16, products
    and sums in fp32 (exact products; only the fp32 summation order differs from the kernels'),
    conv bias + eval BN folded as the kernels fold them, ReLU, max over the K rows.
    grouped [B, S, K, Cin] float32 (device) -> [B, S, Cout] float64 (host)."""
    x = grouped
    for L in layers:
        W = torch.from_numpy(L["W"]).to(x.device)
        alpha = torch.from_numpy(L["gamma"] / np.sqrt(L["var"].astype(np.float64) + L["eps"])).float()
        beta = (alpha.double() * (torch.from_numpy(L["b"]).double() - torch.from_numpy(L["mean"]).double())
                + torch.from_numpy(L["beta"]).double()).float()
        y = x.to(torch.bfloat16).float() @ W.to(torch.bfloat16).float().t()
        x = torch.relu(y * alpha.to(x.device) + beta.to(x.device))
    return x.max(dim=2)[0].double().cpu().numpy()


def _check_layer(mod, p_in, f_in, p_out, f_out, start, check, prec, what):
    from pn2.pointnet2_utils import PointNetSetAbstractionMsg
    pts = p_in.permute(0, 2, 1).numpy()            # [B, N, C] with the module's strides
    feat = None if f_in is None else f_in.permute(0, 2, 1).contiguous().numpy()
    got = f_out.permute(0, 2, 1).numpy()           # [B, S, Cout]
    rtol = 2e-3 if prec == "bf16" else 1e-5
    check = list(check)
    full = prec == "bf16" and len(check) < pts.shape[0]  # every cloud through the torch restatement
    if getattr(mod, "group_all", False):
        rows = pts if feat is None else np.concatenate([pts, feat], -1)
        layers = _layers(mod.mlp_convs, mod.mlp_bns)
        for c0 in range(0, len(check), 8):
            cl = check[c0:c0 + 8]
            want = _mlp(rows[cl][:, None], layers, prec)
            _close(got[cl], want, rtol, what + " group_all features")
        if full:
            want = _torch_mlp_max_bf16(torch.from_numpy(np.ascontiguousarray(rows)).to(DEV)[:, None], layers)
            _close(got, want, rtol, what + " group_all features, every cloud (torch bf16)")
        assert float(np.abs(p_out.numpy()).max()) == 0.0
        return
    S = mod.point_number
    fi = oracle.farthest_point_sample(pts, S, start.numpy())
    ctr = oracle.index_points(pts, fi)
    np.testing.assert_array_equal(p_out.permute(0, 2, 1).numpy().view(np.uint32), ctr.view(np.uint32),
                                  err_msg=what + " centroids")
    if isinstance(mod, PointNetSetAbstractionMsg):
        scales = [(r, k, mod.conv_blocks[i], mod.bn_blocks[i], True)
                  for i, (r, k) in enumerate(zip(mod.radius_list, mod.sample_number_list))]
    else:
        scales = [(mod.radius, mod.sample_number, mod.mlp_convs, mod.mlp_bns, False)]
    col = 0
    for r, K, convs, bns, ff in scales:
        idx = oracle.query_ball_point(r, K, pts, ctr)
        layers = _layers(convs, bns)
        cout = layers[-1]["W"].shape[0]
        step = max(1, 2 ** 21 // (S * K))  # clouds per float64 chunk (~2M grouped rows)
        for c0 in range(0, len(check), step):
            cl = check[c0:c0 + step]
            grouped = oracle.group(pts[cl], None if feat is None else feat[cl], idx[cl], ctr[cl],
                                   feature_first=ff)
            _close(got[cl, :, col:col + cout], _mlp(grouped, layers, prec), rtol,
                   "%s r=%g K=%d features, clouds %s" % (what, r, K, cl[:3]))
        if full:
            for c0 in range(0, pts.shape[0], 32):
                cl = list(range(c0, min(c0 + 32, pts.shape[0])))
                grouped = oracle.group(pts[cl], None if feat is None else feat[cl], idx[cl], ctr[cl],
                                       feature_first=ff)
                want = _torch_mlp_max_bf16(torch.from_numpy(np.ascontiguousarray(grouped, np.float32)).to(DEV),
                                           layers)
                _close(got[cl, :, col:col + cout], want, rtol,
                       "%s r=%g K=%d features, clouds %d.. (torch bf16)" % (what, r, K, c0))
        col += cout
    assert col == got.shape[2]


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_config_full_batch_vs_oracle(cfg):
    names, models, x, mean, prec, check = _build(cfg)
    B, N = x.shape[0], x.shape[2]
    torch.manual_seed(55)
    draws = _draws(names, models, B, N)
    rec, hs = _record(models)
    torch.manual_seed(55)
    _forward(names, models, x.to(DEV), mean.to(DEV), prec)
    torch.cuda.synchronize()
    for h in hs:
        h.remove()
    # every SA layer in call order; the non-group_all layers consumed the draws in that order
    d = iter(draws)
    for j, (mod, p_in, f_in, p_out, f_out) in enumerate(rec):
        start = None if getattr(mod, "group_all", False) else next(d)
        _check_layer(mod, p_in, f_in, p_out, f_out, start, check, prec, "%s layer %d" % (cfg, j))
    assert next(d, None) is None


@pytest.mark.parametrize("gb,fuse", [(1, False), (4, True)])
@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_config_full_batch_pipeline_equals_eager(cfg, gb, fuse, monkeypatch):
    """GraphedPipeline -- the bench's headline launch (one batch per launch, 2 compute streams,
    the heads on the tail stream) and its value_fused launch (4 consecutive batches fused into
    every launch) -- over 4 batches with the eager pass's start draws: every batch's outputs
    equal the eager outputs bit for bit."""
    import pn2
    from pn2 import shard
    from pn2.pipeline import GraphedPipeline, MultiHead
    names, models, x, mean, prec, _ = _build(cfg)
    B, N = x.shape[0], x.shape[2]
    torch.manual_seed(56)
    draws = _draws(names, models, B, N)
    cyc = itertools.cycle(draws)

    def fixed_draw(B_, N_, pin=True):
        t = next(cyc)
        assert t.shape[0] == B_ and int(t.max()) < N_
        return t.clone()

    monkeypatch.setattr(shard, "draw_start", fixed_draw)
    # the pipeline writes its draws in place (shard.draw_start_into): the same cycle
    monkeypatch.setattr(shard, "draw_start_into", lambda dst, N: dst.copy_(fixed_draw(dst.shape[0], N)))
    xd, md = x.to(DEV), mean.to(DEV)
    eager = _forward(names, models, xd, md, prec)
    model = models[0] if len(models) == 1 else MultiHead(
        models, [i for i, n in enumerate(names) if n.startswith("translation")])
    takes_mean = any(n.startswith("translation") for n in names)
    n = 4
    with torch.no_grad(), pn2.mlp_precision(prec):
        # the bench's launches: one batch per launch with four geometry streams and the ball
        # queries in each batch's forward; four fused batches with r05's geometry streams
        gp = GraphedPipeline(model, geometry_streams=4 if gb == 1 else 2 if cfg == "stress" else 1,
                             geometry_batches=gb, fuse=fuse, nslots=max(16, 4 * gb),
                             geometry_bq=False if gb == 1 else None,
                             tail_streams=2 if gb == 1 else None)
        outs = gp.run([xd] * n, [(md,)] * n if takes_mean else None)
    torch.cuda.synchronize()
    want = eager[0] if len(models) == 1 else tuple(eager)
    flat_w = [t for t in _flat(want)]
    for i, o in enumerate(outs):
        flat_o = _flat(o)
        assert len(flat_o) == len(flat_w)
        for a, b in zip(flat_o, flat_w):
            np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy(), err_msg="%s batch %d" % (cfg, i))


def _flat(o):
    if isinstance(o, torch.Tensor):
        return [o]
    return [t for x in o for t in _flat(x)]


@pytest.mark.parametrize("gb,fuse", [(1, False), (4, True)])
def test_pose_rank_shards_pipeline_equals_unsharded(gb, fuse, monkeypatch):
    """BASELINE config 4 at the shape each of 8 ranks runs (rotation_ssg.py:24-38,
    translation_ssg.py:28-44): global B=64 sharded 8 ways is B=8 per rank, and each rank's
    GraphedPipeline (one batch per launch, or four fused into each launch: 32-cloud launches)
    draws the FULL batch's FPS starts and keeps its slice (shard.batch_shard).  Every shard's
    outputs, for every pipelined batch, equal its rows of the unsharded eager forward bit for
    bit."""
    import pn2
    from pn2 import shard
    from pn2.pipeline import GraphedPipeline, MultiHead
    names, models, x, mean, prec, _ = _build("pose")
    B, N, W = x.shape[0], x.shape[2], 8
    torch.manual_seed(57)
    draws = _draws(names, models, B, N)
    xd, md = x.to(DEV), mean.to(DEV)
    state = {"i": 0}

    def full_draw(N_):
        t = draws[state["i"] % len(draws)]
        state["i"] += 1
        assert int(t.max()) < N_
        return t

    torch.manual_seed(57)
    eager = _forward(names, models, xd, md, prec)  # the reference's unsharded draws, in order
    flat_w = _flat(tuple(eager))
    model = MultiHead(models, [i for i, n in enumerate(names) if n.startswith("translation")])
    n = 4
    for r in range(W):
        lo, hi = shard.shard_range(B, r, W)
        state["i"] = 0

        def fixed_draw(B_, N_, pin=True, lo=lo):
            assert B_ == hi - lo
            return full_draw(N_)[lo:lo + B_].clone()

        monkeypatch.setattr(shard, "draw_start", fixed_draw)
        monkeypatch.setattr(shard, "draw_start_into", lambda dst, N_: dst.copy_(fixed_draw(dst.shape[0], N_)))
        with torch.no_grad(), pn2.mlp_precision(prec), shard.batch_shard(B, lo):
            gp = GraphedPipeline(model, geometry_batches=gb, fuse=fuse, nslots=max(16, 4 * gb),
                                 geometry_streams=4 if gb == 1 else 1,
                                 geometry_bq=False if gb == 1 else None,
                             tail_streams=2 if gb == 1 else None)
            outs = gp.run([xd[lo:hi]] * n, [(md[lo:hi],)] * n)
        torch.cuda.synchronize()
        del gp
        for i, o in enumerate(outs):
            flat_o = _flat(o)
            assert len(flat_o) == len(flat_w)
            for a, b in zip(flat_o, flat_w):
                np.testing.assert_array_equal(a.cpu().numpy(), b[lo:hi].cpu().numpy(),
                                              err_msg="rank %d batch %d" % (r, i))
