"""Training path: train-mode forward + backward of the SA layers on the
GPU (fused batch-statistics BN / ReLU / max kernels of csrc/train.hip around library GEMMs)
against the reference's own train-mode forward + backward (tests/golden/train_*.npz, made by
make_goldens.py with the reference modules).

Tolerances (float; batch-statistics reductions over all rows run in another order, float64
partials here vs float32 in torch-CPU): forward features and running statistics
|got-ref| <= 1e-4*|ref| + 1e-4*max|ref|; gradients 1e-3 (relative plus the same max-scaled
floor).  Centroids and num_batches_tracked exact."""
import numpy as np
import pytest
import torch

import cases
from conftest import golden_names, load_golden


def _build(name):
    from pn2 import pointnet2_utils as P
    kind, args, B, N, D, wseed, fseed = cases.TRAIN_CASES[name]
    ctor = P.PointNetSetAbstraction if kind == "ssg" else P.PointNetSetAbstractionMsg
    torch.manual_seed(wseed)
    mod = ctor(*args)
    cases.randomize_bn(mod, wseed + 1)
    return mod.train(), (B, N, D, wseed, fseed)


def close(got, want, rtol, what):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    np.testing.assert_allclose(got, want, rtol=rtol, atol=rtol * max(float(np.abs(want).max()), 1e-30),
                               err_msg=what)


@pytest.mark.parametrize("name", golden_names("train_"))
def test_train_modules_rebuild_reference_weights(name):
    mod, _ = _build(name)
    assert cases.state_hash(mod) == str(load_golden("train_%s.npz" % name)["state_hash"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_names("train_"))
def test_train_step_matches_reference(name):
    from pn2 import train
    g = load_golden("train_%s.npz" % name)
    mod, (B, N, D, wseed, fseed) = _build(name)
    mod = mod.cuda()
    pts = torch.from_numpy(g["points"]).cuda()
    feat = None
    if "feature" in g:
        feat = torch.from_numpy(g["feature"]).cuda().requires_grad_(True)
    calls = []
    orig = train.mlp_max_train
    train.mlp_max_train = lambda *a: calls.append(1) or orig(*a)
    try:
        torch.manual_seed(fseed)
        new_points, new_feature = mod(pts, feat)
        (new_feature * torch.from_numpy(g["R"]).cuda()).sum().backward()
    finally:
        train.mlp_max_train = orig
    assert calls, "the fused training kernels did not run"
    np.testing.assert_array_equal(new_points.detach().cpu().numpy(), g["new_points"])
    close(new_feature.detach().cpu().numpy(), g["new_feature"], 1e-4, "new_feature")
    if feat is not None:
        close(feat.grad.cpu().numpy(), g["feature_grad"], 1e-3, "feature grad")
    for k, p in mod.named_parameters():
        if k.endswith(".bias") and ("conv" in k):
            # a conv bias followed by batch-statistics BN has zero gradient analytically (the
            # mean subtraction cancels it): both sides are float noise, bounded by the scale of
            # the layer's weight gradient
            scale = float(np.abs(g["grad." + k[:-5] + ".weight"]).max())
            assert float(p.grad.abs().max()) <= 1e-4 * scale, k
            assert float(np.abs(g["grad." + k]).max()) <= 1e-4 * scale, k
            continue
        close(p.grad.cpu().numpy(), g["grad." + k], 1e-3, "grad " + k)
    for k, b in mod.named_buffers():
        if k.endswith("num_batches_tracked"):
            assert int(b) == int(g["buf." + k]), k
        else:
            close(b.cpu().numpy(), g["buf." + k], 1e-4, k)


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,cins,couts", [(32 * 64 * 32, 32, [3], [64, 64, 128]),
                                            (4 * 128 * 64, 64, [131], [128, 256]),
                                            (3 * 100, 100, [35], [64]),
                                            (8 * 1024, 1024, [64], [128, 1024]),  # v1: max over N
                                            (5 * 300, 300, [16], [64])])
def test_train_mlp_matches_torch_on_device(M, K, cins, couts):
    """The fused Function against torch's own Conv2d/BatchNorm2d/ReLU/max autograd on the same
    device, at SSG-like sizes (sa1 B=32, sa2 B=4) and a K that is no power of two."""
    from pn2 import train
    torch.manual_seed(M)
    dims = cins + couts
    convs = [torch.nn.Conv2d(dims[i], dims[i + 1], 1).cuda() for i in range(len(couts))]
    bns = [torch.nn.BatchNorm2d(c).cuda() for c in couts]
    for bn in bns:
        cases.randomize_bn(bn, 3)
    convs2 = [torch.nn.Conv2d(dims[i], dims[i + 1], 1).cuda() for i in range(len(couts))]
    bns2 = [torch.nn.BatchNorm2d(c).cuda() for c in couts]
    for a, b in zip(convs + bns, convs2 + bns2):
        b.load_state_dict(a.state_dict())
    G = M // K
    x = torch.randn(G, 1, K, cins[0], device="cuda").view(G // 1, 1, K, cins[0])
    x = x.reshape(1, G, K, cins[0])
    xa = x.clone().requires_grad_(True)
    xb = x.clone().requires_grad_(True)
    out_a = train.mlp_max_train(xa, convs, bns)
    h = xb.permute(0, 3, 2, 1)
    for c, b in zip(convs2, bns2):
        h = torch.relu(b(c(h)))
    out_b = torch.max(h, 2)[0]
    # Where a group's two largest values are within float noise the two forwards (library GEMM
    # vs MIOpen conv) may pick different argmax rows and route that (g, c)'s gradient to another
    # row -- a near-tie, not an error (a few dozen of ~1e5 pairs here).  The upstream gradient
    # is zeroed on those pairs, so every remaining gradient must agree element-wise.
    top2 = torch.topk(h, 2, dim=2)[0]
    clear = (top2[:, :, 0] - top2[:, :, 1]) > 1e-4 * (top2[:, :, 0].abs() + 1e-2)
    R = torch.randn_like(out_b) * clear
    (out_a * R).sum().backward()
    (out_b * R).sum().backward()
    close(out_a.detach().cpu(), out_b.detach().cpu(), 1e-4, "out")
    close(xa.grad.cpu(), xb.grad.cpu(), 1e-3, "dx")
    for a, b in zip(convs + bns, convs2 + bns2):
        for (k, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
            if isinstance(a, torch.nn.Conv2d) and k == "bias":  # ~0: see above
                scale = float(a.weight.grad.abs().max())
                assert float(p.grad.abs().max()) <= 1e-4 * scale
                continue
            close(p.grad.cpu(), q.grad.cpu(), 1e-3, k)
        for (k, p), (_, q) in zip(a.named_buffers(), b.named_buffers()):
            close(p.float().cpu(), q.float().cpu(), 1e-4, k)


@pytest.mark.gpu
@pytest.mark.parametrize("G,K,C", [(7, 32, 64), (3, 1024, 200), (2, 300, 64), (4, 257, 5)])
def test_group_max_ties_and_nan(G, K, C):
    """pn2_group_max_f32 (narrow kernel below K = 256, row-split wide kernel from 256) against
    numpy's max / first argmax, on values with many exact ties, -inf rows and NaNs (NaN wins,
    first NaN index, as torch.max)."""
    from pn2 import _lib
    from pn2.ops import _stream
    rng = np.random.default_rng(G * K + C)
    a = rng.integers(-3, 4, (G, K, C)).astype(np.float32)
    a[0, :, 0] = -np.inf
    a[G - 1, rng.integers(0, K, 3), C - 1] = np.nan
    A = torch.from_numpy(a).cuda()
    out = torch.empty(G, C, device="cuda")
    arg = torch.empty(G, C, dtype=torch.int32, device="cuda")
    L = _lib.load()
    _lib.check(L.pn2_group_max_f32(A.data_ptr(), G, K, C, C, out.data_ptr(), C, arg.data_ptr(),
                                   _stream(A)), "pn2_group_max_f32")
    torch.cuda.synchronize()
    key = np.where(np.isnan(a), np.inf, a)  # NaN above everything; ties -> first index
    want_arg = np.where(np.isnan(a).any(1), np.argmax(np.isnan(a), axis=1), np.argmax(key, axis=1))
    want = np.take_along_axis(a, want_arg[:, None, :], 1)[:, 0]
    np.testing.assert_array_equal(arg.cpu().numpy(), want_arg)
    np.testing.assert_array_equal(out.cpu().numpy(), want)


# ------------------------------------------------------------------ PointNet-v1 training
def _build_v1(name):
    from pn2.heads_v1 import HEADS_V1
    head, B, N, kind, wseed, kw = cases.TRAIN_V1_CASES[name]
    return cases.train_v1_model(HEADS_V1[head], wseed, **kw)


def _v1_step(model, g, dev):
    out = model(torch.from_numpy(g["input"]).to(dev))
    outs = [o for o in (out if isinstance(out, tuple) else (out,))
            if torch.is_tensor(o) and o.is_floating_point() and o.requires_grad]
    loss = 0
    for i, o in enumerate(outs):
        loss = loss + (o * torch.from_numpy(g["R%d" % i]).to(dev)).sum()
    loss.backward()
    return outs


def _v1_check(model, g, outs, rtol_out, rtol_grad, pre=""):
    """Outputs, every parameter gradient (large ones through the golden's fixed sample and the
    norm) against the golden's float32 (pre "") or float64 (pre "t.") step; running
    statistics against the float32 step."""
    assert len(outs) == sum(k.startswith("out") for k in g.files)
    for i, o in enumerate(outs):
        close(o.detach().cpu().numpy(), g[pre + "out%d" % i], rtol_out, "out%d" % i)
    for k, p in model.named_parameters():
        full, sub = pre + "grad." + k, pre + "gsub." + k
        if full not in g and sub not in g:
            # no gradient in the reference (rotation.py computes its feature T-Net and drops it)
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, k
            continue
        gr = p.grad.detach().cpu().numpy()
        ref = g[full] if full in g else None
        if k.endswith(".bias"):
            # a bias whose layer feeds a batch-statistics BN (conv -> BN, fc -> BN, and a BN
            # shift that reaches the next BN through the max) has zero gradient analytically:
            # the reference's value is rounding noise (< 3e-6 of its weight's gradient in
            # float32, real ones > 6e-2), and ours must be noise of the same order
            wk = k[:-5] + ".weight"
            scale = float(np.abs(g[pre + "grad." + wk] if pre + "grad." + wk in g
                                 else g[pre + "gsub." + wk]).max())
            if ref is not None and float(np.abs(ref).max()) <= 1e-4 * scale:
                assert float(np.abs(gr).max()) <= 1e-4 * scale, k
                continue
        got = gr if ref is not None else gr.reshape(-1)[cases.grad_sample_index(gr.size)]
        want = ref if ref is not None else g[sub]
        tol = rtol_grad
        if pre:
            # against float64: the tolerance is the larger of rtol_grad and 4x the reference's
            # own float32 error on this tensor (max-scaled), so a gradient the T-Net networks
            # amplify float32 rounding into is held to the reference's accuracy
            f32 = g[full[len(pre):]] if ref is not None else g[sub[len(pre):]]
            ref_err = float(np.abs(f32.astype(np.float64) - want).max() / max(np.abs(want).max(), 1e-30))
            tol = max(rtol_grad, 4.0 * ref_err)
        close(got, want, tol, "grad " + k)
        if ref is None:
            np.testing.assert_allclose(np.linalg.norm(gr.astype(np.float64)), float(g[pre + "gnorm." + k]),
                                       rtol=tol, err_msg="grad norm " + k)
    for k, b in model.named_buffers():
        if k.endswith("num_batches_tracked"):
            assert int(b) == int(g["buf." + k]), k
        elif "buf." + k in g:
            close(b.cpu().numpy(), g["buf." + k], 1e-4, k)


@pytest.mark.parametrize("name", golden_names("trainv1_"))
def test_trainv1_rebuild_reference_weights(name):
    g = load_golden("trainv1_%s.npz" % name)
    assert cases.state_hash(_build_v1(name)) == str(g["state_hash"])
    assert float(g["min_gap"]) >= cases.TRAIN_V1_MIN_GAP  # tie-free maxima (cases.py)


@pytest.mark.parametrize("name", golden_names("trainv1_"))
def test_trainv1_cpu_step_matches_reference(name):
    """On the CPU the v1 modules keep the reference's torch formulation in training: the same
    step as the reference's modules, to float noise."""
    g = load_golden("trainv1_%s.npz" % name)
    model = _build_v1(name)
    outs = _v1_step(model, g, "cpu")
    _v1_check(model, g, outs, 1e-5, 1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_names("trainv1_"))
def test_trainv1_step_matches_reference(name):
    """The v1 heads' train step on the GPU (shared MLPs on pn2.train's fused batch-statistics
    kernels, the encoder's conv3 + bn3 unrectified before its max) against the reference's
    own train step run in float64 (make_goldens.py trainv1): outputs 1e-4; gradients 2e-3, or
    4x the reference's own float32 error where that is larger (relative, plus the same
    max-scaled floor) -- the networks with an input T-Net amplify float32 rounding into some
    gradients: the reference's float32 step is 4-9e-4 from float64 on these cases, up to 1e-1 on
    others (tools/debug/trainv1_diff.py)."""
    from pn2 import train
    g = load_golden("trainv1_%s.npz" % name)
    model = _build_v1(name).cuda()
    calls = []
    orig = train.point_mlp_train
    train.point_mlp_train = lambda *a, **k: calls.append(1) or orig(*a, **k)
    try:
        outs = _v1_step(model, g, "cuda")
    finally:
        train.point_mlp_train = orig
    assert calls, "the fused training kernels did not run"
    _v1_check(model, g, outs, 1e-4, 2e-3, pre="t.")
