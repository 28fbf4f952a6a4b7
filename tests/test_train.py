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
                                            (3 * 100, 100, [35], [64])])
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
