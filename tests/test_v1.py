"""PointNet-v1 path: pn2/pointnet_utils.py (drop-in for
/root/reference/model/pointnet_utils.py) and the v1 head restatements (pn2/heads_v1.py),
against goldens produced by the reference itself (tests/golden/make_goldens.py v1).

CPU tests: seeded weights reproduce the reference's state_dict, the autograd (torch) path
reproduces the goldens, eval on a CPU tensor raises (no CPU fallback), and the reference's own
v1 head files run unchanged on the drop-in.  GPU tests: eval-mode heads on the split-bf16
dense-layer kernels against the goldens, and the kernel features the v1 path adds (rows
source, unpooled output, PN2_LAYER_NO_RELU signed max) against torch fp32 on the same device.

Tolerance (float, as tests/test_gpu_sa.py): |got - ref| <= rtol * |ref| + rtol * max|ref|,
rtol = 1e-5 for encoder features / T-Net outputs, 1e-4 for head outputs (two more GEMM layers
of fp32 library rounding differences)."""
import os
import sys

import numpy as np
import pytest
import torch

import cases
from conftest import golden_names, load_golden

REF = "/root/reference/model"


def _build(name):
    from pn2.heads_v1 import HEADS_V1
    head, B, N, kind, wseed, kw = cases.V1_CASES[name]
    return cases.build_head(HEADS_V1[head], wseed, **kw), head


def _args(g, dev):
    args = [torch.from_numpy(g["input"]).to(dev)]
    if "mean" in g:
        args.append(torch.from_numpy(g["mean"]).to(dev))
    return args


def _hooks(model, acts):
    for tag, sub in (("feat", "feat"), ("tnet", "feat.tnet"), ("ftnet", "feat.ftnet"),
                     ("ftnet", "ftnet"), ("tnet", "tnet")):
        m = model
        try:
            for part in sub.split("."):
                m = getattr(m, part)
        except AttributeError:
            continue

        def f(_m, _i, out, tag=tag):
            for i, o in enumerate(out if isinstance(out, tuple) else (out,)):
                acts["%s_%d" % (tag, i)] = o.detach().cpu().numpy()
        m.register_forward_hook(f)


def assert_close(got, want, rtol):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    np.testing.assert_allclose(got, want, rtol=rtol, atol=rtol * max(float(np.abs(want).max()), 1e-30))


def _check(g, out, acts, rtol_feat, rtol_out):
    for k, v in acts.items():
        assert k in g, k
        assert_close(v, g[k], rtol_feat)
    outs = out if isinstance(out, tuple) else (out,)
    for i, o in enumerate(outs):
        o = o.detach().cpu().numpy()
        if o.dtype == np.int64:
            np.testing.assert_array_equal(o, g["out%d" % i])
        else:
            assert_close(o, g["out%d" % i], rtol_out)


# ---------------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("name", golden_names("v1_"))
def test_v1_heads_rebuild_reference_weights(name):
    model, _ = _build(name)
    assert cases.state_hash(model) == str(load_golden("v1_%s.npz" % name)["state_hash"])


@pytest.mark.parametrize("name", golden_names("v1_"))
def test_v1_autograd_path_matches_goldens(name):
    """Eval forward inside pn2.eval_autograd() = the reference's torch formulation, on the
    CPU."""
    import pn2
    g = load_golden("v1_%s.npz" % name)
    model, _ = _build(name)
    acts = {}
    _hooks(model, acts)
    with pn2.eval_autograd():
        out = model(*_args(g, "cpu"))
    _check(g, out, acts, 1e-6, 1e-6)


def test_v1_eval_on_cpu_raises():
    from pn2.heads_v1 import HEADS_V1
    from pn2.pointnet_utils import PointNetEncoder
    for model, x in ((PointNetEncoder(channel=3).eval(), torch.rand(2, 3, 64)),
                     (HEADS_V1["sign"]().eval(), torch.rand(2, 10, 64))):
        with pytest.raises(RuntimeError, match="ROCm device tensors only"):
            with torch.no_grad():
                model(x)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
@pytest.mark.parametrize("head", ["pointnet_cls", "rotation", "pose"])
def test_reference_v1_heads_import_drop_in_unchanged(head, monkeypatch):
    """The reference's own v1 head files, with `pointnet_utils` resolving to the drop-in, load
    a reference-built state_dict strictly and run (pn2.eval_autograd: the torch path) to the
    reference's numbers;
    eval without autograd reaches the kernels (CPU tensor -> loud error).  (translation / sign
    / width keep their whole conv stack in the head file: only pn2.heads_v1 accelerates them.)"""
    import importlib
    import pn2.pointnet_utils as ours
    monkeypatch.setattr(sys, "dont_write_bytecode", True)
    monkeypatch.syspath_prepend(REF)
    kw = {"mlp_list": [64, 64, 128, 1024], "linear_list": [512, 256, 2], "transform": True,
          "feat_trans": True, "num_category": 0, "normal_channel": False} if head == "pose" else {}
    for m in ("pointnet_utils", head):
        sys.modules.pop(m, None)
    torch.manual_seed(5)
    ref = importlib.import_module(head).get_model(**kw).eval()
    sys.modules.pop(head, None)
    monkeypatch.setitem(sys.modules, "pointnet_utils", ours)
    mod = importlib.import_module(head)
    model = mod.get_model(**kw)
    model.load_state_dict(ref.state_dict(), strict=True)
    sys.modules.pop(head, None)
    model.eval()
    x = torch.rand(2, 3 if head in ("pointnet_cls", "pose") else 10, 64)
    import pn2
    with pn2.eval_autograd():
        a, b = ref(x), model(x)
    for u, v in zip(a if isinstance(a, tuple) else (a,), b if isinstance(b, tuple) else (b,)):
        np.testing.assert_array_equal(u.detach().numpy(), v.detach().numpy())
    with pytest.raises(RuntimeError, match="ROCm device tensors only"):
        with torch.no_grad():
            model(x)


# ---------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_names("v1_"))
def test_v1_heads_match_reference_on_gpu(name):
    from pn2 import _lib
    g = load_golden("v1_%s.npz" % name)
    model, _ = _build(name)
    model = model.to("cuda").eval()
    acts = {}
    _hooks(model, acts)
    with torch.no_grad():
        out = model(*_args(g, "cuda"))
    assert _lib.load().pn2_sa_mlp_last_path() == _lib.PATH_SPLIT_BF16
    _check(g, out, acts, 1e-5, 1e-4)


def _torch_layers(x_cf, convs, bns, relu_last=True):
    h = x_cf
    for i, (c, b) in enumerate(zip(convs, bns)):
        h = b(c(h))
        if relu_last or i < len(convs) - 1:
            h = torch.relu(h)
    return h


def _rand_layers(cins, couts, seed):
    torch.manual_seed(seed)
    convs = [torch.nn.Conv1d(a, b, 1) for a, b in zip(cins, couts)]
    bns = [torch.nn.BatchNorm1d(b) for b in couts]
    for bn in bns:
        cases.randomize_bn(bn, seed)
    return [c.cuda().eval() for c in convs], [b.cuda().eval() for b in bns]


@pytest.mark.gpu
@pytest.mark.parametrize("B,N,cin,couts,pool,relu_last", [
    (3, 1000, 64, [128, 1024], True, False),    # the encoder's conv2/conv3 (signed max)
    (2, 777, 64, [64, 128, 1024], True, True),  # rotation.py layers 2-4 from rows
    (2, 500, 128, [1024], True, False),
    (4, 300, 64, [64], False, True),            # unpooled rows out
    (1, 33, 64, [128, 256], False, False),      # unpooled, signed
    (2, 8, 64, [64, 128], True, True),          # fewer points than 16 (rows, not channels)
])
def test_point_mlp_rows_source(B, N, cin, couts, pool, relu_last):
    from pn2.pointnet_utils import point_mlp
    convs, bns = _rand_layers([cin] + couts[:-1], couts, 11 + N)
    rows = torch.randn(B, N, cin, device="cuda")
    with torch.no_grad():
        got = point_mlp(rows, convs, bns, {}, pool=pool, last_relu=relu_last, rows=True)
        ref = _torch_layers(rows.permute(0, 2, 1), convs, bns, relu_last)
        ref = ref.max(2)[0] if pool else ref.permute(0, 2, 1)
    assert_close(got.cpu().numpy(), ref.cpu().numpy(), 1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("C,N,pool,tview", [(3, 1024, False, False), (10, 2048, True, False),
                                            (13, 100, True, False), (3, 5, False, False),
                                            (10, 1024, True, True), (3, 7, False, True),
                                            (64, 300, True, True)])
def test_point_mlp_channel_first_source(C, N, pool, tview):
    """tview: the input is the transpose(2, 1) view of [B, N, C] storage -- the layout the
    reference's scripts (and pn2.provider.prepare_batch) hand the model."""
    from pn2.pointnet_utils import point_mlp
    convs, bns = _rand_layers([C], [64], 7 + C)
    if tview:
        x = torch.randn(2, N, C, device="cuda").transpose(2, 1)
    else:
        x = torch.randn(2, C, N, device="cuda")
    with torch.no_grad():
        got = point_mlp(x, convs, bns, {}, pool=pool)
        ref = _torch_layers(x, convs, bns)
        ref = ref.max(2)[0] if pool else ref.permute(0, 2, 1)
    assert_close(got.cpu().numpy(), ref.cpu().numpy(), 1e-5)


@pytest.mark.parametrize("relu,affine,extra", [(True, True, False), (False, True, True), (True, False, False)])
def test_linear_bn_folds_eval_batchnorm(relu, affine, extra):
    """linear_bn (the eval FC tails: Linear + BatchNorm1d folded into one GEMM) against the
    modules; plain torch, so it is checked on the CPU.  A BN without running statistics (batch
    statistics even in eval) is not folded: the modules run."""
    from pn2.pointnet_utils import linear_bn
    torch.manual_seed(5)
    fc = torch.nn.Linear(256, 128)
    bn = torch.nn.BatchNorm1d(128, affine=affine)
    cases.randomize_bn(bn, 9) if affine else None
    with torch.no_grad():
        bn.running_mean.uniform_(-0.1, 0.1)
        bn.running_var.uniform_(0.5, 1.5)
    bn.eval()
    x = torch.randn(8, 256)
    e = torch.randn(1, 128) if extra else None
    cache = {}
    with torch.no_grad():
        got = linear_bn(x, fc, bn, cache, relu=relu, extra=e)
        ref = bn(fc(x)) + (e if extra else 0)
        ref = torch.relu(ref) if relu else ref
        assert_close(got.numpy(), ref.numpy(), 1e-5)
        fc.weight.mul_(2)  # a parameter change invalidates the folded copy
        got = linear_bn(x, fc, bn, cache, relu=relu, extra=e)
        ref = bn(fc(x)) + (e if extra else 0)
        ref = torch.relu(ref) if relu else ref
        assert_close(got.numpy(), ref.numpy(), 1e-5)
        nostats = torch.nn.BatchNorm1d(128, track_running_stats=False).eval()
        got = linear_bn(x, fc, nostats, {}, relu=relu)
        ref = nostats(fc(x))
        assert_close(got.numpy(), (torch.relu(ref) if relu else ref).numpy(), 1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("B,K,N,relu", [(8, 1024, 512, True), (8, 512, 256, True), (8, 256, 9, False),
                                        (8, 256, 4096, False), (3, 1024, 7, True), (16, 512, 130, True),
                                        (16, 1024, 512, True), (5, 6, 3, False), (12, 255, 33, True),
                                        (32, 1024, 512, True), (70, 300, 40, False)])
def test_linear_rows_matches_torch(B, K, N, relu):
    """pn2_linear_rows_f32 (the small-batch FC kernel: 16-byte and scalar paths, 2/4 output
    features per wave, row blocks of 16) against float64 torch, fp32 tolerance; every row
    bit-identical to the same row computed in a batch of its own (batch sharding)."""
    from pn2 import ops
    torch.manual_seed(B * K + N)
    x = torch.randn(B, K, device="cuda")
    W = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda")
    got = ops.linear_rows(x, W, b, relu)
    ref = x.double() @ W.double().t() + b.double()
    ref = ref.clamp_min(0) if relu else ref
    assert_close(got.cpu().numpy(), ref.cpu().numpy(), 2e-6)
    one = torch.cat([ops.linear_rows(x[i:i + 1], W, b, relu) for i in range(B)])
    np.testing.assert_array_equal(one.cpu().numpy(), got.cpu().numpy())
    xs = torch.randn(B, K + 3, device="cuda")[:, 1:K + 1]  # strided rows, misaligned base
    got = ops.linear_rows(xs, W, None, False)
    ref = xs.double() @ W.double().t()
    assert_close(got.cpu().numpy(), ref.cpu().numpy(), 2e-6)


@pytest.mark.gpu
def test_v1_pointnet_cls_at_config_batch():
    """BASELINE config 1 runs pointnet_cls at B = 8; the v1 dense kernels pick their tile widths
    by row count, so the B = 8 launch is checked too: the golden's 4 clouds twice over (the
    second copy reversed) must each give the reference's per-cloud outputs, and equal copies
    the same bits."""
    g = load_golden("v1_pointnet_cls.npz")
    model, _ = _build("pointnet_cls")
    model = model.to("cuda").eval()
    x4 = torch.from_numpy(g["input"])
    B0 = x4.shape[0]
    order = list(range(B0)) + list(reversed(range(B0)))
    x8 = x4[order].contiguous().to("cuda")
    with torch.no_grad():
        out = model(x8)
    outs = out if isinstance(out, tuple) else (out,)
    for i, o in enumerate(outs):
        o = o.detach().cpu().numpy()
        want = g["out%d" % i][order]
        if o.dtype == np.int64:
            np.testing.assert_array_equal(o, want)
        else:
            assert_close(o, want, 1e-4)
        for k in range(B0):  # cloud k in both copies: identical bits
            np.testing.assert_array_equal(o[k], o[2 * B0 - 1 - k])
