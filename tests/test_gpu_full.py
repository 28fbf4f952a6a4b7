"""GPU parity at the BASELINE shapes against the reference's own outputs (tests/golden/full_*.npz,
made by make_goldens.py from the imported reference heads):

  cls_ssg_b32            pointnet2_cls_ssg B=32 N=1024 -- the metric's configuration
  cls_msg_n4096          pointnet2_cls_msg N=4096 (B=8)
  rotation_/translation_ssg_n2048   the pose heads at N=2048, 10 channels (B=8)
  cls_ssg_n16384         the stress config's N=16384 (B=2; fp32, and bf16 to a bf16 tolerance)
  translation_msg, sign_ssg, sign_msg   the heads without a small case
  camera_*               the reference's two real scans (camera_test/bed.txt, night_stand.txt)

Both launch paths are checked: the eager modules and pn2.pipeline.GraphedPipeline (the bench's
launch).  Bar: every layer's centroids bit-exact for the whole batch (they are FPS indices
gathered), SA features within 1e-5 relative (+1e-5 * max|ref| absolute), head outputs within
1e-4 relative (three unfused FC layers), integer outputs exact."""
import itertools

import numpy as np
import pytest
import torch

import cases
from conftest import golden_names, load_golden
from test_oracle_golden import full_draws, full_input

pytestmark = pytest.mark.gpu
DEV = "cuda"
FULL = golden_names("full_")


def _close(got, want, rtol, what):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    atol = rtol * max(float(np.abs(want).max()), 1e-30)
    np.testing.assert_allclose(got, want, rtol=rtol, atol=atol, err_msg=what)


def _setup(name):
    from pn2 import heads as H
    head, B, N, kind, wseed, fseed, keep = cases.HEAD_FULL_CASES[name]
    g = load_golden("full_%s.npz" % name)
    model = cases.build_head(H.HEADS[head], wseed)
    assert cases.state_hash(model) == str(g["state_hash"])
    x = full_input(name, g)
    draws = full_draws(model, B, N, fseed)
    args = [x.to(DEV)]
    if "mean" in g:
        args.append(torch.from_numpy(g["mean"]).to(DEV))
    return g, model.to(DEV).eval(), args, draws, fseed


def _hook_acts(model):
    acts = {}
    tags = [t for t in ("sa1", "sa2", "sa3") if hasattr(model, t)]
    def hook(m, i, o, t):
        # first call of each layer only: later calls may be graph captures, where a copy to the
        # host is not allowed
        if t not in acts:
            acts[t] = [(o[0].cpu().numpy(), o[1].cpu().numpy())]
    hs = [getattr(model, t).register_forward_hook(lambda m, i, o, t=t: hook(m, i, o, t))
          for t in tags]
    return acts, tags, hs


def _check(g, acts, tags, outs, k=0, feat_rtol=1e-5, out_rtol=1e-4):
    kept = g["keep"]
    for t in tags:
        p, f = acts[t][k]
        np.testing.assert_array_equal(p.view(np.uint32), g[t + "_points"].view(np.uint32),
                                      err_msg=t + " centroids")
        _close(f if t == tags[-1] else f[kept], g[t + "_feature"], feat_rtol, t + " feature")
    _check_outs(g, outs, out_rtol, "")


def _check_outs(g, outs, rtol, what):
    outs = outs if isinstance(outs, tuple) else (outs,)
    for i, o in enumerate(outs):
        o = o.cpu().numpy()
        want = g["out%d" % i]
        if o.dtype == np.int64:
            np.testing.assert_array_equal(o, want, err_msg=what + "out%d" % i)
        elif i == 1 and want.ndim == 2 and want.shape[1] == 1:
            # sign heads: sign(sigmoid - 0.5) is exact away from 0.5 (sign_ssg.py:34-35)
            far = np.abs(g["out0"] - 0.5) > 1e-4
            np.testing.assert_array_equal(o[far], want[far], err_msg=what + "sign")
        else:
            _close(o, want, rtol, what + "out%d" % i)


@pytest.mark.parametrize("name", FULL)
def test_full_size_head_eager_matches_reference(name):
    g, model, args, draws, fseed = _setup(name)
    acts, tags, hs = _hook_acts(model)
    torch.manual_seed(fseed)
    with torch.no_grad():
        out = model(*args)
    torch.cuda.synchronize()
    for h in hs:
        h.remove()
    _check(g, acts, tags, out)


@pytest.mark.parametrize("mode", ["fused4", "one"])
@pytest.mark.parametrize("name", FULL)
def test_full_size_head_graphed_pipeline_matches_reference(name, mode, monkeypatch):
    """GraphedPipeline over four batches of the golden's input: the first runs eagerly and
    captures the slots, the rest replay the fps / sa / head graphs on their streams.  Every
    batch takes the golden's start draws (shard.draw_start patched to cycle them), so every
    batch must reproduce the reference's outputs.  mode: the class defaults (four batches fused
    per launch), or bench.py's headline launch (one batch per launch, four geometry streams, the
    ball queries in each batch's forward)."""
    from pn2 import shard
    from pn2.pipeline import GraphedPipeline
    g, model, args, draws, fseed = _setup(name)
    cyc = itertools.cycle([torch.from_numpy(d) for d in draws])

    def golden_draw(B, N, pin=True):
        d = next(cyc)
        assert d.shape[0] == B and int(d.max()) < N
        return d.clone()

    monkeypatch.setattr(shard, "draw_start", golden_draw)
    # the pipeline writes its draws in place (shard.draw_start_into): the same cycle
    monkeypatch.setattr(shard, "draw_start_into", lambda dst, N: dst.copy_(golden_draw(dst.shape[0], N)))
    acts, tags, hs = _hook_acts(model)  # fire on the eager first batch only (graphs replay)
    n = 4
    extras = [tuple(args[1:])] * n if len(args) > 1 else None
    gp = GraphedPipeline(model) if mode == "fused4" else GraphedPipeline(
        model, geometry_batches=1, fuse=False, nslots=16, geometry_streams=4, geometry_bq=False,
        tail_streams=2)
    outs = gp.run([args[0]] * n, extras)
    torch.cuda.synchronize()
    for h in hs:
        h.remove()
    _check(g, acts, tags, outs[0])
    for i, o in enumerate(outs[1:]):
        _check_outs(g, o, 1e-4, "batch %d " % (i + 1))
        if "out1" in g and g["out1"].ndim == 3:  # cls heads return l3f: the SA path itself
            _close(o[1].cpu().numpy(), g["out1"], 1e-5, "batch %d l3f" % (i + 1))


def test_stress_shape_bf16_matches_reference_indices():
    """BASELINE config 5 arithmetic (MLP in bf16) at N=16384: centroids still bit-exact (the
    geometry is fp32), features within a bf16 tolerance of the reference's fp32 outputs (three
    layers with bf16 operands: 2e-2 of the layer's max |feature|)."""
    import pn2
    g, model, args, draws, fseed = _setup("cls_ssg_n16384")
    acts, tags, hs = _hook_acts(model)
    torch.manual_seed(fseed)
    with torch.no_grad(), pn2.mlp_precision("bf16"):
        model(*args)
    for h in hs:
        h.remove()
    assert pn2._lib.load().pn2_sa_mlp_last_path() == pn2._lib.PATH_BF16
    for t in tags:
        p, f = acts[t][0]
        np.testing.assert_array_equal(p.view(np.uint32), g[t + "_points"].view(np.uint32))
        want = g[t + "_feature"]
        f = f if t == tags[-1] else f[g["keep"]]
        err = np.abs(f - want).max() / np.abs(want).max()
        assert err < 2e-2, (t, err)
