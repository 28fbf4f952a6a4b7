"""GPU parity of the SA modules and full heads (fused path) against the reference's goldens,
plus full-size BASELINE configs checked through size-independent properties.

Tolerance for float features (north star: 1e-5 relative): |got - ref| <= 1e-5 * |ref| +
1e-5 * max|ref| -- the absolute floor covers near-zero ReLU outputs whose relative error is
meaningless; indices and centroid coordinates are compared bit-for-bit."""
import numpy as np
import pytest
import torch

import cases
import oracle
from conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"
RTOL = 1e-5


def assert_feat_close(got, want, rtol=RTOL):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    atol = rtol * max(float(np.abs(want).max()), 1e-30)
    np.testing.assert_allclose(got, want, rtol=rtol, atol=atol)


def _head(name):
    from pn2 import heads as H
    head, B, N, kind, wseed, fseed = cases.HEAD_CASES[name]
    model = cases.build_head(H.HEADS[head], wseed)
    return model, head, fseed


@pytest.mark.parametrize("name", golden_names("head_"))
def test_head_matches_reference(name):
    g = load_golden("head_%s.npz" % name)
    model, head, fseed = _head(name)
    assert cases.state_hash(model) == str(g["state_hash"])
    model = model.to(DEV).eval()
    acts = {}
    for tag in ("sa1", "sa2", "sa3"):
        if hasattr(model, tag):
            getattr(model, tag).register_forward_hook(
                lambda m, i, o, tag=tag: acts.__setitem__(tag, (o[0].cpu().numpy(), o[1].cpu().numpy())))
    args = [torch.from_numpy(g["input"]).to(DEV)]
    if "mean" in g:
        args.append(torch.from_numpy(g["mean"]).to(DEV))
    torch.manual_seed(fseed)
    with torch.no_grad():
        out = model(*args)
    for tag, (p, f) in acts.items():
        np.testing.assert_array_equal(p.view(np.uint32), g[tag + "_points"].view(np.uint32),
                                      err_msg=tag + " centroids")
        assert_feat_close(f, g[tag + "_feature"])
    outs = out if isinstance(out, tuple) else (out,)
    for i, o in enumerate(outs):
        if o.dtype == torch.int64:
            np.testing.assert_array_equal(o.cpu().numpy(), g["out%d" % i])
        else:
            assert_feat_close(o.cpu().numpy(), g["out%d" % i], rtol=1e-4)


@pytest.mark.parametrize("name", ["cls_ssg", "cls_msg"])
def test_reference_input_layout_transposed(name):
    """The training loop feeds points.transpose(2,1) of a contiguous [B,N,C] tensor
    (train_rotation.py:116); the drop-in must accept that view and give the same numbers."""
    g = load_golden("head_%s.npz" % name)
    model, head, fseed = _head(name)
    model = model.to(DEV).eval()
    x = torch.from_numpy(g["input"])
    xt = x.permute(0, 2, 1).contiguous().to(DEV).permute(0, 2, 1)
    torch.manual_seed(fseed)
    with torch.no_grad():
        a = model(x.to(DEV))
    torch.manual_seed(fseed)
    with torch.no_grad():
        b = model(xt)
    # C=3: both layouts sum the 3 channels in the same order -> identical results
    np.testing.assert_array_equal(a[1].cpu().numpy(), b[1].cpu().numpy())


def _torch_sa_reference(sa, pts_bnc, feat_bnd, start):
    """fp32 torch-GPU evaluation of the reference formulation of one SSG layer (MIOpen conv +
    BN), with the oracle's indices -- the float reference for the fused MLP kernel."""
    from pn2.pointnet2_utils import _torch_group, _torch_mlp_max
    B, N, C = pts_bnc.shape
    f = oracle.farthest_point_sample(pts_bnc.cpu(), sa.point_number, start)
    newp = oracle.index_points(pts_bnc.cpu(), f)
    idx = oracle.query_ball_point(sa.radius, sa.sample_number, pts_bnc.cpu(), newp)
    with torch.no_grad():
        g = _torch_group(pts_bnc, torch.from_numpy(idx).to(DEV), torch.from_numpy(newp).to(DEV),
                         feat_bnd, False)
        return newp, _torch_mlp_max(g, sa.mlp_convs, sa.mlp_bns)


def test_ssg_baseline_config_full_size():
    """BASELINE config 2 (pointnet2_cls_ssg, B=32, N=1024): sa1 indices exact vs oracle for the
    whole batch, features vs the fp32 torch formulation."""
    from pn2 import heads as H
    torch.manual_seed(0)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 1)
    model = model.to(DEV)
    B, N = 32, 1024
    x = cases.cloud("uniform3", B, N, 42).permute(0, 2, 1).contiguous()
    torch.manual_seed(5)
    with torch.no_grad():
        newp, feat = model.sa1(x.to(DEV), None)
    torch.manual_seed(5)
    start = torch.randint(0, N, (B,), dtype=torch.long)
    want_p, want_f = _torch_sa_reference(model.sa1, x.to(DEV).permute(0, 2, 1), None, start)
    np.testing.assert_array_equal(newp.permute(0, 2, 1).cpu().numpy(), want_p)
    assert_feat_close(feat.cpu().numpy(), want_f.cpu().numpy())
    # the whole forward runs and is deterministic
    torch.manual_seed(7)
    with torch.no_grad():
        o1 = model(x.to(DEV))
    torch.manual_seed(7)
    with torch.no_grad():
        o2 = model(x.to(DEV))
    np.testing.assert_array_equal(o1[0].cpu().numpy(), o2[0].cpu().numpy())


def test_pose_heads_sharded_equals_unsharded():
    """BASELINE config 4 semantics on one GPU: rotation_ssg + translation_ssg B=64 N=2048
    one-hot; running the batch as 8 shards (with the full-batch FPS draws sliced) reproduces
    the unsharded result bit-for-bit."""
    from pn2 import heads as H
    from pn2 import shard
    torch.manual_seed(2)
    rot = H.RotationSSG().eval()
    cases.randomize_bn(rot, 3)
    rot = rot.to(DEV)
    B, N, W = 64, 2048, 8
    x = cases.cloud("onehot10", B, N, 44).permute(0, 2, 1).contiguous().to(DEV)
    torch.manual_seed(11)
    with torch.no_grad():
        full = rot(x)
    parts = []
    for r in range(W):
        lo, hi = shard.shard_range(B, r, W)
        torch.manual_seed(11)
        with torch.no_grad(), shard.batch_shard(B, lo):
            parts.append(rot(x[lo:hi]))
    got = torch.cat(parts)
    np.testing.assert_array_equal(got.cpu().numpy(), full.cpu().numpy())


def test_stress_config_geometry():
    """BASELINE config 5 geometry (B=128, N=16384): the FPS/ball-query front end of sa1 on 2
    clouds of the batch vs the oracle (indices bit-exact)."""
    import pn2
    B, N, S, K = 128, 16384, 512, 32
    x = cases.cloud("uniform3", B, N, 45)
    xs = cases.as_layout(x, "strided")
    start = torch.randint(0, N, (B,), generator=torch.Generator().manual_seed(0))
    d = xs.permute(0, 2, 1).contiguous().to(DEV).permute(0, 2, 1)
    idx, newp, cpk, ppk = torch.ops.pn2.fps(d, S, start.to(DEV))
    bq = torch.ops.pn2.ball_query(ppk, cpk, 3, 0.2, K)
    for b in (0, 97):
        f = oracle.farthest_point_sample(xs[b:b + 1], S, start[b:b + 1])
        np.testing.assert_array_equal(idx[b:b + 1].cpu().numpy(), f)
        c = oracle.index_points(xs[b:b + 1], f)
        np.testing.assert_array_equal(bq[b:b + 1].cpu().numpy(), oracle.query_ball_point(0.2, K, xs[b:b + 1], c))
    # sortedness/padding property over the whole batch
    q = bq.cpu().numpy()
    first = q[:, :, :1]
    d_ = np.diff(q, axis=-1)
    assert ((d_ > 0) | ((d_ <= 0) & (q[:, :, 1:] == first))).all()


@pytest.mark.parametrize("head", ["ClsSSG", "ClsMSG"])
def test_geometry_stream_matches_single_stream(head):
    """FPS/ball query on the geometry stream (overlapping the previous layer's MLP) give the
    same bits as running everything on the caller's stream -- over back-to-back forwards whose
    temporaries churn the caching allocator, with the inputs freed right after each launch."""
    from pn2 import heads as H
    torch.manual_seed(4)
    model = getattr(H, head)().eval()
    cases.randomize_bn(model, 4)
    model = model.to(DEV)
    B, N = (16, 1024) if head == "ClsSSG" else (8, 2048)
    clouds = [cases.cloud("uniform3", B, N, 60 + i).permute(0, 2, 1).contiguous() for i in range(4)]

    def run():
        torch.manual_seed(9)
        outs = []
        with torch.no_grad():
            for c in clouds:
                x = c.to(DEV, non_blocking=True)
                outs.append(model(x)[0])
                del x
        torch.cuda.synchronize()
        return [o.cpu().numpy() for o in outs]

    from pn2 import tuning
    with tuning.override(geometry_stream=0):
        want = run()
    with tuning.override(geometry_stream=1):
        for _ in range(2):
            got = run()
            for g, w in zip(got, want):
                np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("head", ["ClsSSG", "ClsMSG", "RotationSSG"])
def test_graph_replay_matches_eager(head):
    """GraphedForward: the first call runs eagerly and captures; replays give the eager bits for
    new inputs, take the FPS start draws from the CPU generator in the eager order (the RNG is
    left in the same state), follow shard.batch_shard slicing, and re-capture after an
    in-place parameter update."""
    from pn2 import heads as H
    from pn2 import shard
    from pn2.graphs import GraphedForward
    torch.manual_seed(6)
    model = getattr(H, head)().eval()
    cases.randomize_bn(model, 6)
    model = model.to(DEV)
    kind = "onehot10" if head.startswith("Rotation") else "uniform3"
    B, N = (8, 2048) if head == "ClsMSG" else (16, 1024)
    xs = [cases.cloud(kind, B, N, 80 + i).permute(0, 2, 1).contiguous().to(DEV) for i in range(4)]

    def first(o):
        return (o[0] if isinstance(o, tuple) else o).clone()

    def run(fn):
        torch.manual_seed(21)
        outs = []
        with torch.no_grad():
            for i, x in enumerate(xs):
                if i == 2:  # sharded call: second half of a 2*B global batch
                    with shard.batch_shard(2 * B, B):
                        outs.append(first(fn(x)))
                else:
                    outs.append(first(fn(x)))
            if head == "ClsSSG":  # in-place parameter change -> recapture
                rm = model.sa1.mlp_bns[0].running_mean
                saved = rm.clone()
                rm.add_(0.25)
                outs.append(first(fn(xs[0])))
                outs.append(first(fn(xs[1])))
                rm.copy_(saved)
        return [o.cpu().numpy() for o in outs], torch.randint(0, 1 << 30, (4,))

    want, rng_want = run(model)
    gm = GraphedForward(model)
    got, rng_got = run(gm)
    assert gm._graph is not None
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
    np.testing.assert_array_equal(rng_got.numpy(), rng_want.numpy())


@pytest.mark.parametrize("head,tail", [("ClsSSG", False), ("ClsSSG", "auto"), ("ClsMSG", False),
                                       ("TranslationSSG", "auto")])
def test_pipelined_forward_matches_eager(head, tail):
    """pn2.pipeline.PipelinedForward (FPS of batch i+1 on its own CUs while batch i runs) returns
    the eager forwards' results for a sequence of batches -- including a sharded call -- and
    leaves the CPU generator where the eager sequence leaves it.  Every SA output (the l3
    feature) and the logits are bit-identical (the FC tail runs on pn2's row kernel, which
    computes every row the same way on any stream)."""
    from pn2 import heads as H
    from pn2 import shard
    from pn2.pipeline import PipelinedForward
    torch.manual_seed(8)
    model = getattr(H, head)().eval()
    cases.randomize_bn(model, 8)
    model = model.to(DEV)
    kind = "onehot10" if head.startswith("Translation") else "uniform3"
    B, N = (8, 2048) if head == "ClsMSG" else (16, 1024)
    xs = [cases.cloud(kind, B, N, 90 + i).permute(0, 2, 1).contiguous().to(DEV) for i in range(4)]
    extras = None
    if head.startswith("Translation"):
        extras = [(torch.randn(B, 3, generator=torch.Generator().manual_seed(i)).to(DEV),) for i in range(4)]

    feats = []
    last_sa = model.sa3 if hasattr(model, "sa3") else model.sa2
    last_sa.register_forward_hook(lambda m, i, o: feats.append(o[1].cpu().numpy()))

    def first(o):
        return (o[0] if isinstance(o, tuple) else o).cpu().numpy()

    torch.manual_seed(31)
    with torch.no_grad(), shard.batch_shard(2 * B, B):
        want = [first(model(x, *(extras[i] if extras else ()))) for i, x in enumerate(xs)]
    rng_want = torch.randint(0, 1 << 30, (4,))
    want_f, feats[:] = list(feats), []
    torch.manual_seed(31)
    with shard.batch_shard(2 * B, B):
        got = [first(o) for o in PipelinedForward(model, geometry_cus=16, tail=tail).run(xs, extras)]
    rng_got = torch.randint(0, 1 << 30, (4,))
    np.testing.assert_array_equal(rng_got.numpy(), rng_want.numpy())
    assert len(feats) == len(want_f) == len(xs)
    for g, w in zip(feats, want_f):
        np.testing.assert_array_equal(g, w)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("head,tail", [("ClsSSG", True), ("ClsSSG", False), ("ClsMSG", True),
                                       ("TranslationSSG", True), ("RotationSSG", True)])
def test_graphed_pipeline_matches_eager(head, tail):
    """pn2.pipeline.GraphedPipeline (fps / SA / head replayed from HIP graphs on the geometry,
    compute and tail streams, two slots) returns the eager forwards' results for a sequence of
    batches -- the first batch eager, the rest replayed through both slots twice, under
    shard.batch_shard -- and walks the CPU generator exactly as the eager sequence does.  The
    cls heads return the last SA feature (l3f); every output is held bit-identical (the FC tail
    runs on pn2's row kernel).  A second run()
    replays without recapturing; an in-place BN change recaptures."""
    from pn2 import heads as H
    from pn2 import shard
    from pn2.pipeline import GraphedPipeline
    torch.manual_seed(8)
    model = getattr(H, head)().eval()
    cases.randomize_bn(model, 8)
    model = model.to(DEV)
    kind = "onehot10" if head in ("TranslationSSG", "RotationSSG") else "uniform3"
    B, N = (8, 2048) if head == "ClsMSG" else (16, 1024)
    xs = [cases.cloud(kind, B, N, 90 + i).permute(0, 2, 1).contiguous().to(DEV) for i in range(6)]
    extras = None
    if head.startswith("Translation"):
        extras = [(torch.randn(B, 3, generator=torch.Generator().manual_seed(i)).to(DEV),)
                  for i in range(6)]

    def as_np(o):
        return [t.cpu().numpy() for t in (o if isinstance(o, tuple) else (o,))
                if isinstance(t, torch.Tensor)]

    torch.manual_seed(31)
    with torch.no_grad(), shard.batch_shard(2 * B, B):
        want = [as_np(model(x, *(extras[i] if extras else ()))) for i, x in enumerate(xs)]
    rng_want = torch.randint(0, 1 << 30, (4,))

    gp = GraphedPipeline(model, geometry_cus=0 if tail else 16, tail=tail)
    torch.manual_seed(31)
    with shard.batch_shard(2 * B, B):
        got = [as_np(o) for o in gp.run(xs[:3], extras[:3] if extras else None)]
        slots = gp._slots
        got += [as_np(o) for o in gp.run(xs[3:], extras[3:] if extras else None)]
        assert gp._slots is slots  # replayed, not recaptured
    rng_got = torch.randint(0, 1 << 30, (4,))
    np.testing.assert_array_equal(rng_got.numpy(), rng_want.numpy())
    assert len(got) == len(want)
    if head.startswith("Cls"):  # l3f: the SA path, bit-exact
        for i, (g, w) in enumerate(zip(got, want)):
            np.testing.assert_array_equal(g[1], w[1], err_msg="l3f of batch %d" % i)
    for i, (g, w) in enumerate(zip(got, want)):
        assert len(g) == len(w)
        for k, (a, b) in enumerate(zip(g, w)):
            np.testing.assert_array_equal(a, b, err_msg="output %d of batch %d" % (k, i))

    # a parameter change recaptures and still matches eager
    next(b for n, b in model.sa1.named_buffers() if n.endswith("running_mean")).add_(0.25)
    torch.manual_seed(5)
    with torch.no_grad():
        want2 = [as_np(model(x, *(extras[i] if extras else ()))) for i, x in enumerate(xs[:3])]
    torch.manual_seed(5)
    old_sa = [sl.sa for grp in gp._slots for sl in grp.halves]
    got2 = [as_np(o) for o in gp.run(xs[:3], extras[:3] if extras else None)]
    # the sa / head graphs were recaptured (the geometry graphs read no parameters and stay)
    new_sa = [sl.sa for grp in gp._slots for sl in grp.halves]
    assert all(a is not b for a, b in zip(new_sa, old_sa))
    for g, w in zip(got2, want2):
        for a, b in zip(g, w):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("layout", ["contig", "tview"])
def test_graphed_pipeline_multihead_matches_eager(layout):
    """BASELINE config 4 (rotation_ssg + translation_ssg over the same clouds) as one
    pn2.pipeline.MultiHead: the FPS chain covers both heads (a group_all layer ends a head's
    chain, the next head restarts from the input; the heads' first FPS run as one launch over
    the repeated input), draws in the order separate eager calls take them, and every output
    matches those calls bit for bit.  tview: the input is the
    transpose view of [B, N, C] storage (the scripts' layout), which the repeated copy keeps."""
    from pn2 import heads as H
    from pn2 import shard
    from pn2.pipeline import GraphedPipeline, MultiHead
    torch.manual_seed(12)
    rot, tra = H.RotationSSG().eval(), H.TranslationSSG().eval()
    cases.randomize_bn(rot, 12)
    cases.randomize_bn(tra, 13)
    rot, tra = rot.to(DEV), tra.to(DEV)
    B, N = 8, 2048
    if layout == "tview":
        xs = [cases.cloud("onehot10", B, N, 70 + i).to(DEV).permute(0, 2, 1) for i in range(5)]
    else:
        xs = [cases.cloud("onehot10", B, N, 70 + i).permute(0, 2, 1).contiguous().to(DEV) for i in range(5)]
    means = [(torch.randn(B, 3, generator=torch.Generator().manual_seed(i)).to(DEV),) for i in range(5)]
    torch.manual_seed(41)
    with torch.no_grad(), shard.batch_shard(4 * B, 2 * B):
        want = [(rot(x).cpu().numpy(), tra(x, *m).cpu().numpy()) for x, m in zip(xs, means)]
    rng_want = torch.randint(0, 1 << 30, (4,))
    gp = GraphedPipeline(MultiHead([rot, tra], [1]))
    torch.manual_seed(41)
    with shard.batch_shard(4 * B, 2 * B):
        got = [tuple(t.cpu().numpy() for t in o) for o in gp.run(xs, means)]
    np.testing.assert_array_equal(torch.randint(0, 1 << 30, (4,)).numpy(), rng_want.numpy())
    for i, (g, w) in enumerate(zip(got, want)):
        for k, (a, b) in enumerate(zip(g, w)):
            np.testing.assert_array_equal(a, b, err_msg="head %d of batch %d" % (k, i))


@pytest.mark.parametrize("compute_streams,geometry_streams", [(1, 2), (2, 1), (2, 2)])
def test_graphed_pipeline_delayed_tail_matches_eager(compute_streams, geometry_streams):
    """A slow tail stream must not let a slot's next fps replay overwrite geometry that the slot's
    head graph still reads: with the group_all split, sa3 (in the head graph) reads sa2's
    centroids, a static output of the fps graph.  `post` runs on the tail stream and sleeps
    there, so every head replay starts late; the geometry streams run ahead as far as the
    events allow.  The l3 features must still be the eager bits.  compute_streams=2: the two
    batches of a geometry group run on different compute streams, and the group's next fps
    replay must wait for both; with two geometry streams too the heads run after their sa
    graph on the compute stream and `post` still on the tail stream, in batch order (the
    collective order every rank must keep)."""
    from pn2 import heads as H
    from pn2.pipeline import GraphedPipeline
    torch.manual_seed(8)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 8)
    model = model.to(DEV)
    B, N = 16, 1024
    xs = [cases.cloud("uniform3", B, N, 200 + i).permute(0, 2, 1).contiguous().to(DEV)
          for i in range(9)]
    torch.manual_seed(17)
    with torch.no_grad():
        want = [model(x)[1].cpu().numpy() for x in xs]

    def slow(i, o):
        torch.cuda._sleep(4_000_000)  # on the tail stream, before the next head replay
        return o

    gp = GraphedPipeline(model, tail=True, compute_streams=compute_streams,
                         geometry_streams=geometry_streams)
    assert gp._split_index() == 1  # sa3 (group_all) is in the head graph
    from pn2 import pipeline
    # the heads get their own stream(s) while every stream has a hardware queue
    assert gp.head_on_tail == (compute_streams + geometry_streams + gp.tail_streams <= pipeline._hw_queues())
    torch.manual_seed(17)
    got = [o[1].cpu().numpy() for o in gp.run(xs, post=slow)]
    for i, (g, w) in enumerate(zip(got, want)):
        np.testing.assert_array_equal(g, w, err_msg="l3f of batch %d" % i)


def test_eval_with_autograd_is_differentiable():
    """model.eval() without torch.no_grad() (mutilthreading/predict_test.py:44-63) is
    differentiable, as the reference's eval forward is: the torch device formulation, within the
    feature tolerance of the no_grad (fused) run, with weight gradients after a backward.
    Inside pn2.fused_eval() the same forward runs the fused split-bf16 kernels and gives the
    no_grad bits -- logits included (the FC tail takes the fused row kernel too) -- with no
    autograd history."""
    import pn2
    from pn2 import _lib
    from pn2 import heads as H
    torch.manual_seed(3)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 3)
    model = model.to(DEV)
    x = cases.cloud("uniform3", 4, 1024, 5).permute(0, 2, 1).contiguous().to(DEV)
    torch.manual_seed(1)
    with torch.no_grad():
        want = model(x)
    torch.manual_seed(1)
    got = model(x)  # autograd on, parameters require grad: the differentiable formulation
    assert got[0].requires_grad
    got[0].sum().backward()
    assert model.sa1.mlp_convs[0].weight.grad is not None
    assert model.sa3.mlp_convs[2].weight.grad is not None
    assert_feat_close(got[1].detach().cpu().numpy(), want[1].cpu().numpy())
    model.zero_grad()
    torch.manual_seed(1)
    with pn2.fused_eval():
        fz = model(x)
    assert _lib.load().pn2_sa_mlp_last_path() == _lib.PATH_SPLIT_BF16
    assert not fz[0].requires_grad
    for a, b in zip(fz, want):
        np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())


@pytest.mark.parametrize("head", ["ClsSSG", "ClsMSG"])
def test_graphed_pipeline_ball_query_in_forward_matches_eager(head):
    """tuning geometry_bq = 0: the geometry graph holds only the FPS launches and each batch's sa
    graph runs its layers' ball queries itself (the module queries when its provided entry holds
    no lists).  Results and generator state are still the eager ones, bit for bit."""
    from pn2 import heads as H
    from pn2 import tuning
    from pn2.pipeline import GraphedPipeline
    torch.manual_seed(8)
    model = getattr(H, head)().eval()
    cases.randomize_bn(model, 8)
    model = model.to(DEV)
    B, N = (8, 2048) if head == "ClsMSG" else (16, 1024)
    xs = [cases.cloud("uniform3", B, N, 300 + i).permute(0, 2, 1).contiguous().to(DEV) for i in range(5)]
    torch.manual_seed(23)
    with torch.no_grad():
        want = [[t.cpu().numpy() for t in model(x)] for x in xs]
    rng_want = torch.randint(0, 1 << 30, (4,))
    with tuning.override(geometry_bq=0):
        gp = GraphedPipeline(model)
        torch.manual_seed(23)
        got = [[t.cpu().numpy() for t in o] for o in gp.run(xs)]
        for ent in gp._slots[0].entries.values():
            assert ent[4] == []  # no ball query in the geometry graph
    np.testing.assert_array_equal(torch.randint(0, 1 << 30, (4,)).numpy(), rng_want.numpy())
    for i, (g, w) in enumerate(zip(got, want)):
        for k, (a, b) in enumerate(zip(g, w)):
            np.testing.assert_array_equal(a, b, err_msg="output %d of batch %d" % (k, i))


def test_graphed_pipeline_recaptures_geometry_on_sa_change():
    """the geometry graphs bake in each SA module's sampling / grouping
    configuration.  Replacing sa1 by a module with another radius, or changing sa2's radius in
    place, between pipelined runs recaptures them: the results equal the eager forwards', and
    the CPU generator walks as the eager sequence walks it."""
    from pn2 import heads as H
    from pn2.pipeline import GraphedPipeline
    from pn2.pointnet2_utils import PointNetSetAbstraction as SA
    torch.manual_seed(9)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 9)
    model = model.to(DEV)
    B, N = 8, 1024
    xs = [cases.cloud("uniform3", B, N, 70 + i).permute(0, 2, 1).contiguous().to(DEV) for i in range(4)]

    def check(gp):
        torch.manual_seed(12)
        with torch.no_grad():
            want = [model(x)[1].cpu() for x in xs]
        rng_want = torch.randint(0, 1 << 30, (4,))
        torch.manual_seed(12)
        got = [o[1].cpu() for o in gp.run(xs)]
        assert torch.equal(torch.randint(0, 1 << 30, (4,)), rng_want)
        for i, (g, w) in enumerate(zip(got, want)):
            assert torch.equal(g, w), "batch %d" % i

    gp = GraphedPipeline(model)
    check(gp)
    slots = gp._slots
    check(gp)
    assert gp._slots is slots  # replayed

    # a replaced module (new identity, another radius): found by the parameter check, the run
    # restarts with a full capture
    torch.manual_seed(3)
    new = SA(512, 32, 0.3, 3, [64, 64, 128], False).eval()
    cases.randomize_bn(new, 3)
    model.sa1 = new.to(DEV)
    check(gp)
    assert gp._slots is not slots and gp.sas[0] is model.sa1
    slots = gp._slots

    # an in-place change of a module's grouping: found by the input signature
    model.sa2.radius = 0.5
    check(gp)
    assert gp._slots is not slots
