"""Generate the golden fixtures by running the REFERENCE (PyTorch-CPU) implementation.

Run only in the survey/build container, where /root/reference exists:
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py
It imports /root/reference/model/pointnet2_utils.py and the head modules read-only (no .pyc
writes) and stores inputs + the reference's outputs as .npz data under tests/golden/.
Nothing from the reference is copied: the fixtures are data only.

Files:
  index_<case>.npz  FPS indices / gathered centroids / ball-query indices / (small) square
                    distance matrices, for the cases in cases.INDEX_CASES
  head_<case>.npz   per-SA-layer outputs and head outputs for cases.HEAD_CASES (eval mode,
                    seeded weights + BN statistics; the weights are regenerated from the seed
                    and pinned by a state_dict SHA-256)
  full_<case>.npz   the same at the BASELINE shapes, for the heads without a small case and on
                    the reference's two real scans (cases.HEAD_FULL_CASES; features of a few
                    clouds per batch, centroids / last feature / outputs of all)
  v1_<case>.npz     PointNet-v1 heads (cases.V1_CASES): encoder / T-Net / head outputs
  e2e.npz           dataset tree -> ModelDataLoader -> preparation -> translation_ssg
                    (cases.E2E_CASE), the reference's whole test-script input path
  prep_<case>.npz   input preparation (cases.PREP_CASES) by provider.py's own functions
  train_<case>.npz  training-mode SA forward + backward (cases.TRAIN_CASES)
  sa_<case>.npz     eval-mode SA layers on points with C > 16 channels (cases.SA_WIDE_CASES)
(`make_goldens.py v1` regenerates only the v1 files, etc.)
  meta.json         torch version, CPU capability, MKL/oneDNN versions, thread count
"""
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
REF_MODEL = "/root/reference/model"

import numpy as np  # noqa: E402
import torch  # noqa: E402

import cases  # noqa: E402


def _ref():
    if REF_MODEL not in sys.path:
        sys.path.insert(0, REF_MODEL)
    import importlib
    return importlib.import_module("pointnet2_utils"), importlib


def _camera_cloud(kind, B, N):
    """The reference's two real scans (camera_test/*.txt, rows 'x,y,z,nx,ny,nz'): np.loadtxt,
    xyz columns, the reference's provider.normalization, float32; 'camera10' adds the one-hot
    of cases.CAMERA_LABELS with the reference's splice_torch.  -> [B, N, C] contiguous."""
    normalization, splice_torch = _provider_functions()
    assert B == len(cases.CAMERA_FILES)
    raw = np.stack([np.loadtxt(os.path.join(os.path.dirname(REF_MODEL), "camera_test", f),
                               delimiter=",")[:N, :3] for f in cases.CAMERA_FILES])
    assert raw.shape == (B, N, 3), raw.shape
    pts = torch.Tensor(normalization(raw))
    if kind == "camera10":
        pts = splice_torch(pts, torch.tensor(cases.CAMERA_LABELS))
    return pts.contiguous()


def _cloud(kind, B, N, seed):
    if kind.startswith("camera"):
        return _camera_cloud(kind, B, N)
    return cases.cloud(kind, B, N, seed)


def gen_index(P):
    for name, (kind, B, N, layout, S, bqs, seed) in cases.INDEX_CASES.items():
        if only_cases and name not in only_cases:
            continue
        pts = cases.as_layout(_cloud(kind, B, N, seed), layout)
        torch.manual_seed(seed + 1000)
        start = torch.randint(0, N, (B,), dtype=torch.long)
        torch.manual_seed(seed + 1000)
        fps_idx = P.farthest_point_sample(pts, S)  # draws the same start
        new_points = P.index_points(pts, fps_idx)
        rec = dict(points=pts.contiguous().numpy(), layout=np.array(layout), start=start.numpy(),
                   S=np.array(S), fps_idx=fps_idx.numpy().astype(np.int32),
                   new_points=new_points.numpy())
        for i, (r, K) in enumerate(bqs):
            try:
                g = P.query_ball_point(r, K, pts, new_points).numpy().astype(np.int32)
            except IndexError:
                g = np.full((0,), -1, np.int32)  # reference raises: K > N
            rec["bq%d_radius" % i] = np.array(r)
            rec["bq%d_K" % i] = np.array(K)
            rec["bq%d_idx" % i] = g
        if B * S * N <= 110_000:
            rec["sqdist"] = P.square_distance(new_points, pts).numpy()
        np.savez_compressed(os.path.join(HERE, "index_%s.npz" % name), **rec)
        print("index", name, {k: v.shape for k, v in rec.items() if hasattr(v, "shape")})


def gen_heads(importlib):
    for name, (head, B, N, kind, wseed, fseed) in cases.HEAD_CASES.items():
        mod = importlib.import_module(head)
        model = cases.build_head(mod.get_model, wseed)
        x = cases.cloud(kind, B, N, wseed + 7)            # [B,N,C]
        xin = x.permute(0, 2, 1).contiguous()             # [B,C,N] model input
        rec = {"input": xin.numpy(), "state_hash": np.array(cases.state_hash(model))}
        acts = {}

        def hook(tag):
            def f(_m, _inp, out):
                acts[tag] = (out[0].detach().contiguous().numpy(), out[1].detach().contiguous().numpy())
            return f
        for tag in ("sa1", "sa2", "sa3"):
            if hasattr(model, tag):
                getattr(model, tag).register_forward_hook(hook(tag))
        args = [xin]
        if head.startswith("translation"):
            mean = torch.randn(B, 3, generator=torch.Generator().manual_seed(wseed + 9))
            rec["mean"] = mean.numpy()
            args.append(mean)
        torch.manual_seed(fseed)
        with torch.no_grad():
            out = model(*args)
        outs = out if isinstance(out, tuple) else (out,)
        for i, o in enumerate(outs):
            rec["out%d" % i] = o.detach().numpy()
        for tag, (p, f) in acts.items():
            rec[tag + "_points"] = p
            rec[tag + "_feature"] = f
        np.savez_compressed(os.path.join(HERE, "head_%s.npz" % name), **rec)
        print("head", name, {k: v.shape for k, v in rec.items() if hasattr(v, "shape")})


def gen_full(importlib):
    """cases.HEAD_FULL_CASES: the reference heads at the BASELINE shapes, the heads without a
    small case (translation_msg, sign_ssg, sign_msg) and the two real scans.  Stored: every
    layer's centroids and the last SA layer's feature for the whole batch, sa1/sa2 features of
    the `keep` clouds, the head outputs; the input itself only for the scans (synthetic clouds
    are regenerated from their seed and pinned by a SHA-256)."""
    import types
    for name, (head, B, N, kind, wseed, fseed, keep) in cases.HEAD_FULL_CASES.items():
        if only_cases and name not in only_cases:
            continue
        mod = importlib.import_module(head)
        if not hasattr(mod, "torch"):  # sign_*.py use torch without importing it (sign_ssg.py:1-3, 34)
            mod.torch = torch
        assert isinstance(mod, types.ModuleType)
        model = cases.build_head(mod.get_model, wseed)
        x = _cloud(kind, B, N, wseed + 7)               # [B,N,C]
        xin = x.permute(0, 2, 1).contiguous()           # [B,C,N] model input
        rec = {"state_hash": np.array(cases.state_hash(model)),
               "input_hash": np.array(cases.tensor_hash(xin))}
        if kind.startswith("camera"):
            rec["input"] = xin.numpy()
        acts = {}
        tags = [t for t in ("sa1", "sa2", "sa3") if hasattr(model, t)]

        def hook(tag):
            def f(_m, _inp, out):
                acts[tag] = (out[0].detach().contiguous().numpy(), out[1].detach().contiguous().numpy())
            return f
        for tag in tags:
            getattr(model, tag).register_forward_hook(hook(tag))
        args = [xin]
        if head.startswith("translation"):
            mean = torch.randn(B, 3, generator=torch.Generator().manual_seed(wseed + 9))
            rec["mean"] = mean.numpy()
            args.append(mean)
        torch.manual_seed(fseed)
        with torch.no_grad():
            out = model(*args)
        outs = out if isinstance(out, tuple) else (out,)
        for i, o in enumerate(outs):
            rec["out%d" % i] = o.detach().numpy()
        kept = np.arange(B) if keep is None else np.array(keep)
        rec["keep"] = kept
        for tag, (p, f) in acts.items():
            rec[tag + "_points"] = p
            rec[tag + "_feature"] = f if tag == tags[-1] else f[kept]
        np.savez_compressed(os.path.join(HERE, "full_%s.npz" % name), **rec)
        print("full", name, {k: v.shape for k, v in rec.items() if hasattr(v, "shape")})


def gen_e2e(importlib):
    """The test script's whole input path (test_translation.py:70-83) by the reference: its
    ModelDataLoader over a synthetic dataset tree (cases.write_dataset_tree), a DataLoader
    batch, the provider preparation, and the translation_ssg head -> e2e.npz (prepared input,
    mean, targets, prediction)."""
    import tempfile
    from types import SimpleNamespace
    e = cases.E2E_CASE
    normalization, splice_torch = _provider_functions()
    sys.path.insert(0, os.path.join(os.path.dirname(REF_MODEL), "data_utils"))
    loader_mod = importlib.import_module("ModelDataLoader")
    head = importlib.import_module(e["head"])
    with tempfile.TemporaryDirectory() as root:
        root = root + "/"
        cases.write_dataset_tree(root, e["items"])
        ds = loader_mod.ModelDataLoader(root=root, args=SimpleNamespace(num_category=7), split="test")
        np.random.seed(e["np_seed"])
        dl = torch.utils.data.DataLoader(torch.utils.data.Subset(ds, list(e["index"])),
                                         batch_size=len(e["index"]))
        points, label, rot, target, sign = next(iter(dl))
    points = points.data.numpy()
    mean = torch.Tensor(np.mean(points[:, :3, :], axis=1))
    points[:, :, 0:3] = normalization(points[:, :, 0:3])
    points = torch.Tensor(points)
    points = splice_torch(points, label)
    points = points.transpose(2, 1)
    model = cases.build_head(head.get_model, e["wseed"])
    torch.manual_seed(e["fseed"])
    with torch.no_grad():
        pred = model(points, mean)
    rec = {"prepared": points.contiguous().numpy(), "mean": mean.numpy(), "label": label.numpy(),
           "target": target.numpy(), "rot": rot.numpy(), "sign": sign.numpy(),
           "pred": pred.numpy(), "state_hash": np.array(cases.state_hash(model))}
    np.savez_compressed(os.path.join(HERE, "e2e.npz"), **rec)
    print("e2e", {k: v.shape for k, v in rec.items()})


def gen_v1(importlib):
    """PointNet-v1 heads (pointnet_utils.py + pointnet_cls / rotation / translation / sign):
    the encoder's (global feature, input transform, feature transform), the T-Nets' outputs and
    the head outputs, eval mode.  sign.py misses `import torch` (sign.py:1-3, like sign_ssg), so
    the harness sets it on the module without editing the file."""
    for name, (head, B, N, kind, wseed, kw) in cases.V1_CASES.items():
        mod = importlib.import_module(head)
        if not hasattr(mod, "torch"):
            mod.torch = torch
        model = cases.build_head(mod.get_model, wseed, **kw)
        x = cases.cloud(kind, B, N, wseed + 7)
        xin = x.permute(0, 2, 1).contiguous()
        rec = {"input": xin.numpy(), "state_hash": np.array(cases.state_hash(model))}
        acts = {}

        def hook(tag):
            def f(_m, _inp, out):
                outs = out if isinstance(out, tuple) else (out,)
                for i, o in enumerate(outs):
                    acts["%s_%d" % (tag, i)] = o.detach().contiguous().numpy()
            return f
        for tag, sub in (("feat", "feat"), ("tnet", "feat.tnet"), ("ftnet", "feat.ftnet"),
                         ("ftnet", "ftnet"), ("tnet", "tnet")):
            m = model
            try:
                for part in sub.split("."):
                    m = getattr(m, part)
            except AttributeError:
                continue
            m.register_forward_hook(hook(tag))
        args = [xin]
        if head == "translation":
            mean = torch.randn(B, 3, generator=torch.Generator().manual_seed(wseed + 9))
            rec["mean"] = mean.numpy()
            args.append(mean)
        with torch.no_grad():
            out = model(*args)
        outs = out if isinstance(out, tuple) else (out,)
        for i, o in enumerate(outs):
            rec["out%d" % i] = o.detach().numpy()
        rec.update(acts)
        np.savez_compressed(os.path.join(HERE, "v1_%s.npz" % name), **rec)
        print("v1", name, {k: v.shape for k, v in rec.items() if hasattr(v, "shape")})


def _provider_functions():
    """normalization / splice_torch from /root/reference/provider.py.  The module imports
    open3d (absent here), so the two functions are compiled from its source text alone (read
    only, nothing copied into the repository) and run with numpy / torch."""
    import ast
    src = open(os.path.join(os.path.dirname(REF_MODEL), "provider.py")).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef)
            and n.name in ("normalization", "splice_torch")]
    ns = {"np": np, "torch": torch}
    exec(compile(ast.Module(body=keep, type_ignores=[]), "provider.py", "exec"), ns)
    return ns["normalization"], ns["splice_torch"]


def gen_prep():
    """The scripts' input preparation (test_translation.py:72-79) with the reference's own
    provider functions: mean of the first 3 points, normalization, float32 cast, splice."""
    normalization, splice_torch = _provider_functions()
    for name, (kind, B, N, C, seed, with_labels) in cases.PREP_CASES.items():
        raw = cases.raw_batch(kind, B, N, seed, C)
        labels = torch.arange(B) % 7 if with_labels else None
        points = raw.copy()
        mean = torch.Tensor(np.mean(points[:, :3, :], axis=1))
        points[:, :, 0:3] = normalization(points[:, :, 0:3])
        points = torch.Tensor(points)
        if labels is not None:
            points = splice_torch(points, labels)
        rec = {"raw": raw, "mean": mean.numpy(), "prepared": points.contiguous().numpy()}
        if labels is not None:
            rec["labels"] = labels.numpy()
        np.savez_compressed(os.path.join(HERE, "prep_%s.npz" % name), **rec)
        print("prep", name, {k: v.shape for k, v in rec.items()})


def gen_train(P):
    """Training-mode forward + backward of SA layers with the reference modules: outputs,
    parameter / feature gradients of loss = sum(out_feature * R), running statistics after."""
    for name, (kind, args, B, N, D, wseed, fseed) in cases.TRAIN_CASES.items():
        ctor = P.PointNetSetAbstraction if kind == 'ssg' else P.PointNetSetAbstractionMsg
        torch.manual_seed(wseed)
        mod = ctor(*args)
        cases.randomize_bn(mod, wseed + 1)
        mod.train()
        pts, feat = cases.train_inputs(B, N, D, wseed + 2)
        rec = {"points": pts.numpy(), "state_hash": np.array(cases.state_hash(mod))}
        if feat is not None:
            rec["feature"] = feat.numpy()
            feat = feat.clone().requires_grad_(True)
        torch.manual_seed(fseed)
        new_points, new_feature = mod(pts, feat)
        R = torch.randn(new_feature.shape, generator=torch.Generator().manual_seed(wseed + 3))
        (new_feature * R).sum().backward()
        rec["new_points"] = new_points.detach().numpy()
        rec["new_feature"] = new_feature.detach().numpy()
        rec["R"] = R.numpy()
        if feat is not None:
            rec["feature_grad"] = feat.grad.numpy()
        for k, p in mod.named_parameters():
            rec["grad." + k] = p.grad.numpy()
        for k, b in mod.named_buffers():
            rec["buf." + k] = b.numpy()
        np.savez_compressed(os.path.join(HERE, "train_%s.npz" % name), **rec)
        print("train", name, {k: v.shape for k, v in rec.items() if hasattr(v, "shape")})


def gen_sa(P):
    """Eval-mode SA layers on points with more than 16 channels (cases.SA_WIDE_CASES): the
    reference module's centroids and features."""
    for name, (kind, args, B, N, C, D, wseed, fseed) in cases.SA_WIDE_CASES.items():
        if only_cases and name not in only_cases:
            continue
        ctor = P.PointNetSetAbstraction if kind == 'ssg' else P.PointNetSetAbstractionMsg
        torch.manual_seed(wseed)
        mod = ctor(*args)
        cases.randomize_bn(mod, wseed + 1)
        mod.eval()
        pts, feat = cases.sa_inputs(B, N, C, D, wseed + 2)
        rec = {"points": pts.numpy(), "state_hash": np.array(cases.state_hash(mod))}
        if feat is not None:
            rec["feature"] = feat.numpy()
        torch.manual_seed(fseed)
        with torch.no_grad():
            new_points, new_feature = mod(pts, feat)
        rec["new_points"] = new_points.numpy()
        rec["new_feature"] = new_feature.numpy()
        np.savez_compressed(os.path.join(HERE, "sa_%s.npz" % name), **rec)
        print("sa", name, {k: v.shape for k, v in rec.items() if hasattr(v, "shape")})


def _v1_step_record(model, x, Rs, prefix, rec):
    """One train step of a v1 head (loss = sum_i out_i * R_i; R drawn here when Rs is empty):
    outputs, parameter gradients (large ones as a fixed sample + norm) under `prefix`."""
    out = model(x)
    outs = [o for o in (out if isinstance(out, tuple) else (out,))
            if torch.is_tensor(o) and o.is_floating_point() and o.requires_grad]
    loss = 0
    for i, o in enumerate(outs):
        if len(Rs) <= i:
            Rs.append(torch.randn(o.shape, generator=torch.Generator().manual_seed(len(Rs) + 77)))
        loss = loss + (o * Rs[i].to(o.dtype)).sum()
        rec[prefix + "out%d" % i] = o.detach().float().numpy()
    loss.backward()
    for k, p in model.named_parameters():
        if p.grad is None:
            continue
        gr = p.grad.float().numpy()
        if gr.size > cases.GRAD_FULL_MAX:  # the FC / conv3 weights: a fixed sample + norm
            rec[prefix + "gsub." + k] = gr.reshape(-1)[cases.grad_sample_index(gr.size)]
            rec[prefix + "gnorm." + k] = np.array(np.linalg.norm(p.grad.double().numpy()))
        else:
            rec[prefix + "grad." + k] = gr
    return len(outs)


def _v1_min_gap(model):
    """Forward hooks on the BatchNorm before each max over the points: the smallest relative
    gap between a (cloud, channel)'s two largest (ReLU'd, except the encoder's conv3) values."""
    gaps = []
    last = "bn_conv.%d" % (len(getattr(model, "conv", [])) - 1)
    for k, m in model.named_modules():
        if not (k.endswith("bn3") or k == last):
            continue
        signed = k.endswith("feat.bn3") or k == "bn3"

        def f(_m, _i, out, signed=signed):
            h = out.detach() if signed else torch.relu(out.detach())
            t2 = torch.topk(h, 2, dim=2)[0]
            rel = (t2[..., 0] - t2[..., 1]) / t2[..., 0].abs().clamp_min(1e-300)
            rel = rel.flatten() if signed else rel[t2[..., 0] > 0]
            if rel.numel():
                gaps.append(float(rel.min()))
        m.register_forward_hook(f)
    return gaps


def gen_train_v1(importlib):
    """Training-mode forward + backward of the PointNet-v1 heads with the reference modules
    (pointnet_utils.py T-Nets / encoder and the heads' conv stacks): outputs, every parameter
    gradient and the running statistics after the step, in float32 (the reference as it runs)
    and the same step in float64 ("t." keys: the precision reference the GPU test measures
    against -- these deep T-Net networks amplify float32 rounding to ~1e-3 in some gradients,
    the reference's own float32 step included)."""
    for name, (head, B, N, kind, wseed, kw) in cases.TRAIN_V1_CASES.items():
        mod = importlib.import_module(head)
        model = cases.train_v1_model(mod.get_model, wseed, **kw)
        x = cases.cloud(kind, B, N, wseed + 7).permute(0, 2, 1).contiguous()
        rec = {"input": x.numpy(), "state_hash": np.array(cases.state_hash(model))}
        Rs = []
        n = _v1_step_record(model, x, Rs, "", rec)
        for i, R in enumerate(Rs):
            rec["R%d" % i] = R.numpy()
        for k, b in model.named_buffers():
            rec["buf." + k] = b.numpy()
        m64 = cases.train_v1_model(mod.get_model, wseed, **kw).double()
        gaps = _v1_min_gap(m64)
        _v1_step_record(m64, x.double(), Rs, "t.", rec)
        rec["min_gap"] = np.array(min(gaps))
        assert min(gaps) >= cases.TRAIN_V1_MIN_GAP, (name, gaps)
        np.savez_compressed(os.path.join(HERE, "trainv1_%s.npz" % name), **rec)
        print("trainv1", name, n, "outputs, min gap %.1e" % min(gaps))


only_cases = set()  # `make_goldens.py full cls_ssg_b32`: just these cases of the chosen kinds


def main():
    torch.set_num_threads(8)
    P, importlib = _ref()
    kinds = ("index", "heads", "full", "e2e", "v1", "prep", "train", "trainv1", "sa")
    only = [a for a in sys.argv[1:] if a in kinds]
    only_cases.update(a for a in sys.argv[1:] if a not in kinds)
    if not only or "index" in only:
        gen_index(P)
    if not only or "heads" in only:
        gen_heads(importlib)
    if not only or "full" in only:
        gen_full(importlib)
    if not only or "e2e" in only:
        gen_e2e(importlib)
    if not only or "v1" in only:
        gen_v1(importlib)
    if not only or "prep" in only:
        gen_prep()
    if not only or "train" in only:
        gen_train(P)
    if not only or "trainv1" in only:
        gen_train_v1(importlib)
    if not only or "sa" in only:
        gen_sa(P)
    meta = {
        "torch": torch.__version__,
        "cpu_capability": torch.backends.cpu.get_cpu_capability(),
        "threads": torch.get_num_threads(),
        "config": torch.__config__.show().splitlines()[:12],
        "generator": "tests/golden/make_goldens.py (reference imported read-only from %s)" % REF_MODEL,
    }
    with open(os.path.join(HERE, "meta.json"), "w") as fh:
        json.dump(meta, fh, indent=1)


if __name__ == "__main__":
    main()
