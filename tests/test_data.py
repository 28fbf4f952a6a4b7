"""Dataset text reader: libpn2io.so via pn2.data, against np.loadtxt
(the reference's parser, data_utils/ModelDataLoader.py:85-90) and the reference's own
ModelDataLoader on a synthetic dataset tree written the way data_build/Cube.py:90-94 writes
it.  CPU only; bar: bit-identical float64 values, same shapes, same numpy RNG consumption."""
import io
import os
import sys
from types import SimpleNamespace

import numpy as np
import pytest
import torch

import cases
from pn2 import data

REF = "/root/reference"


def _bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


def _write(path, text):
    with open(path, "w") as fh:
        fh.write(text)


@pytest.mark.parametrize("fmt", ["%6f", "%.17g", "%.6e", "%.3f", "%.9g"])
def test_loadtxt_bits_match_numpy(tmp_path, fmt):
    rng = np.random.default_rng(hash(fmt) % 1000)
    x = rng.standard_normal((1500, 3)) * 10.0 ** rng.uniform(-4, 4, (1500, 3))
    x[0, 0] = -0.0
    x[1, 1] = 1e-310  # subnormal
    p = tmp_path / "pts.txt"
    np.savetxt(p, x, fmt=fmt, delimiter=",")
    want = np.loadtxt(p, delimiter=",")
    got = data.loadtxt(str(p))
    assert got.shape == want.shape and got.dtype == np.float64
    np.testing.assert_array_equal(_bits(got), _bits(want))


def test_loadtxt_text_details_and_shapes(tmp_path):
    cases = {
        "one_row": "0.123456,-1.500000,2.000000\n",                   # -> (3,), like _rot.txt
        "one_col": "1\n2\n3\n",                                        # -> (3,)
        "scalar": "7.25\n",                                            # -> ()
        "blanks": " 1.0 , +2.5,\t-3e-2 \r\n\n# comment\n4,5,6 # tail\n",
        "special": "inf,-inf,1e400\n-0.0,1e-400,.5\n",
    }
    for name, text in cases.items():
        p = tmp_path / (name + ".txt")
        _write(p, text)
        want = np.loadtxt(p, delimiter=",")
        got = data.loadtxt(str(p))
        assert got.shape == want.shape, name
        np.testing.assert_array_equal(_bits(got), _bits(want), err_msg=name)


def test_loadtxt_errors(tmp_path):
    p = tmp_path / "ragged.txt"
    _write(p, "1,2,3\n4,5\n")
    with pytest.raises(ValueError):
        np.loadtxt(p, delimiter=",")
    with pytest.raises(ValueError):
        data.loadtxt(str(p))
    _write(p, "1,2,x\n")
    with pytest.raises(ValueError):
        data.loadtxt(str(p))
    with pytest.raises(OSError):
        data.loadtxt(str(tmp_path / "missing.txt"))


def test_load_many_threads(tmp_path):
    rng = np.random.default_rng(3)
    paths, arrs = [], []
    for i in range(23):
        a = rng.uniform(-1, 1, (int(rng.integers(1, 3000)), 3))
        p = tmp_path / ("f%d.txt" % i)
        np.savetxt(p, a, fmt="%6f", delimiter=",")
        paths.append(str(p))
        arrs.append(np.loadtxt(p, delimiter=",", ndmin=2))
    for threads in (1, 4, 0):
        got = data.load_many(paths, 3, threads=threads)
        for g, w in zip(got, arrs):
            np.testing.assert_array_equal(_bits(g), _bits(w))


def _make_tree(root, items, n_points=1300):
    """A few test-split items per class (ids 6002.. are test), written like data_build."""
    cases.write_dataset_tree(root, items, n_points)


def _ref_loader_module(monkeypatch):
    monkeypatch.setattr(sys, "dont_write_bytecode", True)
    monkeypatch.syspath_prepend(os.path.join(REF, "data_utils"))
    sys.modules.pop("ModelDataLoader", None)
    import importlib
    return importlib.import_module("ModelDataLoader")


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
def test_dataset_matches_reference(tmp_path, monkeypatch):
    root = str(tmp_path) + "/"
    _make_tree(root, [6002, 6003, 6004])
    args = SimpleNamespace(num_category=7)
    ref_mod = _ref_loader_module(monkeypatch)
    ref = ref_mod.ModelDataLoader(root=root, args=args, split="test")
    ours = data.ModelDataLoader(root=root, args=args, split="test")
    assert ours.datapath == ref.datapath and len(ours) == len(ref)
    train = data.ModelDataLoader(root=root, args=args, split="train")
    assert train.datapath == ref_mod.ModelDataLoader(root=root, args=args, split="train").datapath
    idx = [0, 1, 2, 1999, 2000, 2001, 13992]  # cube_6002..6004, cuboid_6002..
    idx = [i for i in idx if os.path.exists(ref.datapath[i][1])]
    np.random.seed(5)
    want = [ref[i] for i in idx]
    np.random.seed(5)
    got = [ours[i] for i in idx]
    for w, g in zip(want, got):
        np.testing.assert_array_equal(_bits(g[0]), _bits(w[0]))
        assert g[1] == w[1]
        for a, b in zip(g[2:], w[2:]):
            np.testing.assert_array_equal(_bits(a), _bits(b))
    # batch API == the reference dataset through a DataLoader (num_workers=0, no shuffle)
    np.random.seed(9)
    dl = torch.utils.data.DataLoader(torch.utils.data.Subset(ref, idx), batch_size=len(idx))
    wb = next(iter(dl))
    np.random.seed(9)
    gb = ours.load_batch(idx, threads=3)
    for a, b in zip(gb, wb):
        assert a.dtype == b.dtype and a.shape == b.shape
        np.testing.assert_array_equal(a.numpy(), b.numpy())


def _e2e_batch(tmp_path):
    """The E2E case's DataLoader batch through pn2.data (libpn2io reader, thread pool)."""
    e = cases.E2E_CASE
    root = str(tmp_path) + "/"
    cases.write_dataset_tree(root, e["items"])
    ds = data.ModelDataLoader(root=root, args=SimpleNamespace(num_category=7), split="test")
    np.random.seed(e["np_seed"])
    return ds.load_batch(list(e["index"]), threads=4)


def test_e2e_reader_and_oracle_preparation_match_reference(tmp_path):
    """f4 -> f2 on the CPU: the reader's batch, prepared by the oracle restatement of the
    scripts' steps, equals the reference's whole test-script input path (e2e.npz: the
    reference's ModelDataLoader + DataLoader + provider functions), bit for bit."""
    import oracle
    from conftest import load_golden
    g = load_golden("e2e.npz")
    points, label, rot, target, sign = _e2e_batch(tmp_path)
    np.testing.assert_array_equal(label.numpy(), g["label"])
    for a, k in ((rot, "rot"), (target, "target"), (sign, "sign")):
        np.testing.assert_array_equal(_bits(a.numpy()), _bits(g[k]))
    prepared, mean = oracle.prepare_points(points.numpy(), label.numpy(), 7, with_mean=True)
    np.testing.assert_array_equal(_bits(prepared.transpose(0, 2, 1)), _bits(g["prepared"]))
    np.testing.assert_array_equal(_bits(mean), _bits(g["mean"]))


@pytest.mark.gpu
def test_e2e_reader_prepare_head_on_gpu(tmp_path):
    """f4 -> f2 -> head on the GPU box: pn2.data reads the dataset tree, pn2.provider
    prepare_batch prepares it on the device (bit-exact to the reference's prepared input), and
    the translation_ssg head on the fused kernels reproduces the reference's prediction."""
    from conftest import load_golden
    from pn2 import heads as H
    from pn2.provider import prepare_batch
    e = cases.E2E_CASE
    g = load_golden("e2e.npz")
    points, label, rot, target, sign = _e2e_batch(tmp_path)
    x, mean = prepare_batch(points, label, with_mean=True)
    np.testing.assert_array_equal(_bits(x.cpu().numpy()), _bits(g["prepared"]))
    np.testing.assert_array_equal(_bits(mean.cpu().numpy()), _bits(g["mean"]))
    model = cases.build_head(H.HEADS[e["head"]], e["wseed"])
    assert cases.state_hash(model) == str(g["state_hash"])
    model = model.to("cuda").eval()
    torch.manual_seed(e["fseed"])
    with torch.no_grad():
        pred = model(x, mean)
    want = g["pred"]
    np.testing.assert_allclose(pred.cpu().numpy(), want, rtol=1e-4, atol=1e-4 * np.abs(want).max())
