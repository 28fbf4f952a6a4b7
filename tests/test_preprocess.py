"""Input preparation: pn2.provider.prepare_batch on the GPU against the
reference's own provider.normalization / splice_torch (tests/golden/prep_*.npz, made by
make_goldens.py from /root/reference/provider.py) and the oracle's numpy restatement.

Bar: bit-exact (float32 bits of the model input and of the translation heads' mean) -- the
kernel computes in float64 with numpy's operation order and rounds to float32 once."""
import numpy as np
import pytest
import torch

import cases
import oracle
from conftest import golden_names, load_golden


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


# ---------------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("name", golden_names("prep_"))
def test_oracle_matches_reference_preparation(name):
    g = load_golden("prep_%s.npz" % name)
    labels = g["labels"] if "labels" in g else None
    prepared, mean = oracle.prepare_points(g["raw"], labels, 7, with_mean=True)
    np.testing.assert_array_equal(_bits(prepared), _bits(g["prepared"]))
    np.testing.assert_array_equal(_bits(mean), _bits(g["mean"]))


def test_numpy_reduction_orders():
    """The orders the kernel restates (csrc/preprocess.hip header), probed on this numpy:
    axis-0 mean = sequential row sum / N; 3-column sum = (x + y) + z."""
    rng = np.random.default_rng(7)
    x = rng.standard_normal((4096, 3)) * 10.0 ** rng.uniform(-3, 3, (4096, 3))
    acc = x[0].copy()
    for i in range(1, len(x)):
        acc = acc + x[i]
    np.testing.assert_array_equal(np.mean(x, axis=0), acc / len(x))
    q = x ** 2
    np.testing.assert_array_equal(np.sum(q, axis=1), (q[:, 0] + q[:, 1]) + q[:, 2])
    p = rng.standard_normal((8, 50, 3)) * 100
    np.testing.assert_array_equal(np.mean(p[:, :3, :], axis=1), ((p[:, 0] + p[:, 1]) + p[:, 2]) / 3)


def test_prepare_batch_rejects_cpu_and_bad_input():
    from pn2.provider import prepare_batch
    x = torch.rand(2, 16, 3, dtype=torch.float64)
    with pytest.raises(TypeError):
        prepare_batch(x.float())
    with pytest.raises(IndexError):
        prepare_batch(x, label=[0, 7])  # the reference's class_vector[i, 7, :] raises
    with pytest.raises(RuntimeError, match="ROCm"):
        prepare_batch(x, device="cpu")


# ---------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_names("prep_"))
def test_prepare_batch_matches_reference(name):
    from pn2.provider import prepare_batch
    g = load_golden("prep_%s.npz" % name)
    labels = torch.from_numpy(g["labels"]) if "labels" in g else None
    for src in (torch.from_numpy(g["raw"]), torch.from_numpy(g["raw"]).cuda()):
        x, mean = prepare_batch(src, labels, with_mean=True)
        assert x.is_cuda and x.shape == (g["raw"].shape[0], g["prepared"].shape[2], g["raw"].shape[1])
        assert x.stride(1) == 1  # the reference's transpose(2,1) view of [B,N,C+K] storage
        np.testing.assert_array_equal(_bits(x.transpose(2, 1).cpu().numpy()), _bits(g["prepared"]))
        np.testing.assert_array_equal(_bits(mean.cpu().numpy()), _bits(g["mean"]))


@pytest.mark.gpu
@pytest.mark.parametrize("B,N,C,kind,strided", [(8, 16384, 3, "raw", False), (16, 2048, 3, "dup", True),
                                                 (5, 1, 3, "raw", False), (3, 777, 9, "raw", True)])
def test_prepare_batch_matches_oracle(B, N, C, kind, strided):
    from pn2.provider import prepare_batch
    raw = cases.raw_batch(kind, B, N, 50 + N, C)
    labels = np.arange(B) % 7
    want, want_mean = oracle.prepare_points(raw, labels, 7, with_mean=True)
    t = torch.from_numpy(raw).cuda()
    if strided:  # a [B,N,C] view of [B,C,N] storage
        t = t.permute(0, 2, 1).contiguous().permute(0, 2, 1)
    x, mean = prepare_batch(t, torch.from_numpy(labels), with_mean=True)
    np.testing.assert_array_equal(_bits(x.transpose(2, 1).cpu().numpy()), _bits(want))
    np.testing.assert_array_equal(_bits(mean.cpu().numpy()), _bits(want_mean))
    x2, none = prepare_batch(t, normalize=False)
    assert none is None
    np.testing.assert_array_equal(_bits(x2.transpose(2, 1).cpu().numpy()), _bits(raw.astype(np.float32)))


@pytest.mark.gpu
def test_prepared_batch_feeds_the_head_unchanged():
    """prepare_batch -> rotation_ssg forward == the reference-prepared input -> forward, bit for
    bit (same input bits, same layout, so the same FPS / ball-query sums)."""
    from pn2 import heads as H
    from pn2.provider import prepare_batch
    g = load_golden("prep_raw.npz")
    model = cases.build_head(H.HEADS["rotation_ssg"], 11).cuda().eval()
    x, _ = prepare_batch(torch.from_numpy(g["raw"]), torch.from_numpy(g["labels"]))
    ref = torch.from_numpy(g["prepared"]).transpose(2, 1).cuda()
    with torch.no_grad():
        torch.manual_seed(3)
        a = model(x)
        torch.manual_seed(3)
        b = model(ref)
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
