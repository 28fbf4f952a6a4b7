"""Input preparation on the GPU: the host-side steps the reference's
scripts run on every batch before the forward, as one kernel (csrc/preprocess.hip).

The reference does, per batch (test_translation.py:72-84; test_rotation.py:71-80 and
test_sign.py:69-76 without the mean; test_classification.py:71-78 without the splice):

    points = points.data.numpy()                                  # float64 [B,N,C]
    mean = torch.Tensor(np.mean(points[:,:3,:], axis=1))          # translation heads
    points[:, :, 0:3] = provider.normalization(points[:, :, 0:3]) # per-cloud numpy loop
    points = provider.splice_torch(torch.Tensor(points), label)   # per-cloud python loop
    points = points.transpose(2, 1).cuda()

``prepare_batch`` returns the same model input (bit-identical: float64 arithmetic in numpy's
operation order, one rounding to float32) and the same ``mean``, computed on the device from
the float64 batch (host or device tensor, or numpy array).  The points come back as the
reference's [B, C+K, N] view of [B, N, C+K] storage -- the layout its models receive, which
the SA path's FPS / ball-query sum orders depend on.
"""
import numpy as np
import torch

from . import _lib
from .ops import _stream


def prepare_batch(points, label=None, num_category=7, with_mean=False, normalize=True,
                  device=None):
    """points: float64 [B, N, C] (torch tensor on any device, or numpy), C >= 3.
    label: [B] class indices (one-hot spliced after the C channels when given; values must be
    in [0, num_category) -- the reference raises IndexError otherwise).
    Returns (model input [B, C+K, N] float32 on the device, mean [B, C] float32 or None)."""
    if isinstance(points, np.ndarray):
        points = torch.from_numpy(points)
    if points.dtype != torch.float64:
        raise TypeError("pn2.provider.prepare_batch: points must be float64 (np.loadtxt rows), "
                        "got %s" % points.dtype)
    if points.dim() != 3:
        raise ValueError("pn2.provider.prepare_batch: points must be [B, N, C]")
    B, N, C = points.shape
    if normalize and C < 3:
        raise ValueError("pn2.provider.prepare_batch: normalising needs C >= 3")
    K = 0
    lab = None
    if label is not None:
        lab = torch.as_tensor(label).reshape(-1).to(torch.int64)
        if lab.numel() != B:
            raise ValueError("pn2.provider.prepare_batch: %d labels for %d clouds" % (lab.numel(), B))
        # host labels (the DataLoader's) are range-checked like the reference; device labels
        # are not (that would synchronise): an out-of-range one gets an all-zero one-hot
        lab_host = lab if not lab.is_cuda else None
        if B and lab_host is not None and (int(lab_host.min()) < 0 or int(lab_host.max()) >= num_category):
            raise IndexError("index %d is out of bounds for dimension 1 with size %d" % (
                int(lab_host.max()) if int(lab_host.max()) >= num_category else int(lab_host.min()),
                num_category))
        K = int(num_category)
    if device is not None:
        dev = torch.device(device)
    elif points.is_cuda:
        dev = points.device
    elif torch.cuda.is_available():
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    if dev.type != "cuda":
        raise RuntimeError("pn2.provider.prepare_batch: runs on ROCm devices only (got %s); "
                           "there is no CPU path" % dev)
    if lab is not None:
        lab = lab.to(dev, non_blocking=True)
    pts = points.to(dev, non_blocking=True)
    out = torch.empty(B, N, C + K, dtype=torch.float32, device=dev)
    mean = torch.empty(B, C, dtype=torch.float32, device=dev) if with_mean else None
    if B and N:
        L = _lib.load()
        _lib.check(L.pn2_prepare_points_f64(
            pts.data_ptr(), B, N, C, pts.stride(0), pts.stride(1), pts.stride(2),
            1 if normalize else 0, 0 if lab is None else lab.data_ptr(), K, out.data_ptr(),
            0 if mean is None else mean.data_ptr(), _stream(out)), "pn2_prepare_points_f64")
    return out.transpose(2, 1), mean


__all__ = ["prepare_batch"]
