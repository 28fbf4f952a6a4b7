"""CPU oracle for the PointNet++ set-abstraction path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker (never as the product).

Two parts:
  * ``libpn2_oracle.so`` (pn2_oracle.c): the exact float32 index path -- FPS,
    square_distance, ball query -- restated with the reference's rounding
    sequence (see the C file header for the rules and citations).
  * numpy restatements of the grouping and the shared-MLP + max of
    /root/reference/model/pointnet2_utils.py:92-223 in float64 (the float path is
    checked with a tolerance, not bit-for-bit).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libpn2_oracle.so")
_lib = None

_i64 = ctypes.c_int64
_fp = ctypes.POINTER(ctypes.c_float)
_ip = ctypes.POINTER(ctypes.c_int64)


def build():
    """Compile the C oracle (gcc) into oracle/_build/."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.pn2o_ssq.argtypes = [_fp, _i64, _i64, _i64, _i64, _i64, _i64, _fp]
        L.pn2o_fps.argtypes = [_fp, _i64, _i64, _i64, _i64, _i64, _i64, _ip, _i64, _ip]
        L.pn2o_ball_query.argtypes = [_fp, _i64, _i64, _i64, _i64, _i64, _i64,
                                      _fp, _i64, _i64, _i64, _i64, ctypes.c_double, _i64, _ip]
        L.pn2o_ball_query.restype = ctypes.c_int
        L.pn2o_square_distance.argtypes = [_fp, _i64, _i64, _i64, _i64, _i64, _i64,
                                           _fp, _i64, _i64, _i64, _i64, _fp]
        _lib = L
    return _lib


def _view(a):
    """(pointer, element strides) of a float32 numpy [B, N, C] view (any strides)."""
    assert a.dtype == np.float32 and a.ndim == 3
    st = [s // 4 for s in a.strides]
    return a.ctypes.data_as(_fp), st


def _np(t):
    """Accept numpy arrays or CPU torch tensors; keeps the strides of a view."""
    if hasattr(t, "detach"):
        t = t.detach().cpu().numpy()
    return t


def ssq(points):
    """torch.sum(points**2, -1) with the reference's layout-dependent order. [B,N,C] -> [B,N]."""
    p = _np(points)
    B, N, C = p.shape
    out = np.empty((B, N), np.float32)
    ptr, st = _view(p)
    lib().pn2o_ssq(ptr, B, N, C, st[0], st[1], st[2], out.ctypes.data_as(_fp))
    return out


def farthest_point_sample(points, number, start):
    """pointnet2_utils.py:47-68.  points [B,N,C] (any strides), start [B] int64 -> [B,number] int64."""
    p = _np(points)
    B, N, C = p.shape
    start = np.ascontiguousarray(_np(start), dtype=np.int64)
    out = np.empty((B, number), np.int64)
    ptr, st = _view(p)
    lib().pn2o_fps(ptr, B, N, C, st[0], st[1], st[2], start.ctypes.data_as(_ip), number,
                   out.ctypes.data_as(_ip))
    return out


def square_distance(src, dst):
    """pointnet2_utils.py:5-26, float32-exact.  src [B,S,C], dst [B,N,C] -> [B,S,N]."""
    s, d = _np(src), _np(dst)
    B, S, C = s.shape
    N = d.shape[1]
    out = np.empty((B, S, N), np.float32)
    sp, ss = _view(s)
    dp, ds = _view(d)
    lib().pn2o_square_distance(sp, B, S, C, ss[0], ss[1], ss[2], dp, N, ds[0], ds[1], ds[2],
                               out.ctypes.data_as(_fp))
    return out


def query_ball_point(radius, number, points, new_points):
    """pointnet2_utils.py:70-90.  Raises IndexError when number > N, like the reference."""
    p, q = _np(points), _np(new_points)
    B, N, C = p.shape
    S = q.shape[1]
    out = np.empty((B, S, number), np.int64)
    pp, ps = _view(p)
    qp, qs = _view(q)
    rc = lib().pn2o_ball_query(pp, B, N, C, ps[0], ps[1], ps[2], qp, S, qs[0], qs[1], qs[2],
                               float(radius), number, out.ctypes.data_as(_ip))
    if rc != 0:
        raise IndexError("query_ball_point: sample_number %d > N %d" % (number, N))
    return out


def index_points(points, idx):
    """pointnet2_utils.py:28-45: points[b, idx[b, ...], :]."""
    p = np.asarray(_np(points))
    idx = np.asarray(_np(idx))
    b = np.arange(p.shape[0]).reshape((-1,) + (1,) * (idx.ndim - 1))
    return p[b, idx, :]


def group(points, feature, idx, centers, feature_first=False):
    """sample_and_group grouping (pointnet2_utils.py:107-116) and the MSG variant
    (pointnet2_utils.py:204-209): [B,S,K,C(+D)], centred xyz, exact float32."""
    g = index_points(points, idx) - np.asarray(_np(centers))[:, :, None, :]
    if feature is None:
        return g
    f = index_points(feature, idx)
    return np.concatenate([f, g] if feature_first else [g, f], axis=-1)


def mlp_max(grouped, layers):
    """Shared 1x1-conv MLP + eval BatchNorm + ReLU, then max over the K axis
    (pointnet2_utils.py:167-172, 211-218), in float64.

    grouped: [B,S,K,Cin]; layers: list of dicts with numpy W [out,in], b, gamma, beta,
    mean, var, eps.  Returns [B,S,Cout] float64.
    """
    x = grouped.astype(np.float64)
    for L in layers:
        y = x @ L["W"].astype(np.float64).T + L["b"].astype(np.float64)
        inv = 1.0 / np.sqrt(L["var"].astype(np.float64) + L["eps"])
        y = (y - L["mean"]) * inv * L["gamma"] + L["beta"]
        x = np.maximum(y, 0.0)
    return x.max(axis=2)


def bf16_round(x):
    """float32 -> the nearest bfloat16 value (round-to-nearest-even), returned as float32."""
    b = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    b = (b + 0x7FFF + ((b >> 16) & 1)) & 0xFFFF0000
    return b.astype(np.uint32).view(np.float32)


def mlp_max_bf16(grouped, layers):
    """mlp_max in the bf16 arithmetic of pn2_sa_mlp_max_bf16 (BASELINE config 5; the reference
    has no bf16 path, so this defines it): every layer's float32 input and its weights are
    rounded to bfloat16 (RNE), the products summed exactly (float64 here, fp32 accumulation on
    the GPU), bias / BatchNorm / ReLU applied to the fp32 sum.  Returns [B,S,Cout] float64."""
    x = np.asarray(grouped, np.float32)
    for L in layers:
        W = bf16_round(L["W"]).astype(np.float64)
        y = bf16_round(x).astype(np.float64) @ W.T + L["b"].astype(np.float64)
        inv = 1.0 / np.sqrt(L["var"].astype(np.float64) + L["eps"])
        y = (y - L["mean"]) * inv * L["gamma"] + L["beta"]
        x = np.maximum(y, 0.0).astype(np.float32)
    return x.max(axis=2).astype(np.float64)


# ---------------------------------------------------------------------- input preparation
def normalization(point_cloud):
    """/root/reference/provider.py:5-21, restated with the same numpy calls (provider.py itself
    imports open3d, absent here, so it cannot be imported): per cloud, centroid = np.mean over
    points, centre, m = max of the Euclidean norms, divide.  float64 in, float64 out."""
    B, N, C = point_cloud.shape
    normalize = np.zeros((B, N, C))
    for i in range(B):
        pc = point_cloud[i]
        centroid = np.mean(pc, axis=0)
        pc = pc - centroid
        m = np.max(np.sqrt(np.sum(pc ** 2, axis=1)))
        pc = pc / m
        normalize[i] = pc
    return normalize


def prepare_points(points, labels=None, num_category=7, with_mean=False, normalize=True):
    """The scripts' preparation of a DataLoader batch (test_translation.py:72-79;
    test_rotation.py:71-77 and test_classification.py:71-72 without the mean / splice):
    float64 [B,N,C] numpy -> (float32 [B,N,C+K] storage of the model input, float32 mean [B,C]
    or None).  splice_torch (provider.py:166-180) appends the one-hot as float32 channels."""
    import torch
    points = np.array(points, dtype=np.float64, copy=True)
    mean = None
    if with_mean:
        mean = torch.Tensor(np.mean(points[:, :3, :], axis=1)).numpy()
    if normalize:
        points[:, :, 0:3] = normalization(points[:, :, 0:3])
    pts = torch.Tensor(points)
    if labels is not None and num_category:
        B, N, _ = pts.shape
        oh = torch.zeros(B, N, num_category)
        for i in range(B):
            oh[i, :, int(labels[i])] = 1
        pts = torch.cat([pts, oh], 2)
    return pts.numpy(), mean
