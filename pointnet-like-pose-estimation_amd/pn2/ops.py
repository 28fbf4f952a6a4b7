"""PyTorch custom ops (namespace ``pn2``) over the libpn2.so C ABI.

Each op takes/returns torch tensors, checks shapes in Python (raising the exception the
reference raises for the same misuse), and calls the HIP entry point asynchronously on torch's
current stream.  ``<op>_direct`` is the same function without the torch.library dispatcher
(the SA modules' eager path calls it: the dispatcher costs more host time per call than the
kernels it launches take on the GPU at these sizes).  Device tensors only: there is no CPU implementation and no fallback -- a CPU
tensor or a missing library is an error.

Ops (reference code each replaces, in /root/reference/model/pointnet2_utils.py):
  pn2::fps            farthest_point_sample :47-68 (+ index_points of the samples, :106)
  pn2::pack_points    the torch.sum(points**2, -1) terms of square_distance :24-25
  pn2::ball_query     query_ball_point :70-90
  pn2::square_distance square_distance :5-26
  pn2::index_points   index_points :28-45
  pn2::group          grouping in sample_and_group :107-116 / the MSG module :204-209
  pn2::pack_layer     Conv2d 1x1 + BatchNorm2d (eval) parameters :150-156, :184-193
  pn2::sa_mlp_max_    gathered shared MLP + max :167-172, :211-218 (writes into `out`)
"""
import contextlib
import ctypes
import threading
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from ._lib import MlpLayer, SaSrc, check, load

_L = load()  # fail at import, loudly, if the native library is unavailable

# ------------------------------------------------------------------------------ MLP precision
# "fp32": the reference's arithmetic (split-bf16 products at fp32 accuracy, or fp32 MFMA);
# "bf16": bf16 operands, fp32 accumulation (BASELINE config 5) -- an explicit caller choice.
PRECISIONS = ("fp32", "bf16")
_prec = threading.local()


def current_precision() -> str:
    return getattr(_prec, "value", "fp32")


@contextlib.contextmanager
def mlp_precision(precision: str):
    """Within this context (this thread) SA modules without their own ``mlp_precision``
    attribute run their shared MLPs at `precision` ("fp32" or "bf16")."""
    if precision not in PRECISIONS:
        raise ValueError("pn2: precision must be one of %s, got %r" % (PRECISIONS, precision))
    prev = current_precision()
    _prec.value = precision
    try:
        yield
    finally:
        _prec.value = prev


class KernelTimer:
    """HIP-event timing of every libpn2 launch, recorded on the stream the launch is issued on
    (torch's current stream), with each launch's algorithmic FLOPs / bytes and, for the MLP
    calls, the planes per operand its kernels ran with (pn2_sa_mlp_last_planes)."""

    def __init__(self):
        self.records = []  # (name, start_event, end_event, flops, bytes[, planes])

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for rec in self.records:
            name, e0, e1, flops, nbytes = rec[:5]
            d = out.setdefault(name, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0,
                                      "flops_by_planes": {}})
            d["launches"] += 1
            d["ms"] += e0.elapsed_time(e1)
            d["flops"] += flops
            d["bytes"] += nbytes
            if len(rec) > 5:
                fp = d["flops_by_planes"]
                fp[rec[5]] = fp.get(rec[5], 0.0) + flops
        return out


_TIMER = None


@contextlib.contextmanager
def kernel_timer():
    """Within this context every pn2 op launch is bracketed by HIP events."""
    global _TIMER
    prev, _TIMER = _TIMER, KernelTimer()
    try:
        yield _TIMER
    finally:
        _TIMER = prev


def _run(name, fn, args, device, flops=0.0, nbytes=0.0):
    t = _TIMER
    if t is None:
        check(fn(*args), name)
        return
    s = torch.cuda.current_stream(device)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(s)
    rc = fn(*args)
    e1.record(s)
    check(rc, name)
    t.records.append((name, e0, e1, float(flops), float(nbytes)))


def _dev(t: Tensor, what: str):
    if t.device.type != "cuda":
        raise RuntimeError("%s: pn2 runs on ROCm device tensors only (got %s); there is no CPU "
                           "path" % (what, t.device))
    if t.dtype != torch.float32 and t.dtype != torch.int64:
        raise TypeError("%s: unsupported dtype %s" % (what, t.dtype))


def _stream(t: Tensor) -> int:
    # this thread's device error slot first (a dict lookup once bound): kernels raise into it
    return _lib.stream_ptr(t.device)


def packed_stride(C: int) -> int:
    return int(_L.pn2_packed_stride(C))


def cin_pad(cin: int) -> int:
    return int(_L.pn2_layer_cin_pad(cin))


# ------------------------------------------------------------------------------ fps
def fps_direct(points: Tensor, npoint: int, start: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """points [B,N,C] float32 (any strides), start [B] int64 -> (fps_idx [B,S] int64,
    new_points [B,S,C], packed centroids [B,S,cp], packed points [B,N,cp]).  A CPU start (the
    reference's host draw) goes to pn2_fps_host_ws_f32 in the launch's arguments; a device start
    (and any start under graph capture, whose replays must read a device slot) to pn2_fps_ws_f32."""
    _dev(points, "pn2::fps")
    B, N, C = points.shape
    cp = packed_stride(C)
    host = start.device.type == "cpu" and not torch.cuda.is_current_stream_capturing()
    if host:
        start = start.to(dtype=torch.int64).contiguous()
    else:
        start = start.to(device=points.device, dtype=torch.int64).contiguous()
    idx = torch.empty(B, npoint, dtype=torch.int64, device=points.device)
    newp = torch.empty(B, npoint, C, dtype=torch.float32, device=points.device)
    cpk = torch.empty(B, npoint, cp, dtype=torch.float32, device=points.device)
    ppk = torch.empty(B, N, cp, dtype=torch.float32, device=points.device)
    sb, sn, sc = points.stride()
    # past the register-resident shapes (N > 16384, npoint > 8192) the streamed kernel; past
    # N = 40896 it keeps the running distances in this workspace
    nws = int(_L.pn2_fps_workspace_bytes(B, N, C, npoint))
    ws = torch.empty(max(nws, 0) // 4, dtype=torch.float32, device=points.device) if nws > 0 else None
    _run("pn2_fps_f32", _L.pn2_fps_host_ws_f32 if host else _L.pn2_fps_ws_f32,
         (points.data_ptr(), B, N, C, sb, sn, sc, start.data_ptr(), npoint, idx.data_ptr(),
          newp.data_ptr(), cpk.data_ptr(), ppk.data_ptr(), 0 if ws is None else ws.data_ptr(),
          max(nws, 0), _stream(points)), points.device,
         flops=float(B) * npoint * N * (3 * C + 2))
    return idx, newp, cpk, ppk


fps = torch.library.custom_op("pn2::fps", fps_direct, mutates_args=())


@fps.register_fake
def _(points, npoint, start):
    B, N, C = points.shape
    cp = packed_stride(C)
    e = points.new_empty
    return (e(B, npoint, dtype=torch.int64), e(B, npoint, C), e(B, npoint, cp), e(B, N, cp))


# ------------------------------------------------------------------------------ pack_points
def pack_points_direct(points: Tensor) -> Tensor:
    """[B,N,C] (any strides) -> [B,N,cp] records (coords, ssq in the reference's order, pad)."""
    _dev(points, "pn2::pack_points")
    B, N, C = points.shape
    out = torch.empty(B, N, packed_stride(C), dtype=torch.float32, device=points.device)
    sb, sn, sc = points.stride()
    _run("pn2_pack_points_f32", _L.pn2_pack_points_f32,
         (points.data_ptr(), B, N, C, sb, sn, sc, out.data_ptr(), _stream(points)), points.device)
    return out


pack_points = torch.library.custom_op("pn2::pack_points", pack_points_direct, mutates_args=())


@pack_points.register_fake
def _(points):
    B, N, C = points.shape
    return points.new_empty(B, N, packed_stride(C))


# ------------------------------------------------------------------------------ ball query
def ball_query_direct(pts_packed: Tensor, ctr_packed: Tensor, C: int, radius: float, nsample: int,
                      with_count: bool = False):
    """Packed points [B,N,cp] and centroids [B,S,cp] -> group_idx [B,S,nsample] int64 (the
    reference's query_ball_point); with with_count the SA layers' fused-path form: the lists as
    int32 (half the bytes; sa_mlp_max_direct reads either) and the distinct neighbours per
    centroid, [B,S] int32 (entries past them repeat entry 0; sa_mlp_max_direct(cnt=...) then
    computes only those rows)."""
    _dev(pts_packed, "pn2::ball_query")
    B, N, _ = pts_packed.shape
    S = ctr_packed.shape[1]
    if nsample > N:
        # the reference's `group_idx[mask] = group_first[mask]` fails the same way (:89)
        raise IndexError("query_ball_point: sample_number %d > number of points %d" % (nsample, N))
    out = torch.empty(B, S, nsample, dtype=torch.int32 if with_count else torch.int64,
                      device=pts_packed.device)
    cnt = torch.empty(B, S, dtype=torch.int32, device=pts_packed.device) if with_count else None
    cp = pts_packed.shape[2]
    fn = _L.pn2_ball_query_i32 if with_count else _L.pn2_ball_query_cnt_f32
    _run("pn2_ball_query_f32", fn,
         (pts_packed.data_ptr(), ctr_packed.data_ptr(), B, N, S, C, float(radius), nsample,
          out.data_ptr(), 0 if cnt is None else cnt.data_ptr(), _stream(pts_packed)),
         pts_packed.device, nbytes=4.0 * cp * B * (N + S) + out.element_size() * B * S * nsample +
         (4.0 * B * S if with_count else 0.0),
         flops=float(B) * S * N * (2 * C + 3))  # pairs x (2C + 3)
    return (out, cnt) if with_count else out


def ball_query_multi_direct(pts_packed: Tensor, ctr_packed: Tensor, C: int, radii, nsamples):
    """ball_query_direct(..., with_count=True) for several radii of one centroid set (an MSG
    layer's scales) in one launch (pn2_ball_query_multi_i32, up to 3 radii per launch): a list of
    (group_idx [B,S,nsample] int32, counts [B,S] int32), the same as one call per radius."""
    _dev(pts_packed, "pn2::ball_query")
    B, N, cp = pts_packed.shape
    S = ctr_packed.shape[1]
    res = []
    for i0 in range(0, len(radii), 3):
        rs, ks = list(radii[i0:i0 + 3]), list(nsamples[i0:i0 + 3])
        for k in ks:
            if k > N:
                raise IndexError("query_ball_point: sample_number %d > number of points %d" % (k, N))
        outs = [torch.empty(B, S, k, dtype=torch.int32, device=pts_packed.device) for k in ks]
        cnts = [torch.empty(B, S, dtype=torch.int32, device=pts_packed.device) for _ in ks]
        nr = len(ks)
        radii_c = (ctypes.c_double * nr)(*[float(r) for r in rs])
        ks_c = (ctypes.c_int64 * nr)(*[int(k) for k in ks])
        outs_c = (ctypes.c_void_p * nr)(*[t.data_ptr() for t in outs])
        cnts_c = (ctypes.c_void_p * nr)(*[t.data_ptr() for t in cnts])
        _run("pn2_ball_query_f32", _L.pn2_ball_query_multi_i32,
             (pts_packed.data_ptr(), ctr_packed.data_ptr(), B, N, S, C, nr, radii_c, ks_c, outs_c, cnts_c,
              _stream(pts_packed)), pts_packed.device,
             nbytes=4.0 * cp * B * (N + S) + sum(4.0 * B * S * (k + 1) for k in ks),
             flops=float(B) * S * N * (2 * C + 3))  # one distance per pair for all radii
        res.extend(zip(outs, cnts))
    return res


def _ball_query_op(pts_packed: Tensor, ctr_packed: Tensor, C: int, radius: float, nsample: int) -> Tensor:
    return ball_query_direct(pts_packed, ctr_packed, C, radius, nsample)


ball_query = torch.library.custom_op("pn2::ball_query", _ball_query_op, mutates_args=())


@ball_query.register_fake
def _(pts_packed, ctr_packed, C, radius, nsample):
    return pts_packed.new_empty(pts_packed.shape[0], ctr_packed.shape[1], nsample, dtype=torch.int64)


# ------------------------------------------------------------------------------ square_distance
def square_distance_direct(src_packed: Tensor, dst_packed: Tensor, C: int) -> Tensor:
    _dev(src_packed, "pn2::square_distance")
    B, S, _ = src_packed.shape
    N = dst_packed.shape[1]
    out = torch.empty(B, S, N, dtype=torch.float32, device=src_packed.device)
    _run("pn2_square_distance_f32", _L.pn2_square_distance_f32,
         (src_packed.data_ptr(), dst_packed.data_ptr(), B, S, N, C, out.data_ptr(),
          _stream(src_packed)), src_packed.device)
    return out


square_distance = torch.library.custom_op("pn2::square_distance", square_distance_direct, mutates_args=())


@square_distance.register_fake
def _(src_packed, dst_packed, C):
    return src_packed.new_empty(src_packed.shape[0], src_packed.shape[1], dst_packed.shape[1])


# ------------------------------------------------------------------------------ index_points
def index_points_direct(points: Tensor, idx: Tensor) -> Tensor:
    """points [B,N,C] (any strides), idx [B,M] int64 -> [B,M,C] contiguous."""
    _dev(points, "pn2::index_points")
    B, N, C = points.shape
    M = idx.shape[1]
    idx = idx.contiguous()
    out = torch.empty(B, M, C, dtype=torch.float32, device=points.device)
    sb, sn, sc = points.stride()
    _run("pn2_index_points_f32", _L.pn2_index_points_f32,
         (points.data_ptr(), B, N, C, sb, sn, sc, idx.data_ptr(), M, out.data_ptr(),
          _stream(points)), points.device)
    return out


index_points = torch.library.custom_op("pn2::index_points", index_points_direct, mutates_args=())


@index_points.register_fake
def _(points, idx):
    return points.new_empty(points.shape[0], idx.shape[1], points.shape[2])


# ------------------------------------------------------------------------------ group
def group_direct(points: Tensor, feature: Optional[Tensor], centers: Tensor, idx: Tensor,
          feature_first: bool) -> Tensor:
    """[B,S,K,C+D]: [xyz(idx) - centre, feature(idx)] (or feature first, the MSG order)."""
    _dev(points, "pn2::group")
    B, N, C = points.shape
    S, K = idx.shape[1], idx.shape[2]
    D = 0 if feature is None else feature.shape[2]
    centers = centers.contiguous()
    idx = idx.contiguous()
    out = torch.empty(B, S, K, C + D, dtype=torch.float32, device=points.device)
    sb, sn, sc = points.stride()
    if feature is None:
        fp, fb, fn, fd = 0, 0, 0, 0
    else:
        fp = feature.data_ptr()
        fb, fn, fd = feature.stride()
    _run("pn2_group_f32", _L.pn2_group_f32,
         (points.data_ptr(), B, N, C, sb, sn, sc, fp, D, fb, fn, fd, centers.data_ptr(), S,
          idx.data_ptr(), K, int(feature_first), out.data_ptr(), _stream(points)), points.device)
    return out


group = torch.library.custom_op("pn2::group", group_direct, mutates_args=())


@group.register_fake
def _(points, feature, centers, idx, feature_first):
    D = 0 if feature is None else feature.shape[2]
    return points.new_empty(points.shape[0], idx.shape[1], idx.shape[2], points.shape[2] + D)


# ------------------------------------------------------------------------------ pack_layer
def pack_layer_direct(weight: Tensor, bias: Optional[Tensor], gamma: Optional[Tensor],
               beta: Optional[Tensor], mean: Optional[Tensor], var: Optional[Tensor],
               eps: float, rot: int) -> Tuple[Tensor, Tensor, Tensor]:
    """Conv2d 1x1 weight [cout,cin,1,1] (+ bias) and eval BatchNorm2d stats -> (W^T pair-packed
    [cin_pad/2,cout,2], alpha [cout], beta [cout]) with layer(x) = relu(alpha*(W x) + beta).
    rot: leading xyz input channels moved behind the features (the kernels' row order)."""
    _dev(weight, "pn2::pack_layer")
    cout, cin = weight.shape[0], weight.shape[1]
    w = weight.reshape(cout, cin).contiguous()
    dev = weight.device
    wt = torch.empty(cin_pad(cin) // 2, cout, 2, dtype=torch.float32, device=dev)
    al = torch.empty(cout, dtype=torch.float32, device=dev)
    be = torch.empty(cout, dtype=torch.float32, device=dev)

    def p(t):
        return 0 if t is None else t.contiguous().data_ptr()
    keep = [None if t is None else t.contiguous() for t in (bias, gamma, beta, mean, var)]
    _run("pn2_pack_layer_f32", _L.pn2_pack_layer_f32,
         (w.data_ptr(), *[p(t) for t in keep], float(eps), cout, cin, int(rot), wt.data_ptr(),
          al.data_ptr(), be.data_ptr(), _stream(weight)), weight.device)
    return wt, al, be


pack_layer = torch.library.custom_op("pn2::pack_layer", pack_layer_direct, mutates_args=())


@pack_layer.register_fake
def _(weight, bias, gamma, beta, mean, var, eps, rot):
    cout, cin = weight.shape[0], weight.shape[1]
    e = weight.new_empty
    return e(cin_pad(cin) // 2, cout, 2), e(cout), e(cout)


def pack_layer_split_direct(weight: Tensor, xyz: int, xyz_first: bool) -> Tensor:
    """Conv2d 1x1 weight [cout,cin,1,1] -> the split image of pn2_pack_layer_split_bf16 (three
    bf16 planes hi/mid/lo, two fp16 planes of the row-scaled weights and the rows' inverse
    scales, in MFMA fragment order), flat 16-bit storage.  xyz: the xyz channels
    of a first layer (its rows are [xyz | features] in the chain kernel; 0 for hidden layers),
    xyz_first: W's own order is [xyz, features] (SSG) rather than [features, xyz] (MSG)."""
    _dev(weight, "pn2::pack_layer_split")
    cout, cin = weight.shape[0], weight.shape[1]
    w = weight.reshape(cout, cin).contiguous()
    nbytes = int(_L.pn2_layer_split_bytes(cout, cin, xyz))
    if nbytes < 0:
        raise ValueError("pn2::pack_layer_split: bad shape cout=%d cin=%d xyz=%d" % (cout, cin, xyz))
    out = torch.empty(nbytes // 2, dtype=torch.bfloat16, device=weight.device)
    _run("pn2_pack_layer_split_bf16", _L.pn2_pack_layer_split_bf16,
         (w.data_ptr(), cout, cin, int(xyz), 1 if xyz_first else 0, out.data_ptr(),
          _stream(weight)), weight.device)
    return out


pack_layer_split = torch.library.custom_op("pn2::pack_layer_split", pack_layer_split_direct, mutates_args=())


@pack_layer_split.register_fake
def _(weight, xyz, xyz_first):
    cout, cin = weight.shape[0], weight.shape[1]
    return weight.new_empty(int(_L.pn2_layer_split_bytes(cout, cin, xyz)) // 2, dtype=torch.bfloat16)


# ------------------------------------------------------------------------------ sa_mlp_max_
def _src(mode, points, feature, centers, idx, rows, B, N, C, D, S, K, cnt=None):
    s = SaSrc()
    if cnt is not None:
        if cnt.dtype != torch.int32 or not cnt.is_contiguous() or cnt.numel() != B * S:
            raise ValueError("pn2::sa_mlp_max_: cnt must be a contiguous int32 [B, S] tensor")
        s.cnt = cnt.data_ptr()
    s.mode = mode
    if points is not None:
        s.pts = points.data_ptr()
        s.pb, s.pn, s.pc = points.stride()
    if feature is not None:
        if feature.stride(2) != 1:
            raise ValueError("pn2::sa_mlp_max_: features must be channels-last (stride 1)")
        s.feat = feature.data_ptr()
        s.fb, s.fn = feature.stride(0), feature.stride(1)
    if centers is not None:
        s.ctr = centers.data_ptr()
    if idx is not None:
        if idx.dtype == torch.int32:
            s.idx32 = idx.data_ptr()
        else:
            s.idx = idx.data_ptr()
    if rows is not None:
        s.rows = rows.data_ptr()
        s.rs = rows.stride(0)
    s.B, s.N, s.C, s.D, s.S, s.K = B, N, C, D, S, K
    return s


def fps_side_job(points: Tensor, npoint: int, start: Tensor):
    """The next SA layer's farthest point sampling as a side job of an SA MLP call (pn2_fps_side):
    points [B,N,C] (any strides), start [B] int64 on the CPU -> (job, (fps_idx, new_points,
    packed centroids, packed points)); pass `job` as sa_mlp_max_impl(..., fps_side=job).  The
    outputs are fps_direct's, filled by the MLP call's launches."""
    _dev(points, "pn2::fps")
    B, N, C = points.shape
    cp = packed_stride(C)
    start = start.to(dtype=torch.int64).contiguous()
    if start.device.type != "cpu" or start.shape != (B,):
        raise ValueError("pn2::fps side job: start must be a [B] CPU tensor")
    dev = points.device
    outs = (torch.empty(B, npoint, dtype=torch.int64, device=dev),
            torch.empty(B, npoint, C, dtype=torch.float32, device=dev),
            torch.empty(B, npoint, cp, dtype=torch.float32, device=dev),
            torch.empty(B, N, cp, dtype=torch.float32, device=dev))
    sb, sn, sc = points.stride()
    job = _lib.FpsSide(points.data_ptr(), B, N, C, sb, sn, sc, start.data_ptr(), npoint,
                       *(t.data_ptr() for t in outs))
    job._keep = (points, start)  # alive until the MLP call has read them
    return job, outs


def sa_mlp_max_direct(out: Tensor, mode: int, points: Optional[Tensor], feature: Optional[Tensor],
                centers: Optional[Tensor], idx: Optional[Tensor], wts: List[Tensor],
                alphas: List[Tensor], betas: List[Tensor], cins: List[int],
                splits: List[Tensor], precision: str = "fp32", flags: Optional[List[int]] = None,
                rows: Optional[Tensor] = None, pool: bool = True,
                cnt: Optional[Tensor] = None, zero: Optional[Tensor] = None) -> None:
    """sa_mlp_max_impl without a side job (the signature torch.library registers)."""
    sa_mlp_max_impl(out, mode, points, feature, centers, idx, wts, alphas, betas, cins, splits,
                    precision, flags, rows, pool, cnt, zero)


def sa_mlp_max_impl(out, mode, points, feature, centers, idx, wts, alphas, betas, cins, splits,
                    precision="fp32", flags=None, rows=None, pool=True, cnt=None, zero=None,
                    fps_side=None):
    """Fused gather -> MLP (conv1x1+BN+ReLU)* -> max over each group, written channels-last
    into `out` ([G, >=cout] view with unit column stride; G = B*S groups, or B for
    group_all).  mode: 0 SSG grouping, 1 MSG grouping, 2 group_all, 3 rows (`rows` [B, R, cin]
    with unit column stride: B groups of R rows, `points` unused).  splits: the
    pack_layer_split images of the same layers (empty list: fp32 kernels only).
    precision: "fp32" (pn2_sa_mlp_max_f32) or "bf16" (pn2_sa_mlp_max_bf16, needs splits).
    flags: per-layer PN2_LAYER_* bits (LAYER_NO_RELU).  pool=False: `out` gets every row's
    last-layer output ([M, >=cout], group_all / rows sources).  cnt: the ball query's
    distinct-neighbour counts ([B, S] int32, grouping modes) -- only those rows of each group are
    computed (the rest repeat the first neighbour; same result).  zero: a contiguous float32
    tensor one of the call's launches fills with zeros (group_all's new_points).  fps_side: a
    fps_side_job() the call also runs (sa_mlp_max_impl only; the SA modules' lookahead)."""
    if precision not in PRECISIONS:
        raise ValueError("pn2::sa_mlp_max_: precision must be one of %s" % (PRECISIONS,))
    bf16 = precision == "bf16"
    if bf16 and not splits:
        raise ValueError("pn2::sa_mlp_max_: bf16 needs the split weight images (none for points "
                         "with more than 16 channels)")
    if mode == _lib.SRC_ROWS:
        _dev(rows, "pn2::sa_mlp_max_")
        if rows.dim() != 3 or rows.stride(2) != 1 or rows.stride(0) != rows.shape[1] * rows.stride(1):
            raise ValueError("pn2::sa_mlp_max_: rows must be [B, R, cin] with unit column stride "
                             "and uniform row stride")
        B, K = rows.shape[0], rows.shape[1]
        src = _src(mode, None, None, None, None, rows.view(B * K, -1) if B * K else rows[0],
                   B, K, 0, 0, 1, K)
        dev_t = rows
        S = 1
    else:
        _dev(points, "pn2::sa_mlp_max_")
        B, N, C = points.shape
        D = 0 if feature is None else feature.shape[2]
        if mode == _lib.SRC_GROUP_ALL:
            S, K = 1, N
        else:
            S, K = idx.shape[1], idx.shape[2]
            idx = idx.contiguous()
            centers = centers.contiguous()
        src = _src(mode, points, feature, centers, idx, None, B, N, C, D, S, K,
                   cnt if mode in (_lib.SRC_GROUP_XYZ_FIRST, _lib.SRC_GROUP_FEAT_FIRST) else None)
        dev_t = points
    if zero is not None:
        if zero.dtype != torch.float32 or not zero.is_contiguous() or zero.device != dev_t.device:
            raise ValueError("pn2::sa_mlp_max_: zero must be a contiguous float32 device tensor")
        src.zero_out, src.zero_count = zero.data_ptr(), zero.numel()
    if fps_side is not None:
        src.fps_side = ctypes.addressof(fps_side)
    n = len(wts)
    layers = (MlpLayer * n)()
    for i in range(n):
        layers[i].wt = wts[i].data_ptr()
        layers[i].alpha = alphas[i].data_ptr()
        layers[i].beta = betas[i].data_ptr()
        layers[i].cin = cins[i]
        layers[i].cout = wts[i].shape[1]  # [cin_pad/2, cout, 2]
        layers[i].wt_split = splits[i].data_ptr() if splits else 0
        layers[i].flags = int(flags[i]) if flags else 0
    if out.stride(-1) != 1:
        raise ValueError("pn2::sa_mlp_max_: out must have unit column stride")
    ws_fn = _L.pn2_sa_mlp_workspace_bytes_bf16 if bf16 else _L.pn2_sa_mlp_workspace_bytes
    ws_bytes = int(ws_fn(src, layers, n))
    if ws_bytes < 0:
        check(-1, "pn2_sa_mlp_workspace_bytes")
    ws = torch.empty(ws_bytes // 4, dtype=torch.float32, device=dev_t.device) if ws_bytes else None
    M = B * S * K
    flops = 2.0 * M * sum(cins[i] * wts[i].shape[1] for i in range(n))  # algorithmic, cin unpadded
    # compulsory bytes: every source element, index and weight read once, the output written once
    if mode == _lib.SRC_ROWS:
        nbytes = 4.0 * B * K * cins[0]
    else:
        nbytes = 4.0 * B * N * (C + D)
        if mode != _lib.SRC_GROUP_ALL:
            nbytes += 4.0 * B * S * C + 8.0 * B * S * K + (4.0 * B * S if cnt is not None else 0.0)
    nbytes += sum(4.0 * (cins[i] + 2) * wts[i].shape[1] for i in range(n))
    nbytes += 4.0 * (B * S if pool else M) * wts[-1].shape[1]
    name = "pn2_sa_mlp_max_bf16" if bf16 else "pn2_sa_mlp_max_f32"
    _run(name, getattr(_L, name),
         (src, layers, n, 1 if pool else 0, out.data_ptr(), out.stride(-2),
          0 if ws is None else ws.data_ptr(), ws_bytes, _stream(dev_t)), dev_t.device, flops=flops,
         nbytes=nbytes)
    if _TIMER is not None and _TIMER.records and _TIMER.records[-1][0] == name:
        _TIMER.records[-1] = _TIMER.records[-1] + (int(_L.pn2_sa_mlp_last_planes()),)


sa_mlp_max_ = torch.library.custom_op("pn2::sa_mlp_max_", sa_mlp_max_direct, mutates_args=("out", "zero"))


@sa_mlp_max_.register_fake
def _(out, mode, points, feature, centers, idx, wts, alphas, betas, cins, splits, precision="fp32",
      flags=None, rows=None, pool=True, cnt=None, zero=None):
    return None


def linear_rows(x: Tensor, weight: Tensor, bias: Optional[Tensor], relu: bool) -> Tensor:
    """act(x @ weight^T + bias) on pn2_linear_rows_f32 (rows in blocks of 16; each output
    element computed the same way whatever the row count, so batch shards are bit-identical):
    x [B, K] (unit column stride), weight [N, K] contiguous, bias [N] or None -> [B, N]."""
    _dev(x, "pn2::linear_rows")
    B, K = x.shape
    N = weight.shape[0]
    if B < 1 or x.stride(1) != 1 or not weight.is_contiguous() or \
            weight.shape[1] != K or (bias is not None and not bias.is_contiguous()):
        raise ValueError("pn2::linear_rows: x [B, K] with unit column stride, weight [N, K] "
                         "contiguous")
    out = torch.empty(B, N, device=x.device, dtype=torch.float32)
    check(_L.pn2_linear_rows_f32(x.data_ptr(), x.stride(0), B, K, weight.data_ptr(),
                                 0 if bias is None else bias.data_ptr(), out.data_ptr(), N, N,
                                 _lib.LINEAR_RELU if relu else 0, _stream(x)),
          "pn2_linear_rows_f32")
    return out


def fc_tail(x: Tensor, layers, logsoftmax: bool):
    """The heads' eval FC tail on pn2_fc_tail_f32 (two launches): x [B, K] (unit column stride),
    layers = ((W1, b1), (W2, b2), (W3, b3)) folded float32 (bn1 / bn2 in W1 / W2), fc1 and fc2
    with ReLU -> (out [B, N3], argmax [B] int64 or None).  logsoftmax: out is
    log_softmax(fc3(...), -1) and argmax its first per-row maximum (the classifiers' tail,
    pointnet2_cls_ssg.py:36-38)."""
    _dev(x, "pn2::fc_tail")
    (w1, b1), (w2, b2), (w3, b3) = layers
    B, K = x.shape
    N1, N2, N3 = w1.shape[0], w2.shape[0], w3.shape[0]
    if x.stride(1) != 1 or w1.shape[1] != K or w2.shape[1] != N1 or w3.shape[1] != N2:
        raise ValueError("pn2::fc_tail: x [B, K] with unit column stride and chained layer shapes")
    nbytes = int(_L.pn2_fc_tail_workspace_bytes(B, N1, N2))
    ws = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=x.device)
    out = torch.empty(B, N3, dtype=torch.float32, device=x.device)
    amax = torch.empty(B, dtype=torch.int64, device=x.device) if logsoftmax else None

    def p(t):
        return 0 if t is None else t.data_ptr()
    _run("pn2_fc_tail_f32", _L.pn2_fc_tail_f32,
         (x.data_ptr(), x.stride(0), B, K, w1.data_ptr(), p(b1), N1, w2.data_ptr(), p(b2), N2,
          w3.data_ptr(), p(b3), N3, _lib.TAIL_LOGSOFTMAX if logsoftmax else 0, out.data_ptr(), N3,
          p(amax), ws.data_ptr(), nbytes, _stream(x)), x.device,
         flops=2.0 * B * (K * N1 + N1 * N2 + N2 * N3))
    return out, amax
