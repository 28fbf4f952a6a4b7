"""Drop-in replacement for /root/reference/model/pointnet2_utils.py on MI355X.

Same public names, signatures, return shapes, ``state_dict`` keys and CPU-RNG consumption as
the reference, so its heads (pointnet2_cls_ssg/msg, rotation_/translation_/sign_*) run
unchanged when this module is importable as ``pointnet2_utils`` (see the shim
``pointnet-like-pose-estimation_amd/pointnet2_utils.py``).

Eval-mode inference (``model.eval()`` / no autograd) of an SA layer is three HIP launches
(FPS and ball query on the geometry stream, see geometry.py, overlapping the previous layer's
MLP):
  pn2::fps            FPS + gathered centroids + packed (coords, ssq) records
  pn2::ball_query     first-K-in-radius neighbour indices
  pn2::sa_mlp_max_    fused gather -> conv1x1/BN/ReLU chain -> max over neighbours
(+ per scale for the MSG module).  Hidden activations stay in registers (the chain kernel) or
pass through an HBM workspace between the dense-layer launches (group_all layers); the
per-layer ``[B, C, K, S]`` tensors of the reference are never materialised.

Training (``model.train()`` or autograd through the weights) keeps the reference's semantics
(batch-statistics BatchNorm, autograd through the MLP and the feature gather): FPS and the ball
query still run as HIP kernels (they are index ops with no gradient); in train mode the
grouping and the MLP + max run forward and backward on the training kernels of pn2/train.py
(csrc/train.hip around library GEMMs).  As in the reference, an eval-mode forward with
autograd enabled (``model.eval()`` without ``torch.no_grad()``, parameters requiring grad) is
differentiable: it runs the torch device formulation.  The fused inference kernels serve
eval-mode forwards under ``torch.no_grad()`` / ``torch.inference_mode()``, with parameters that
need no gradient, or inside ``pn2.fused_eval()`` (the mutilthreading/predict_test.py pattern
made fast: its outputs carry no autograd history).

Device tensors only -- the reference's CPU execution is not re-implemented here.
"""
import contextlib
import threading

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import geometry
from . import ops
from . import shard
from . import train
from . import tuning


# ----------------------------------------------------------------------------- helpers
def _draw_start(B, N, device):
    """The reference's FPS start draw: torch.randint(0, N, (B,), dtype=long) on the CPU default
    generator (pointnet2_utils.py:59) -- one draw per FPS call, sliced when sharded.  A CPU
    tensor (ops.fps_direct passes host starts in the launch's arguments), or a device slot under
    graph capture."""
    return shard.host_start(B, N, device)


def _fps_ahead(module, new_points):
    """The side job that runs the next SA layer's FPS (geometry.fps_ahead) on this layer's
    centroids `new_points` [B, S, C] inside this layer's MLP call, or None: registered so the next
    layer's forward takes its results instead of sampling."""
    nxt = geometry.ahead_of(module)
    if nxt is None or getattr(nxt, "group_all", False) or nxt.point_number is None:
        return None
    if _needs_autograd(nxt, new_points) or shard.recording():  # (graph records: device starts)
        return None
    B, N, _ = new_points.shape
    start = shard.host_start(B, N, new_points.device)
    job, (_, newp, cpk, ppk) = ops.fps_side_job(new_points, nxt.point_number, start)
    geometry.put_ahead(nxt, new_points, newp, cpk, ppk)
    return job


def msg_ball_queries(ppk, cpk, C, radii, nsamples):
    """The ball queries of an MSG layer's scales (pointnet2_utils.py:197-203): one launch over
    all radii (ops.ball_query_multi_direct; host tuning bq_multi = 0: one call per radius), the
    same (int32 lists, counts) per radius either way."""
    if tuning.get("bq_multi") and len(radii) > 1:
        return ops.ball_query_multi_direct(ppk, cpk, C, radii, nsamples)
    return [ops.ball_query_direct(ppk, cpk, C, r, k, True) for r, k in zip(radii, nsamples)]


def _channels_last(feature):
    """[B, D, N] feature -> a [B, N, D] view with unit channel stride (copy only if needed)."""
    f = feature.permute(0, 2, 1)
    return f if f.stride(2) == 1 else f.contiguous()


def _precision(module):
    """The module's MLP arithmetic: its own ``mlp_precision`` if set, else the thread's
    ``pn2.ops.mlp_precision`` context ("fp32" unless changed)."""
    p = getattr(module, "mlp_precision", None)
    return ops.current_precision() if p is None else p


_fused = threading.local()


@contextlib.contextmanager
def fused_eval(enabled=True):
    """Within this context (this thread) eval-mode forwards run the fused inference kernels even
    with autograd enabled (``model.eval()`` without ``torch.no_grad()``, the
    mutilthreading/predict_test.py pattern): the no_grad bits, no autograd history (a backward
    through the outputs finds nothing that requires grad).  Outside it such a forward is
    differentiable, as in the reference."""
    prev = getattr(_fused, "on", False)
    _fused.on = bool(enabled)
    try:
        yield
    finally:
        _fused.on = prev


@contextlib.contextmanager
def eval_autograd(enabled=True):
    """Round-2 name kept for callers: eval-mode forwards with autograd enabled are
    differentiable (the default now); ``enabled=False`` is ``fused_eval()``."""
    with fused_eval(not enabled):
        yield


def _needs_autograd(module, *tensors):
    """Whether a forward must be differentiable: training mode, or autograd on (outside
    ``fused_eval()``) with an input or a parameter that needs a gradient -- the reference's
    eval forward is differentiable whenever autograd is."""
    if module.training:
        return True
    if not torch.is_grad_enabled() or getattr(_fused, "on", False):
        return False
    if any(t is not None and t.requires_grad for t in tensors):
        return True
    return any(p.requires_grad for p in module.parameters())


_SPLIT_MAX_XYZ = 16  # point channels of a split-bf16 first layer (csrc/sa_chain.hip)


def _pack_chain(convs, bns, cache, rot0, xyz=0, xyz_first=True):
    """Fold each Conv2d-1x1 + eval BatchNorm2d into (W^T, alpha, beta) for the fp32 kernels and
    the split-bf16 image for the chain kernel; cached until any parameter/buffer changes
    (data_ptr or in-place version).  rot0: xyz channels leading the first layer's input in the
    reference's order (the fp32 kernels put them behind the features); xyz / xyz_first: the
    first layer's xyz channel count and order for the chain kernel (rows [xyz | features]).
    Points with more than 16 channels get no split images: the split-bf16 kernels hold at most
    16 point channels (pn2_layer_split_kblocks), so those layers run the fp32 kernels only and
    precision "bf16" fails loudly for them (sa_mlp_max_impl)."""
    tensors = []
    for conv, bn in zip(convs, bns):
        tensors += [conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var]
    key = (rot0, xyz, xyz_first) + tuple((None if t is None else (t.data_ptr(), t._version))
                                         for t in tensors)
    if cache.get("key") != key:
        wts, als, bes, cins, splits = [], [], [], [], []
        with torch.no_grad():
            for li, (conv, bn) in enumerate(zip(convs, bns)):
                rot = rot0 if li == 0 else 0
                wt, al, be = ops.pack_layer_direct(conv.weight, conv.bias, bn.weight, bn.bias,
                                            bn.running_mean, bn.running_var, float(bn.eps), rot)
                wts.append(wt)
                als.append(al)
                bes.append(be)
                cins.append(conv.weight.shape[1])
                if xyz <= _SPLIT_MAX_XYZ:
                    splits.append(ops.pack_layer_split_direct(conv.weight, xyz if li == 0 else 0,
                                                              xyz_first))
        cache["key"] = key
        cache["layers"] = (wts, als, bes, cins, splits)
    return cache["layers"]


def _torch_group(points, idx, centers, feature, feature_first):
    """Differentiable grouping for the training path: the HIP grouping kernel with an
    index_add_ backward for the features (pn2/train.py), or torch device gathers when the
    coordinates need a gradient too."""
    g = train.group_train(points, idx, centers, feature, feature_first)
    if g is not None:
        return g
    B = points.shape[0]
    b = torch.arange(B, device=points.device).view(B, 1, 1)
    g = points[b, idx, :] - centers.unsqueeze(2)
    if feature is None:
        return g
    f = feature[b, idx, :]
    return torch.cat([f, g] if feature_first else [g, f], dim=-1)


def _torch_mlp_max(grouped, convs, bns):
    """grouped [B,S,K,C] -> [B, Cout, S].  Training on the device: the fused batch-statistics
    BN / ReLU / max kernels around library GEMMs (pn2/train.py); otherwise (eval with autograd,
    exotic BN configs) the reference's torch formulation."""
    if train.eligible(grouped, convs, bns):
        return train.mlp_max_train(grouped, convs, bns)
    x = grouped.permute(0, 3, 2, 1)  # [B, C, K, S] as the reference (:167)
    for conv, bn in zip(convs, bns):
        x = F.relu(bn(conv(x)))
    return torch.max(x, 2)[0]


# ----------------------------------------------------------------------------- public functions
def square_distance(src, dst):
    """pointnet2_utils.py:5-26 -> [B, N, M], bit-identical to the reference's float32 result."""
    C = src.shape[-1]
    return ops.square_distance_direct(ops.pack_points_direct(src), ops.pack_points_direct(dst), C)


def index_points(points, idx):
    """pointnet2_utils.py:28-45: points [B,N,C], idx [B, ...] -> [B, ..., C]."""
    B = points.shape[0]
    out = ops.index_points_direct(points, idx.reshape(B, -1))
    return out.view(*idx.shape, points.shape[-1])


def farthest_point_sample(points, number):
    """pointnet2_utils.py:47-68: [B,N,C] -> [B, number] int64 (consumes one CPU randint)."""
    B, N, _ = points.shape
    return ops.fps_direct(points, number, _draw_start(B, N, points.device))[0]


def query_ball_point(radius, number, points, new_points):
    """pointnet2_utils.py:70-90: [B,S,number] int64; IndexError if number > N (as the
    reference)."""
    C = points.shape[-1]
    return ops.ball_query_direct(ops.pack_points_direct(points), ops.pack_points_direct(new_points),
                                 C, radius, number)


def sample_and_group(points, feature, point_number, sample_number, radius, returnfps=False):
    """pointnet2_utils.py:92-120.  points [B,N,C], feature [B,N,D] or None."""
    B, N, C = points.shape
    fps_idx, new_points, cpk, ppk = ops.fps_direct(points, point_number, _draw_start(B, N, points.device))
    idx = ops.ball_query_direct(ppk, cpk, C, radius, sample_number)
    new_feature = ops.group_direct(points, feature, new_points, idx, False)
    if returnfps:
        grouped = index_points(feature if feature is not None else points, idx)
        return new_points, new_feature, grouped, fps_idx
    return new_points, new_feature


def sample_and_group_all(points, feature):
    """pointnet2_utils.py:122-141: centroid at the origin, raw xyz (not centred) first."""
    B, N, C = points.shape
    new_points = torch.zeros(B, 1, C, device=points.device, dtype=points.dtype)
    grouped = points.reshape(B, 1, N, C)
    if feature is not None:
        return new_points, torch.cat([grouped, feature.reshape(B, 1, N, -1)], dim=-1)
    return new_points, grouped


# ----------------------------------------------------------------------------- modules
class PointNetSetAbstraction(nn.Module):
    """pointnet2_utils.py:143-174 (same ctor, submodule names and forward contract)."""

    def __init__(self, point_number, sample_number, radius, in_channel, mlp, group_all=False):
        super(PointNetSetAbstraction, self).__init__()
        self.point_number = point_number
        self.radius = radius
        self.sample_number = sample_number
        self.group_all = group_all
        self.mlp_convs = nn.ModuleList()
        self.mlp_bns = nn.ModuleList()
        last = in_channel
        for out_channel in mlp:
            self.mlp_convs.append(nn.Conv2d(last, out_channel, 1))
            self.mlp_bns.append(nn.BatchNorm2d(out_channel))
            last = out_channel
        self._pack_cache = {}
        self.mlp_precision = None  # None: ops.mlp_precision context ("fp32" by default)

    def forward(self, points, feature):
        """points [B,C,N], feature [B,D,N] or None -> (new_points [B,C,S], new_feature
        [B,mlp[-1],S]).  Both outputs are channel-first views of channels-last buffers."""
        if _needs_autograd(self, points, feature):
            return self._forward_autograd(points, feature)
        pts = points.permute(0, 2, 1)
        feat = None if feature is None else _channels_last(feature)
        B, N, C = pts.shape
        # reference row order is [xyz, feature] (:114, :139); kernels use [feature, xyz]
        rot0 = C if feat is not None else 0
        xyz = C  # split-bf16 rows are [xyz | features] for grouped and group_all layers alike
        wts, als, bes, cins, splits = _pack_chain(self.mlp_convs, self.mlp_bns, self._pack_cache,
                                                  rot0, xyz, True)
        cout = wts[-1].shape[1]
        dev = pts.device
        if self.group_all:
            out = torch.empty(B, cout, device=dev, dtype=torch.float32)
            # new_points = the reference's zeros (:136), filled by the MLP's last launch
            new_points = torch.empty(B, C, 1, device=dev, dtype=torch.float32)
            ops.sa_mlp_max_direct(out, _lib.SRC_GROUP_ALL, pts, feat, None, None, wts, als, bes, cins,
                                  splits, _precision(self), zero=new_points)
            return new_points, out.view(B, 1, cout).permute(0, 2, 1)
        S, K = self.point_number, self.sample_number
        pre = geometry.take(self, pts)  # FPS (+ ball query) precomputed by pn2.pipeline
        if pre is not None:
            new_points, cpk, ppk, idxs = pre
            idx, cnt = idxs[0] if idxs else ops.ball_query_direct(ppk, cpk, C, self.radius, K, True)
        else:
            with geometry.Span(dev, [pts]) as span:  # overlaps the previous layer's MLP
                _, new_points, cpk, ppk = ops.fps_direct(pts, S, _draw_start(B, N, dev))
                idx, cnt = ops.ball_query_direct(ppk, cpk, C, self.radius, K, True)
            span.finish([new_points], [new_points, idx, cnt])
        out = torch.empty(B * S, cout, device=dev, dtype=torch.float32)
        ops.sa_mlp_max_impl(out, _lib.SRC_GROUP_XYZ_FIRST, pts, feat, new_points, idx, wts, als, bes,
                            cins, splits, _precision(self), cnt=cnt, fps_side=_fps_ahead(self, new_points))
        return new_points.permute(0, 2, 1), out.view(B, S, cout).permute(0, 2, 1)

    def _forward_autograd(self, points, feature):
        pts = points.permute(0, 2, 1)
        feat = None if feature is None else feature.permute(0, 2, 1)
        if self.group_all:
            new_points, grouped = sample_and_group_all(pts, feat)
        else:
            B, N, C = pts.shape
            _, new_points, cpk, ppk = ops.fps_direct(pts.detach(), self.point_number,
                                              _draw_start(B, N, pts.device))
            idx = ops.ball_query_direct(ppk, cpk, C, self.radius, self.sample_number)
            grouped = _torch_group(pts, idx, new_points, feat, False)
        return new_points.permute(0, 2, 1), _torch_mlp_max(grouped, self.mlp_convs, self.mlp_bns)


class PointNetSetAbstractionMsg(nn.Module):
    """pointnet2_utils.py:176-223 (same ctor, submodule names and forward contract)."""

    def __init__(self, point_number, sample_number_list, radius_list, in_channel, mlp_list,
                 num_category=0):
        super(PointNetSetAbstractionMsg, self).__init__()
        self.point_number = point_number
        self.radius_list = radius_list
        self.sample_number_list = sample_number_list
        self.conv_blocks = nn.ModuleList()
        self.bn_blocks = nn.ModuleList()
        for widths in mlp_list:
            convs = nn.ModuleList()
            bns = nn.ModuleList()
            last = in_channel + 3 + num_category
            for out_channel in widths:
                convs.append(nn.Conv2d(last, out_channel, 1))
                bns.append(nn.BatchNorm2d(out_channel))
                last = out_channel
            self.conv_blocks.append(convs)
            self.bn_blocks.append(bns)
        self._pack_cache = [{} for _ in mlp_list]
        self.mlp_precision = None  # None: ops.mlp_precision context ("fp32" by default)

    def forward(self, points, feature):
        if _needs_autograd(self, points, feature):
            return self._forward_autograd(points, feature)
        pts = points.permute(0, 2, 1)
        feat = None if feature is None else _channels_last(feature)
        B, N, C = pts.shape
        S = self.point_number
        dev = pts.device
        # MSG row order is already [feature, xyz] (:209): no rotation
        chains = [_pack_chain(self.conv_blocks[i], self.bn_blocks[i], self._pack_cache[i], 0, C,
                              False)
                  for i in range(len(self.radius_list))]
        total = sum(ch[0][-1].shape[1] for ch in chains)
        pre = geometry.take(self, pts)  # FPS (+ ball queries) precomputed by pn2.pipeline
        if pre is not None:
            new_points, cpk, ppk, idxs = pre
            if not idxs:
                idxs = msg_ball_queries(ppk, cpk, C, self.radius_list, self.sample_number_list)
        else:
            with geometry.Span(dev, [pts]) as span:  # overlaps the previous layer's MLP
                _, new_points, cpk, ppk = ops.fps_direct(pts, S, _draw_start(B, N, dev))
                idxs = msg_ball_queries(ppk, cpk, C, self.radius_list, self.sample_number_list)
            span.finish([new_points], [new_points] + [t for ic in idxs for t in ic])
        out = torch.empty(B * S, total, device=dev, dtype=torch.float32)
        prec = _precision(self)
        col = 0
        side = _fps_ahead(self, new_points)  # rides on the longest scale's launch (largest K)
        longest = max(range(len(idxs)), key=lambda i: self.sample_number_list[i])
        for i, (idx, cnt) in enumerate(idxs):
            wts, als, bes, cins, splits = chains[i]
            cout = wts[-1].shape[1]
            ops.sa_mlp_max_impl(out[:, col:col + cout], _lib.SRC_GROUP_FEAT_FIRST, pts, feat,
                                new_points, idx, wts, als, bes, cins, splits, prec, cnt=cnt,
                                fps_side=side if i == longest else None)
            col += cout
        return new_points.permute(0, 2, 1), out.view(B, S, total).permute(0, 2, 1)

    def _forward_autograd(self, points, feature):
        pts = points.permute(0, 2, 1)
        feat = None if feature is None else feature.permute(0, 2, 1)
        B, N, C = pts.shape
        _, new_points, cpk, ppk = ops.fps_direct(pts.detach(), self.point_number,
                                          _draw_start(B, N, pts.device))
        outs = []
        for i, radius in enumerate(self.radius_list):
            idx = ops.ball_query_direct(ppk, cpk, C, radius, self.sample_number_list[i])
            grouped = _torch_group(pts, idx, new_points, feat, True)
            outs.append(_torch_mlp_max(grouped, self.conv_blocks[i], self.bn_blocks[i]))
        return new_points.permute(0, 2, 1), torch.cat(outs, dim=1)


__all__ = [
    "square_distance", "index_points", "farthest_point_sample", "query_ball_point",
    "sample_and_group", "sample_and_group_all", "PointNetSetAbstraction",
    "PointNetSetAbstractionMsg",
]
