"""Drop-in for /root/reference/model/pointnet_utils.py (PointNet v1: T-Nets + shared-MLP
encoder) on MI355X -- SURVEY.md §8(f) rank 1.

Same public names, constructor signatures, submodule names (so ``state_dict`` keys match the
reference's checkpoints) and forward contracts:

  TNet3d(channel)        pointnet_utils.py:9-43   x [B,C,N] -> transform [B,3,3]
  TNetkd(channel)        pointnet_utils.py:45-81  x [B,k,N] -> transform [B,k,k]
  PointNetEncoder(global_feat=True, channel=3)
                         pointnet_utils.py:83-138 x [B,D,N] -> (global [B,1024] or
                                                  [B,1088,N], transform, trans_feat)
  feature_transform_reguliarzer(transform)        pointnet_utils.py:140-147

The hot part of every v1 network is the same as a group_all SA layer (pointnet2_utils.py
:163-172): a per-point shared MLP (Conv1d 1x1 + BatchNorm1d + ReLU)* followed by a max over
the N points.  In eval mode it runs on pn2's split-bf16 dense-layer kernels (pn2_sa_mlp_max_f32
with a group_all source for a channel-first [B,C<=16,N] input, or a rows source for per-point
features already in HBM), one launch per layer, the max fused into the last layer's epilogue;
the encoder's conv3 + bn3 without ReLU before its max uses PN2_LAYER_NO_RELU (signed pooling).
The small per-cloud transforms (torch.bmm of a 3x3 / 64x64 matrix with the points) and the
T-Nets' FC layers are plain library GEMMs (torch on the GPU).  Training on the GPU runs the same
shared MLPs through pn2.train.point_mlp_train (library GEMMs + the fused batch-statistics BN /
ReLU / max kernels, forward and backward) in the same rows layout; eval with autograd (and
exotic BN configurations) keeps the reference's torch formulation.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import ops
from . import train
from .pointnet2_utils import _needs_autograd, _precision


# ----------------------------------------------------------------------------- eval-mode MLPs
def _pack(convs, bns, cache, xyz):
    """Folded (W^T, alpha, beta) and split images of Conv1d + BatchNorm1d layers; cached until a
    parameter changes.  xyz: channels of a channel-first first-layer input (group_all source,
    all of them in the split image's first block), 0 for a rows source."""
    tensors = []
    for conv, bn in zip(convs, bns):
        tensors += [conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var]
    key = (xyz,) + tuple((t.data_ptr(), t._version) for t in tensors if t is not None)
    if cache.get("key") != key:
        wts, als, bes, cins, splits = [], [], [], [], []
        with torch.no_grad():
            for li, (conv, bn) in enumerate(zip(convs, bns)):
                wt, al, be = ops.pack_layer_direct(conv.weight, conv.bias, bn.weight, bn.bias,
                                                   bn.running_mean, bn.running_var, float(bn.eps), 0)
                wts.append(wt)
                als.append(al)
                bes.append(be)
                cins.append(conv.weight.shape[1])
                splits.append(ops.pack_layer_split_direct(conv.weight, xyz if li == 0 else 0, True))
        cache["key"] = key
        cache["layers"] = (wts, als, bes, cins, splits)
    return cache["layers"]


def point_mlp(x, convs, bns, cache, pool=True, last_relu=True, module=None, rows=False):
    """relu(bn(conv(x))) over every point (the last layer without ReLU if not last_relu), then
    the max over the points when pool.  x: channel-first [B, C, N] (rows=False, any strides:
    C <= 16 is read in place as a group_all source, wider inputs as rows) or per-point rows
    [B, N, C] (rows=True, unit column stride, as a previous point_mlp returns them).
    Returns [B, cout] (pool) or rows [B, N, cout]."""
    if not rows and x.shape[1] > 16:
        x, rows = _cf_to_rows(x), True
    chan_first = not rows
    if chan_first:
        B, C, N = x.shape
        pts = x.permute(0, 2, 1)
        layers = _pack(convs, bns, cache, C)
    else:
        B, N, C = x.shape
        layers = _pack(convs, bns, cache, 0)
    wts, als, bes, cins, splits = layers
    cout = wts[-1].shape[1]
    n = len(wts)
    flags = [0] * n
    if not last_relu:
        flags[-1] = _lib.LAYER_NO_RELU
    out = torch.empty((B if pool else B * N), cout, device=x.device, dtype=torch.float32)
    prec = "fp32" if module is None else _precision(module)
    # the kernels take <= 4 layers per call: longer chains go through a rows intermediate
    if n > 4:
        mid = point_mlp(x, convs[:n - 3], bns[:n - 3], cache.setdefault("head", {}), pool=False,
                        module=module, rows=rows)
        return point_mlp(mid, convs[n - 3:], bns[n - 3:], cache.setdefault("tail", {}), pool,
                         last_relu, module, rows=True)
    if chan_first:
        ops.sa_mlp_max_direct(out, _lib.SRC_GROUP_ALL, pts, None, None, None, wts, als, bes, cins,
                              splits, prec, flags, pool=pool)
    else:
        ops.sa_mlp_max_direct(out, _lib.SRC_ROWS, None, None, None, None, wts, als, bes, cins,
                              splits, prec, flags, rows=x, pool=pool)
    return out if pool else out.view(B, N, cout)


def mlp_mode(module, x, convs, bns):
    """How a v1 module runs its shared MLPs on x: "fused" (eval without autograd: the split-bf16
    kernels; a CPU tensor raises), "train" (training on the device: pn2.train), or "torch" (the
    reference's formulation: eval with autograd, CPU training, BN configs pn2.train does not
    cover)."""
    if not _needs_autograd(module, x):
        return "fused"
    if module.training and train.eligible(x, convs, bns):
        return "train"
    return "torch"


def run_mlp(mode, x, convs, bns, cache, pool=True, last_relu=True, module=None, rows=False):
    """point_mlp ("fused") or train.point_mlp_train ("train") on x: channel-first [B, C, N]
    as the module received it (rows=False), or rows [B, N, C] from a previous run_mlp
    (rows=True).  Same results layout: [B, cout] (pool) or rows [B, N, cout]."""
    if mode == "train":
        return train.point_mlp_train(x, convs, bns, rows, pool, last_relu)
    return point_mlp(x, convs, bns, cache, pool, last_relu, module, rows)


def _fold_linear(fc, bn, cache, extra=None):
    """Linear + eval BatchNorm1d folded into one (W', b') in float64, then float32:
    W' = a*W, b' = a*(b - running_mean) + beta (+ extra), a = gamma / sqrt(running_var + eps).
    Cached until a parameter or buffer changes.  None when bn normalises with batch statistics
    (no running stats), which cannot fold."""
    tensors = [fc.weight, fc.bias]
    if bn is not None:
        if bn.running_mean is None or bn.running_var is None:
            return None
        tensors += [bn.weight, bn.bias, bn.running_mean, bn.running_var]
    if extra is not None:
        tensors.append(extra)
    key = tuple((t.data_ptr(), t._version) for t in tensors if t is not None)
    if cache.get("key") != key:
        with torch.no_grad():
            W = fc.weight.double()
            b = fc.bias.double() if fc.bias is not None else torch.zeros(W.shape[0], dtype=torch.float64,
                                                                         device=W.device)
            if bn is not None:
                a = torch.rsqrt(bn.running_var.double() + bn.eps)
                if bn.weight is not None:
                    a = a * bn.weight.double()
                W = W * a[:, None]
                b = (b - bn.running_mean.double()) * a
                if bn.bias is not None:
                    b = b + bn.bias.double()
            if extra is not None:
                b = b + extra.double().reshape(-1)
            cache["key"] = key
            cache["wb"] = (W.float().contiguous(), b.float().contiguous())
    return cache["wb"]


def linear_bn(x, fc, bn, cache, relu=True, extra=None):
    """Eval-mode ``relu(bn(fc(x)))`` (``bn`` may be None; ``extra`` a bias added after) as one
    folded GEMM with the ReLU in its epilogue: the v1 FC tails (pointnet_utils.py:33-40, the
    heads' fc / bn_fc) on B rows are launch-bound, and BatchNorm1d's eval kernels cost more than
    the GEMM.  Device tensors run on pn2_linear_rows_f32 (the library GEMMs picked for these
    shapes take 5-13 us; CPU tensors, in tests, on F.linear).  Falls back to the modules when
    the BN cannot fold."""
    wb = _fold_linear(fc, bn, cache, extra) if x.dtype == torch.float32 else None
    if wb is None:  # BN without running statistics, or a non-float32 model: the modules
        y = bn(fc(x)) if bn is not None else fc(x)
        if extra is not None:
            y = y + extra
        return F.relu(y) if relu else y
    if x.is_cuda and x.dim() == 2 and x.shape[0] >= 1 and x.stride(1) == 1:
        return ops.linear_rows(x, wb[0], wb[1], relu)
    y = F.linear(x, wb[0], wb[1])
    return y.relu_() if relu else y


def _rows_to_cf(rows):
    """[B, N, C] rows -> the reference's channel-first [B, C, N] view (no copy)."""
    return rows.permute(0, 2, 1)


def _cf_to_rows(x):
    """[B, C, N] channel-first -> [B, N, C] rows with unit column stride (copy unless it is
    already the permuted view of rows)."""
    r = x.permute(0, 2, 1)
    return r if r.stride(2) == 1 and r.stride(0) == r.shape[1] * r.stride(1) else r.contiguous()


# ----------------------------------------------------------------------------- modules
class _TNet(nn.Module):
    """Shared body of TNet3d / TNetkd (pointnet_utils.py:9-81): conv 64-128-1024 + max, FC
    512-256-k*k, + identity."""

    def _build(self, channel, k):
        self.conv1 = nn.Conv1d(channel, 64, 1)
        self.conv2 = nn.Conv1d(64, 128, 1)
        self.conv3 = nn.Conv1d(128, 1024, 1)
        self.fc1 = nn.Linear(1024, 512)
        self.fc2 = nn.Linear(512, 256)
        self.fc3 = nn.Linear(256, k * k)
        self.bn1 = nn.BatchNorm1d(64)
        self.bn2 = nn.BatchNorm1d(128)
        self.bn3 = nn.BatchNorm1d(1024)
        self.bn4 = nn.BatchNorm1d(512)
        self.bn5 = nn.BatchNorm1d(256)
        self._k = k
        self._cache = {}
        self._fc_cache = {}
        # the reference rebuilds eye(k) from numpy and copies it to the device every forward
        # (pointnet_utils.py:37-40); here it is a non-persistent buffer (state_dict unchanged)
        # that moves with the module, so the forward has no host copy and captures in a graph
        self.register_buffer("_iden", torch.from_numpy(np.eye(k).flatten().astype(np.float32)).view(1, k * k),
                             persistent=False)

    def forward(self, x):
        """x: [B, C, N] (any strides: a rows view is read as rows, not copied)."""
        B = x.size()[0]
        convs, bns = [self.conv1, self.conv2, self.conv3], [self.bn1, self.bn2, self.bn3]
        mode = mlp_mode(self, x, convs, bns)
        if mode == "torch":
            h = F.relu(self.bn1(self.conv1(x)))
            h = F.relu(self.bn2(self.conv2(h)))
            h = F.relu(self.bn3(self.conv3(h)))
            g = torch.max(h, 2, keepdim=True)[0].view(-1, 1024)
        else:
            g = run_mlp(mode, x, convs, bns, self._cache, module=self)
        if mode == "fused":  # FC + BN folded, the identity in fc3's bias
            g = linear_bn(g, self.fc1, self.bn4, self._fc_cache.setdefault(1, {}))
            g = linear_bn(g, self.fc2, self.bn5, self._fc_cache.setdefault(2, {}))
            g = linear_bn(g, self.fc3, None, self._fc_cache.setdefault(3, {}), relu=False, extra=self._iden)
            return g.view(-1, self._k, self._k)
        g = F.relu(self.bn4(self.fc1(g)))
        g = F.relu(self.bn5(self.fc2(g)))
        g = self.fc3(g)
        g = g + self._iden.expand(B, -1)
        return g.view(-1, self._k, self._k)


class TNet3d(_TNet):
    def __init__(self, channel):
        super(TNet3d, self).__init__()
        self._build(channel, 3)


class TNetkd(_TNet):
    def __init__(self, channel):
        super(TNetkd, self).__init__()
        self._build(channel, channel)
        self.channel = channel


class PointNetEncoder(nn.Module):
    """pointnet_utils.py:83-138 (same submodules, same forward, including its D > 3 branch)."""

    def __init__(self, global_feat=True, channel=3):
        super(PointNetEncoder, self).__init__()
        self.tnet = TNet3d(channel=channel)
        self.ftnet = TNetkd(channel=64)
        self.conv1 = nn.Conv1d(channel, 64, 1)
        self.conv2 = nn.Conv1d(64, 128, 1)
        self.conv3 = nn.Conv1d(128, 1024, 1)
        self.bn1 = nn.BatchNorm1d(64)
        self.bn2 = nn.BatchNorm1d(128)
        self.bn3 = nn.BatchNorm1d(1024)
        self.global_feat = global_feat
        self._c1, self._c23 = {}, {}

    def forward(self, x):
        B, D, N = x.size()
        transform = self.tnet(x)
        if D > 3:
            normal = x[:, 3:, :]
            x = x[:, :3, :]
        x = torch.bmm(transform, x)
        if D > 3:
            x = torch.cat([x, normal], dim=2)  # the reference's concatenation axis (:112)
        mode = mlp_mode(self, x, [self.conv1, self.conv2, self.conv3], [self.bn1, self.bn2, self.bn3])
        if mode == "torch":
            x = F.relu(self.bn1(self.conv1(x)))
            trans_feat = self.ftnet(x)
            x = torch.bmm(trans_feat, x)
            pointfeat = x
            x = F.relu(self.bn2(self.conv2(x)))
            x = self.bn3(self.conv3(x))
            x = torch.max(x, 2, keepdim=True)[0].view(-1, 1024)
        else:
            # conv1 + bn1 + relu per point -> rows [B, N, 64]
            r1 = run_mlp(mode, x, [self.conv1], [self.bn1], self._c1, pool=False, module=self)
            trans_feat = self.ftnet(_rows_to_cf(r1))
            # bmm(trans_feat, x) in the rows layout: x2 rows = x1 rows . trans_feat^T
            r2 = torch.bmm(r1, trans_feat.transpose(1, 2))
            pointfeat = _rows_to_cf(r2)
            # conv2 + bn2 + relu, conv3 + bn3 (no ReLU, :126-127), max over the points
            x = run_mlp(mode, r2, [self.conv2, self.conv3], [self.bn2, self.bn3], self._c23,
                        last_relu=False, module=self, rows=True)
        if self.global_feat:
            return x, transform, trans_feat
        x = x.view(-1, 1024, 1).repeat(1, 1, N)
        return torch.cat([x, pointfeat], 1), transform, trans_feat


def feature_transform_reguliarzer(transform):
    """pointnet_utils.py:140-147 (name kept as spelled in the reference)."""
    d = transform.size()[1]
    I = torch.eye(d, device=transform.device)[None, :, :]
    return torch.mean(torch.norm(torch.bmm(transform, transform.transpose(2, 1)) - I, dim=(1, 2)))


__all__ = ["TNet3d", "TNetkd", "PointNetEncoder", "feature_transform_reguliarzer", "point_mlp",
           "mlp_mode", "run_mlp", "linear_bn"]
