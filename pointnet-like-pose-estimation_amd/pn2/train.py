"""Training path of the SA layers' shared MLP: forward and backward of
(Conv 1x1 -> train-mode BatchNorm -> ReLU)* -> max over the K neighbours on channels-last rows.

Reference: pointnet2_utils.py:167-172 (and the MSG scales :211-221) run under autograd by the
training loops (train_rotation.py:99-133): Conv2d on the [B, C, K, S] grouped tensor,
BatchNorm2d with batch statistics over all B*S*K rows, ReLU, torch.max over K.

Here the rows stay channels-last [M = B*S*K, C] (the grouping's natural layout -- no [B,C,K,S]
permute copies).  The three GEMMs of each layer (Y = X W^T + b, dW = dY^T X, dX = dY W) are plain
library GEMMs (torch.mm -> hipBLASLt); the batch-statistics BatchNorm, ReLU, running-stat update,
max + argmax and their backward are the fused HIP kernels of csrc/train.hip (one pass over the
activations each).  BatchNorm semantics follow torch's train mode: biased variance normalises,
running_var takes the unbiased one, momentum None = cumulative average, num_batches_tracked += 1.

The PointNet-v1 shared MLPs (Conv1d 1x1 -> train-mode BatchNorm1d -> ReLU, /root/reference/
model/pointnet_utils.py:31-35, 118-128, and the v1 heads' conv stacks, rotation.py:37-43) are the
same computation on [M = B*N, C] rows with K = N (the max over a cloud's points) or no max at all
(the encoder's per-point conv1); the encoder's conv3 + bn3 before its max has no ReLU
(PN2_LAYER_NO_RELU): point_mlp_train.

Used by the SA modules' and the v1 modules' autograd path when a module is training on a ROCm
device (pn2/pointnet2_utils.py, pn2/pointnet_utils.py, pn2/heads_v1.py); eval with autograd
keeps the reference's torch formulation.
"""
import torch

from . import _lib
from . import ops
from .ops import _stream


def eligible(grouped, convs, bns):
    """The fused training path covers: device rows, 1x1 convs (Conv2d or Conv1d) with bias,
    affine train-mode BN."""
    if not grouped.is_cuda or grouped.dtype != torch.float32:
        return False
    for conv, bn in zip(convs, bns):
        if conv.bias is None or tuple(conv.weight.shape[2:]) not in ((1, 1), (1,)) or not bn.affine:
            return False
        if not bn.training:
            return False
    return True


def _bn_factor(bn):
    """torch's exponential_average_factor for a train-mode forward (and the counter update)."""
    if not bn.track_running_stats:
        return 0.0
    if bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    if bn.momentum is None:
        return 1.0 / float(bn.num_batches_tracked)
    return float(bn.momentum)


_CHUNK = 2048


def _grad_weight(dY, X):
    """dW = dY^T X over M rows.  A single library GEMM of this tall-skinny shape (K = M up to
    5e5, output 64x64) runs on one or two workgroups (780-850 us at SSG sa1, measured); M is cut
    into 2048-row chunks summed after a batched GEMM instead (61-151 us,
    tools/debug/gemm_shapes.py)."""
    M = dY.shape[0]
    q = M // _CHUNK
    if q < 4:
        return torch.mm(dY.t(), X)
    n = q * _CHUNK
    g = torch.bmm(dY[:n].view(q, _CHUNK, -1).transpose(1, 2), X[:n].view(q, _CHUNK, -1)).sum(0)
    if n < M:
        g += torch.mm(dY[n:].t(), X[n:])
    return g


_WS = {}


def _workspace(L, M, C, device, stream):
    """The BN sweeps' float64 partials, one grow-only buffer per (device, stream): every use is
    ordered on that stream, so forward and backward layers can share it (one allocation per
    step instead of one per call)."""
    need = int(L.pn2_bn_train_workspace_bytes(M, C))
    key = (device, stream)
    ws = _WS.get(key)
    if ws is None or ws.numel() < need:
        ws = torch.empty(max(need, 1 << 20), dtype=torch.uint8, device=device)
        _WS[key] = ws
    return ws


class _MlpMaxTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x0, K, cfg, *params):
        """x0 [M, Cin] rows; cfg[l] = (eps, momentum factor, running_mean, running_var, flags);
        params = (W, b, gamma, beta) per layer.  -> [M / K, Cout] max over each K rows, or the
        last layer's [M, Cout] rows when K == 0."""
        L = _lib.load()
        n = len(cfg)
        M = x0.shape[0]
        st = _stream(x0)
        xs, ys, stats = [x0], [], []
        x = x0
        for l in range(n):
            W, b, g, be = params[4 * l:4 * l + 4]
            eps, mom, rm, rv, flags = cfg[l]
            cout = W.shape[0]
            Y = torch.addmm(b, x, W.reshape(cout, -1).t())
            ws = _workspace(L, M, cout, x0.device, st)
            st_mi = torch.empty(2 * cout, device=x0.device)  # [mean | invstd]
            sxhat = torch.empty(cout, dtype=torch.float64, device=x0.device)
            upd = mom > 0.0 and rm is not None
            A = torch.empty_like(Y)
            _lib.check(L.pn2_bn_train_forward_f32(
                Y.data_ptr(), M, cout, cout, float(eps), float(mom) if upd else 0.0,
                rm.data_ptr() if upd else 0, rv.data_ptr() if upd else 0, g.data_ptr(),
                be.data_ptr(), A.data_ptr(), cout, flags, st_mi.data_ptr(), sxhat.data_ptr(),
                ws.data_ptr(), ws.numel(), st), "pn2_bn_train_forward_f32")
            ys.append(Y)
            stats += [st_mi[:cout], st_mi[cout:], sxhat]
            x = A
            if l + 1 < n:
                xs.append(A)
        ctx.K, ctx.n = K, n
        ctx.flags = tuple(c[4] for c in cfg)
        if not K:
            ctx.save_for_backward(*xs, *ys, *stats, *params)
            return x
        G = M // K
        cout = x.shape[1]
        out = torch.empty(G, cout, device=x0.device)
        arg = torch.empty(G, cout, dtype=torch.int32, device=x0.device)
        _lib.check(L.pn2_group_max_f32(x.data_ptr(), G, K, cout, cout, out.data_ptr(), cout,
                                       arg.data_ptr(), st), "pn2_group_max_f32")
        ctx.save_for_backward(*xs, *ys, *stats, arg, *params)
        return out

    @staticmethod
    def backward(ctx, dout):
        L = _lib.load()
        n, K = ctx.n, ctx.K
        saved = ctx.saved_tensors
        xs = saved[:n]
        ys = saved[n:2 * n]
        stats = saved[2 * n:5 * n]
        arg = saved[5 * n] if K else None
        params = saved[5 * n + (1 if K else 0):]
        dout = dout.contiguous()
        M = xs[0].shape[0]
        st = _stream(dout)
        grads = [None] * (4 * n)
        dA = None if K else dout  # K == 0: the rows' gradient is dense
        for l in reversed(range(n)):
            W, b, g, be = params[4 * l:4 * l + 4]
            Y = ys[l]
            mean, invstd, sxhat = stats[3 * l], stats[3 * l + 1], stats[3 * l + 2]
            cout = Y.shape[1]
            ws = _workspace(L, M, cout, Y.device, st)
            dY = torch.empty_like(Y)
            dgamma = torch.empty(cout, device=Y.device)
            dbeta = torch.empty(cout, device=Y.device)
            dbias = torch.empty(cout, device=Y.device)
            last = l == n - 1 and K
            _lib.check(L.pn2_bn_relu_backward_f32(
                Y.data_ptr(), M, cout, cout, mean.data_ptr(), invstd.data_ptr(), g.data_ptr(),
                be.data_ptr(), 0 if last else dA.data_ptr(), cout,
                dout.data_ptr() if last else 0, cout, arg.data_ptr() if last else 0, K,
                sxhat.data_ptr(), dY.data_ptr(), cout, dgamma.data_ptr(), dbeta.data_ptr(),
                dbias.data_ptr(), ws.data_ptr(), ws.numel(), ctx.flags[l], st),
                "pn2_bn_relu_backward_f32")
            X = xs[l]
            W2 = W.reshape(cout, -1)
            grads[4 * l] = _grad_weight(dY, X).view_as(W)
            grads[4 * l + 1] = dbias  # sum_r dY, from the BN sums (no extra pass over dY)
            grads[4 * l + 2] = dgamma
            grads[4 * l + 3] = dbeta
            if l > 0 or ctx.needs_input_grad[0]:
                dA = torch.mm(dY, W2)
        return (dA if ctx.needs_input_grad[0] else None, None, None, *grads)


class _GroupTrain(torch.autograd.Function):
    """Grouping with a gradient for the features only (coordinates and centroids carry none in
    the SA layers: they come from index ops of the input).  Forward: pn2_group_f32 (the same
    rows as the reference's index_points + cat, pointnet2_utils.py:107-116 / 204-209);
    backward: the feature rows' gradients added back to their source points (index_add_ --
    atomic adds, instead of advanced indexing's sort-based backward)."""

    @staticmethod
    def forward(ctx, feature, points, centers, idx, feature_first):
        ctx.save_for_backward(idx)
        ctx.meta = (feature.shape, points.shape[2], bool(feature_first))
        return ops.group_direct(points, feature, centers, idx, feature_first)

    @staticmethod
    def backward(ctx, dgrouped):
        idx, = ctx.saved_tensors
        (B, N, D), C, ff = ctx.meta
        dfeat = dgrouped[..., :D] if ff else dgrouped[..., C:]
        flat = (idx + torch.arange(B, device=idx.device).view(B, 1, 1) * N).reshape(-1)
        out = torch.zeros(B * N, D, device=dgrouped.device, dtype=dgrouped.dtype)
        out.index_add_(0, flat, dfeat.reshape(-1, D))
        return out.view(B, N, D), None, None, None, None


def group_train(points, idx, centers, feature, feature_first):
    """[B,S,K,C+D] grouped rows for the training path (pn2/pointnet2_utils._torch_group's
    contract), or None when this path does not apply (no features needing a gradient, or
    coordinates that need one)."""
    if (feature is None or not feature.requires_grad or points.requires_grad or
            centers.requires_grad or not points.is_cuda):
        return None
    return _GroupTrain.apply(feature, points, centers, idx, feature_first)


def _apply(x0, K, convs, bns, last_relu=True):
    cfg, params = [], []
    n = len(convs)
    for l, (conv, bn) in enumerate(zip(convs, bns)):
        mom = _bn_factor(bn)
        flags = _lib.LAYER_NO_RELU if (l == n - 1 and not last_relu) else 0
        cfg.append((bn.eps, mom, bn.running_mean if mom > 0 else None,
                    bn.running_var if mom > 0 else None, flags))
        params += [conv.weight, conv.bias, bn.weight, bn.bias]
    return _MlpMaxTrain.apply(x0, K, tuple(cfg), *params)


def mlp_max_train(grouped, convs, bns):
    """grouped [B, S, K, Cin] (any float32 device tensor, autograd-tracked) -> [B, Cout, S]:
    the reference's ``torch.max(relu(bn(conv(x)))..., 2)[0]`` in train mode (:167-172)."""
    B, S, K, Cin = grouped.shape
    x0 = grouped.reshape(B * S * K, Cin)
    if not x0.is_contiguous():
        x0 = x0.contiguous()
    out = _apply(x0, K, convs, bns)
    return out.view(B, S, -1).permute(0, 2, 1)


def point_mlp_train(x, convs, bns, rows, pool=True, last_relu=True):
    """The v1 shared MLP in train mode, pn2.pointnet_utils.point_mlp's contract: x channel-first
    [B, C, N] (rows=False) or per-point rows [B, N, C] (rows=True), autograd-tracked; returns
    the max over the points [B, Cout] (pool) or rows [B, N, Cout].  The reference's
    relu(bn(conv(x)))* (+ torch.max(x, 2)) with Conv1d / BatchNorm1d in train mode
    (pointnet_utils.py:31-35, 118-128); last_relu=False drops the last ReLU (:127)."""
    if rows:
        B, N, C = x.shape
        x0 = x.reshape(B * N, C)
    else:
        B, C, N = x.shape
        x0 = x.permute(0, 2, 1).reshape(B * N, C)
    if not x0.is_contiguous():
        x0 = x0.contiguous()
    out = _apply(x0, N if pool else 0, convs, bns, last_relu)
    return out if pool else out.view(B, N, -1)


__all__ = ["mlp_max_train", "point_mlp_train", "group_train", "eligible"]
