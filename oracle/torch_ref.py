"""PyTorch-CPU restatement of the reference's PointNet++ forward FORMULATION, used as the
cpu_baseline leg of bench.py (the reference itself never travels to the GPU box).

TEST/BENCH INFRASTRUCTURE ONLY -- never imported by the product.

It performs the same op sequence as /root/reference/model/pointnet2_utils.py, so it costs what
the reference costs on the same cores:
  FPS       Python loop of S dependent iterations of small torch ops      (:47-68)
  distances matmul + two channel sums, [B,S,N] materialised             (:5-26)
  ball query mask + full sort of every [N] row, first K, pad            (:70-90)
  grouping  advanced-index gathers + subtraction + concat               (:92-141)
  MLP       Conv2d 1x1 -> BatchNorm2d (eval) -> ReLU per layer, max(K)  (:158-174)
and the pointnet2_cls_ssg head (/root/reference/model/pointnet2_cls_ssg.py:22-38).  Weights
come from a state_dict with the reference's keys (any pn2 / reference model's).
"""
import torch
import torch.nn.functional as F


def _gather(points, idx):
    B = points.shape[0]
    bidx = torch.arange(B).view((B,) + (1,) * (idx.dim() - 1)).expand_as(idx)
    return points[bidx, idx, :]


def _sqdist(src, dst):
    d = -2 * torch.matmul(src, dst.transpose(1, 2))
    d += torch.sum(src ** 2, -1).unsqueeze(-1)
    d += torch.sum(dst ** 2, -1).unsqueeze(1)
    return d


def _fps(points, S):
    B, N, C = points.shape
    out = torch.zeros(B, S, dtype=torch.long)
    dist = torch.full((B, N), 1e10)
    far = torch.randint(0, N, (B,), dtype=torch.long)
    ar = torch.arange(B)
    for i in range(S):
        out[:, i] = far
        c = points[ar, far, :].view(B, 1, C)
        d = torch.sum((points - c) ** 2, -1)
        m = d < dist
        dist[m] = d[m]
        far = torch.max(dist, -1)[1]
    return out


def _ball(radius, K, points, centers):
    B, N, _ = points.shape
    S = centers.shape[1]
    idx = torch.arange(N).view(1, 1, N).repeat(B, S, 1)
    idx[_sqdist(centers, points) > radius ** 2] = N
    idx = idx.sort(dim=-1)[0][:, :, :K]
    first = idx[:, :, :1].expand(-1, -1, K)
    pad = idx == N
    idx[pad] = first[pad]
    return idx


def _mlp_max(x, sd, prefix, n):
    x = x.permute(0, 3, 2, 1)
    for i in range(n):
        w = sd["%s.mlp_convs.%d.weight" % (prefix, i)]
        b = sd["%s.mlp_convs.%d.bias" % (prefix, i)]
        x = F.conv2d(x, w, b)
        x = F.batch_norm(x, sd["%s.mlp_bns.%d.running_mean" % (prefix, i)],
                         sd["%s.mlp_bns.%d.running_var" % (prefix, i)],
                         sd["%s.mlp_bns.%d.weight" % (prefix, i)],
                         sd["%s.mlp_bns.%d.bias" % (prefix, i)], False, 0.1, 1e-5)
        x = F.relu(x)
    return torch.max(x, 2)[0]


def sa_ssg(sd, prefix, points, feature, S, K, radius, n_layers, group_all=False):
    """One PointNetSetAbstraction forward; points [B,C,N], feature [B,D,N] or None."""
    p = points.permute(0, 2, 1)
    f = None if feature is None else feature.permute(0, 2, 1)
    B, N, C = p.shape
    if group_all:
        newp = torch.zeros(B, 1, C)
        g = p.reshape(B, 1, N, C)
        if f is not None:
            g = torch.cat([g, f.reshape(B, 1, N, -1)], -1)
    else:
        newp = _gather(p, _fps(p, S))
        idx = _ball(radius, K, p, newp)
        g = _gather(p, idx) - newp.view(B, S, 1, C)
        if f is not None:
            g = torch.cat([g, _gather(f, idx)], -1)
    return newp.permute(0, 2, 1), _mlp_max(g, sd, prefix, n_layers)


def cls_ssg_forward(sd, points):
    """pointnet2_cls_ssg.get_model.forward (eval): returns log-probabilities [B, k]."""
    B = points.shape[0]
    l1p, l1f = sa_ssg(sd, "sa1", points, None, 512, 32, 0.2, 3)
    l2p, l2f = sa_ssg(sd, "sa2", l1p, l1f, 128, 64, 0.4, 3)
    _, l3f = sa_ssg(sd, "sa3", l2p, l2f, None, None, None, 3, group_all=True)
    x = l3f.view(B, 1024)
    for i, (fc, bn) in enumerate((("fc1", "bn1"), ("fc2", "bn2"))):
        x = F.linear(x, sd[fc + ".weight"], sd[fc + ".bias"])
        x = F.batch_norm(x, sd[bn + ".running_mean"], sd[bn + ".running_var"], sd[bn + ".weight"],
                         sd[bn + ".bias"], False, 0.1, 1e-5)
        x = F.relu(x)
    x = F.linear(x, sd["fc3.weight"], sd["fc3.bias"])
    return F.log_softmax(x, -1)
