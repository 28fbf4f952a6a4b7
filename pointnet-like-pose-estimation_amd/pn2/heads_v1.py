"""Layer-config restatements of the reference's PointNet-v1 heads,
built on pn2's v1 drop-in (pn2/pointnet_utils.py).

Like heads.py: submodules are created in the reference's order, so ``torch.manual_seed``
before construction gives the identical parameters (pinned by the state_dict hash in the
v1_*.npz goldens) and the ``state_dict`` keys match the reference's checkpoints.  The per-point
shared MLP + max over the points -- the whole cost of these networks -- runs on the split-bf16
dense-layer kernels through ``point_mlp`` in eval mode on the GPU, and on pn2.train's fused
batch-statistics kernels when training on the GPU; the FC tails are [B, 1024] library GEMMs
(torch), each Linear + eval BatchNorm1d folded into one GEMM in eval (``linear_bn``).

  PointNetCls    /root/reference/model/pointnet_cls.py:7-32
  RotationV1     /root/reference/model/rotation.py:7-50 (its T-Net output is computed and
                 unused, as in the reference)
  TranslationV1  /root/reference/model/translation.py:6-50
  SignV1         /root/reference/model/sign.py:6-44
  WidthV1        /root/reference/model/width.py:7-44
  PoseV1         /root/reference/model/pose.py:7-91
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .pointnet2_utils import _needs_autograd
from .pointnet_utils import (PointNetEncoder, TNet3d, TNetkd, _rows_to_cf, linear_bn, mlp_mode,
                             run_mlp)


class _ConvStack(nn.Module):
    """The v1 heads' ``conv`` / ``bn_conv`` ModuleLists and the ``fc`` / ``bn_fc`` tail
    (rotation.py:12-25 and the same blocks in translation / sign / width / pose)."""

    def _build(self, channel, mlp_list, linear_list):
        self.conv = nn.ModuleList()
        self.bn_conv = nn.ModuleList()
        cin = channel
        for cout in mlp_list:
            self.conv.append(nn.Conv1d(cin, cout, 1))
            self.bn_conv.append(nn.BatchNorm1d(cout))
            cin = cout
        self.fc = nn.ModuleList()
        self.bn_fc = nn.ModuleList()
        for cout in linear_list:
            self.fc.append(nn.Linear(cin, cout))
            self.bn_fc.append(nn.BatchNorm1d(cout))
            cin = cout
        self._caches = {}
        self._fc_cache = {}

    def _mode(self, x):
        """mlp_mode over the whole conv stack: "fused" (eval without autograd: the HIP kernels,
        device tensors only -- a CPU tensor raises, there is no CPU fallback), "train" (training
        on the device: pn2.train) or "torch" (the reference's formulation)."""
        return mlp_mode(self, x, list(self.conv), list(self.bn_conv))

    def _layers(self, x, lo, hi, pool, mode, rows=False):
        """relu(bn_conv[i](conv[i](x))) for i in [lo, hi), then the max over the points when
        pool.  "fused" / "train": x channel-first [B, C, N] as the head received it, or rows
        [B, N, C] (rows=True) from a previous call; returns [B, 1024] (pool) or rows
        [B, N, cout].  "torch": the reference's ops on channel-first tensors."""
        if mode == "torch":
            for i in range(lo, hi):
                x = F.relu(self.bn_conv[i](self.conv[i](x)))
            return torch.max(x, 2, keepdim=True)[0].view(-1, x.shape[1]) if pool else x
        return run_mlp(mode, x, list(self.conv[lo:hi]), list(self.bn_conv[lo:hi]),
                       self._caches.setdefault((lo, hi), {}), pool=pool, module=self, rows=rows)

    def _tail(self, x, mode=None):
        """fc / bn_fc / dropout / relu for all but the last fc (rotation.py:45-49); "fused":
        each fc + bn_fc folded into one GEMM (dropout is the identity in eval)."""
        if mode == "fused":
            n = len(self.fc)
            for i in range(n):
                x = linear_bn(x, self.fc[i], self.bn_fc[i] if i < n - 1 else None,
                              self._fc_cache.setdefault(i, {}), relu=i < n - 1)
            return x
        for i in range(len(self.fc)):
            if i < len(self.fc) - 1:
                x = F.relu(self.dropout(self.bn_fc[i](self.fc[i](x))))
            else:
                x = self.fc[i](x)
        return x

    def _split_ftnet(self, x, mode):
        """Layers 0-1, the feature T-Net on their output, layers 2.. + max (rotation.py:37-43,
        pose.py:59-69).  Returns (layer-1 output -- rows unless mode is "torch", then
        channel-first -- and the T-Net's T)."""
        h = self._layers(x, 0, 2, False, mode)
        if mode != "torch":
            return h, self.ftnet(_rows_to_cf(h))
        return h, self.ftnet(h)


class PointNetCls(nn.Module):
    def __init__(self, num_category=7):
        super().__init__()
        self.feat = PointNetEncoder(channel=3)
        self.fc1 = nn.Linear(1024, 512)
        self.fc2 = nn.Linear(512, 256)
        self.fc3 = nn.Linear(256, num_category)
        self.dropout = nn.Dropout(p=0.4)
        self.bn1 = nn.BatchNorm1d(512)
        self.bn2 = nn.BatchNorm1d(256)
        self._fc_cache = {}

    def forward(self, x):
        x, _, trans_feat = self.feat(x)
        if not _needs_autograd(self, x):  # eval: fc + bn folded (dropout is the identity)
            x = linear_bn(x, self.fc1, self.bn1, self._fc_cache.setdefault(1, {}))
            x = linear_bn(x, self.fc2, self.bn2, self._fc_cache.setdefault(2, {}))
            x = linear_bn(x, self.fc3, None, self._fc_cache.setdefault(3, {}), relu=False)
        else:
            x = F.relu(self.bn1(self.fc1(x)))
            x = F.relu(self.bn2(self.dropout(self.fc2(x))))
            x = self.fc3(x)
        x = F.log_softmax(x, dim=1)
        return x, trans_feat, x.data.max(1)[1]


class RotationV1(_ConvStack):
    def __init__(self, mlp_list=(64, 64, 64, 128, 1024), linear_list=(512, 256, 3), num_category=7):
        super().__init__()
        self._build(3 + num_category, mlp_list, linear_list)
        self.ftnet = TNetkd(channel=64)
        self.dropout = nn.Dropout(p=0.4)

    def forward(self, x):
        mode = self._mode(x)
        h, _ = self._split_ftnet(x, mode)
        return self._tail(self._layers(h, 2, len(self.conv), True, mode, rows=mode != "torch"), mode)


class TranslationV1(_ConvStack):
    def __init__(self, mlp_list=(64, 64, 64, 128, 1024), linear_list=(512, 256, 3), num_category=7,
                 mean_mlp='True'):
        super().__init__()
        self.mean_mlp = mean_mlp
        self._build(3 + num_category, mlp_list, linear_list)
        if mean_mlp == 'True':  # string compare, as the reference (translation.py:27)
            self.fc1 = nn.Linear(3, 6)
            self.fc2 = nn.Linear(6, 3)
            self.bn1 = nn.BatchNorm1d(6)
        self.dropout = nn.Dropout(p=0.4)

    def forward(self, x, mean):
        if self.mean_mlp == 'True':
            mean = self.fc2(F.relu(self.bn1(self.fc1(mean))))
        mode = self._mode(x)
        return self._tail(self._layers(x, 0, len(self.conv), True, mode), mode) + mean


class SignV1(_ConvStack):
    def __init__(self, mlp_list=(64, 64, 64, 128, 1024), linear_list=(512, 256, 1), num_category=7):
        super().__init__()
        self._build(3 + num_category, mlp_list, linear_list)
        self.dropout = nn.Dropout(p=0.4)

    def forward(self, x):
        mode = self._mode(x)
        x = torch.sigmoid(self._tail(self._layers(x, 0, len(self.conv), True, mode), mode))
        return x, torch.sign(x - 0.5)


class WidthV1(_ConvStack):
    def __init__(self, mlp_list=(64, 64, 64, 128, 1024), linear_list=(512, 256, 1), num_category=7,
                 normal_channel=True):
        super().__init__()
        self._build((6 if normal_channel else 3) + num_category, mlp_list, linear_list)
        self.dropout = nn.Dropout(p=0.4)

    def forward(self, x):
        mode = self._mode(x)
        return self._tail(self._layers(x, 0, len(self.conv), True, mode), mode)


class PoseV1(_ConvStack):
    """pose.py's configurable head.  Its ``mean`` branch indexes the 2-D FC output with three
    subscripts (pose.py:79) and raises in the reference; it raises the same IndexError here."""

    def __init__(self, mlp_list, linear_list, mean=False, classify=False, num_category=7,
                 normal_channel=True, transform=False, feat_trans=False):
        super().__init__()
        channel = (6 if normal_channel else 3) + num_category
        if transform:
            self.tnet = TNet3d(channel=channel)
        if feat_trans:
            self.ftnet = TNetkd(channel=64)
        self._build(channel, mlp_list, linear_list)
        if mean:
            self.fc1 = nn.Linear(3, 6)
            self.fc2 = nn.Linear(6, 3)
            self.bn1 = nn.BatchNorm1d(6)
        self.dropout = nn.Dropout(p=0.4)
        self.mean = mean
        self.classify = classify
        self.transform = transform
        self.feat_trans = feat_trans

    def forward(self, x):
        B, D, N = x.size()
        if self.transform:
            transform = self.tnet(x)
            if D > 3:
                normal = x[:, 3:, :]
                x = x[:, :3, :]
            x = torch.bmm(transform, x)
            if D > 3:
                x = torch.cat([x, normal], dim=2)  # the reference's axis (pose.py:57)
        mode = self._mode(x)
        if self.feat_trans:
            h, trans_feat = self._split_ftnet(x, mode)
            if mode != "torch":  # bmm(trans_feat, x) in the rows layout
                h = torch.bmm(h, trans_feat.transpose(1, 2))
            else:
                h = torch.bmm(trans_feat, h)
            x = self._layers(h, 2, len(self.conv), True, mode, rows=mode != "torch")
        else:
            x = self._layers(x, 0, len(self.conv), True, mode)
        x = self._tail(x, mode)
        if self.mean:
            mean = torch.mean(x[:, :3, :], dim=2)
            mean = self.fc2(F.relu(self.bn1(self.fc1(mean))))
            return mean + x
        if self.classify:
            x = F.log_softmax(x, dim=1)
            pred_choice = x.data.max(1)[1]
            return x, (-1) ** pred_choice, pred_choice
        return x


HEADS_V1 = {
    "pointnet_cls": PointNetCls,
    "rotation": RotationV1,
    "translation": TranslationV1,
    "sign": SignV1,
    "width": WidthV1,
    "pose": PoseV1,
}

__all__ = ["PointNetCls", "RotationV1", "TranslationV1", "SignV1", "WidthV1", "PoseV1", "HEADS_V1"]
