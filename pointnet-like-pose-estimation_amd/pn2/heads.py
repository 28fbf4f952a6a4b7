"""Layer-config restatements of the reference's PointNet++ heads, built on pn2's SA modules.

The reference heads import ``pointnet2_utils`` by bare name and run unchanged on the drop-in
(tests/test_host.py loads their checkpoints into these classes strictly and checks the
constructor draws; tests/golden/make_goldens.py runs the reference heads themselves to make the
head_*/full_* goldens the GPU tests compare against); the reference sources never travel to the GPU box, so
the benchmark and the on-box parity tests build the same networks from these restatements.
Submodules are created in the reference's order, so a ``torch.manual_seed`` before
construction yields the identical parameters (pinned by a state_dict hash in the goldens) and
the ``state_dict`` keys match the reference's checkpoints.

  ClsSSG          /root/reference/model/pointnet2_cls_ssg.py:5-38
  ClsMSG          /root/reference/model/pointnet2_cls_msg.py:5-38
  RotationSSG     /root/reference/model/rotation_ssg.py:5-38
  TranslationSSG  /root/reference/model/translation_ssg.py:5-44
  RotationMSG     /root/reference/model/rotation_msg.py:5-38
  TranslationMSG  /root/reference/model/translation_msg.py:5-44
  SignSSG         /root/reference/model/sign_ssg.py:5-36 (with the missing `import torch`)
  SignMSG         /root/reference/model/sign_msg.py:5-36 (likewise)
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .pointnet2_utils import PointNetSetAbstraction as SA
from .pointnet2_utils import PointNetSetAbstractionMsg as SAMsg
from .pointnet2_utils import _needs_autograd
from . import geometry
from . import ops
from . import tuning
from .pointnet_utils import _fold_linear, linear_bn


class _FCHead(nn.Module):
    """fc1/bn1/relu/drop -> fc2/bn2/relu/drop -> fc3, shared by every head.  Eval without
    autograd: each fc + bn folded into one (W', b') and the whole tail in three launches
    (pn2.ops.fc_tail: fc1 and fc2 as row kernels, then fc3 fused with the classifiers'
    log_softmax and argmax; dropout is the identity in eval).  Otherwise, or when a layer cannot fold, the reference's modules."""

    def _folded(self):
        c = self._fc_cache
        wb = [_fold_linear(self.fc1, self.bn1, c.setdefault(1, {})),
              _fold_linear(self.fc2, self.bn2, c.setdefault(2, {})),
              _fold_linear(self.fc3, None, c.setdefault(3, {}))]
        return None if any(t is None for t in wb) else wb

    def _fused_ok(self, x):
        return (tuning.get("fc_tail") and not _needs_autograd(self, x) and x.is_cuda and x.dtype == torch.float32 and
                x.dim() == 2 and x.stride(1) == 1 and self.fc3.out_features <= 819)

    def _fc(self, x):
        if self._fused_ok(x):
            wb = self._folded()
            if wb is not None:
                return ops.fc_tail(x, wb, False)[0]
        if not _needs_autograd(self, x):
            x = linear_bn(x, self.fc1, self.bn1, self._fc_cache.setdefault(1, {}))
            x = linear_bn(x, self.fc2, self.bn2, self._fc_cache.setdefault(2, {}))
            return linear_bn(x, self.fc3, None, self._fc_cache.setdefault(3, {}), relu=False)
        x = self.drop(F.relu(self.bn1(self.fc1(x))))
        x = self.drop(F.relu(self.bn2(self.fc2(x))))
        return self.fc3(x)

    def _mean_mlp(self, mean):
        """translation_ssg.py:23-33's mean MLP, mean_fc2(relu(mean_bn1(mean_fc1(mean)))).  Eval
        without autograd: mean_fc1 + mean_bn1 folded, ReLU in the epilogue, then mean_fc2, on
        pn2_linear_rows_f32 -- a [B, 3] x [3, 6] product is not worth two library GEMM launches
        and BatchNorm1d's kernels.  Otherwise (or when mean_bn1 cannot fold) the modules."""
        if not _needs_autograd(self, mean) and mean.is_cuda:
            c = self._fc_cache
            h = linear_bn(mean, self.mean_fc1, self.mean_bn1, c.setdefault("mean1", {}))
            return linear_bn(h, self.mean_fc2, None, c.setdefault("mean2", {}), relu=False)
        return self.mean_fc2(F.relu(self.mean_bn1(self.mean_fc1(mean))))

    def _fc_log_softmax(self, x):
        """(F.log_softmax(fc(x), -1), its first argmax per row): pointnet2_cls_ssg.py:36-38."""
        if self._fused_ok(x):
            wb = self._folded()
            if wb is not None:
                return ops.fc_tail(x, wb, True)
        y = F.log_softmax(self._fc(x), -1)
        return y, y.data.max(1)[1]

    def _make_fc(self, out):
        self.fc1 = nn.Linear(1024, 512)
        self.fc2 = nn.Linear(512, 256)
        self.fc3 = nn.Linear(256, out)
        self.drop = nn.Dropout(0.4)
        self.bn1 = nn.BatchNorm1d(512)
        self.bn2 = nn.BatchNorm1d(256)
        self._fc_cache = {}


class ClsSSG(_FCHead):
    def __init__(self, num_category=7):
        super().__init__()
        self.sa1 = SA(512, 32, 0.2, 3, [64, 64, 128], False)
        self.sa2 = SA(128, 64, 0.4, 128 + 3, [128, 128, 256], False)
        self.sa3 = SA(None, None, None, 256 + 3, [256, 512, 1024], True)
        self._make_fc(num_category)

    def forward(self, points):
        B = points.shape[0]
        with geometry.fps_ahead(self.sa1, self.sa2):  # sa2's FPS inside sa1's MLP launch
            l1p, l1f = self.sa1(points, None)
            l2p, l2f = self.sa2(l1p, l1f)
        _, l3f = self.sa3(l2p, l2f)
        x, pred = self._fc_log_softmax(l3f.reshape(B, 1024))
        return x, l3f, pred


class ClsMSG(_FCHead):
    def __init__(self, num_category=7):
        super().__init__()
        self.sa1 = SAMsg(512, [16, 32, 128], [0.1, 0.2, 0.4], 0, [[32, 32, 64], [64, 64, 128], [64, 96, 128]])
        self.sa2 = SAMsg(128, [32, 64, 128], [0.2, 0.4, 0.8], 320, [[64, 64, 128], [128, 128, 256], [128, 128, 256]])
        self.sa3 = SA(None, None, None, 640 + 3, [256, 512, 1024], True)
        self._make_fc(num_category)

    def forward(self, points):
        B = points.shape[0]
        with geometry.fps_ahead(self.sa1, self.sa2):  # sa2's FPS inside sa1's MLP launch
            l1p, l1f = self.sa1(points, None)
            l2p, l2f = self.sa2(l1p, l1f)
        _, l3f = self.sa3(l2p, l2f)
        x, pred = self._fc_log_softmax(l3f.reshape(B, 1024))
        return x, l3f, pred


class RotationSSG(_FCHead):
    def __init__(self, num_category=7):
        super().__init__()
        ch = 3 + num_category
        self.sa1 = SA(512, 32, 0.2, ch, [64, 64, 128], False)
        self.sa2 = SA(128, 64, 0.4, 128 + ch, [128, 128, 256], False)
        self.sa3 = SA(None, None, None, 256 + ch, [256, 512, 1024], True)
        self._make_fc(3)

    def forward(self, points):
        B = points.shape[0]
        with geometry.fps_ahead(self.sa1, self.sa2):  # sa2's FPS inside sa1's MLP launch
            l1p, l1f = self.sa1(points, None)
            l2p, l2f = self.sa2(l1p, l1f)
        _, l3f = self.sa3(l2p, l2f)
        return self._fc(l3f.reshape(B, 1024))


class TranslationSSG(_FCHead):
    def __init__(self, num_category=7, mean_mlp='True'):
        super().__init__()
        self.mean_mlp = mean_mlp
        ch = 3 + num_category
        self.sa1 = SA(512, 32, 0.2, ch, [64, 64, 128], False)
        self.sa2 = SA(None, None, None, 128 + ch, [256, 512, 1024], True)
        self._make_fc(3)
        if mean_mlp == 'True':  # string compare, as the reference (translation_ssg.py:23)
            self.mean_fc1 = nn.Linear(3, 6)
            self.mean_fc2 = nn.Linear(6, 3)
            self.mean_bn1 = nn.BatchNorm1d(6)

    def forward(self, points, mean):
        B = points.shape[0]
        if self.mean_mlp == 'True':
            mean = self._mean_mlp(mean)
        l1p, l1f = self.sa1(points, None)
        _, l2f = self.sa2(l1p, l1f)
        return self._fc(l2f.reshape(B, 1024)) + mean


class RotationMSG(_FCHead):
    def __init__(self, num_category=7):
        super().__init__()
        ch = 3 + num_category
        self.sa1 = SAMsg(512, [16, 32, 128], [0.1, 0.2, 0.4], 0, [[32, 32, 64], [64, 64, 128], [64, 96, 128]], num_category=num_category)
        self.sa2 = SAMsg(128, [32, 64, 128], [0.2, 0.4, 0.8], 320, [[64, 64, 128], [128, 128, 256], [128, 128, 256]], num_category=num_category)
        self.sa3 = SA(None, None, None, 640 + ch, [256, 512, 1024], True)
        self._make_fc(3)

    def forward(self, points):
        B = points.shape[0]
        with geometry.fps_ahead(self.sa1, self.sa2):  # sa2's FPS inside sa1's MLP launch
            l1p, l1f = self.sa1(points, None)
            l2p, l2f = self.sa2(l1p, l1f)
        _, l3f = self.sa3(l2p, l2f)
        return self._fc(l3f.reshape(B, 1024))


class TranslationMSG(_FCHead):
    def __init__(self, num_category=7, mean_mlp='True'):
        super().__init__()
        self.mean_mlp = mean_mlp
        ch = 3 + num_category
        self.sa1 = SAMsg(512, [16, 32, 64], [0.1, 0.2, 0.4], 0, [[32, 64, 128], [64, 128, 256], [96, 128, 256]], num_category=num_category)
        self.sa2 = SA(None, None, None, 640 + ch, [256, 512, 1024], True)
        self._make_fc(3)
        if mean_mlp == 'True':
            self.mean_fc1 = nn.Linear(3, 6)
            self.mean_fc2 = nn.Linear(6, 3)
            self.mean_bn1 = nn.BatchNorm1d(6)

    def forward(self, points, mean):
        B = points.shape[0]
        if self.mean_mlp == 'True':
            mean = self._mean_mlp(mean)
        l1p, l1f = self.sa1(points, None)
        _, l2f = self.sa2(l1p, l1f)
        return self._fc(l2f.reshape(B, 1024)) + mean


class SignSSG(_FCHead):
    def __init__(self, num_category=7):
        super().__init__()
        ch = 3 + num_category
        self.sa1 = SA(512, 32, 0.2, ch, [64, 64, 128], False)
        self.sa2 = SA(None, None, None, 128 + ch, [256, 512, 1024], True)
        self._make_fc(1)

    def forward(self, points):
        B = points.shape[0]
        l1p, l1f = self.sa1(points, None)
        _, l2f = self.sa2(l1p, l1f)
        x = torch.sigmoid(self._fc(l2f.reshape(B, 1024)))
        return x, torch.sign(x - 0.5)


class SignMSG(_FCHead):
    def __init__(self, num_category=7):
        super().__init__()
        ch = 3 + num_category
        self.sa1 = SAMsg(512, [16, 32, 64], [0.1, 0.2, 0.4], 0, [[32, 64, 128], [64, 128, 256], [96, 128, 256]], num_category=num_category)
        self.sa2 = SA(None, None, None, 640 + ch, [256, 512, 1024], True)
        self._make_fc(1)

    def forward(self, points):
        B = points.shape[0]
        l1p, l1f = self.sa1(points, None)
        _, l2f = self.sa2(l1p, l1f)
        x = torch.sigmoid(self._fc(l2f.reshape(B, 1024)))
        return x, torch.sign(x - 0.5)


class ReferenceForward(nn.Module):
    """What the reference's own head file computes through the drop-in: its forward restated
    call for call -- the SA modules one after the other (no FPS side job: an unchanged
    reference head never enters ``geometry.fps_ahead``) and the FC tail as the torch modules
    fc/bn/relu/drop, log_softmax and ``x.data.max(1)[1]``.  Wraps one of the heads above (same
    parameters); bench.py's ``eager_value_reference_head`` times it.

      pointnet2_cls_ssg.py:22-38, pointnet2_cls_msg.py:22-38, rotation_ssg.py:24-38,
      rotation_msg.py:24-38, translation_ssg.py:28-44, translation_msg.py:28-44
    """

    def __init__(self, head):
        super().__init__()
        self.head = head

    def _tail(self, x):
        h = self.head
        x = h.drop(F.relu(h.bn1(h.fc1(x))))
        x = h.drop(F.relu(h.bn2(h.fc2(x))))
        return h.fc3(x)

    def forward(self, points, mean=None):
        h = self.head
        B = points.shape[0]
        if isinstance(h, (TranslationSSG, TranslationMSG)) and h.mean_mlp == 'True':
            mean = h.mean_fc2(F.relu(h.mean_bn1(h.mean_fc1(mean))))
        l1p, l1f = h.sa1(points, None)
        l2p, l2f = h.sa2(l1p, l1f)
        if hasattr(h, "sa3"):
            _, feat = h.sa3(l2p, l2f)
        else:
            feat = l2f
        x = self._tail(feat.view(B, 1024))
        if isinstance(h, (ClsSSG, ClsMSG)):
            x = F.log_softmax(x, -1)
            return x, feat, x.data.max(1)[1]
        if isinstance(h, (TranslationSSG, TranslationMSG)):
            return x + mean
        if isinstance(h, (SignSSG, SignMSG)):
            x = torch.sigmoid(x)
            return x, torch.sign(x - 0.5)
        return x


HEADS = {
    "pointnet2_cls_ssg": ClsSSG,
    "pointnet2_cls_msg": ClsMSG,
    "rotation_ssg": RotationSSG,
    "translation_ssg": TranslationSSG,
    "rotation_msg": RotationMSG,
    "translation_msg": TranslationMSG,
    "sign_ssg": SignSSG,
    "sign_msg": SignMSG,
}
