"""Deterministic inputs shared by the golden generator (make_goldens.py, run in the survey
container against the imported reference) and the tests (run anywhere, incl. the GPU box).

Everything is derived from seeds with torch's CPU generators, so the same torch version
regenerates the same tensors; the goldens also store the inputs, and tests check both.
"""
import hashlib

import numpy as np
import torch


def cloud(kind, B, N, seed, labels=None):
    """A [B, N, C] float32 cloud (contiguous), unit-sphere normalised like provider.normalization
    (/root/reference/provider.py:5-21).  kind:
      'uniform3'  U[-1,1)^3
      'dup3'      uniform, then provider.random_point_dropout-style duplication of point 0
                  (/root/reference/provider.py:157-164): many exact duplicates -> FPS ties
      'onehot10'  xyz + 7-way one-hot of `labels` (provider.splice_torch, provider.py:166-180)
      'randn<C>'  N(0,1) in all C channels (not a real input; pins the channel-sum order:
                  randn10, and randn24 / randn40 / randn64 past the register-resident C <= 16)
    """
    g = torch.Generator().manual_seed(seed)
    if kind.startswith('randn'):
        return torch.randn(B, N, int(kind[5:]), generator=g)
    xyz = torch.rand(B, N, 3, generator=g) * 2 - 1
    if kind == 'dup3':
        for b in range(B):
            ratio = float(torch.rand(1, generator=g)) * 0.875
            drop = torch.rand(N, generator=g) <= ratio
            xyz[b, drop] = xyz[b, 0].clone()
    xyz = xyz - xyz.mean(1, keepdim=True)
    xyz = xyz / xyz.norm(dim=2).max(1)[0].view(B, 1, 1)
    if kind in ('uniform3', 'dup3'):
        return xyz.contiguous()
    if kind == 'onehot10':
        if labels is None:
            labels = torch.arange(B) % 7
        oh = torch.zeros(B, N, 7)
        oh[torch.arange(B), :, labels] = 1.0
        return torch.cat([xyz, oh], 2).contiguous()
    raise ValueError(kind)


def as_layout(pts_bnc, layout):
    """[B,N,C] view with the requested storage: 'contig' ([B,N,C] storage) or 'strided'
    ([B,C,N] storage, i.e. the permute(0,2,1) of the reference's model input)."""
    if layout == 'contig':
        return pts_bnc.contiguous()
    return pts_bnc.permute(0, 2, 1).contiguous().permute(0, 2, 1)


def randomize_bn(model, seed):
    """Non-trivial eval-mode BatchNorm statistics/affine, in module order."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)):
                n = m.num_features
                m.running_mean.copy_(torch.rand(n, generator=g) * 0.2 - 0.1)
                m.running_var.copy_(torch.rand(n, generator=g) + 0.5)
                m.weight.copy_(torch.rand(n, generator=g) + 0.5)
                m.bias.copy_(torch.rand(n, generator=g) * 0.2 - 0.1)


def build_head(factory, w_seed, **kw):
    torch.manual_seed(w_seed)
    model = factory(**kw)
    randomize_bn(model, w_seed + 1)
    return model.eval()


def state_hash(model):
    h = hashlib.sha256()
    for k, v in sorted(model.state_dict().items()):
        h.update(k.encode())
        h.update(np.ascontiguousarray(v.detach().cpu().numpy()).tobytes())
    return h.hexdigest()


# ----------------------------------------------------------------------- case tables
# op-level index cases: name -> (kind, B, N, layout, S, [(radius, K), ...], seed)
INDEX_CASES = {
    'u3_strided':   ('uniform3', 4, 1024, 'strided', 512, [(0.2, 32), (0.4, 64), (0.1, 16), (0.8, 128)], 11),
    'u3_contig':    ('uniform3', 3, 512, 'contig', 128, [(0.4, 64), (0.2, 32), (0.8, 128)], 12),
    'dup3_strided': ('dup3', 4, 1024, 'strided', 512, [(0.2, 32), (0.4, 64)], 13),
    'oh10_strided': ('onehot10', 7, 1024, 'strided', 512, [(0.2, 32), (0.1, 16), (0.4, 128)], 14),
    'oh10_contig':  ('onehot10', 7, 512, 'contig', 128, [(0.4, 64), (0.8, 128)], 15),
    'r10_contig':   ('randn10', 2, 1000, 'contig', 256, [(2.0, 32), (3.0, 64)], 16),
    'r10_strided':  ('randn10', 2, 1000, 'strided', 256, [(2.0, 32), (3.0, 64)], 17),
    'small_smoke':  ('uniform3', 2, 100, 'strided', 512, [(0.2, 32), (0.9, 100)], 18),
    'tiny':         ('uniform3', 1, 10, 'contig', 4, [(0.5, 2), (2.0, 10)], 19),
    'pose2048':     ('onehot10', 2, 2048, 'strided', 512, [(0.2, 32)], 20),
    'stress16k':    ('uniform3', 1, 16384, 'strided', 512, [(0.2, 32)], 21),
    # the reference's real scans (points stored in the fixture): clustered, non-uniform density
    'camera_strided': ('camera', 2, 10000, 'strided', 512, [(0.2, 32), (0.1, 16), (0.4, 128)], 22),
    'camera10_contig': ('camera10', 2, 10000, 'contig', 512, [(0.2, 32), (0.4, 64)], 23),
    # point dimensions past the register-resident 16 (the streamed FPS, the wide ball query):
    # both layouts, N off the 16-point strided-tail boundary, radii around the median distance
    'r24_contig':   ('randn24', 2, 1000, 'contig', 256, [(6.0, 32), (7.5, 64)], 24),
    'r24_strided':  ('randn24', 2, 1000, 'strided', 256, [(6.0, 32), (7.5, 64)], 25),
    'r40_contig':   ('randn40', 2, 600, 'contig', 128, [(8.0, 32), (9.5, 64)], 26),
    'r40_strided':  ('randn40', 1, 600, 'strided', 128, [(8.0, 32), (9.5, 64)], 27),
    'r64_contig':   ('randn64', 1, 500, 'contig', 128, [(10.5, 32), (12.0, 64)], 28),
    'r64_strided':  ('randn64', 2, 500, 'strided', 128, [(10.5, 32), (12.0, 64)], 29),
    # strided clouds whose point count is not a multiple of 32: ATen sums whole 32-point
    # blocks vectorised (the first 4 points of a 4..7-point cloud), the rest in row_sum order
    'r10_n600_strided': ('randn10', 1, 600, 'strided', 128, [(2.0, 32), (3.0, 64)], 30),
    'r10_n48_strided':  ('randn10', 3, 48, 'strided', 16, [(3.0, 8), (4.0, 16)], 31),
    'r10_n20_strided':  ('randn10', 3, 20, 'strided', 8, [(3.0, 4), (4.5, 20)], 32),
    'r10_n6_strided':   ('randn10', 4, 6, 'strided', 6, [(3.0, 2), (5.0, 6)], 33),
}

# head-level cases: name -> (head, B, N, cloud kind, weight seed, forward seed)
HEAD_CASES = {
    'cls_ssg': ('pointnet2_cls_ssg', 2, 1024, 'uniform3', 100, 200),
    'cls_msg': ('pointnet2_cls_msg', 2, 1024, 'uniform3', 101, 201),
    'rotation_ssg': ('rotation_ssg', 2, 1024, 'onehot10', 102, 202),
    'translation_ssg': ('translation_ssg', 2, 1024, 'onehot10', 103, 203),
    'rotation_msg': ('rotation_msg', 2, 1024, 'onehot10', 104, 204),
}

# head cases at the BASELINE shapes, the heads without a small case, and the reference's two
# real scans: name -> (head, B, N, cloud kind, weight seed, forward seed, keep).  keep: the
# clouds whose sa1 / sa2 features are stored (None: all) -- centroids of every layer, the last
# SA feature and the head outputs are stored for the whole batch.  Synthetic inputs are
# regenerated from the seed (the fixture holds their SHA-256); kind 'camera' / 'camera10' clouds
# are /root/reference/camera_test/{bed,night_stand}.txt (np.loadtxt, xyz columns, the reference's
# provider.normalization; 'camera10' + a one-hot label), stored in the fixture.
HEAD_FULL_CASES = {
    'cls_ssg_b32': ('pointnet2_cls_ssg', 32, 1024, 'uniform3', 110, 210, (0, 31)),
    'cls_msg_n4096': ('pointnet2_cls_msg', 8, 4096, 'uniform3', 111, 211, (5,)),
    'rotation_ssg_n2048': ('rotation_ssg', 8, 2048, 'onehot10', 112, 212, (0, 6)),
    'translation_ssg_n2048': ('translation_ssg', 8, 2048, 'onehot10', 113, 213, (3, 7)),
    'cls_ssg_n16384': ('pointnet2_cls_ssg', 2, 16384, 'uniform3', 114, 214, None),
    'translation_msg': ('translation_msg', 2, 1024, 'onehot10', 115, 215, (1,)),
    'sign_ssg': ('sign_ssg', 2, 1024, 'onehot10', 116, 216, None),
    'sign_msg': ('sign_msg', 2, 1024, 'onehot10', 117, 217, (0,)),
    'camera_cls_ssg': ('pointnet2_cls_ssg', 2, 10000, 'camera', 118, 218, None),
    'camera_rotation_ssg': ('rotation_ssg', 2, 10000, 'camera10', 119, 219, None),
}
CAMERA_FILES = ('bed.txt', 'night_stand.txt')
CAMERA_LABELS = (1, 4)  # one-hot classes of the two scans in 'camera10'


def tensor_hash(t):
    return hashlib.sha256(np.ascontiguousarray(t.detach().cpu().numpy()).tobytes()).hexdigest()


# PointNet-v1 cases (/root/reference/model/pointnet_utils.py and the v1
# heads): name -> (head module, B, N, cloud kind, weight seed, get_model kwargs)
V1_CASES = {
    'pointnet_cls': ('pointnet_cls', 4, 1024, 'uniform3', 300, {}),
    'rotation_v1': ('rotation', 2, 1024, 'onehot10', 301, {}),
    'translation_v1': ('translation', 2, 1024, 'onehot10', 302, {}),
    'sign_v1': ('sign', 2, 1024, 'onehot10', 303, {}),
    'width_v1': ('width', 2, 1024, 'onehot10', 304, {'normal_channel': False}),
    # pose.py with both T-Nets on a 3-channel cloud (D > 3 with transform=True fails in the
    # reference: its cat is along the points axis, pose.py:57) and the classify tail
    'pose_v1': ('pose', 2, 1024, 'uniform3', 305,
                {'mlp_list': [64, 64, 64, 128, 1024], 'linear_list': [512, 256, 2],
                 'classify': True, 'num_category': 0, 'normal_channel': False,
                 'transform': True, 'feat_trans': True}),
}


def raw_batch(kind, B, N, seed, C=3):
    """A float64 [B, N, C] batch as the DataLoader yields it (np.loadtxt rows: sensor points in
    metres, off-centre, scale varying per cloud).  kind: 'raw', 'dup' (many exact duplicates,
    as random_point_dropout leaves them), 'tiny' (a few points, one scale)."""
    rng = np.random.default_rng(seed)
    scale = rng.uniform(0.05, 2.0, (B, 1, 1))
    off = rng.uniform(-3.0, 3.0, (B, 1, C))
    x = rng.uniform(-1.0, 1.0, (B, N, C)) * scale + off
    if kind == 'dup':
        for b in range(B):
            x[b, rng.random(N) < 0.6] = x[b, 0]
    return x


# the dataset tree of data_utils/ModelDataLoader.py (classes in its order, ModelDataLoader.py:51)
CATEGORIES = ['cube', 'cuboid', 'cylinder', 'h_structure', 'double_cube', 'double_cylinder',
              'cube_cylinder']


def write_dataset_tree(root, items, n_points=1300, seed=11):
    """<root>/<cls>/<cls>_NNNN{,_rot,_tran}.txt for every class, written the way
    data_build/Cube.py:90-94 writes them (np.savetxt '%6f', comma-separated).  Deterministic:
    the same call writes the same bytes anywhere (ids >= 6002 are the test split)."""
    import os
    rng = np.random.default_rng(seed)
    for cls in CATEGORIES:
        os.makedirs(os.path.join(root, cls), exist_ok=True)
        for i in items:
            base = os.path.join(root, cls, "%s_%04d" % (cls, i))
            np.savetxt(base + ".txt", rng.uniform(-0.2, 0.2, (n_points + i % 50, 3)) + 0.5,
                       fmt="%6f", delimiter=",")
            np.savetxt(base + "_tran.txt", rng.normal(0, 0.1, (1, 3)), fmt="%6f", delimiter=",")
            np.savetxt(base + "_rot.txt", rng.uniform(-3, 3, (1, 3)), fmt="%6f", delimiter=",")


# end-to-end case (f4 -> f2 -> head, test_translation.py:70-83): the tree of
# write_dataset_tree(items), the test split's items `index` loaded with np.random.seed(np_seed)
# (random_sample draws), prepared, and run through `head` (weight seed, forward seed)
E2E_CASE = dict(items=(6002, 6003), index=tuple(c * 1999 + j for c in range(7) for j in (1, 0)),
                np_seed=5, head='translation_ssg', wseed=120, fseed=220)


# input-preparation cases (provider.normalization + splice_torch + the translation mean):
# name -> (kind, B, N, C, seed, with labels)
PREP_CASES = {
    'raw': ('raw', 4, 1024, 3, 400, True),
    'dup': ('dup', 3, 2048, 3, 401, True),
    'nolabel': ('raw', 2, 1000, 3, 402, False),
    'c6': ('raw', 2, 512, 6, 403, True),
    'tiny': ('tiny', 2, 2, 3, 404, True),
}


# training-mode SA layers: name -> (kind: 'ssg' | 'msg', ctor args, B, N,
# feature channels D, weight seed, forward seed)
TRAIN_CASES = {
    'ssg_xyz': ('ssg', (64, 32, 0.4, 3, [32, 32, 64], False), 2, 512, 0, 500, 600),
    'ssg_feat': ('ssg', (32, 16, 0.5, 3 + 16, [32, 64], False), 2, 256, 16, 501, 601),
    'group_all': ('ssg', (None, None, None, 3 + 32, [64, 128], True), 3, 128, 32, 502, 602),
    'msg': ('msg', (32, [8, 16], [0.3, 0.6], 16, [[16, 32], [32, 32]]), 2, 256, 16, 503, 603),
}


# eval-mode SA layers on points with more than 16 channels (the streamed FPS, the wide ball
# query, the generic MLP path): name -> (kind, ctor args, B, N, C, D, weight seed, forward seed).
# points [B, C, N] and features [B, D, N] are N(0,1) (sa_inputs); radii around the median
# distance of C-dimensional normal points.  MSG in_channel = D, num_category = C - 3.
SA_WIDE_CASES = {
    'ssg_c24': ('ssg', (64, 32, 6.0, 24 + 8, [32, 64], False), 2, 512, 24, 8, 700, 800),
    'ssg_c40_xyz': ('ssg', (32, 16, 8.5, 40, [32, 32, 64], False), 2, 300, 40, 0, 701, 801),
    'group_all_c20': ('ssg', (None, None, None, 20 + 16, [64, 128], True), 3, 128, 20, 16, 702, 802),
    'msg_c24': ('msg', (32, [8, 16], [5.5, 7.0], 8, [[32, 32], [32, 64]], 21), 2, 256, 24, 8, 703, 803),
}


def sa_inputs(B, N, C, D, seed):
    """points [B, C, N] and feature [B, D, N] (or None), N(0,1), channel-first."""
    g = torch.Generator().manual_seed(seed)
    pts = torch.randn(B, C, N, generator=g)
    return pts, (torch.randn(B, D, N, generator=g) if D else None)


# PointNet-v1 training cases: name -> (head module, B, N, cloud kind, weight seed, get_model
# kwargs).  Train mode with every Dropout switched to eval (its mask is device-RNG dependent);
# loss = sum_i (out_i * R_i) over the head's float outputs.  Seeds are chosen so that every max
# over the points is tie-free: the smallest relative gap between a (cloud, channel)'s two largest
# values is >= TRAIN_V1_MIN_GAP in the float64 forward (a pair closer than float32 noise may
# route that channel's gradient to another point in any fp32 implementation, the reference's
# own included); make_goldens.py records and checks it.
TRAIN_V1_CASES = {
    'cls': ('pointnet_cls', 4, 96, 'uniform3', 3010, {}),
    'rotation': ('rotation', 4, 96, 'onehot10', 1011, {}),
    'pose': ('pose', 4, 96, 'uniform3', 1286,
             {'mlp_list': [64, 64, 64, 128, 1024], 'linear_list': [512, 256, 2],
              'classify': True, 'num_category': 0, 'normal_channel': False,
              'transform': True, 'feat_trans': True}),
}
TRAIN_V1_MIN_GAP = 2e-5


def train_v1_model(factory, wseed, **kw):
    """build_head, then train mode with the dropouts off."""
    model = build_head(factory, wseed, **kw).train()
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.eval()
    return model


GRAD_FULL_MAX = 32768   # larger gradients are kept as a fixed sample + their norm
GRAD_SAMPLE = 8192


def grad_sample_index(n):
    """The flat indices of an n-element gradient kept in the trainv1 goldens (sorted, fixed by
    n alone)."""
    return np.sort(np.random.default_rng(n).choice(n, GRAD_SAMPLE, replace=False))


def train_inputs(B, N, D, seed):
    """points [B, 3, N] (unit-sphere cloud, channel-first), feature [B, D, N] or None, and the
    loss weights R are drawn by the caller once the output shape is known."""
    pts = cloud('uniform3', B, N, seed).permute(0, 2, 1).contiguous()
    feat = None
    if D:
        g = torch.Generator().manual_seed(seed + 1)
        feat = torch.randn(B, D, N, generator=g)
    return pts, feat
