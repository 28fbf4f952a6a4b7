"""pn2 -- MI355X-native PointNet++ set-abstraction path (drop-in for the reference's
model/pointnet2_utils.py).  See DESIGN.md at the repository root."""
from . import _lib, ops, shard, tuning  # noqa: F401  (ops loads libpn2.so and registers torch.ops.pn2.*)
from ._lib import check_device_errors  # noqa: F401
from .ops import mlp_precision  # noqa: F401
from .pointnet2_utils import (  # noqa: F401
    eval_autograd, fused_eval, PointNetSetAbstraction, PointNetSetAbstractionMsg, farthest_point_sample, index_points,
    query_ball_point, sample_and_group, sample_and_group_all, square_distance)

__version__ = "0.1.0"
