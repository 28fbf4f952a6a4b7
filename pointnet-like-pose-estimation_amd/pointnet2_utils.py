"""Import shim: with this directory on sys.path, ``from pointnet2_utils import
PointNetSetAbstraction`` (how every reference head imports it, e.g.
/root/reference/model/pointnet2_cls_ssg.py:3) resolves to the MI355X implementation."""
import os as _os
import sys as _sys

_here = _os.path.dirname(_os.path.abspath(__file__))
if _here not in _sys.path:
    _sys.path.insert(0, _here)

from pn2.pointnet2_utils import *  # noqa: E402,F401,F403
from pn2.pointnet2_utils import __all__  # noqa: E402,F401
