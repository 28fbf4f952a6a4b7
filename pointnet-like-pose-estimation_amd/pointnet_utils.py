"""Import shim: with this directory on sys.path, ``from pointnet_utils import PointNetEncoder``
(how the reference's v1 heads import it, e.g. /root/reference/model/pointnet_cls.py:5)
resolves to the MI355X implementation."""
import os as _os
import sys as _sys

_here = _os.path.dirname(_os.path.abspath(__file__))
if _here not in _sys.path:
    _sys.path.insert(0, _here)

from pn2.pointnet_utils import *  # noqa: E402,F401,F403
from pn2.pointnet_utils import __all__  # noqa: E402,F401
