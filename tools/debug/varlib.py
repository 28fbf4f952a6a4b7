"""Run a diagnostic tool against a diagnostic build of libpn2 (tools/debug/build_*.sh ->
pn2/var/*.so: timeline stamps and the like) without any switch in the product: the tool imports
pn2 from a scratch copy of the package whose libpn2.so is that build.

    PN2_DEBUG_LIB=<path to the .so> python tools/debug/<tool>.py ...

Call setup() before the first `import pn2`."""
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "pointnet-like-pose-estimation_amd")


def setup():
    path = os.environ.get("PN2_DEBUG_LIB")
    if not path:
        return None
    tmp = tempfile.mkdtemp(prefix="pn2var_")
    shutil.copytree(os.path.join(PKG, "pn2"), os.path.join(tmp, "pn2"),
                    ignore=shutil.ignore_patterns("libpn2.so", "__pycache__", "var"))
    shutil.copy(path, os.path.join(tmp, "pn2", "libpn2.so"))
    sys.path.insert(0, tmp)
    return tmp
