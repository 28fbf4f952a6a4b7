"""Eager SSG forwards (B=32, N=1024) on whatever library PN2_DEBUG_LIB names (a variant build,
tools/debug/build_var.sh) or the default one -- for rocprofv3 kernel timing of a build variant:
    rocprofv3 --kernel-trace --stats -d gpurun_out/x -- python3 tools/debug/eager_run.py
FORWARDS=<n> (default 20) forwards after 5 warm-up ones."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import cases  # noqa: E402
import varlib  # noqa: E402
varlib.setup()
from pn2 import heads as H  # noqa: E402

DEV = torch.device("cuda", 0)
torch.manual_seed(8)
model = H.ClsSSG().eval()
cases.randomize_bn(model, 8)
model = model.to(DEV)
x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
with torch.no_grad():
    for _ in range(5):
        model(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = int(os.environ.get("FORWARDS", "20"))
    e0.record()
    for _ in range(n):
        model(x)
    e1.record()
    torch.cuda.synchronize()
print("eager forward %.1f us (%s)" % (e0.elapsed_time(e1) * 1e3 / n, os.environ.get("PN2_DEBUG_LIB", "default lib")))
