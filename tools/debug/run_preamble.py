"""Host time of GraphedPipeline.run before its first geometry replay (SSG B=32, the bench's
launch): each step of the preamble timed with perf_counter through wrappers, over a few runs.
    python tools/debug/run_preamble.py"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import cases  # noqa: E402
from pn2 import heads as H  # noqa: E402
from pn2 import pipeline  # noqa: E402
from pn2.pipeline import GraphedPipeline  # noqa: E402

DEV = torch.device("cuda", 0)
log = []


def wrap(obj, name):
    f = getattr(obj, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        log.append((name, (time.perf_counter() - t0) * 1e6))
        return r
    setattr(obj, name, g)


def main():
    torch.manual_seed(8)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 8)
    model = model.to(DEV)
    x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
    gp = GraphedPipeline(model)
    gp.run([x] * 6)
    torch.cuda.synchronize()
    wrap(gp._params, "key")
    wrap(gp, "_draw_all")
    wrap(gp, "_draw_row")
    wrap(pipeline, "_streams")
    grp = gp._slots[0]
    orig = grp.fps.replay

    def rep():
        log.append(("fps.replay called", (time.perf_counter() - T[0]) * 1e6))
        t0 = time.perf_counter()
        orig()
        log.append(("fps.replay", (time.perf_counter() - t0) * 1e6))
    grp.fps.replay = rep
    T = [0.0]
    for it in range(4):
        torch.cuda.synchronize()
        time.sleep(0.01)
        del log[:]
        T[0] = time.perf_counter()
        gp.run([x] * 20)
        torch.cuda.synchronize()
        first = [e for e in log if e[0] == "fps.replay called"][0][1]
        parts = {}
        for n, us in log:
            if n == "fps.replay called":
                break
            parts[n] = parts.get(n, 0.0) + us
        print("run %d: first fps replay issued %.1f us after run(); before it: %s" % (
            it, first, ", ".join("%s %.1f" % kv for kv in parts.items())))


if __name__ == "__main__":
    main()
