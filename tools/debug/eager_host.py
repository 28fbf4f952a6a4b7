"""Is the eager SSG forward (B=32 N=1024, the bench's eager_value) host-bound?  Host time to
issue N forwards without synchronising (the GPU runs behind) against the time to the final
synchronize, and torch.profiler's host-side split of one forward.
    python tools/debug/eager_host.py [--profile]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import cases  # noqa: E402
from pn2 import heads as H  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    torch.manual_seed(8)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 8)
    model = model.to(DEV)
    x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
    with torch.no_grad():
        for _ in range(10):
            model(x)
        torch.cuda.synchronize()
        for rep in range(3):
            n = 50
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                model(x)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print("rep %d: host issue %.1f us/forward, wall %.1f us/forward" % (
                rep, (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6), flush=True)
        if "--profile" in sys.argv:
            from torch.profiler import ProfilerActivity, profile
            with profile(activities=[ProfilerActivity.CPU]) as prof:
                for _ in range(20):
                    model(x)
                torch.cuda.synchronize()
            print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))


if __name__ == "__main__":
    main()
