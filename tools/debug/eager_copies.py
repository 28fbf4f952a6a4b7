"""Which host calls launch the copies in the eager SSG forward (VERDICT r05 "unattributed work")?
Runs the bench's eager step (head forward + the world-size-1 logits gather) under the torch
profiler and prints every copy / fill / elementwise device activity with its host call stack.
    python tools/debug/eager_copies.py [--ref]   (--ref: pn2.heads.ReferenceForward)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import cases  # noqa: E402
import pn2  # noqa: E402,F401
from pn2 import heads as H, shard  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    torch.manual_seed(1000)
    m = H.ClsSSG()
    cases.randomize_bn(m, 2000)
    m = m.eval().to(DEV)
    if "--ref" in sys.argv:
        m = H.ReferenceForward(m)
    x = cases.cloud("uniform3", 32, 1024, 7).permute(0, 2, 1).contiguous().to(DEV)

    def step():
        with torch.no_grad(), shard.batch_shard(32, 0):
            o = m(x)
            shard.all_gather_rows(o[0], sizes="shard")

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(3):
            step()
        torch.cuda.synchronize()
    keys = ("copy", "Memcpy", "Memset", "fill", "elementwise", "Copy")
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA and any(k in ev.name for k in keys):
            par = ev.cpu_parent
            chain = []
            while par is not None and len(chain) < 6:
                chain.append(par.name)
                par = par.cpu_parent
            stack = [f for f in (ev.cpu_parent.stack if ev.cpu_parent is not None else [])
                     if "pointnet" in f or "bench" in f or "pn2" in f][:4]
            print("%-50s %7.1f us  <- %s  %s" % (ev.name[:50], ev.device_time, " < ".join(chain), " | ".join(stack)))
    print(prof.key_averages().table(sort_by="device_time_total", row_limit=25))


if __name__ == "__main__":
    main()
