"""The eager SSG forward's kernel sequence (run under rocprofv3 --kernel-trace): 5 warm-up
forwards, then 5 marked ones.  python tools/debug/eager_seq.py [trace.csv]
  without an argument: run the forwards (profile this);
  with the kernel-trace CSV: print the last forward's kernels in order with their durations and
  the gaps between them."""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    import torch
    sys.path.insert(0, ROOT)
    import bench  # noqa: F401
    import cases
    from pn2 import heads as H
    dev = torch.device("cuda", 0)
    torch.manual_seed(8)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 8)
    model = model.to(dev)
    x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(dev)
    with torch.no_grad():
        for _ in range(10):
            model(x)
    torch.cuda.synchronize()


def show(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    fps = [i for i, r in enumerate(rows) if "fps_kernel" in r[2]]
    a = fps[-2]  # the last forward starts at its first FPS
    prev = None
    for s, e, n in rows[a:]:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print("%8.2f us  (gap %6.2f)  %s" % ((e - s) / 1e3, gap, n[:100]))
        prev = e
    print("forward span %.1f us" % ((rows[-1][1] - rows[a][0]) / 1e3))


if __name__ == "__main__":
    if len(sys.argv) > 1:
        show(sys.argv[1])
    else:
        run()
