"""Cold (after 300 ms idle) vs warm pipelined runs of K = 20 batches (SSG): host issue time
(until GraphedPipeline.run returns) against the run's total time (until the device is done).
Issue ~ total in the cold runs = the host is the bound while the SOC clock climbs; issue well
below total = the device is.  Also the eager forward cold vs warm.
python tools/debug/cold_host.py"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402,F401  (its sys.path setup)
import cases  # noqa: E402
from pn2 import heads as H  # noqa: E402
from pn2 import shard  # noqa: E402
from pn2.pipeline import GraphedPipeline  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    torch.manual_seed(8)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 8)
    model = model.to(DEV)
    x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
    torch.manual_seed(1234)
    gp = GraphedPipeline(model)
    post = lambda i, o: shard.all_gather_rows(o[0], sizes="shard")  # noqa: E731
    K = 20
    with shard.batch_shard(32, 0):
        gp.run([x] * 10, post=post)
    torch.cuda.synchronize()
    for mode in ("cold", "warm", "cold", "warm"):
        rows = []
        for _ in range(3):
            if mode == "cold":
                time.sleep(0.3)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with shard.batch_shard(32, 0):
                gp.run([x] * K, post=post)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            rows.append("issue %6.0f us  total %6.0f us  %6.0f clouds/s" % (
                (t1 - t0) * 1e6, (t2 - t0) * 1e6, 32 * K / (t2 - t0)))
        print("pipelined %s K=%d: %s" % (mode, K, " | ".join(rows)))
    with torch.no_grad():
        for _ in range(5):
            model(x)
        torch.cuda.synchronize()
        for mode in ("cold", "warm"):
            rows = []
            for _ in range(3):
                if mode == "cold":
                    time.sleep(0.3)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(K):
                    model(x)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                rows.append("issue %6.0f us  total %6.0f us  %6.0f clouds/s" % (
                    (t1 - t0) * 1e6, (t2 - t0) * 1e6, 32 * K / (t2 - t0)))
            print("eager %s K=%d: %s" % (mode, K, " | ".join(rows)))


if __name__ == "__main__":
    main()
