"""Where bench.py's pipelined rate and a bare GraphedPipeline loop part ways (SSG, K = 100):
one variant per process (process state -- stream/queue binding, the allocator -- is part of
it).  python tools/debug/bench_gap.py VARIANT
  bare     ClsSSG(seed 8), cloud seed 90, pipeline warm-up then timed runs
  benchin  bench.py's model and input (build_models / make_inputs), otherwise bare
  eagerw   benchin + bench's 10 eager warm-up steps before the pipeline
  batched  eagerw + bench's BatchedGather(8) post
  prec     batched + pn2.mlp_precision('fp32') entered for the whole run, as bench does
  warmk    bare with a 100-batch pipelined warm-up
  empty    bare, torch.cuda.empty_cache() before every timed run
  sleep    bare, 200 ms idle before every timed run
  spin     bare, 200 ms host busy-wait (GPU idle) before every timed run
  gpubusy  bare, 200 ms of GPU matmuls (host asleep) before every timed run
(The first timed run after a short warm-up reads ~5 % below the later ones in every variant
above; these three ask why.)"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (its sys.path setup)
import cases  # noqa: E402
import pn2  # noqa: E402
from pn2 import heads as H  # noqa: E402
from pn2 import shard  # noqa: E402
from pn2.pipeline import GraphedPipeline  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    v = sys.argv[1]
    order = ["bare", "benchin", "eagerw", "batched", "prec"]
    lvl = order.index(v) if v in order else 0
    if lvl >= 4:
        pn2.mlp_precision("fp32").__enter__()
    if lvl >= 1:
        names, models = bench.build_models("ssg", DEV)
        x, mean = bench.make_inputs("ssg", 32, 0, DEV, 0, 32)
        model = models[0]
    else:
        torch.manual_seed(8)
        model = H.ClsSSG().eval()
        cases.randomize_bn(model, 8)
        model = model.to(DEV)
        x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
    torch.manual_seed(1234)
    if lvl >= 2:
        for _ in range(10):
            bench.step(["pointnet2_cls_ssg"], [model], x, None, 32, 0)
    gp = GraphedPipeline(model)

    def post_for(k):
        if lvl >= 3:
            bg = shard.BatchedGather(8, total=k)
            return lambda i, o: bg(i, o[0])
        return lambda i, o: shard.all_gather_rows(o[0], sizes="shard")

    nw = 100 if v == "warmk" else 10
    with shard.batch_shard(32, 0):
        gp.run([x] * nw, post=post_for(nw))
    torch.cuda.synchronize()
    res = []
    for _ in range(3):
        if v == "empty":
            torch.cuda.empty_cache()
        if v == "sleep":
            time.sleep(0.2)
        if v == "spin":
            t1 = time.perf_counter() + 0.2
            while time.perf_counter() < t1:
                pass
        if v == "gpubusy":
            a = torch.randn(4096, 4096, device="cuda")
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(20):
                a = a @ a
                a = a / a.norm()
            torch.cuda.synchronize()
            n = max(1, int(0.2 / max(time.perf_counter() - t1, 1e-4) * 20))
            for _ in range(n):
                a = a @ a
                a = a / a.norm()
            time.sleep(0.15)
            torch.cuda.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with shard.batch_shard(32, 0):
            gp.run([x] * 100, post=post_for(100))
        torch.cuda.synchronize()
        res.append(3200 / (time.perf_counter() - t0))
    print("%-8s K=100 %s clouds/s" % (v, " ".join("%.0f" % r for r in res)))


if __name__ == "__main__":
    main()
