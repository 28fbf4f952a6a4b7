"""Where bench.py's pipelined rate and a bare GraphedPipeline loop part ways (SSG, K = 100):
one variant per process (process state -- stream/queue binding, the allocator -- is part of
it).  python tools/debug/bench_gap.py VARIANT
  bare     ClsSSG(seed 8), cloud seed 90, pipeline warm-up then timed runs
  benchin  bench.py's model and input (build_models / make_inputs), otherwise bare
  eagerw   benchin + bench's 10 eager warm-up steps before the pipeline
  batched  eagerw + bench's BatchedGather(8) post
  prec     batched + pn2.mlp_precision('fp32') entered for the whole run, as bench does"""
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
    lvl = order.index(v)
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

    with shard.batch_shard(32, 0):
        gp.run([x] * 10, post=post_for(10))
    torch.cuda.synchronize()
    res = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with shard.batch_shard(32, 0):
            gp.run([x] * 100, post=post_for(100))
        torch.cuda.synchronize()
        res.append(3200 / (time.perf_counter() - t0))
    print("%-8s K=100 %s clouds/s" % (v, " ".join("%.0f" % r for r in res)))


if __name__ == "__main__":
    main()
