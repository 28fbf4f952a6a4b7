"""Which stream bounds the pipelined SSG run (timing only, wrong outputs): the GraphedPipeline
at K = 100 with one stream's work removed -- the head's FC tail (identity), then sa3 too; the
geometry's FPS (a copy of a cached result), then its ball queries too -- beside the full model,
interleaved.
    python tools/debug/pipe_ablate.py"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import cases  # noqa: E402
from pn2 import heads as H  # noqa: E402
from pn2.pipeline import GraphedPipeline  # noqa: E402

DEV = torch.device("cuda", 0)


def build(kind):
    torch.manual_seed(8)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 8)
    model = model.to(DEV)
    if kind in ("nofc", "nohead"):
        model._fc_log_softmax = lambda x: (x[:, :7].contiguous(), x[:, :7].contiguous())
    if kind == "nohead":
        def sa3(p, f):
            return p[:, :, :1], f[:, :, :1].repeat(1, 4, 1)  # [B, 1024, 1], no MLP
        model.sa3.forward = sa3
    return model


def main():
    from pn2 import ops
    x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
    kinds = ("full", "nofc", "nohead", "nofps", "nogeo")
    gps = {k: GraphedPipeline(build(k)) for k in kinds}
    real_fps, real_bq = ops.fps_direct, ops.ball_query_direct
    cache = {}

    def fake_fps(pts, S, start):  # the first real result per shape, copied (timing only)
        key = ("fps", tuple(pts.shape), S)
        if key not in cache:
            cache[key] = [t.clone() for t in real_fps(pts, S, start)]
        return tuple(t.clone() for t in cache[key])

    def fake_bq(ppk, cpk, C, r, k, cnt):
        key = ("bq", tuple(ppk.shape), tuple(cpk.shape), r, k)
        if key not in cache:
            cache[key] = [t.clone() for t in real_bq(ppk, cpk, C, r, k, cnt)]
        return tuple(t.clone() for t in cache[key])

    with torch.no_grad():
        for k, gp in gps.items():
            if k in ("nofps", "nogeo"):
                ops.fps_direct = fake_fps
            if k == "nogeo":
                ops.ball_query_direct = fake_bq
            gp.run([x] * 12)  # captures the graphs with the stand-ins
            ops.fps_direct, ops.ball_query_direct = real_fps, real_bq
    torch.cuda.synchronize()
    K = int(os.environ.get("K", "100"))
    for rnd in range(3):
        for k, gp in gps.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with torch.no_grad():
                gp.run([x] * K)
            torch.cuda.synchronize()
            print("round %d %-7s K=%d %8.0f clouds/s" % (rnd, k, K, 32 * K / (time.perf_counter() - t0)))


if __name__ == "__main__":
    main()
