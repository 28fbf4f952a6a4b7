"""Eager SSG forward (B = 32, N = 1024) under kernel-tuning variants, interleaved in one
process after a settle: which launch choices the eager forward prefers (several defaults were
tuned in the pipelined launch).  python tools/debug/eager_ab.py [rounds]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402,F401  (its sys.path setup)
import cases  # noqa: E402
from pn2 import heads as H  # noqa: E402
from pn2 import tuning  # noqa: E402

DEV = torch.device("cuda", 0)
VARIANTS = [
    ("default", {}),
    ("pool8", dict(compact_pool=8)),
    ("pool0", dict(compact_pool=0)),
    ("stages2", dict(compact_stages=2)),
    ("pool8_st2", dict(compact_pool=8, compact_stages=2)),
    ("minwg512", dict(dense_minwg=512)),
    ("minwg128", dict(dense_minwg=128)),
    ("maxntc1", dict(dense_maxntc=1)),
    ("dense_lds", dict(dense_lds=1)),
    ("bq16", dict(bq_waves=16)),
    ("lds_bq16", dict(dense_lds=1, bq_waves=16)),
    ("lds_bq16_mw512", dict(dense_lds=1, bq_waves=16, dense_minwg=512)),
]
if os.environ.get("EAGER_AB_SET") == "profile":
    VARIANTS = [("default", {}), ("mincin0", dict(dense_lds_mincin=0)), ("mincin128", dict(dense_lds_mincin=128)),
                ("pipeline_profile", dict(fps_mid=256, dense_lds=0, bq_waves=0)),
                ("no_lds", dict(dense_lds=0)), ("bq8", dict(bq_waves=0))]
if os.environ.get("EAGER_AB_SET") == "more":
    VARIANTS = [("default", {}), ("lds_st4", dict(dense_lds_stages=4)), ("lds_xcd2d", dict(dense_lds_xcd2d=1)),
                ("tile44", dict(dense_lds_tile=44)), ("tile42", dict(dense_lds_tile=42)),
                ("tile22", dict(dense_lds_tile=22)), ("tile82", dict(dense_lds_tile=82)),
                ("minwg512", dict(dense_minwg=512)), ("no_prepass", dict(chain_prepass=0)),
                ("rowbuf0", dict(bq_rowbuf_kb=0))]
if os.environ.get("EAGER_AB_SET") == "short":
    VARIANTS = [v for v in VARIANTS if v[0] in ("default", "dense_lds", "bq16", "lds_bq16", "lds_bq16_mw512")]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    torch.manual_seed(8)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 8)
    model = model.to(DEV)
    x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
    K = 40
    res = {n: [] for n, _ in VARIANTS}
    with torch.no_grad():
        torch.manual_seed(5)  # the FPS start draws
        ref = model(x)[0].clone()
        t1 = time.perf_counter() + 0.15  # settle: ~150 ms of forwards
        while time.perf_counter() < t1:
            model(x)
        torch.cuda.synchronize()
        for _ in range(rounds):
            for name, kw in VARIANTS:
                with tuning.override(**kw):
                    for _ in range(2):
                        model(x)
                    torch.manual_seed(5)
                    out = model(x)[0]
                    torch.cuda.synchronize()
                    if not torch.allclose(out, ref, rtol=1e-5, atol=1e-5 * float(ref.abs().max())):
                        raise SystemExit("%s: output differs" % name)
                    t0 = time.perf_counter()
                    for _ in range(K):
                        model(x)
                    torch.cuda.synchronize()
                    res[name].append(32 * K / (time.perf_counter() - t0))
    for name, _ in VARIANTS:
        print("%-10s %s clouds/s" % (name, " ".join("%.0f" % v for v in res[name])))


if __name__ == "__main__":
    main()
