"""Time the group_all SA layer (sa3 of pointnet2_cls_ssg: 259 -> 256 -> 512 -> 1024 + max over
128 points, B = 32) and the FC tail, eager, for each tuning variant named on the command line
(`key=value[;key=value]`, default: the current defaults), interleaved over rounds.  A variant's
l3 feature must be bit-identical to the first variant's of the same arithmetic (the keys that
change it: mlp_f32, chain_f16, dense_f16) and within the north star's 1e-5 of the first
variant's otherwise (split fp16 and split bf16 are different roundings of the same product).  One JSON line per
variant: median microseconds per sa3 call (HIP events over 50 calls) and the split-bf16
fraction of its algorithmic FLOPs.  Run under rocprofv3 --kernel-trace --stats for kernel
times."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import cases  # noqa: E402
import pn2  # noqa: E402,F401
from pn2 import heads, tuning  # noqa: E402


def parse(v):
    return {} if v in ("", "default") else {k: int(x) for k, x in (t.split("=") for t in v.split(";"))}


def main():
    dev = torch.device("cuda")
    variants = sys.argv[1:] or ["default"]
    B = int(os.environ.get("B", "32"))
    torch.manual_seed(1000)
    model = heads.ClsSSG()
    cases.randomize_bn(model, 2000)
    model = model.eval().to(dev)
    g = torch.Generator().manual_seed(3)
    l2p = torch.rand(B, 3, 128, generator=g).to(dev)
    l2f = torch.relu(torch.randn(B, 128, 256, generator=g)).to(dev).permute(0, 2, 1)  # channels-last view
    flops = 2.0 * B * 128 * (259 * 256 + 256 * 512 + 512 * 1024)
    ARITH = ("mlp_f32", "chain_f16", "dense_f16")

    def arith(v):
        return tuple(parse(v).get(k, tuning.kernel_default(k)) for k in ARITH)

    ref, refs, res = None, {}, {v: [] for v in variants}
    for rnd in range(5):
        for v in variants:
            with tuning.override(**parse(v)), torch.no_grad():
                out = model.sa3(l2p, l2f)[1]
                torch.cuda.synchronize()
                got = out.cpu().numpy()
                if ref is None:
                    ref = got
                a = arith(v)
                if a not in refs:
                    refs[a] = got
                assert np.array_equal(got.view(np.uint32), refs[a].view(np.uint32)), v
                np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5 * float(np.abs(ref).max()), err_msg=v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    model.sa3(l2p, l2f)
                e1.record()
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) * 1e3 / 50)
    for v in variants:
        us = float(np.median(res[v]))
        print(json.dumps({"variant": v, "B": B, "sa3_us": round(us, 2), "min_us": round(min(res[v]), 2),
                          "tflops": round(flops / us * 1e-6, 1),
                          "frac_split_peak": round(flops / us * 1e-6 / 419.5, 3)}))


if __name__ == "__main__":
    main()
