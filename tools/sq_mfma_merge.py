"""Merge gpurun_out/sqmfma/sq_mfma_<cfg>.json into profiles/sq_mfma.json ({cfg: {kernel: {...}}}),
the counters bench.py reports as roofline.mfma_busy.  python tools/sq_mfma_merge.py DIR"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "sqmfma")
dst = os.path.join(ROOT, "profiles", "sq_mfma.json")
out = {}
if os.path.exists(dst):
    out = json.load(open(dst))
for f in sorted(glob.glob(os.path.join(src, "sq_mfma_*.json"))):
    cfg = os.path.basename(f)[len("sq_mfma_"):-5]
    out[cfg] = json.load(open(f))
json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
print("wrote", dst, sorted(out))
