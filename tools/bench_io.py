"""Dataset reader: np.loadtxt (the reference, data_utils/ModelDataLoader.py:85) vs
pn2.data.loadtxt (libpn2io, one thread) vs pn2.data.load_many (native thread pool) on files
written like data_build/Cube.py:92 (np.savetxt fmt='%6f').  Checks the values are bit-identical
and prints one JSON line per thread count."""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
from pn2 import data  # noqa: E402

n_files, rows = int(os.environ.get("FILES", "96")), int(os.environ.get("ROWS", "4096"))
d = tempfile.mkdtemp(prefix="pn2io_")
rng = np.random.default_rng(0)
paths = []
for i in range(n_files):
    p = os.path.join(d, "cube_%04d.txt" % i)
    np.savetxt(p, rng.uniform(-0.3, 0.3, (rows, 3)) + 0.5, fmt="%6f", delimiter=",")
    paths.append(p)
t = time.perf_counter()
want = [np.loadtxt(p, delimiter=",") for p in paths]
t_np = time.perf_counter() - t
t = time.perf_counter()
one = [data.loadtxt(p) for p in paths]
t_one = time.perf_counter() - t
assert all((a.view(np.uint64) == b.view(np.uint64)).all() for a, b in zip(want, one))
threads = len(os.sched_getaffinity(0))
for th in sorted({1, 4, min(16, threads)}):
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        got = data.load_many(paths, 3, threads=th)
        best = min(best, time.perf_counter() - t)
    assert all((a.view(np.uint64) == b.view(np.uint64)).all() for a, b in zip(want, got))
    print(json.dumps({"files": n_files, "rows": rows, "np_loadtxt_ms": round(t_np * 1e3, 1),
                      "pn2_loadtxt_ms": round(t_one * 1e3, 1), "load_many_threads": th,
                      "load_many_ms": round(best * 1e3, 1),
                      "speedup_vs_np": round(t_np / best, 1), "cpus": threads}))
