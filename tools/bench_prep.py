"""Input preparation: pn2.provider.prepare_batch (device-resident float64 batch -> model input)
against the reference's host steps (oracle.prepare_points: numpy normalization loop + torch
splice, the same calls as provider.py / test_translation.py:72-79).  Prints one JSON line per
config: GPU kernel time (HIP events, input already in HBM), H2D-inclusive time, CPU time."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"),
                os.path.join(ROOT, "tests", "golden")]
import cases  # noqa: E402
import oracle  # noqa: E402
from pn2.provider import prepare_batch  # noqa: E402

for B, N in ((32, 1024), (64, 2048), (128, 16384)):
    raw = cases.raw_batch("raw", B, N, 9)
    labels = torch.arange(B) % 7
    host = torch.from_numpy(raw)
    dev = host.cuda()
    dlab = labels.cuda()
    for _ in range(3):
        prepare_batch(dev, dlab, with_mean=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        prepare_batch(dev, dlab, with_mean=True)
    e1.record()
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        prepare_batch(host, labels, with_mean=True)
    torch.cuda.synchronize()
    h2d_ms = (time.perf_counter() - t0) / reps * 1e3
    k = 1 if B * N > 1e6 else 3
    t0 = time.perf_counter()
    for _ in range(k):
        oracle.prepare_points(raw, labels.numpy(), 7, with_mean=True)
    cpu_ms = (time.perf_counter() - t0) / k * 1e3
    bytes_ = B * N * 3 * 8 + B * N * 10 * 4
    print(json.dumps({"B": B, "N": N, "gpu_ms": round(gpu_ms, 4), "gpu_GBps": round(bytes_ / gpu_ms / 1e6, 1),
                      "h2d_inclusive_ms": round(h2d_ms, 4), "cpu_ms": round(cpu_ms, 2),
                      "cpu_over_gpu": round(cpu_ms / gpu_ms, 1)}))
