"""Probe (this container only: imports /root/reference read-only): does the oracle's restatement
of square_distance (pointnet2_utils.py:5-26) hold for point dimensions C > 16?  Prints, per C and
layout, how many [S,N] entries differ bit-wise from the reference, split into the sum of squares
(torch.sum(x**2, -1)) and the matmul (fma chain in k order).  Round 6 result: the matmul chain
holds to C = 64; the sum-of-squares orders past 16 channels are ATen's vectorised reductions --
point-contiguous rows ("strided" views) sum 16-channel chunks sequentially and add the chunk
sums in order for the points of whole 32-point blocks (the first 4 of a 4..7-point cloud; the
other points in the row_sum order -- rounds 1-5 assumed 16-point blocks) (differs from a plain sequential sum from C = 18), channel-contiguous rows put
whole 32-channel blocks of 8-lane vectors into 4 vector accumulators (differs from C = 40).
The oracle (oracle/pn2_oracle.c) and the kernels (csrc/pn2_internal.h) restate both; after
that every count printed here is 0 up to C = 64.
    PYTHONDONTWRITEBYTECODE=1 python tools/probe/sum_orders_past_16.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, "/root/reference/model")
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
import pointnet2_utils as ref  # noqa: E402  (the reference, read-only)


def main():
    torch.manual_seed(0)
    for C in (16, 17, 18, 20, 24, 32, 40, 64):
        for layout in ("contig", "strided"):
            B, S, N = 2, 64, 200
            src, dst = torch.randn(B, S, C), torch.randn(B, N, C)
            if layout == "strided":
                dst = dst.permute(0, 2, 1).contiguous().permute(0, 2, 1)
            want = ref.square_distance(src, dst).numpy()
            got = np.asarray(oracle.square_distance(src, dst), np.float32)
            ssq_bad = int((torch.sum(dst ** 2, -1).numpy() != np.asarray(oracle.ssq(dst), np.float32)).sum())
            print("C=%2d %-7s square_distance mismatches %5d of %d (sum-of-squares mismatches %d of %d)" % (
                C, layout, int((want.view(np.uint32) != got.view(np.uint32)).sum()), want.size, ssq_bad, B * N))
    # which strided points ATen's vectorised body sums: 32-point blocks (4 of a 4..7-point cloud)
    for C in (5, 10, 24, 64):
        bad = 0
        for N in list(range(1, 70)) + [95, 600, 1000, 1040, 10000]:
            x = torch.randn(4, C, N).permute(0, 2, 1)
            bad += int((torch.sum(x ** 2, -1).numpy() != np.asarray(oracle.ssq(x), np.float32)).sum())
        print("C=%2d strided sum-of-squares mismatches over N = 1..69, 95, 600, 1000, 1040, 10000: %d" % (C, bad))


if __name__ == "__main__":
    main()
