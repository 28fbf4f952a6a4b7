"""Which hardware queue each pipeline stream's kernels ran on: reads a rocprofv3 kernel trace
(`--kernel-trace --output-format csv`) and prints, per (queue id, stream id), the dispatch
count and the most frequent kernels.  Two pipeline streams on one queue serialise.
    python tools/debug/queue_map.py <dir with *kernel_trace.csv>"""
import collections
import csv
import glob
import os
import sys


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    keys = [k for k in rows[0] if k.lower() in ("queue_id", "stream_id")]
    print("columns:", keys)
    by = collections.defaultdict(collections.Counter)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
        by[tuple(r[k] for k in keys)][name] += 1
    for k in sorted(by):
        c = by[k]
        print(k, sum(c.values()), "; ".join("%s x%d" % (n, m) for n, m in c.most_common(5)))


if __name__ == "__main__":
    main()
