"""From a rocprofv3 kernel-trace CSV of a pipelined run: over the last `span_ms` of kernel
activity, the fraction of time with at least one kernel running, the mean number of kernels
in flight, and the idle gaps' distribution -- is the steady state bound by execution (busy ~1)
or by issue / dependencies (gaps)?  python tools/debug/busy_union.py kernel_trace.csv [span_ms]"""
import csv
import sys


def main():
    path = sys.argv[1]
    span = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    iv = []
    with open(path) as f:
        for r in csv.DictReader(f):
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    iv.sort()
    t1 = max(e for _, e, _ in iv)
    t0 = t1 - span * 1e6
    sel = [(max(s, t0), e, n) for s, e, n in iv if e > t0]
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e, _ in sel:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    total = t1 - t0
    inflight = sum(e - s for s, e, _ in sel) / total
    gaps.sort()
    print("last %.1f ms: %d kernels, busy %.1f %%, mean kernels in flight %.2f" % (
        span, len(sel), 100.0 * busy / total, inflight))
    if gaps:
        print("idle gaps: %d, total %.1f us, median %.2f us, p90 %.2f us, max %.1f us" % (
            len(gaps), sum(gaps) / 1e3, gaps[len(gaps) // 2] / 1e3, gaps[int(len(gaps) * 0.9)] / 1e3,
            gaps[-1] / 1e3))
    names = {}
    for s, e, n in sel:
        k = n.split("(")[0][:60]
        a = names.setdefault(k, [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e3
    for k, (c, t) in sorted(names.items(), key=lambda x: -x[1][1])[:25]:
        print("%-62s n %5d  sum %9.1f us  avg %7.2f us" % (k, c, t, t / c))


if __name__ == "__main__":
    main()
