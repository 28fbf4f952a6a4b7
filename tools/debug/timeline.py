"""Per-stream timeline of one rocprofv3 kernel trace: for the last `--steps` chain<4,4,9>
launches, print each kernel's start (relative, us), duration, stream and queue."""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--from-kernel", default="sa_chain_kernel<2, 2, 1>")
    ap.add_argument("--count", type=int, default=3, help="periods to print")
    ap.add_argument("--skip", type=int, default=8, help="periods to skip (warm-up)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.from_kernel in r["Kernel_Name"]]
    lo = marks[a.skip]
    hi = marks[min(a.skip + a.count, len(marks) - 1)]
    t0 = int(rows[lo]["Start_Timestamp"])
    for r in rows[lo:hi]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("void ", "").split("(")[0][:48]
        print("%9.1f %9.1f %7.1f  s%-3s q%-3s %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3,
                                                r["Stream_Id"], r["Queue_Id"], name))
    periods = [(int(rows[marks[i + 1]]["Start_Timestamp"]) - int(rows[marks[i]]["Start_Timestamp"])) / 1e3
               for i in range(a.skip, len(marks) - 1)]
    if periods:
        periods.sort()
        print("period between marks: median %.1f us, min %.1f, max %.1f (n=%d)" % (
            periods[len(periods) // 2], periods[0], periods[-1], len(periods)))


if __name__ == "__main__":
    main()
