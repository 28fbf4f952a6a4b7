"""Per-(kernel, grid) median durations from a rocprofv3 kernel trace:
python tools/kstats.py <dir with *kernel_trace.csv> [name filter]"""
import collections
import csv
import glob
import sys

d = collections.defaultdict(list)
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for x in csv.DictReader(open(f)):
        if flt not in x["Kernel_Name"]:
            continue
        key = (x["Kernel_Name"].split("(")[0][:60], x["Grid_Size_X"], x["Workgroup_Size_X"], x["LDS_Block_Size"])
        d[key].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print("%-60s grid %7s wg %4s lds %6s  n %4d  med %7.2f us  min %7.2f" % (k + (len(v), v[len(v) // 2], v[0])))
