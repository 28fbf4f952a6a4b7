"""Per-(kernel, grid) average durations from a rocprofv3 kernel_trace.csv: separates the calls
of one template instance at different shapes (e.g. the dense layer's pre-pass and sa3 layers).
    python tools/debug/trace_shapes.py <run_kernel_trace.csv> [name-substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(list)
for r in rows:
    if pat and pat not in r["Kernel_Name"]:
        continue
    key = (r["Kernel_Name"][:60], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])),
           int(r["Grid_Size_Y"]), int(r["LDS_Block_Size"]))
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (name, gx, gy, lds), d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    d.sort()
    print("%-60s grid %5dx%-3d lds %6d  n %4d  avg %8.1f  med %8.1f us" % (name, gx, gy, lds, len(d), sum(d) / len(d), d[len(d) // 2]))
