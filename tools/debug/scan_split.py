import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "compact_scan" in r["Kernel_Name"] or "u_table" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows:
    k = r["Kernel_Name"][:30] + " grid " + r.get("Grid_Size_X", r.get("Grid_Size", "?"))
    by.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in by.items():
    v.sort()
    print("%-50s n %3d med %7.2f us" % (k, len(v), v[len(v) // 2]))
