"""Per-kernel summary of rocprofv3 SQ counter passes (tools/sq_pmc.sh): per-call means and
per-wave rates.  SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles per wave
(MI355X_MICROARCH.md); SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs, so
mfma_busy = it / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)."""
import collections
import csv
import glob
import json
import sys

# --json PATH: also write {kernel: {mfma_busy, gui_us, calls}} (bench.py's roofline.mfma_busy)
jpath = None
if "--json" in sys.argv:
    i = sys.argv.index("--json")
    jpath = sys.argv[i + 1]
    del sys.argv[i:i + 2]

agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(collections.Counter)
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k][r["Counter_Name"]] += 1
rows = []
for k, v in agg.items():
    c = {n: v[n] / max(1, calls[k][n]) for n in v}
    waves = c.get("SQ_WAVES", 0) or 1
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    gui = c.get("GRBM_GUI_ACTIVE", 0)
    rows.append((gui, k, c, waves, wc))
rows.sort(reverse=True)
print("%-58s %6s %7s %6s %6s %6s %6s %7s %7s %7s %6s %6s %7s" % (
    "kernel", "waves", "gui_us", "wait", "winst", "active", "mfma", "valu/w", "salu/w", "lds/w", "vmrd/w", "ldsbc",
    "ldsact"))
for gui, k, c, waves, wc in rows[:25]:
    mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
    lact = c.get("SQ_LDS_IDX_ACTIVE")
    print("%-58s %6d %7.1f %6.2f %6.2f %6.2f %6s %7.0f %7.0f %7.0f %6.0f %6.3f %7s" % (
        k[:58], waves, gui / 8 / 2.4e3, c.get("SQ_WAIT_ANY", 0) / wc, c.get("SQ_WAIT_INST_ANY", 0) / wc,
        c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        "%.3f" % (mf / (gui / 8 * 1024)) if mf and gui else "-",
        c.get("SQ_INSTS_VALU", 0) / waves, c.get("SQ_INSTS_SALU", 0) / waves,
        c.get("SQ_INSTS_LDS", 0) / waves, c.get("SQ_INSTS_VMEM_RD", 0) / waves,
        c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, c.get("SQ_LDS_IDX_ACTIVE", 0)),
        # LDS-array cycles per CU-cycle of the kernel (256 CUs): the LDS's busy fraction
        "%.3f" % (lact / (gui / 8 * 256)) if lact and gui else "-"))

if jpath:
    out = {}
    for gui, k, c, waves, wc in rows:
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        if mf and gui:
            out[k] = {"mfma_busy": round(mf / (gui / 8 * 1024), 4), "gui_us": round(gui / 8 / 2.4e3, 2),
                      "calls": int(calls[k]["GRBM_GUI_ACTIVE"])}
    with open(jpath, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
