"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE: they do not fit
one gfx950 TCC pass), corrected as /opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes:
FETCH_SIZE is reported in KB and counts half the bytes of wide coalesced reads on gfx950
(doubled here); WRITE_SIZE (KB) is taken as is.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py ...
    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --config ssg

Writes profiles/pmc_traffic.json[config] = {"pn2_sa_mlp_max_f32": bytes per API call (sum over
the MLP kernel dispatches one call issues), "kernels": {name: {...}}}.
bench.py reads the per-call figure into roofline.traffic.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# pn2_sa_mlp_max_f32 calls per forward for each bench config (SSG: sa1, sa2, sa3)
CALLS_PER_FORWARD = {"ssg": 3, "msg": 7, "pose": 6, "stress": 3}
FORWARD_MARKER = "fps_kernel"  # one launch per sampled SA layer, counted below
# kernels one pn2_sa_mlp_max_f32 call may dispatch
MLP_KERNELS = ("sa_mlp_kernel", "dense_layer_kernel", "sa_chain_kernel", "dense_split_kernel",
               "dense_lds_kernel", "dense_pair_kernel", "compact_scan_kernel", "u_table_kernel", "unkey_kernel")
FPS_PER_FORWARD = {"ssg": 2, "msg": 2, "pose": 3, "stress": 2}
# pn2_ball_query_f32 calls per forward (one per radius of every grouping SA layer)
BQ_PER_FORWARD = {"ssg": 2, "msg": 6, "pose": 3, "stress": 2}
# the MLP entry point each config's bench line names (config 5 runs the bf16 MLP)
MLP_NAME = {"stress": "pn2_sa_mlp_max_bf16"}


def read(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under %s" % d)
    per = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--config", default="ssg")
    ap.add_argument("--no-save", action="store_true", help="print only (A/B passes)")
    ap.add_argument("--forwards", type=float, default=0.0,
                    help="forwards the profiled run made (bench --steps + --warmup, eager); default: "
                         "counted from the FPS launches (not valid where the next layer's FPS rides "
                         "on the MLP launch, pn2_fps_side)")
    a = ap.parse_args()
    if a.config not in FPS_PER_FORWARD:
        raise SystemExit("pmc_traffic: no per-forward launch counts for config %r" % a.config)
    fetch = read(a.fetch_dir, "FETCH_SIZE")
    write = read(a.write_dir, "WRITE_SIZE")
    kernels = {}
    mlp_total = 0.0
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        fb = 2 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        kernels[short(name)] = {"dispatches": max(len(f), len(w)), "fetch_bytes": fb,
                                "write_bytes": wb}
    n_fps = sum(len(v) for k, v in fetch.items() if FORWARD_MARKER in k)
    forwards = a.forwards or n_fps / FPS_PER_FORWARD[a.config]
    for name, v in fetch.items():
        if any(k in name for k in MLP_KERNELS):
            mlp_total += 2 * 1024 * sum(v)
    for name, v in write.items():
        if any(k in name for k in MLP_KERNELS):
            mlp_total += 1024 * sum(v)
    per_call = mlp_total / (forwards * CALLS_PER_FORWARD[a.config]) if forwards else None
    bq_total = sum(2 * 1024 * sum(v) for k, v in fetch.items() if "ball_query_kernel" in k) + \
        sum(1024 * sum(v) for k, v in write.items() if "ball_query_kernel" in k)
    bq_call = bq_total / (forwards * BQ_PER_FORWARD[a.config]) if forwards else None
    if not a.no_save:
        out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        data = json.load(open(out_path)) if os.path.exists(out_path) else {}
        data[a.config] = {MLP_NAME.get(a.config, "pn2_sa_mlp_max_f32"): per_call,
                          "pn2_ball_query_f32": bq_call, "forwards": forwards, "kernels": kernels,
                          "note": "bytes per dispatch; FETCH_SIZE x2 (gfx950), KB->bytes"}
        json.dump(data, open(out_path, "w"), indent=1, sort_keys=True)
    print(json.dumps({"config": a.config, "per_call_bytes": per_call, "forwards": forwards}))
    for k, v in kernels.items():
        print("%-60s %6d  fetch %12s  write %12s" % (k[:60], v["dispatches"],
              "%.3e" % v["fetch_bytes"] if v["fetch_bytes"] is not None else "-",
              "%.3e" % v["write_bytes"] if v["write_bytes"] is not None else "-"))


if __name__ == "__main__":
    main()
