"""The GPU's shader clock and power around pipelined runs (SSG, K = 100): does the first timed
run after a short warm-up, or one after an idle gap, run at a lower clock?
A host thread samples the card's sysfs (pp_dpm_sclk's current level, hwmon power) every ~2 ms
while the main thread runs: idle 0.3 s, 10-batch warm-up, 4 timed K = 100 runs back to back,
idle 0.3 s, 1 timed run.  python tools/debug/clock_trace.py"""
import glob
import os
import re
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402,F401  (its sys.path setup)
import cases  # noqa: E402
from pn2 import heads as H  # noqa: E402
from pn2 import shard  # noqa: E402
from pn2.pipeline import GraphedPipeline  # noqa: E402

DEV = torch.device("cuda", 0)


def card_dir():
    p = torch.cuda.get_device_properties(0)
    bus = getattr(p, "pci_bus_id", None)
    dom = getattr(p, "pci_domain_id", 0)
    dev = getattr(p, "pci_device_id", 0)
    if bus is not None:
        d = "/sys/bus/pci/devices/%04x:%02x:%02x.0" % (dom, bus, dev)
        if os.path.exists(os.path.join(d, "pp_dpm_sclk")):
            return d
    c = sorted(glob.glob("/sys/class/drm/card*/device/pp_dpm_sclk"))
    print("pci id lookup failed (%r); sysfs cards: %d" % (bus, len(c)))
    return os.path.dirname(c[0]) if len(c) == 1 else None


def reader(d):
    f_sclk = os.path.join(d, "pp_dpm_sclk")
    fs = [os.path.join(d, "pp_dpm_%s" % k) for k in ("sclk", "mclk", "fclk", "socclk")]
    fs = [f for f in fs if os.path.exists(f)]
    for f in fs:
        try:
            print(f, open(f).read().replace("\n", " | "))
        except OSError as e:
            print(f, e)
    hw = glob.glob(os.path.join(d, "hwmon", "hwmon*"))
    f_pw = None
    for name in ("power1_input", "power1_average"):
        if hw and os.path.exists(os.path.join(hw[0], name)):
            f_pw = os.path.join(hw[0], name)
            break
    print("sysfs:", f_sclk, f_pw)

    def level(f):
        try:
            with open(f) as fh:
                for line in fh:
                    if "*" in line:
                        m = re.search(r"(\d+)\s*[Mm]hz", line)
                        return int(m.group(1)) if m else None
        except OSError:
            pass
        return None

    def read_all():
        return tuple(level(f) for f in fs)
    read_all.names = [os.path.basename(f)[7:] for f in fs]

    def read():
        mhz = None
        try:
            with open(f_sclk) as f:
                for line in f:
                    if "*" in line:
                        m = re.search(r"(\d+)\s*[Mm]hz", line)
                        mhz = int(m.group(1)) if m else None
        except OSError:
            pass
        w = None
        if f_pw:
            try:
                with open(f_pw) as f:
                    w = int(f.read()) / 1e6
            except (OSError, ValueError):
                pass
        return mhz, w
    return read, read_all


def main():
    d = card_dir()
    if d is None:
        print("no sysfs card found")
        return
    read, read_all = reader(d)
    print("first sample:", read())
    samples, marks = [], []
    stop = threading.Event()
    t0 = time.perf_counter()

    def loop():
        while not stop.is_set():
            mhz, w = read()
            samples.append((time.perf_counter() - t0, mhz, w))
            time.sleep(0.002)

    th = threading.Thread(target=loop, daemon=True)
    torch.manual_seed(8)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 8)
    model = model.to(DEV)
    x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
    torch.manual_seed(1234)
    gp = GraphedPipeline(model)
    post = lambda i, o: None  # noqa: E731
    torch.cuda.synchronize()
    th.start()
    time.sleep(0.3)

    def timed(tag, k):
        torch.cuda.synchronize()
        a = time.perf_counter()
        with shard.batch_shard(32, 0):
            gp.run([x] * k, post=post)
        torch.cuda.synchronize()
        b = time.perf_counter()
        marks.append((tag, a - t0, b - t0, 32 * k / (b - a)))

    timed("warm10", 10)
    for i in range(4):
        timed("run%d" % i, 100)
    time.sleep(0.3)
    timed("after_idle", 100)
    time.sleep(0.05)
    stop.set()
    th.join()
    # the ramp after idle at 2 ms resolution: consecutive K = 10 runs, with every clock domain
    # read between runs (sysfs reads ~tens of us each)
    for gap in (0.3, 0.3):
        time.sleep(gap)
        rows = []
        for i in range(16):
            timed("k10_%d" % i, 10)
            rows.append((marks[-1][3], read_all()))
        print("after %.0f ms idle, K=10 runs: (clouds/s, %s)" % (gap * 1e3, "/".join(read_all.names)))
        print("  " + "  ".join("%.0fk %s" % (r / 1e3, "/".join(str(v) for v in c)) for r, c in rows))
    marks[:] = [m for m in marks if not m[0].startswith("k10")]
    for tag, a, b, r in marks:
        s = [m for (t, m, w) in samples if a <= t <= b and m is not None]
        p = [w for (t, m, w) in samples if a <= t <= b and w is not None]
        print("%-10s %7.1f-%7.1f ms %8.0f clouds/s  sclk n=%d min %s max %s mean %s  power mean %s"
              % (tag, a * 1e3, b * 1e3, r, len(s), min(s) if s else "-", max(s) if s else "-",
                 "%.0f" % (sum(s) / len(s)) if s else "-", "%.0f" % (sum(p) / len(p)) if p else "-"))
    # the whole series, coarsened to 5 ms bins
    bins = {}
    for t, m, w in samples:
        bins.setdefault(int(t * 200), []).append((m, w))
    for k in sorted(bins):
        ms = [m for m, _ in bins[k] if m is not None]
        ws = [w for _, w in bins[k] if w is not None]
        print("t=%6.0f ms sclk %s power %s" % (k * 5, "%.0f" % (sum(ms) / len(ms)) if ms else "-",
                                               "%.0f" % (sum(ws) / len(ws)) if ws else "-"))


if __name__ == "__main__":
    main()
