"""Per-kernel VGPR / AGPR / scratch / occupancy of one HIP source, from the compiler's
kernel-resource-usage remarks:  python tools/kernel_resources.py csrc/fps.hip [filter]"""
import os
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
csrc = os.path.dirname(os.path.abspath(src))
flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I" + os.path.join(csrc, "../../include"),
         "-I" + csrc, "-c", src, "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage",
         "--offload-device-only"]
if os.path.basename(src) not in ("sa_mlp.hip", "sa_chain.hip", "sa_dense.hip", "linear.hip"):
    flags.append("-ffp-contract=off")
if os.path.basename(src) == "sa_dense.hip":  # csrc/Makefile DENSEFLAGS
    flags += ["-mllvm", "-amdgpu-mfma-vgpr-form"]
out = subprocess.run(["/opt/rocm/bin/hipcc"] + flags, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(.+?): (-?\d+) \[-Rpass", line)
    if cur and m:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        dem = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
        print("%-90s vgpr=%s agpr=%s scratch=%s occ=%s lds=%s" % (
            dem[:90], v.get("VGPRs"), v.get("AGPRs"), v.get("ScratchSize [bytes/lane]"),
            v.get("Occupancy [waves/SIMD]"), v.get("LDS Size [bytes/block]")))
