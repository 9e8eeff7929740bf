"""VGPR / AGPR / spill / LDS / occupancy of the kernels of one csrc file (gfx950).
    python tools/resource_usage.py gemm_bf16.hip [name-filter]"""
import os
import re
import subprocess
import sys

csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "sequential-variational-autoencoder_amd", "csrc")
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I../../include", "-I.",
                    "-x", "hip", "-c", sys.argv[1], "-o", "/tmp/ru.o", "-Rpass-analysis=kernel-resource-usage"],
                   cwd=csrc, capture_output=True, text=True)
cur = None
out = []
for line in r.stderr.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": subprocess.run(["c++filt", t.split(":", 1)[1].strip()], capture_output=True,
                                      text=True).stdout.strip()}
        out.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for d in out:
    if flt in d["name"]:
        print("%-90s VGPR %4s AGPR %4s spill %3s/%3s occ %s LDS %s" % (
            d["name"][:90], d.get("VGPRs"), d.get("AGPRs"), d.get("VGPRs Spill"), d.get("SGPRs Spill"),
            d.get("Occupancy [waves/SIMD]"), d.get("LDS Size [bytes/block]")))
