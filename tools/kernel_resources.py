#!/usr/bin/env python3
"""VGPRs, occupancy and spills of every dycore kernel, from hipcc's kernel-resource-usage remarks.

    python tools/kernel_resources.py [name-substring ...]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def resources():
    src = os.path.join(ROOT, "mpas-model_amd", "csrc", "dycore.hip")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-ffp-contract=off", "-Wno-unused-result", "--cuda-device-only", "-c", src, "-o", "/dev/null",
                        "-Rpass-analysis=kernel-resource-usage"] + os.environ.get("KR_EXTRA", "").split(), capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"mangled": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+(VGPRs|Occupancy \[waves/SIMD\]|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]): (\d+)",
                      line)
        if m and cur is not None:
            cur[m.group(1).split()[0] + ("Spill" if "Spill" in m.group(1) else "")] = int(m.group(2))
    names = subprocess.run(["c++filt"], input="\n".join(x["mangled"] for x in rows), capture_output=True,
                           text=True).stdout.splitlines()
    for x, n in zip(rows, names):
        x["name"] = n.split("(")[0].replace("void ", "").replace("mpas::", "")
    return rows


if __name__ == "__main__":
    pats = sys.argv[1:] or ["k_"]
    for x in resources():
        if any(p in x["name"] for p in pats):
            print(f'{x["name"][:56]:56s} VGPR={x.get("VGPRs")} occ={x.get("Occupancy")} '
                  f'spill S/V={x.get("SGPRsSpill")}/{x.get("VGPRsSpill")} LDS={x.get("LDS")}')
