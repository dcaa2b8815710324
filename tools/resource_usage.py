#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table of a HIP source (hipcc -Rpass-analysis=kernel-resource-usage).

usage: python tools/resource_usage.py monotonic-rnnt_amd/csrc/mrnnt_grad.hip [filter]
"""
import re, subprocess, sys, os

here = os.path.dirname(os.path.abspath(__file__))
pkg = os.path.join(here, "..", "monotonic-rnnt_amd")
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
       "-I" + os.path.join(pkg, "..", "include"), "-I" + os.path.join(pkg, "csrc"),
       "-c", src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|SGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        dem = subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()
        cur = {"name": dem}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt in r["name"]:
        print(f'{r.get("VGPRs","?"):>4} vgpr {r.get("AGPRs","?"):>3} agpr occ {r.get("Occupancy [waves/SIMD]","?"):>2} '
              f'sspill {r.get("SGPRs Spill","?"):>3} vspill {r.get("VGPRs Spill","?"):>3} scratch {r.get("ScratchSize [bytes/lane]","?"):>4} '
          f'lds {r.get("LDS Size [bytes/block]","?"):>6}  {r["name"]}')
