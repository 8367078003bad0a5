#!/usr/bin/env python3
"""Per-kernel VGPR / spill / LDS / occupancy summary of one HIP source for gfx950
(hipcc -Rpass-analysis=kernel-resource-usage), optionally filtered by a name substring.

  python scripts/kernel_resources.py csrc/attn_prefill.hip [substring]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-Icsrc", "--offload-arch=gfx950", "-ffp-contract=fast",
       "--cuda-device-only", "-c", src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"remark: (?:\s*)([^\[]+?) \[-Rpass", line)
    if not m:
        continue
    txt = m.group(1).strip()
    if txt.startswith("Function Name:"):
        cur = {"name": txt.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt in r["name"]:
        print(f'{r["name"][:90]:90s} vgpr={r.get("VGPRs")} agpr={r.get("AGPRs")} spill={r.get("VGPRs Spill")} '
              f'scratch={r.get("ScratchSize [bytes/lane]")} lds={r.get("LDS Size [bytes/block]")} '
              f'occ={r.get("Occupancy [waves/SIMD]")}')
