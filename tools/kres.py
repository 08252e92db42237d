#!/usr/bin/env python3
"""Per-kernel register use of a HIP source for gfx950 (hipcc -Rpass-analysis=
kernel-resource-usage): name, VGPRs, scratch, VGPR/SGPR spills, occupancy.
  python3 tools/kres.py lsm_storage_engine_amd/csrc/lsmck_crc32.hip"""
import re
import subprocess
import sys

src = sys.argv[1]
p = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-Iinclude",
                    "-Ilsm_storage_engine_amd/csrc", "-c", src, "-o", "/tmp/kres.o"] + sys.argv[2:] + [
                    "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur = None
rows = {}
for line in p.stderr.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\S+) \[", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    name = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
    print(f"{name[:80]:80s} vgpr {v.get('VGPRs', '?'):>4s} scratch {v.get('ScratchSize [bytes/lane]', '?'):>4s} "
          f"vspill {v.get('VGPRs Spill', '?'):>3s} sspill {v.get('SGPRs Spill', '?'):>3s} occ {v.get('Occupancy [waves/SIMD]', '?')}")
