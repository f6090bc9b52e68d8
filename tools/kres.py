"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: python tools/kres.py <file.hip> [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", "/tmp/kres.o", *sys.argv[3:],
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\])?: (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        dm = subprocess.run(["c++filt"], input=k, capture_output=True, text=True).stdout.strip() or k
        print(f"VGPR {v.get('VGPRs', 0):3d} AGPR {v.get('AGPRs', 0):3d} spill {v.get('VGPRs Spill', 0):3d} "
              f"scratch {v.get('ScratchSize', 0):4d}  {dm[:110]}")
