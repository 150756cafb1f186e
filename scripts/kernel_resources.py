"""Per-kernel register / scratch / occupancy table of one HIP source file,
from the compiler's kernel-resource-usage remarks (device-only gfx950 build).
Usage: python scripts/kernel_resources.py srcdsp_amd/csrc/decim.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src,
       "-Isrcdsp_amd/csrc", "-Iinclude", "--offload-device-only", "-Rpass-analysis=kernel-resource-usage",
       "-o", "/dev/null"]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in err.splitlines():
    m = re.search(r"remark: \s*([^:]+): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
try:
    dem = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows),
                         capture_output=True, text=True).stdout.splitlines()
except OSError:
    dem = [r["name"] for r in rows]
for r, d in zip(rows, dem):
    if filt in d:
        print(f"{d[:int(sys.argv[3]) if len(sys.argv) > 3 else 90]:90s} VGPR {r.get('VGPRs','?'):>4s} AGPR {r.get('AGPRs','?'):>3s} "
              f"scratch {r.get('ScratchSize [bytes/lane]','?'):>4s} occ {r.get('Occupancy [waves/SIMD]','?')}")
