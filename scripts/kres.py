"""Compact per-kernel resource report (VGPRs, AGPRs, spills, occupancy, LDS) of one source file.
    python scripts/kres.py x2-gnn_amd/csrc/attention.hip [name-regex]"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o",
                      "/dev/null", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark:\s+(\w[^:]*?):\s+(.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for name, r in rows.items():
    dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    short = re.sub(r"\(.*", "", dem.replace("(anonymous namespace)::", "")).replace("x2g::", "").replace("void ", "")
    if pat and not pat.search(short):
        continue
    print(f"{short:60s} vgpr {r.get('VGPRs','?'):>4s} agpr {r.get('AGPRs','?'):>3s} spill {r.get('VGPRs Spill','?'):>3s}"
          f" scratch {r.get('ScratchSize [bytes/lane]','?'):>4s} occ {r.get('Occupancy [waves/SIMD]','?'):>2s}"
          f" lds {r.get('LDS Size [bytes/block]','?')}")
