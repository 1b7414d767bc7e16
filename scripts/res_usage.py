"""Per-kernel register / spill / occupancy summary of one HIP source (hipcc -Rpass-analysis):
    python scripts/res_usage.py x2-gnn_amd/csrc/attention_center.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o",
                      "/dev/null", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for ln in out.splitlines():
    m = re.search(r"remark:\s+(.*?)(?: \[-Rpass)", ln)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.strip()
for name, r in rows.items():
    dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    if flt and flt not in dm:
        continue
    dm = re.sub(r"x2g::\(anonymous namespace\)::", "", dm)
    print(f"{dm[:90]:90s} vgpr {r.get('VGPRs', '?'):>4s} agpr {r.get('AGPRs', '?'):>3s} spill {r.get('VGPRs Spill', '?'):>3s} "
          f"occ {r.get('Occupancy [waves/SIMD]', '?')} lds {r.get('LDS Size [bytes/block]', '?')}")
