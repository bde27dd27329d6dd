"""Per-kernel VGPR / scratch / LDS table from hipcc -Rpass-analysis (build check)."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "vector_amd/csrc/xcorr.hip"
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src,
                      "-o", "/tmp/_regs.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1)
        k = re.match(r"_ZN4vsig\d+([a-z_]+)INS_4PlanILi(\d+)ELi(\d+)EJ([^E]*)EEE(?:Li(\d)E)?", name)
        cur = {"name": f"{k.group(1)} N={k.group(2)} E={k.group(3)} V={k.group(5)}" if k else name[:60]}
        rows.append(cur)
        continue
    for key in ("VGPRs", "ScratchSize \\[bytes/lane\\]", "LDS Size \\[bytes/block\\]", "Occupancy \\[waves/SIMD\\]"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0]] = int(m.group(1))
for r in rows:
    if flt in r["name"]:
        print(f"{r['name']:40s} vgpr={r.get('VGPRs')} scratch={r.get('ScratchSize')} lds={r.get('LDS')} occ={r.get('Occupancy')}")
