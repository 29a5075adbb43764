"""Per-kernel register / occupancy table of one .hip file (hipcc -Rpass-analysis=kernel-resource-usage).

usage: python tools/kres.py paddle_infer_amd/csrc/kernels/layernorm.hip [name-filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics",
       "-c", src, "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"]
with open(src) as f:
    for line in f.read().splitlines()[:40]:
        if line.startswith("// piamd-hipcc-flags:"):
            cmd[1:1] = line.split(":", 1)[1].split()
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                       text=True).stdout.splitlines()
print(f"{'kernel':70s} {'VGPR':>5s} {'AGPR':>5s} {'spill':>5s} {'occ':>4s} {'LDS':>6s}")
for r, n in zip(rows, names):
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))
    if flt and flt not in n:
        continue
    print(f"{n[:70]:70s} {r.get('VGPRs', '?'):>5s} {r.get('AGPRs', '?'):>5s} {r.get('VGPRs Spill', '?'):>5s} "
          f"{r.get('Occupancy [waves/SIMD]', '?'):>4s} {r.get('LDS Size [bytes/block]', '?'):>6s}")
