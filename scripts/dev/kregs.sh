#!/bin/bash
# Register / LDS / spill summary of the kl:: kernels of one source (development aid).
# usage: scripts/dev/kregs.sh kaolin-windows_amd/csrc/softmask.hip
set -e
src=$(readlink -f "$1")
t=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -x hip --cuda-device-only \
  --no-gpu-bundle-output -c "$src" -o "$t/k.co"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$t/k.co" | python3 -c '
import sys, re, subprocess
cur = {}
out = []
for line in sys.stdin:
    m = re.match(r"\s+\.(name|vgpr_count|sgpr_count|group_segment_fixed_size|vgpr_spill_count|agpr_count):\s+(\S+)", line)
    if m:
        cur[m.group(1)] = m.group(2)
        if m.group(1) == "vgpr_spill_count":
            out.append(dict(cur)); cur = {}
for d in out:
    n = d.get("name", "")
    if "_ZN2kl" not in n: continue
    dm = subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    print("%-90s vgpr=%s agpr=%s sgpr=%s lds=%s spill=%s" % (dm[:90], d.get("vgpr_count"), d.get("agpr_count"), d.get("sgpr_count"), d.get("group_segment_fixed_size"), d.get("vgpr_spill_count")))
'
rm -rf "$t"
