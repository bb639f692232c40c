#!/bin/bash
# Register / LDS / spill usage of the gfx950 kernels in a hipcc object:
#   tools/kstats.sh zkevm-prover_amd/build/stark.o [kernel-substring]
set -e
LLVM=/opt/rocm/lib/llvm/bin
d=$(mktemp -d)
$LLVM/llvm-objcopy --dump-section=.hip_fatbin=$d/fb.bin "$1"
$LLVM/clang-offload-bundler --unbundle --type=o --input=$d/fb.bin \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$d/k.co
$LLVM/llvm-readelf --notes $d/k.co | python3 -c '
import sys, re
pat = sys.argv[1] if len(sys.argv) > 1 else ""
cur = {}
for line in sys.stdin:
    m = re.match(r"\s+\.(\w+):\s+(.*)", line)
    if m: cur[m.group(1)] = m.group(2)
    if line.strip().startswith("- .agpr_count") or line.strip() == "-" :
        pass
    if "vgpr_spill_count" in line:
        nm = cur.get("name", "?")
        if pat in nm:
            print("%-60s vgpr=%s agpr=%s sgpr=%s spill=%s lds=%s scratch=%s" % (nm[:60], cur.get("vgpr_count"), cur.get("agpr_count"),
                  cur.get("sgpr_count"), cur.get("vgpr_spill_count"), cur.get("group_segment_fixed_size"), cur.get("private_segment_fixed_size")))
' "${2:-}"
rm -rf $d
