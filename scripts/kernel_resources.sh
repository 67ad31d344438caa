#!/bin/bash
# Per-kernel VGPR / SGPR / LDS / scratch of a built library's gfx950 code object:
#   scripts/kernel_resources.sh LIB [kernel-name-regex]
set -e
LIB=$1
PAT=${2:-.}
T=$(mktemp -d)
objcopy --dump-section .hip_fatbin="$T/fat.bin" "$LIB"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --input="$T/fat.bin" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/k.co" --unbundle
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$T/k.co" | python3 -c '
import re, sys
pat = re.compile(sys.argv[1])
cur = {}
rows = []
for line in sys.stdin:
    m = re.match(r"\s+- \.agpr_count:", line)
    if m and cur:
        rows.append(cur); cur = {}
    m = re.match(r"\s+\.(name|vgpr_count|sgpr_count|group_segment_fixed_size|private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count):\s+(\S+)", line)
    if m: cur[m.group(1)] = m.group(2)
if cur: rows.append(cur)
for r in rows:
    n = r.get("name", "?")
    if pat.search(n):
        g = lambda k: r.get(k, "?")
        print("%4s vgpr %4s sgpr lds %6s scratch %5s spill %s  %s" % (g("vgpr_count"), g("sgpr_count"),
              g("group_segment_fixed_size"), g("private_segment_fixed_size"), g("vgpr_spill_count"), n[:110]))
' "$PAT"
rm -rf "$T"
