#!/bin/bash
# Prints VGPR/SGPR/scratch/LDS of the kernels in a hipcc object matching a pattern (default: all).
# usage: scripts/kernel_resources.sh incubator-pinot_amd/build/scan.o [regex]
set -e
OBJ=$1; PAT=${2:-.}
D=$(mktemp -d)
cp "$OBJ" "$D/o.o"
(cd "$D" && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading o.o > /dev/null)
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$D"/o.o.0.hipv4-amdgcn-amd-amdhsa--gfx950 | python3 -c "
import sys,re
t=sys.stdin.read()
for blk in t.split('- .agpr_count')[1:]:
    name=re.search(r'\.name:\s+(\S+)',blk).group(1)
    if re.search(sys.argv[1], name):
        g=lambda k: (re.search(r'\.'+k+r':\s+(\S+)',blk) or [None,None])[1]
        print('%-70s vgpr %-4s sgpr %-4s scratch %-5s lds %-6s spill %s' % (name[:70], g('vgpr_count'), g('sgpr_count'), g('private_segment_fixed_size'), g('group_segment_fixed_size'), g('vgpr_spill_count')))
" "$PAT"
rm -rf "$D"
