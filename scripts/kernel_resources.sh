#!/bin/bash
# Register / LDS / scratch use of the gfx950 kernels in an object built by the Makefile:
#   scripts/kernel_resources.sh fury_amd/lib/varlen.o [name-regex]
set -e
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy -O binary --only-section=.hip_fatbin "$1" $T/fb
$B/clang-offload-bundler --unbundle --type=o --input=$T/fb --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/co
$B/llvm-readelf --notes $T/co | grep -E "^ +\.(name|vgpr_count|sgpr_count|vgpr_spill_count|group_segment_fixed_size|private_segment_fixed_size):" |
  awk '/\.name:/{if(n)print n, v, s, sp, p; n=$2; v=s=sp=p=""} /vgpr_count/{v="vgpr="$2} /\.sgpr_count/{s="sgpr="$2} /vgpr_spill/{sp="spill="$2} /private_segment/{p="scratch="$2} END{print n, v, s, sp, p}' |
  c++filt | grep -E "${2:-.}" || true
rm -rf $T
