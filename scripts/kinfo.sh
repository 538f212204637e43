#!/bin/bash
# Register / LDS / spill metadata of the kernels whose name matches $2 in library $1.
set -e
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy --dump-section .hip_fatbin=$T/fb.bin "$1" /dev/null
$B/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$T/fb.bin --output=$T/co.o
$B/llvm-readelf --notes $T/co.o | awk -v pat="$2" '
  /\.name:/ {name=$2} /\.vgpr_count:/ {v=$2} /\.sgpr_count:/ {s=$2} /\.vgpr_spill_count:/ {vs=$2} /\.sgpr_spill_count:/ {ss=$2}
  /\.agpr_count:/ {a=$2} /\.group_segment_fixed_size:/ {g=$2} /\.private_segment_fixed_size:/ {pr=$2}
  /\.wavefront_size:/ { if (name ~ pat) printf "%-60s vgpr %s agpr %s sgpr %s vspill %s sspill %s scratch %s\n", substr(name,1,60), v, a, s, vs, ss, pr }'
rm -rf $T
