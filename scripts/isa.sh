#!/bin/bash
# Disassembles the gfx950 code object of an engine library: scripts/isa.sh <lib.so> <out.s>
set -e
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy --dump-section .hip_fatbin=$T/fb.bin "$1" /dev/null
$B/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$T/fb.bin --output=$T/co.o
$B/llvm-objdump -d --no-show-raw-insn $T/co.o > "$2"
rm -rf $T
