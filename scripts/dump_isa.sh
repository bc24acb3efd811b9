#!/bin/bash
# Disassemble the gfx950 code object of a built object file: scripts/dump_isa.sh build/native/gemm.hip.o out.s
B=/opt/rocm/lib/llvm/bin
$B/llvm-objcopy --dump-section=.hip_fatbin=/tmp/_fatbin.bin "$1" && \
$B/clang-offload-bundler --unbundle --input=/tmp/_fatbin.bin --output=/tmp/_dev.co --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 && \
$B/llvm-objdump -d /tmp/_dev.co > "$2"
