#!/bin/bash
# Fast ISA inspection of gemm_p4<NT, bf16>: one-instantiation build + disassembly + resource usage.
set -eo pipefail
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -fPIC -O3 -munsafe-fp-atomics -DTDL_GEMM_ISA_ONLY $ISA_FLAGS -I csrc \
  -c csrc/gemm.hip -o /tmp/gemm_isa.o -Rpass-analysis=kernel-resource-usage 2>&1 | grep -A9 "Name: _ZN12_GLOBAL__N_17gemm_p4" | grep "VGPRs\|AGPRs\|Scratch\|Spill"
scripts/dump_isa.sh /tmp/gemm_isa.o /tmp/gemm_isa.s
awk '/^[0-9a-f]+ <_ZN12_GLOBAL__N_17gemm_p4/{f=1;print;next} f&&/^[0-9a-f]+ <_ZN/{exit} f' /tmp/gemm_isa.s > /tmp/p4.s
echo "lines $(wc -l < /tmp/p4.s) mfma $(grep -c v_mfma /tmp/p4.s) scratch $(grep -c scratch_ /tmp/p4.s) accw $(grep -c v_accvgpr_write /tmp/p4.s) accr $(grep -c v_accvgpr_read /tmp/p4.s)"
