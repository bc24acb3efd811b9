#!/bin/bash
# Interleaved bench.py A/B over environment variants (3 rounds, one box):
#   VARIANTS="A=;B=TDL_NATIVE_PROJ=1" bash scripts/gpu_bench_env_ab.sh
mkdir -p gpurun_out
out=gpurun_out/bench_env_ab.txt
: > $out
IFS=';' read -ra VS <<< "${VARIANTS}"
for r in 1 2 3; do
  for v in "${VS[@]}"; do
    name=${v%%=*}; envs=${v#*=}
    line=$(env $envs timeout -k 10 300 python -u ${BENCH:-bench.py} --steps ${STEPS:-10} --warmup ${WARMUP:-3} 2>/dev/null | grep '^{') || { echo "round $r $name failed" >> $out; exit 1; }
    val=$(echo "$line" | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
    echo "round $r $name [$envs] value ms/step: $val" >> $out
  done
done
cat $out
