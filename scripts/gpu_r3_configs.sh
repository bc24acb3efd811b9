#!/bin/bash
# Round-3 attack-config evidence, one GPU, every stage local:
#   detect : configs 3/4/5 x 3 seeds, re-sharding off so every injection is scored (300 steps,
#            attacks from step 100 with p=0.3 -> >= 20 injections per run)
#   reshard: configs 3/4/5 x 3 seeds, full flow (detect -> quarantine -> re-shard)
#   clean  : GPT-2-medium 8 stages, Markov data, 500 steps, no attacker, audit on and off
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out && rm -f gpurun_out/r3_cfg_*.jsonl
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name timeout args...
    local name=$1 t=$2; shift 2
    timeout -k 10 $t python -u scripts/run_attack_configs.py --out gpurun_out/r3_cfg_$name.jsonl "$@" \
        > gpurun_out/r3_cfg_$name.log 2>&1 || { tail -20 gpurun_out/r3_cfg_$name.log; return 1; }
    echo "$name: $(grep -c '^{' gpurun_out/r3_cfg_$name.log) records"
}
run clean 600 --configs clean --seeds 3 --steps 500 &&
run clean_noaudit 600 --configs clean --seeds 3 --steps 500 --no-audit &&
run detect 1100 --configs 3,4,5 --seeds 1,2,3 --steps 300 --no-reassign &&
run reshard 900 --configs 3,4,5 --seeds 1,2,3 --steps 200
