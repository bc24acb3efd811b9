#!/bin/bash
# Round-3 attack-config evidence, one GPU, every stage local.  Two calls (each
# under gpurun's 20-minute limit):  PART=a  clean runs + full-flow re-shard runs;  PART=b  detection-only.
#   clean  : GPT-2-medium 8 stages, Markov data, 500 steps, no attacker, audit on and off
#   reshard: configs 3/4/5 x 3 seeds, full flow (detect -> quarantine -> re-shard), 200 steps
#   detect : configs 3/4/5 x 3 seeds, re-sharding off so every injection is scored (300 steps,
#            attacks from step 100 with p=0.3 -> >= 20 injections per run)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name timeout args...
    local name=$1 t=$2; shift 2
    rm -f gpurun_out/r3_cfg_$name.jsonl
    timeout -k 10 $t python -u scripts/run_attack_configs.py --out gpurun_out/r3_cfg_$name.jsonl "$@" \
        > gpurun_out/r3_cfg_$name.log 2>&1 || { tail -20 gpurun_out/r3_cfg_$name.log; return 1; }
    echo "$name: $(grep -c '^{' gpurun_out/r3_cfg_$name.log) records"
}
if [ "${PART:-a}" = a ]; then
    run clean 300 --configs clean --seeds 3 --steps 500 &&
    run clean_noaudit 300 --configs clean --seeds 3 --steps 500 --no-audit &&
    run reshard 560 --configs 3,4,5 --seeds 1,2,3 --steps 200
else
    run detect 900 --configs 3,4,5 --seeds 1,2,3 --steps 300 --no-reassign &&
    run clean200 150 --configs clean --seeds 4 --steps 200 &&
    run clean200_noaudit 150 --configs clean --seeds 4 --steps 200 --no-audit
fi
