#!/bin/bash
# BASELINE config 2 at N=1 (GPT-2-small, T=1024, batch 64) and the headline GPT-2-medium, verification
# on vs --no-verify, interleaved on one box (2 rounds), with the default native MLP GEMMs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
out=gpurun_out/small_verify_ab.txt
: > $out
for round in $(seq 1 ${ROUNDS:-2}); do
  for model in ${MODELS:-gpt2-small gpt2-medium}; do
    for v in on off; do
      flag=""; [ $v = off ] && flag="--no-verify"
      timeout -k 10 200 python -u bench.py --model $model --steps 10 --warmup 3 $flag > gpurun_out/sv.json 2> gpurun_out/sv.err || { echo "$model $v failed"; tail -5 gpurun_out/sv.err; exit 1; }
      echo "round $round $model verify=$v $(tail -1 gpurun_out/sv.json)" >> $out
      tail -1 $out | cut -c1-200
    done
  done
done
