#!/bin/bash
# Round 5, box p: groups of 4 micro-batches per weight-gradient GEMM (PICO_WGRAD_GROUP=4) against pairs, plain and
# DataParallelBucket at one rank, 3 alternating rounds on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r05_p_ab.jsonl
for r in 1 2 3; do
  for v in "plain_g2 2" "plain_g4 4" "dp_g2 2 --dp-bucket" "dp_g4 4 --dp-bucket"; do
    set -- $v
    PICO_WGRAD_GROUP=$2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-kernel-timing ${3:-} > gpurun_out/r05_p_$1_$r.json 2> gpurun_out/r05_p_$1_$r.log \
      || { tail -20 gpurun_out/r05_p_$1_$r.log; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r05_p_$1_$r.json')); print(json.dumps({'variant': '$1', 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'mfu_pct': d['mfu_pct'], 'loss_last': d['loss_last']}))" >> gpurun_out/r05_p_ab.jsonl
  done
done
cat gpurun_out/r05_p_ab.jsonl
