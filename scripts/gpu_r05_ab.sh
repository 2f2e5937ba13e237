#!/bin/bash
# Round 5, box ab: issue order inside the pipelined graph's iterations (PICO_MB_FWD_FIRST), 3 alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r05_ab_ab.jsonl
for r in 1 2 3; do
  for f in 0 1; do
    PICO_MB_FWD_FIRST=$f timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-kernel-timing > gpurun_out/r05_ab_f${f}_$r.json 2> gpurun_out/r05_ab_f${f}_$r.log \
      || { tail -20 gpurun_out/r05_ab_f${f}_$r.log; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r05_ab_f${f}_$r.json')); print(json.dumps({'fwd_first': $f, 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'mfu_pct': d['mfu_pct'], 'loss_last': d['loss_last']}))" >> gpurun_out/r05_ab_ab.jsonl
  done
done
cat gpurun_out/r05_ab_ab.jsonl
