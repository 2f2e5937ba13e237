#!/bin/bash
# Round 5, box ag: slot 1's stream priority in the pipelined graph (PICO_SLOT1_PRIORITY -1 = high vs 0), 3 alternating
# rounds; first the priority range and whether a captured graph keeps it.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())" || exit 1
rm -f gpurun_out/r05_ag_ab.jsonl
for r in 1 2 3; do
  for o in 0 -1; do
    PICO_SLOT1_PRIORITY=$o timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-kernel-timing > gpurun_out/r05_ag_p${o}_$r.json 2> gpurun_out/r05_ag_p${o}_$r.log \
      || { tail -20 gpurun_out/r05_ag_p${o}_$r.log; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r05_ag_p${o}_$r.json')); print(json.dumps({'slot1_priority': $o, 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'mfu_pct': d['mfu_pct'], 'loss_last': d['loss_last']}))" >> gpurun_out/r05_ag_ab.jsonl
  done
done
cat gpurun_out/r05_ag_ab.jsonl
