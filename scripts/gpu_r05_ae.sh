#!/bin/bash
# Round 5, box ae: layer-ordered backwards in the pipelined graph (PICO_LAYER_ORDER) — bit-identity tests, then a
# 3-round alternating step A/B, then a kernel trace of the layer-ordered step for scripts/trace_overlap.py.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_model_gpu.py \
  -k "layer_ordered or graph_replay_matches_eager or graph_replay_with_dp_bucket" > gpurun_out/r05_ae_tests.log 2>&1 \
  || { tail -40 gpurun_out/r05_ae_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r05_ae_tests.log
rm -f gpurun_out/r05_ae_ab.jsonl
for r in 1 2 3; do
  for o in 0 1; do
    PICO_LAYER_ORDER=$o timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-kernel-timing > gpurun_out/r05_ae_o${o}_$r.json 2> gpurun_out/r05_ae_o${o}_$r.log \
      || { tail -20 gpurun_out/r05_ae_o${o}_$r.log; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r05_ae_o${o}_$r.json')); print(json.dumps({'layer_order': $o, 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'mfu_pct': d['mfu_pct'], 'loss_last': d['loss_last']}))" >> gpurun_out/r05_ae_ab.jsonl
  done
done
cat gpurun_out/r05_ae_ab.jsonl
