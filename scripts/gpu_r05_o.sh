#!/bin/bash
# Round 5, box o: the weight-gradient stream in the pipelined graph — the capture pattern with plain tensor ops,
# the equality tests, then the step with PICO_WGRAD_STREAM=0 / 1 and groups of 2 / 4 micro-batches per wgrad GEMM
# (plain and DataParallelBucket), 2 alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/dbg_wstream_capture.py > gpurun_out/r05_o_capture.log 2>&1 || { cat gpurun_out/r05_o_capture.log; exit 1; }
cat gpurun_out/r05_o_capture.log
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_model_gpu.py \
  -k "wgrad_stream or wgrad_pairs or pipelined" > gpurun_out/r05_o_tests.log 2>&1 || { tail -40 gpurun_out/r05_o_tests.log; exit 1; }
grep "wgrad-stream\|passed\|failed" gpurun_out/r05_o_tests.log
rm -f gpurun_out/r05_o_ab.jsonl
for r in 1 2; do
  for v in "plain_ws0 0 2" "plain_ws1 1 2" "plain_ws1_g4 1 4" "dp_ws0 0 2 --dp-bucket" "dp_ws1 1 2 --dp-bucket" "dp_ws1_g4 1 4 --dp-bucket"; do
    set -- $v
    PICO_WGRAD_STREAM=$2 PICO_WGRAD_GROUP=$3 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-kernel-timing ${4:-} > gpurun_out/r05_o_$1_$r.json 2> gpurun_out/r05_o_$1_$r.log \
      || { tail -20 gpurun_out/r05_o_$1_$r.log; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r05_o_$1_$r.json')); print(json.dumps({'variant': '$1', 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'mfu_pct': d['mfu_pct'], 'loss_last': d['loss_last']}))" >> gpurun_out/r05_o_ab.jsonl
  done
done
cat gpurun_out/r05_o_ab.jsonl
