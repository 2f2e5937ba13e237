#!/bin/bash
# Round 5, box s: the LM head's weight gradient grouped like the projections' (one dW GEMM per four micro-batches,
# the final norm's y^T in the head's x^T slot) — model tests, then the step with PICO_LM_WGRAD_GROUP=0 / 1, plain and
# DataParallelBucket, 2 alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 400 --timeout-method thread tests/test_model_gpu.py tests/test_dp_hip_gpu.py \
  > gpurun_out/r05_s_tests.log 2>&1 || { tail -40 gpurun_out/r05_s_tests.log; exit 1; }
grep "loss-overlay\|passed\|failed" gpurun_out/r05_s_tests.log
rm -f gpurun_out/r05_s_ab.jsonl
for r in 1 2; do
  for v in "plain_lm0 0" "plain_lm1 1" "dp_lm0 0 --dp-bucket" "dp_lm1 1 --dp-bucket"; do
    set -- $v
    PICO_LM_WGRAD_GROUP=$2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-kernel-timing ${3:-} > gpurun_out/r05_s_$1_$r.json 2> gpurun_out/r05_s_$1_$r.log \
      || { tail -20 gpurun_out/r05_s_$1_$r.log; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r05_s_$1_$r.json')); print(json.dumps({'variant': '$1', 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'mfu_pct': d['mfu_pct'], 'loss_last': d['loss_last']}))" >> gpurun_out/r05_s_ab.jsonl
  done
done
cat gpurun_out/r05_s_ab.jsonl
