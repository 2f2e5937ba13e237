#!/bin/bash
# Round 5, box n: row-stacked weight gradients as fp32-output GEMMs into main_grad and the chained RMSNorm dw on
# non-syncing micro-batches under DataParallelBucket — DP / composition GPU tests, then the step plain / DP /
# DP with the previous stacked form (PICO_DP_STACKED=accum), 3 alternating rounds on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_dp_hip_gpu.py tests/test_pp_dp_gpu.py \
  tests/test_composition_gpu.py > gpurun_out/r05_n_tests.log 2>&1 || { tail -30 gpurun_out/r05_n_tests.log; exit 1; }
tail -2 gpurun_out/r05_n_tests.log
rm -f gpurun_out/r05_n_ab.jsonl
for r in 1 2 3; do
  for v in "plain gemm" "dp gemm --dp-bucket" "dpaccum accum --dp-bucket"; do
    set -- $v
    PICO_DP_STACKED=$2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-kernel-timing ${3:-} > gpurun_out/r05_n_$1_$r.json 2> gpurun_out/r05_n_$1_$r.log \
      || { tail -20 gpurun_out/r05_n_$1_$r.log; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r05_n_$1_$r.json')); print(json.dumps({'variant': '$1', 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'mfu_pct': d['mfu_pct'], 'loss_last': d['loss_last']}))" >> gpurun_out/r05_n_ab.jsonl
  done
done
cat gpurun_out/r05_n_ab.jsonl
