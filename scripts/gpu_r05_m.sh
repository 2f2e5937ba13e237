#!/bin/bash
# Round 5, box m: the 64-row dK/dV kernel as the D = 64 default — attention tests; then the step with and without
# DataParallelBucket at one rank (bench --dp-bucket), 3 alternating rounds on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_configs_gpu.py \
  tests/test_cp_ring_gpu.py -k "attn or attention or ring or C2 or C4" > gpurun_out/r05_m_tests.log 2>&1 || { tail -30 gpurun_out/r05_m_tests.log; exit 1; }
tail -2 gpurun_out/r05_m_tests.log
rm -f gpurun_out/r05_m_ab.jsonl
for r in 1 2 3; do
  for v in "plain " "dp --dp-bucket"; do
    set -- $v
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-kernel-timing ${2:-} > gpurun_out/r05_m_$1_$r.json 2> gpurun_out/r05_m_$1_$r.log \
      || { tail -20 gpurun_out/r05_m_$1_$r.log; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r05_m_$1_$r.json')); print(json.dumps({'variant': '$1', 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'mfu_pct': d['mfu_pct']}))" >> gpurun_out/r05_m_ab.jsonl
  done
done
cat gpurun_out/r05_m_ab.jsonl
