#!/bin/bash
# Round-4 probes on one GPU: the pipelined micro-batch graph (parity tests, then a same-box step A/B), the
# forward GEMMs with a transposed activation operand, HBM kernels hot vs cold (MALL flushed between launches).
# Output under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_model_gpu.py \
  tests/test_kernels_gpu.py -k "graph_replay or transposed" > gpurun_out/pipe_tests.log 2>&1 &&
VARIANTS="base:PICO_MB_PIPELINE=0 pipe:PICO_MB_PIPELINE=1" \
  STEP_ROUNDS=2 STEPS=5 timeout -k 10 1000 bash scripts/gpu_ab_env.sh &&
timeout -k 10 240 python -u scripts/gemm_at_probe.py > gpurun_out/gemm_at_probe.jsonl 2> gpurun_out/gemm_at_probe.log &&
timeout -k 10 240 python -u scripts/kernel_bench.py > gpurun_out/kernel_bench_hot.jsonl 2> gpurun_out/kernel_bench_hot.log &&
timeout -k 10 240 python -u scripts/kernel_bench.py --cold > gpurun_out/kernel_bench_cold.jsonl 2> gpurun_out/kernel_bench_cold.log
rc=$?
tail -8 gpurun_out/pipe_tests.log
cat gpurun_out/gemm_at_probe.jsonl 2>/dev/null
exit $rc
