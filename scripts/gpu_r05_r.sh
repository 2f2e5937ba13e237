#!/bin/bash
# Round 5, box r: the round's defaults (64-row dK/dV kernel for D = 64 up to 2048 keys, groups of four micro-batches
# per wgrad GEMM) through smoke, the whole GPU suite, the default bench line and an in-step rocprof of the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof gpurun_out/status.log
STAGES="smoke tests bench prof" PYTEST_ARGS="-s" bash scripts/gpu_run.sh; rc=$?
tail -3 gpurun_out/pytest_gpu.log
cat gpurun_out/bench.json
exit $rc
