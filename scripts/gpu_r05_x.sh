#!/bin/bash
# Round 5, box x: the round's final tree — smoke, the whole GPU suite, the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/status.log
STAGES="smoke tests bench" PYTEST_ARGS="-s" bash scripts/gpu_run.sh; rc=$?
tail -3 gpurun_out/pytest_gpu.log
cat gpurun_out/bench.json
exit $rc
