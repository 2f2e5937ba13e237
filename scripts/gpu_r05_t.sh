#!/bin/bash
# Round 5, box t: after removing the measured-slower opt-in paths — the whole GPU suite and smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/status.log
STAGES="smoke tests" PYTEST_ARGS="-s" bash scripts/gpu_run.sh; rc=$?
tail -3 gpurun_out/pytest_gpu.log
exit $rc
