#!/bin/bash
# Round-end measurement on one box: smoke, GPU tests, bench (defaults), in-step rocprof stats, attention PMC.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STAGES="smoke tests bench prof" bash scripts/gpu_run.sh; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
ATTN_CONFIGS=c2 bash scripts/pmc_attn.sh
