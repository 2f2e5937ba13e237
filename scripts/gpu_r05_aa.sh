#!/bin/bash
# Round 5, box aa: the attention GPU tests on the dK/dV defaults (64-row kernel, 4 / 8 waves by length).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_configs_gpu.py \
  tests/test_cp_ring_gpu.py -k "attn or attention or ring or C2 or C4 or C5" > gpurun_out/r05_aa_tests.log 2>&1 || { tail -30 gpurun_out/r05_aa_tests.log; exit 1; }
tail -2 gpurun_out/r05_aa_tests.log
timeout -k 10 300 python -u scripts/attn_bench.py --iters 30 --configs c2,c2_full,gqa4,s4096_full > gpurun_out/r05_aa_bench.jsonl 2> gpurun_out/r05_aa_bench.log || exit 1
cat gpurun_out/r05_aa_bench.jsonl
