#!/bin/bash
# Same-box A/B of library variants on the HBM kernel micro-bench (scripts/kernel_bench.py):
# parity tests (-k TEST_K) on each variant, then ROUNDS interleaved rounds, lines matching KB_GREP.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  PICO_LIB_PATH=picotron_amd/lib/variants/$v.so timeout -k 10 300 python -u -m pytest tests -q -m gpu -k "${TEST_K}" --timeout 120 --timeout-method thread > gpurun_out/t_$v.log 2>&1 || exit $?
done
for r in $(seq 1 ${ROUNDS:-3}); do for v in ${VARIANTS}; do
  PICO_LIB_PATH=picotron_amd/lib/variants/$v.so timeout -k 10 120 python scripts/kernel_bench.py 2>/dev/null | grep "${KB_GREP}" | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/hbm_ab.jsonl || exit $?
done; done
