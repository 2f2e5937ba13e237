#!/bin/bash
# D = 64 dQ backward A/B on one box: numerics (attn_check + the attention GPU tests) then attn_bench, new vs old dQ kernel.
# then attn_bench with the ping-pong kernel and with the 128-row kernel (PICO_ATTN_BWDQ64=0), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PICO_ATTN_BWDQ64=1 timeout -k 10 300 python scripts/attn_check.py --cases ${CHECK_CASES:-c2,odd,ragged,gqa4,s4096,full} > gpurun_out/bwdq64_check.jsonl 2> gpurun_out/bwdq64_check.log || { echo "check failed rc=$?"; exit 1; }
if [ -n "${PYTEST_K:-}" ]; then
  PICO_ATTN_BWDQ64=1 timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/bwdq64_pytest.log 2>&1 || { echo "pytest failed rc=$?"; exit 1; }
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in 1 0; do
    PICO_ATTN_BWDQ64=$v timeout -k 10 300 python scripts/attn_bench.py --configs ${ATTN_CONFIGS:-c2,c2_full,gqa4,s4096} | sed "s/^{/{\"bwdq64\": $v, \"round\": $r, /" >> gpurun_out/bwdq64_bench.jsonl || exit $?
  done
done
echo "== bwdq64 done"
