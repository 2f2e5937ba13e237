#!/bin/bash
# Attention backward A/B over environment settings (AB="name=ENV=VAL ..."): numerics (attn_check cases) per
# setting, optional GPU tests (PYTEST_K, default setting only), then interleaved attn_bench rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in ${AB}; do
  name=${spec%%=*}; kv=${spec#*=}
  env $kv timeout -k 10 300 python scripts/attn_check.py --cases ${CHECK_CASES:-d128,d128_ragged,d128_full,odd,ragged,c2} > gpurun_out/check_$name.jsonl 2> gpurun_out/check_$name.log || { echo "check $name failed rc=$?"; exit 1; }
done
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/ab_pytest.log 2>&1 || { echo "pytest failed rc=$?"; exit 1; }
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in ${AB}; do
    name=${spec%%=*}; kv=${spec#*=}
    env $kv timeout -k 10 300 python scripts/attn_bench.py --configs ${ATTN_CONFIGS:-d128,d128_full,d128_s4096,d128_gqa4} | sed "s/^{/{\"variant\": \"$name\", \"round\": $r, /" >> gpurun_out/ab.jsonl || exit $?
  done
done
echo "== ab done"
