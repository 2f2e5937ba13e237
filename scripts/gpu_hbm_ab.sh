#!/bin/bash
# Same-box A/B of HBM kernels under environment switches: ROUNDS x (each "NAME=ENV" in AB) of scripts/kernel_bench.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for spec in ${AB}; do
    name=${spec%%=*}; envs=${spec#*=}
    env ${envs//,/ } timeout -k 10 120 python scripts/kernel_bench.py 2>/dev/null | sed "s/^{/{\"variant\": \"$name\", \"round\": $r, /" >> gpurun_out/hbm_ab.jsonl || exit $?
  done
done
echo "== hbm ab done"
