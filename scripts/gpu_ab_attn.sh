#!/bin/bash
# Numerics gate + same-box timing A/B of attention library variants (picotron_amd/lib/variants/<v>.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  PICO_LIB_PATH=picotron_amd/lib/variants/$v.so timeout -k 10 300 python scripts/attn_check.py --cases ${CHECK_CASES:-c2,odd,ragged,gqa4,s4096,full} > gpurun_out/check_$v.jsonl 2> gpurun_out/check_$v.log || { echo "check $v failed rc=$?"; exit 1; }
done
ROUNDS=${ROUNDS:-3} ATTN_CONFIGS=${ATTN_CONFIGS:-c2,s4096} bash scripts/ab_attn.sh || exit $?
echo "== ab done"
