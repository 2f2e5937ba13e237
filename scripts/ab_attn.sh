#!/bin/bash
# Same-box A/B of library variants on the attention micro-bench: ROUNDS interleaved rounds over
# picotron_amd/lib/variants/<v>.so (VARIANTS="a b c"), one process per (round, variant).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS}; do
    PICO_LIB_PATH=picotron_amd/lib/variants/$v.so timeout -k 10 120 python scripts/attn_bench.py --configs ${ATTN_CONFIGS:-c2} --iters ${ITERS:-30} 2>/dev/null | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> gpurun_out/ab.jsonl
    rc=${PIPESTATUS[0]}
    if [ "$rc" -ne 0 ]; then echo "variant $v failed rc=$rc"; exit $rc; fi
  done
done
