#!/bin/bash
# Same-box A/B of library variants inside the training step: bench.py once per variant (PICO_LIB_PATH), interleaved
# rounds; one JSON line per run in gpurun_out/ab_step.jsonl (with the variant and round).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${STEP_ROUNDS:-1}); do
  for v in ${VARIANTS}; do
    PICO_LIB_PATH=picotron_amd/lib/variants/$v.so timeout -k 10 400 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline 2> gpurun_out/ab_step_$v.log | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> gpurun_out/ab_step.jsonl
    rc=${PIPESTATUS[0]}
    if [ "$rc" -ne 0 ]; then echo "bench $v failed rc=$rc"; tail -20 gpurun_out/ab_step_$v.log; exit $rc; fi
  done
done
