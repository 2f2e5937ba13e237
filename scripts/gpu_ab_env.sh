#!/bin/bash
# Same-box A/B of environment settings inside the training step: bench.py once per variant, interleaved rounds.
# VARIANTS="base:X=0 pipe:PICO_MB_PIPELINE=1" (name:VAR=val,VAR=val; "name:" for no change); one JSON line per
# run in gpurun_out/ab_env.jsonl (with the variant and round).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${STEP_ROUNDS:-1}); do
  for spec in ${VARIANTS}; do
    v=${spec%%:*}
    envs=${spec#*:}
    timeout -k 10 400 env ${envs//,/ } python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline \
      2> gpurun_out/ab_env_$v.log | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> gpurun_out/ab_env.jsonl
    rc=${PIPESTATUS[0]}
    if [ "$rc" -ne 0 ]; then echo "bench $v failed rc=$rc"; tail -20 gpurun_out/ab_env_$v.log; exit $rc; fi
  done
done
cat gpurun_out/ab_env.jsonl
