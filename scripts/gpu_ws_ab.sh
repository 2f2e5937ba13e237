#!/bin/bash
# hipBLASLt workspace A/B: the GEMM micro-bench and the C2 step with the default workspace and with
# HIPBLASLT_WORKSPACE_SIZE=${WS_KIB:-262144} KiB, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in def big; do
  if [ $v = big ]; then export HIPBLASLT_WORKSPACE_SIZE=${WS_KIB:-262144}; else unset HIPBLASLT_WORKSPACE_SIZE; fi
  timeout -k 10 300 python scripts/gemm_bench.py | sed "s/^{/{\"ws\": \"$v\", /" >> gpurun_out/ws_gemm.jsonl || exit $?
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in def big; do
    if [ $v = big ]; then export HIPBLASLT_WORKSPACE_SIZE=${WS_KIB:-262144}; else unset HIPBLASLT_WORKSPACE_SIZE; fi
    timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline 2> gpurun_out/ws_bench_$v$r.log | sed "s/^{/{\"ws\": \"$v\", \"round\": $r, /" >> gpurun_out/ws_bench.jsonl || exit $?
  done
done
echo "== ws ab done"
