#!/bin/bash
# One GPU session on the box: smoke -> GPU parity tests -> short bench (-> optional profile).
# Every GPU step has its own time limit; a crash / abort / timeout stops the script (a plain test
# failure, exit 1, does not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGES="${STAGES:-smoke tests bench}"
ok_or_stop() {  # $1 = exit code, $2 = step name
  local rc=$1
  echo "== $2 exit $rc" | tee -a gpurun_out/status.log
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $2 (rc=$rc)"; exit "$rc"; fi
}
for s in $STAGES; do
  case "$s" in
    smoke)
      timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      ok_or_stop $? smoke ;;
    tests)
      PICO_LOSS_OUT=gpurun_out/loss_curve_gpu.json timeout -k 10 1200 python -u -m pytest tests -q -m gpu --timeout 400 --timeout-method thread ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
      ok_or_stop $? pytest ;;
    bench)
      timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.log
      ok_or_stop $? bench ;;
    attn)
      timeout -k 10 300 python scripts/attn_bench.py --configs ${ATTN_CONFIGS:-c2,c2_full,d128,gqa4} > gpurun_out/attn_bench.jsonl 2> gpurun_out/attn_bench.log
      ok_or_stop $? attn ;;
    gemm)
      timeout -k 10 300 python scripts/gemm_bench.py > gpurun_out/gemm_default.jsonl 2>&1
      ok_or_stop $? gemm_default
      PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv timeout -k 10 900 python scripts/gemm_bench.py > gpurun_out/gemm_tunable.jsonl 2>&1
      ok_or_stop $? gemm_tunable ;;
    prof)
      export TMPDIR=/tmp
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
      ok_or_stop $? prof ;;
  esac
done
echo "== done" | tee -a gpurun_out/status.log
