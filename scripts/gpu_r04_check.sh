#!/bin/bash
# GPU suite + a short bench (round 4 checks). Output under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/r04_pytest.log 2>&1
rc=$?
grep -E "passed|failed|PASSED|FAILED|Error" gpurun_out/r04_pytest.log | tail -15
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -60 gpurun_out/r04_pytest.log; exit 1; }
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup 2 $BENCH_ARGS > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.log || { echo "bench rc=$?"; tail -30 gpurun_out/r04_bench.log; exit 1; }
  cat gpurun_out/r04_bench.json | head -c 3000
fi
