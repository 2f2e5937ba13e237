#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass, --kernel-trace only besides --pmc) on the attention micro-bench
# (PMC_BENCH=kernel: the HBM kernel micro-bench, scripts/kernel_bench.py, instead).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
if [ "${PMC_BENCH:-attn}" = kernel ]; then BENCH="scripts/kernel_bench.py"; else BENCH="scripts/attn_bench.py --iters 5 --configs ${ATTN_CONFIGS:-c2}"; fi
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $line --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 $BENCH > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i ($line) exit $rc" | tee -a gpurun_out/pmc/status.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done < "${PMC_FILE:-scripts/pmc_attn.txt}"
