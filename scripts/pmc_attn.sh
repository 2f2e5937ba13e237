#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass, --kernel-trace only besides --pmc) on the attention micro-bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $line --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 scripts/attn_bench.py --iters 5 --configs ${ATTN_CONFIGS:-c2} > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i ($line) exit $rc" | tee -a gpurun_out/pmc/status.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done < "${PMC_FILE:-scripts/pmc_attn.txt}"
