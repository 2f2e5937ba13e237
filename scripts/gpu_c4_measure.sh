#!/bin/bash
# C4 (Llama-2-7B per-rank attention: D = 128, 16 heads, the reference's micro-batch 4 (and 2), S = 1024) measurements: the attention
# micro-bench (library HIP-event timers), a rocprofv3 kernel-stats run of it, and the PMC passes + summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs d128,d128_b2,d128_gqa4,d128_s4096 > gpurun_out/c4_attn_bench.jsonl 2> gpurun_out/c4_attn_bench.log || exit $?
rm -rf gpurun_out/c4_prof
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c4_prof" -o c4 -- python3 "$R/scripts/attn_bench.py" --iters 20 --configs d128 > gpurun_out/c4_prof.log 2>&1 || exit $?
find gpurun_out/c4_prof -name "*kernel_trace.csv" -delete
rm -rf gpurun_out/pmc
ATTN_CONFIGS=d128 timeout -k 10 900 bash scripts/pmc_attn.sh || exit $?
python scripts/pmc_summary.py --dir gpurun_out/pmc --match attn_ --json gpurun_out/c4_pmc.json > gpurun_out/c4_pmc_summary.txt
find gpurun_out/pmc -name "*.csv" -size +1M -delete
cat gpurun_out/c4_attn_bench.jsonl
