#!/bin/bash
# Round 5 measurement set on one box: the default bench line, in-step rocprof of the pipelined step and of the
# serial per-micro-batch step (PICO_MB_PIPELINE=0: kernel durations without the other micro-batch beside them),
# the attention micro-bench at C2, and the attention PMC passes at C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/final_prof gpurun_out/final_prof_serial gpurun_out/pmc
timeout -k 10 900 python3 bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.log || { tail -20 gpurun_out/final_bench.log; exit 1; }
cat gpurun_out/final_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_prof -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/final_prof.json 2> gpurun_out/final_prof.log || { tail -20 gpurun_out/final_prof.log; exit 1; }
PICO_MB_PIPELINE=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_prof_serial -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/final_prof_serial.json 2> gpurun_out/final_prof_serial.log || { tail -20 gpurun_out/final_prof_serial.log; exit 1; }
timeout -k 10 300 python3 scripts/attn_bench.py --configs c2,c2_full,gqa4,s4096,d128,d128_b2 > gpurun_out/final_attn_bench.jsonl 2> gpurun_out/final_attn_bench.log || exit 1
cat gpurun_out/final_attn_bench.jsonl
ATTN_CONFIGS=c2 bash scripts/pmc_attn.sh || exit 1
python3 scripts/pmc_summary.py --json gpurun_out/final_pmc_attn_c2.json > gpurun_out/final_pmc_attn_c2_summary.txt
cat gpurun_out/final_pmc_attn_c2_summary.txt
