#!/bin/bash
# Round 5, box aj: in-step rocprof kernel stats of the final tree — the pipelined step (what bench.py times) and the
# serial per-micro-batch step (PICO_MB_PIPELINE=0: kernel durations without the other micro-batch beside them),
# plus the bench line of the same box.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/aj_prof gpurun_out/aj_prof_serial
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/aj_bench.json 2> gpurun_out/aj_bench.log || { tail -20 gpurun_out/aj_bench.log; exit 1; }
cat gpurun_out/aj_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/aj_prof -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/aj_prof.json 2> gpurun_out/aj_prof.log || { tail -20 gpurun_out/aj_prof.log; exit 1; }
PICO_MB_PIPELINE=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/aj_prof_serial -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/aj_prof_serial.json 2> gpurun_out/aj_prof_serial.log || { tail -20 gpurun_out/aj_prof_serial.log; exit 1; }
python3 scripts/trace_overlap.py gpurun_out/aj_prof/run_kernel_trace.csv
