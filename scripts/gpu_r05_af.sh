#!/bin/bash
# Round 5, box af: kernel trace of the layer-ordered pipelined step (PICO_LAYER_ORDER=1) for scripts/trace_overlap.py.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r05_af_prof
PICO_LAYER_ORDER=1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05_af_prof -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > gpurun_out/r05_af_prof.json 2> gpurun_out/r05_af_prof.log \
  || { tail -20 gpurun_out/r05_af_prof.log; exit 1; }
python3 scripts/trace_overlap.py $(ls gpurun_out/r05_af_prof/*kernel_trace.csv gpurun_out/r05_af_prof/*/*kernel_trace.csv 2>/dev/null | head -1)
