#!/bin/bash
# Kernel trace of the C2 training step (pipelined graph, then the per-micro-batch graph) and its occupancy
# summary (scripts/trace_busy.py). Output under gpurun_out/trace_*.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
for v in ${TRACE_VARIANTS:-pipe:1 serial:0}; do
  name=${v%%:*}; flag=${v#*:}
  rm -rf "$R/gpurun_out/trace_$name"
  PICO_MB_PIPELINE=$flag timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace_$name" \
    -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/trace_$name.json" \
    2> "$R/gpurun_out/trace_$name.log" || exit $?
  f=$(find "$R/gpurun_out/trace_$name" -name "*kernel_trace.csv" | head -1)
  python "$R/scripts/trace_busy.py" "$f" --steps 2 --json "$R/gpurun_out/trace_busy_$name.json" > /dev/null || exit $?
  rm -f "$f"
done
cat "$R/gpurun_out/trace_busy_pipe.json" "$R/gpurun_out/trace_busy_serial.json"
