#!/bin/bash
# Round 5, box l: where the DP wrapper's per-step cost goes — in-step kernel stats of the default step with and
# without DataParallelBucket at one rank (bench --dp-bucket), same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "plain " "dp --dp-bucket"; do
  set -- $v
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05_l_$1 -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing ${2:-} > gpurun_out/r05_l_$1.json 2> gpurun_out/r05_l_$1.log \
    || { tail -20 gpurun_out/r05_l_$1.log; exit 1; }
  cat gpurun_out/r05_l_$1.json
done
