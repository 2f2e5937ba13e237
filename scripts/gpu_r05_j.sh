#!/bin/bash
# Round 5, box j: the whole GPU suite (the DP stacked-gradient path, the new tests), then the default bench step
# with the shipped dK/dV kernel vs the pipelined 64-row one (PICO_ATTN_KVP), alternating, 2 x 2 runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -q -m gpu --timeout 400 --timeout-method thread -rf > gpurun_out/r05_j_pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r05_j_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2; do
  for k in 0 1; do
    PICO_ATTN_KVP=$k timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/r05_j_bench_kvp${k}_$r.json 2>> gpurun_out/r05_j_bench.log || { tail -20 gpurun_out/r05_j_bench.log; exit 1; }
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05_j_bench_*.json")):
    d = json.loads(open(f).read())
    k = d["kernels"]
    print(f, d["value"], d["ms_per_step"], d["mfu_pct"], "frac", d["roofline"]["frac"],
          {n: k[n]["avg_us"] for n in ("attn_fwd", "attn_bwd_q", "attn_bwd_kv", "rope", "rmsnorm_bwd") if n in k})
PY
