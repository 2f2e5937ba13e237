#!/bin/bash
# Round 5, box v: block groups up to 16 per head now also cover D = 128 at S 4096 (one workgroup per CU, 16 heads):
# numerics, then PICO_ATTN_GROUPS=0 / 1 on d128_s4096 and the C4 shapes, 3 interleaved rounds; the D = 64 default
# (64-row dK/dV kernel also for non-causal blocks up to 4096 keys) on the attention tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/attn_check.py --cases d128_s4096,d128,d128_ragged,s4096_full,c2 \
  > gpurun_out/r05_v_check.jsonl 2> gpurun_out/r05_v_check.log || { cat gpurun_out/r05_v_check.jsonl; tail -20 gpurun_out/r05_v_check.log; exit 1; }
cat gpurun_out/r05_v_check.jsonl
rm -f gpurun_out/r05_v_ab.jsonl
for r in 1 2 3; do
  for g in 0 1; do
    PICO_ATTN_GROUPS=$g timeout -k 10 240 python -u scripts/attn_bench.py --iters 30 --configs d128_s4096,d128,d128_b2 \
      2>> gpurun_out/r05_v_ab.log | sed "s/^{/{\"groups\": $g, \"round\": $r, /" >> gpurun_out/r05_v_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_v_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["groups"])].append((r["attn_bwd_q_us"], r["attn_bwd_kv_us"], r["bwd_wall_us"]))
for k, v in sorted(agg.items()):
    print(k, "dQ", [x[0] for x in v], "dKdV", [x[1] for x in v], "wall", [x[2] for x in v])
PY
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_configs_gpu.py \
  tests/test_cp_ring_gpu.py -k "attn or attention or ring or C2 or C4 or C5" > gpurun_out/r05_v_tests.log 2>&1 || { tail -30 gpurun_out/r05_v_tests.log; exit 1; }
tail -2 gpurun_out/r05_v_tests.log
