#!/bin/bash
# Round 5, box d: the pipelined 64-row dK/dV kernel (PICO_ATTN_KVP=1) — numerics, the attention GPU tests under it,
# then a same-box A/B against the shipped kernel (3 interleaved rounds); the AccumulateGrad probe (node pre-hooks).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PICO_ATTN_KVP=1 timeout -k 10 300 python -u scripts/attn_check.py --cases c2,grp_ragged,grp_10,odd,ragged,gqa4,s4096,full,fold5,fold_ragged \
  > gpurun_out/r05_d_check.jsonl 2> gpurun_out/r05_d_check.log || { cat gpurun_out/r05_d_check.jsonl; tail -20 gpurun_out/r05_d_check.log; exit 1; }
cat gpurun_out/r05_d_check.jsonl
PICO_ATTN_KVP=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_configs_gpu.py \
  tests/test_cp_ring_gpu.py -k "attn or attention or ring or C2" > gpurun_out/r05_d_tests.log 2>&1 || { tail -30 gpurun_out/r05_d_tests.log; exit 1; }
tail -2 gpurun_out/r05_d_tests.log
rm -f gpurun_out/r05_d_ab.jsonl
for r in 1 2 3; do
  for v in "0 1" "1 1" "1 0"; do
    set -- $v
    PICO_ATTN_KVP=$1 PICO_ATTN_GROUPS=$2 timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs c2,gqa4,s4096,c2_full \
      2>> gpurun_out/r05_d_ab.log | sed "s/^{/{\"kvp\": $1, \"groups\": $2, \"round\": $r, /" >> gpurun_out/r05_d_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_d_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["kvp"], r["groups"])].append((r["attn_bwd_q_us"], r["attn_bwd_kv_us"], r["bwd_wall_us"]))
for k, v in sorted(agg.items()):
    print(k, "dQ", [x[0] for x in v], "dKdV", [x[1] for x in v], "wall", [x[2] for x in v])
PY
timeout -k 10 300 python -u scripts/dbg_accgrad_stream.py > gpurun_out/r05_d_accgrad.log 2>&1 || { tail -20 gpurun_out/r05_d_accgrad.log; exit 1; }
grep "^\[" gpurun_out/r05_d_accgrad.log
