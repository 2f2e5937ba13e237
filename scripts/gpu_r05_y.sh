#!/bin/bash
# Round 5, box y: the 64-row dK/dV kernel with 8 waves (one 256-key workgroup per CU, PICO_KVP_WAVES=8) —
# numerics, then the attention micro-bench with 4 / 8 waves, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PICO_KVP_WAVES=8 PICO_ATTN_KVP=1 timeout -k 10 300 python -u scripts/attn_check.py --cases c2,grp_ragged,grp_10,odd,ragged,gqa4,full,fold5,s4096,s3000 \
  > gpurun_out/r05_y_check.jsonl 2> gpurun_out/r05_y_check.log || { cat gpurun_out/r05_y_check.jsonl; tail -20 gpurun_out/r05_y_check.log; exit 1; }
cat gpurun_out/r05_y_check.jsonl
rm -f gpurun_out/r05_y_ab.jsonl
for r in 1 2 3; do
  for w in 4 8; do
    PICO_KVP_WAVES=$w PICO_ATTN_KVP=1 timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs c2,gqa4,c2_full,s2048,s4096 \
      2>> gpurun_out/r05_y_ab.log | sed "s/^{/{\"waves\": $w, \"round\": $r, /" >> gpurun_out/r05_y_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_y_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["waves"])].append((r["attn_bwd_q_us"], r["attn_bwd_kv_us"], r["bwd_wall_us"]))
for k, v in sorted(agg.items()):
    print(k, "dQ", [x[0] for x in v], "dKdV", [x[1] for x in v], "wall", [x[2] for x in v])
PY
