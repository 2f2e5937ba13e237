#!/bin/bash
# Round 5, box u: block groups up to 16 per head, and the 64-row dK/dV kernel beyond 2048 keys — numerics with it
# forced (PICO_ATTN_KVP=1), then the attention micro-bench with it forced off / on, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PICO_ATTN_KVP=1 timeout -k 10 300 python -u scripts/attn_check.py --cases c2,s4096,s4096_full,s3000,grp_ragged,ragged \
  > gpurun_out/r05_u_check.jsonl 2> gpurun_out/r05_u_check.log || { cat gpurun_out/r05_u_check.jsonl; tail -20 gpurun_out/r05_u_check.log; exit 1; }
cat gpurun_out/r05_u_check.jsonl
rm -f gpurun_out/r05_u_ab.jsonl
for r in 1 2 3; do
  for kvp in 0 1; do
    PICO_ATTN_KVP=$kvp timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs c2,s2048,s4096,s4096_full \
      2>> gpurun_out/r05_u_ab.log | sed "s/^{/{\"kvp\": $kvp, \"round\": $r, /" >> gpurun_out/r05_u_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_u_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["kvp"])].append((r["attn_bwd_q_us"], r["attn_bwd_kv_us"], r["bwd_wall_us"]))
for k, v in sorted(agg.items()):
    print(k, "dQ", [x[0] for x in v], "dKdV", [x[1] for x in v], "wall", [x[2] for x in v])
PY
