#!/bin/bash
# Round 5, box z: long sequences — the 32-row dK/dV kernel vs the 64-row kernel with 4 / 8 waves, causal and
# non-causal, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r05_z_ab.jsonl
for r in 1 2 3; do
  for v in "kv32 0 4" "kvp4 1 4" "kvp8 1 8"; do
    set -- $v
    PICO_ATTN_KVP=$2 PICO_KVP_WAVES=$3 timeout -k 10 240 python -u scripts/attn_bench.py --iters 30 --configs s2048,s4096,s4096_full \
      2>> gpurun_out/r05_z_ab.log | sed "s/^{/{\"variant\": \"$1\", \"round\": $r, /" >> gpurun_out/r05_z_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_z_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["variant"])].append((r["attn_bwd_q_us"], r["attn_bwd_kv_us"], r["bwd_wall_us"]))
for k, v in sorted(agg.items()):
    print(k, "dQ", [x[0] for x in v], "dKdV", [x[1] for x in v], "wall", [x[2] for x in v])
PY
