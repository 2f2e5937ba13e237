#!/bin/bash
# Round 5, box ad: the 64-row dK/dV kernel's prologue waiting for tile 0 and K / V only (the other prologue tile issued
# after) — numerics, then A/B against the previous prologue (variant library), 3 interleaved rounds.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/attn_check.py --cases c2,grp_ragged,grp_10,odd,ragged,gqa4,full,fold5,s4096_full,s3000 \
  > gpurun_out/r05_ad_check.jsonl 2> gpurun_out/r05_ad_check.log || { cat gpurun_out/r05_ad_check.jsonl; tail -20 gpurun_out/r05_ad_check.log; exit 1; }
PICO_ATTN_KVP=1 PICO_KVP_WAVES=8 timeout -k 10 300 python -u scripts/attn_check.py --cases c2,gqa4,ragged,s3000 \
  >> gpurun_out/r05_ad_check.jsonl 2>> gpurun_out/r05_ad_check.log || { cat gpurun_out/r05_ad_check.jsonl; tail -20 gpurun_out/r05_ad_check.log; exit 1; }
cat gpurun_out/r05_ad_check.jsonl
rm -f gpurun_out/r05_ad_ab.jsonl
for r in 1 2 3; do
  for v in "new " "prev picotron_amd/lib/variants/kvp_before.so"; do
    set -- $v
    PICO_LIB_PATH=${2:-} timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs c2,gqa4,c2_full,s4096_full \
      2>> gpurun_out/r05_ad_ab.log | sed "s/^{/{\"variant\": \"$1\", \"round\": $r, /" >> gpurun_out/r05_ad_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_ad_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["variant"])].append((r["attn_bwd_q_us"], r["attn_bwd_kv_us"], r["bwd_wall_us"]))
for k, v in sorted(agg.items()):
    print(k, "dQ", [x[0] for x in v], "dKdV", [x[1] for x in v], "wall", [x[2] for x in v])
PY
