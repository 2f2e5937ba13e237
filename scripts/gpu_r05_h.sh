#!/bin/bash
# Round 5, box h: the pipelined kernels with their DMA issued in the last MFMA phase's gaps — numerics, then a
# same-box A/B: shipped (kvp 0, qp 0), kvp (M2(B) DMA), kvp_front (DMA after the barrier), kvp + qp; kvp stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=picotron_amd/lib/variants
PICO_ATTN_KVP=1 PICO_ATTN_QP=1 timeout -k 10 300 python -u scripts/attn_check.py --cases c2,grp_ragged,grp_10,odd,ragged,gqa4,s4096,full,fold5,fold_ragged \
  > gpurun_out/r05_h_check.jsonl 2> gpurun_out/r05_h_check.log || { cat gpurun_out/r05_h_check.jsonl; tail -20 gpurun_out/r05_h_check.log; exit 1; }
cat gpurun_out/r05_h_check.jsonl
rm -f gpurun_out/r05_h_ab.jsonl
for r in 1 2 3; do
  for v in "base 0 0" "base 1 0" "kvp_front 1 0" "base 1 1"; do
    set -- $v
    LIB=""; [ "$1" != base ] && LIB=$V/$1.so
    PICO_LIB_PATH=$LIB PICO_ATTN_KVP=$2 PICO_ATTN_QP=$3 timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs c2,gqa4,s4096,c2_full \
      2>> gpurun_out/r05_h_ab.log | sed "s/^{/{\"lib\": \"$1\", \"kvp\": $2, \"qp\": $3, \"round\": $r, /" >> gpurun_out/r05_h_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_h_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["lib"], r["kvp"], r["qp"])].append((r["attn_bwd_q_us"], r["attn_bwd_kv_us"], r["bwd_wall_us"]))
for k, v in sorted(agg.items()):
    print(k, "dQ", [x[0] for x in v], "dKdV", [x[1] for x in v], "wall", [x[2] for x in v])
PY
PICO_LIB_PATH=$V/kvpstamp.so PICO_ATTN_KVP=1 timeout -k 10 120 python -u scripts/kvp_stamps.py > gpurun_out/r05_h_kvpstamps.json 2> gpurun_out/r05_h_kvpstamps.log || { tail -20 gpurun_out/r05_h_kvpstamps.log; exit 1; }
cat gpurun_out/r05_h_kvpstamps.json
