#!/bin/bash
# Round 5, box f: ring depth (prefetch distance) of the dK/dV and dQ kernels — 3-slot vs 4-slot rings for the
# pipelined kernels (PICO_ATTN_KVP / PICO_ATTN_QP) and for the shipped 32-row dK/dV kernel; numerics of the 4-slot
# variants first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=picotron_amd/lib/variants
PICO_LIB_PATH=$V/v_nb4.so PICO_ATTN_KVP=1 PICO_ATTN_QP=1 timeout -k 10 300 python -u scripts/attn_check.py --cases c2,grp_ragged,odd,ragged,gqa4,s4096,full \
  > gpurun_out/r05_f_check1.jsonl 2> gpurun_out/r05_f_check1.log || { cat gpurun_out/r05_f_check1.jsonl; tail -20 gpurun_out/r05_f_check1.log; exit 1; }
PICO_LIB_PATH=$V/v_kvnb4.so timeout -k 10 300 python -u scripts/attn_check.py --cases c2,grp_ragged,odd,ragged,gqa4,s4096,full \
  > gpurun_out/r05_f_check2.jsonl 2> gpurun_out/r05_f_check2.log || { cat gpurun_out/r05_f_check2.jsonl; tail -20 gpurun_out/r05_f_check2.log; exit 1; }
cat gpurun_out/r05_f_check1.jsonl gpurun_out/r05_f_check2.jsonl
rm -f gpurun_out/r05_f_ab.jsonl
for r in 1 2 3; do
  for v in "base 0 0" "base 1 0" "v_nb4 1 0" "v_nb4 1 1" "v_kvnb4 0 0"; do
    set -- $v
    LIB=""; [ "$1" != base ] && LIB=$V/$1.so
    PICO_LIB_PATH=$LIB PICO_ATTN_KVP=$2 PICO_ATTN_QP=$3 timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs c2,gqa4,s4096 \
      2>> gpurun_out/r05_f_ab.log | sed "s/^{/{\"lib\": \"$1\", \"kvp\": $2, \"qp\": $3, \"round\": $r, /" >> gpurun_out/r05_f_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_f_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["lib"], r["kvp"], r["qp"])].append((r["attn_bwd_q_us"], r["attn_bwd_kv_us"], r["bwd_wall_us"]))
for k, v in sorted(agg.items()):
    print(k, "dQ", [x[0] for x in v], "dKdV", [x[1] for x in v], "wall", [x[2] for x in v])
PY
PICO_LIB_PATH=$V/kvpstamp.so PICO_ATTN_KVP=1 timeout -k 10 120 python -u scripts/kvp_stamps.py > gpurun_out/r05_f_kvpstamps.json 2> gpurun_out/r05_f_kvpstamps.log || { tail -20 gpurun_out/r05_f_kvpstamps.log; exit 1; }
cat gpurun_out/r05_f_kvpstamps.json
PICO_LIB_PATH=$V/kvpstamp.so PICO_ATTN_KVP=1 PICO_ATTN_GROUPS=0 timeout -k 10 120 python -u scripts/kvp_stamps.py > gpurun_out/r05_f_kvpstamps_g0.json 2>> gpurun_out/r05_f_kvpstamps.log || exit 1
cat gpurun_out/r05_f_kvpstamps_g0.json
