#!/bin/bash
# Round 5, box k: kvp as one tile stream across the group's key blocks — numerics, A/B against the previous kvp
# (per-block prologue) and the shipped 32-row kernel, stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=picotron_amd/lib/variants
PICO_ATTN_KVP=1 timeout -k 10 300 python -u scripts/attn_check.py --cases c2,grp_ragged,grp_10,odd,ragged,gqa4,s4096,full,fold5,fold_ragged \
  > gpurun_out/r05_k_check.jsonl 2> gpurun_out/r05_k_check.log || { cat gpurun_out/r05_k_check.jsonl; tail -20 gpurun_out/r05_k_check.log; exit 1; }
cat gpurun_out/r05_k_check.jsonl
PICO_ATTN_KVP=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_configs_gpu.py \
  tests/test_cp_ring_gpu.py -k "attn or attention or ring or C2" > gpurun_out/r05_k_tests.log 2>&1 || { tail -30 gpurun_out/r05_k_tests.log; exit 1; }
tail -2 gpurun_out/r05_k_tests.log
rm -f gpurun_out/r05_k_ab.jsonl
for r in 1 2 3; do
  for v in "base 0" "kvp_prev 1" "base 1"; do
    set -- $v
    LIB=""; [ "$1" != base ] && LIB=$V/$1.so
    PICO_LIB_PATH=$LIB PICO_ATTN_KVP=$2 timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs c2,gqa4,s4096,c2_full \
      2>> gpurun_out/r05_k_ab.log | sed "s/^{/{\"lib\": \"$1\", \"kvp\": $2, \"round\": $r, /" >> gpurun_out/r05_k_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_k_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["lib"], r["kvp"])].append((r["attn_bwd_q_us"], r["attn_bwd_kv_us"], r["bwd_wall_us"]))
for k, v in sorted(agg.items()):
    print(k, "dQ", [x[0] for x in v], "dKdV", [x[1] for x in v], "wall", [x[2] for x in v])
PY
PICO_LIB_PATH=$V/kvpstamp.so PICO_ATTN_KVP=1 timeout -k 10 120 python -u scripts/kvp_stamps.py > gpurun_out/r05_k_kvpstamps.json 2> gpurun_out/r05_k_stamps.log || { tail -20 gpurun_out/r05_k_stamps.log; exit 1; }
cat gpurun_out/r05_k_kvpstamps.json
