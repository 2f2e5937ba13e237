#!/bin/bash
# Round 5, box i: register-staged kvp tiles (PICO_KVP_STAGE) vs LDS-DMA — numerics, A/B, stamps; rope variants
# in eager micro-batches (streaming loads, two heads per thread).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=picotron_amd/lib/variants
PICO_LIB_PATH=$V/kvp_stage.so PICO_ATTN_KVP=1 timeout -k 10 300 python -u scripts/attn_check.py --cases c2,grp_ragged,grp_10,odd,ragged,gqa4,s4096,full,fold5,fold_ragged \
  > gpurun_out/r05_i_check.jsonl 2> gpurun_out/r05_i_check.log || { cat gpurun_out/r05_i_check.jsonl; tail -20 gpurun_out/r05_i_check.log; exit 1; }
cat gpurun_out/r05_i_check.jsonl
rm -f gpurun_out/r05_i_ab.jsonl
for r in 1 2 3; do
  for v in "base 0" "base 1" "kvp_stage 1"; do
    set -- $v
    LIB=""; [ "$1" != base ] && LIB=$V/$1.so
    PICO_LIB_PATH=$LIB PICO_ATTN_KVP=$2 timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs c2,gqa4,s4096,c2_full \
      2>> gpurun_out/r05_i_ab.log | sed "s/^{/{\"lib\": \"$1\", \"kvp\": $2, \"round\": $r, /" >> gpurun_out/r05_i_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_i_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["lib"], r["kvp"])].append((r["attn_bwd_q_us"], r["attn_bwd_kv_us"], r["bwd_wall_us"]))
for k, v in sorted(agg.items()):
    print(k, "dQ", [x[0] for x in v], "dKdV", [x[1] for x in v], "wall", [x[2] for x in v])
PY
for v in kvpstamp kvpstamp_stage; do
  PICO_LIB_PATH=$V/$v.so PICO_ATTN_KVP=1 timeout -k 10 120 python -u scripts/kvp_stamps.py > gpurun_out/r05_i_$v.json 2> gpurun_out/r05_i_stamps.log || { tail -20 gpurun_out/r05_i_stamps.log; exit 1; }
  echo $v; cat gpurun_out/r05_i_$v.json
done
rm -f gpurun_out/r05_i_hbm.jsonl
for r in 1 2; do
  for v in "base 1" "rope_nt 1" "base 2"; do
    set -- $v
    LIB=""; [ "$1" != base ] && LIB=$V/$1.so
    PICO_LIB_PATH=$LIB PICO_ROPE_HPT=$2 timeout -k 10 240 python -u scripts/hbm_instep.py --layers 4 --mb 4 | sed "s/^{/{\"hpt\": $2, /" >> gpurun_out/r05_i_hbm.jsonl 2>> gpurun_out/r05_i_hbm.log || { tail -20 gpurun_out/r05_i_hbm.log; exit 1; }
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r05_i_hbm.jsonl"):
    d = json.loads(l)
    print(d["lib"], d["hpt"], {k: v["avg_us"] for k, v in d["kernels"].items()})
PY
