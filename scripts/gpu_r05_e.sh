#!/bin/bash
# Round 5, box e: the pipelined dQ tile (PICO_ATTN_QP=1) — numerics; A/B of the four (kvp, qp) combinations;
# PMC passes of the pipelined pair on C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PICO_ATTN_KVP=1 PICO_ATTN_QP=1 timeout -k 10 300 python -u scripts/attn_check.py --cases c2,grp_ragged,grp_10,odd,ragged,gqa4,s4096,full,fold5,fold_ragged \
  > gpurun_out/r05_e_check.jsonl 2> gpurun_out/r05_e_check.log || { cat gpurun_out/r05_e_check.jsonl; tail -20 gpurun_out/r05_e_check.log; exit 1; }
cat gpurun_out/r05_e_check.jsonl
rm -f gpurun_out/r05_e_ab.jsonl
for r in 1 2 3; do
  for v in "0 0" "1 0" "0 1" "1 1"; do
    set -- $v
    PICO_ATTN_KVP=$1 PICO_ATTN_QP=$2 timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs c2,gqa4,s4096 \
      2>> gpurun_out/r05_e_ab.log | sed "s/^{/{\"kvp\": $1, \"qp\": $2, \"round\": $r, /" >> gpurun_out/r05_e_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_e_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["kvp"], r["qp"])].append((r["attn_bwd_q_us"], r["attn_bwd_kv_us"], r["bwd_wall_us"]))
for k, v in sorted(agg.items()):
    print(k, "dQ", [x[0] for x in v], "dKdV", [x[1] for x in v], "wall", [x[2] for x in v])
PY
rm -rf gpurun_out/pmc
PICO_ATTN_KVP=1 PICO_ATTN_QP=1 ATTN_CONFIGS=c2 timeout -k 10 900 bash scripts/pmc_attn.sh || exit $?
python scripts/pmc_summary.py --dir gpurun_out/pmc --match attn_ --json gpurun_out/r05_e_pmc.json > gpurun_out/r05_e_pmc_summary.txt
find gpurun_out/pmc -name "*.csv" -size +1M -delete
grep -E "==|MFMA busy|WAIT_ANY/|WAIT_INST_ANY/|ACTIVE_INST_VALU/|INSTS_VALU |INSTS_MFMA |INSTS_SALU |INSTS_LDS " gpurun_out/r05_e_pmc_summary.txt
