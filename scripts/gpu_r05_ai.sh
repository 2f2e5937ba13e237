#!/bin/bash
# Round 5, box ai: per-CU pairing of the dK/dV block groups (PICO_GRP_PAIR: heaviest first-round group with the
# lightest second-round one) — numerics, 3 interleaved rounds of the attention micro-bench, then the step A/B.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r05_ai_*.jsonl
timeout -k 10 300 python -u scripts/attn_check.py --cases c2,grp_ragged,grp_10,odd,ragged,gqa4 \
  > gpurun_out/r05_ai_check.jsonl 2> gpurun_out/r05_ai_check.log || { cat gpurun_out/r05_ai_check.jsonl; tail -20 gpurun_out/r05_ai_check.log; exit 1; }
cat gpurun_out/r05_ai_check.jsonl
for r in 1 2 3; do
  for p in 0 1; do
    PICO_GRP_PAIR=$p timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs c2,gqa4 \
      2>> gpurun_out/r05_ai_ab.log | sed "s/^{/{\"pair\": $p, \"round\": $r, /" >> gpurun_out/r05_ai_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_ai_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["pair"])].append((r["attn_bwd_kv_us"], r["bwd_wall_us"]))
for k, v in sorted(agg.items()):
    print(k, "dKdV", [x[0] for x in v], "wall", [x[1] for x in v])
PY
for r in 1 2 3; do
  for p in 0 1; do
    PICO_GRP_PAIR=$p timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-kernel-timing > gpurun_out/r05_ai_p${p}_$r.json 2> gpurun_out/r05_ai_p${p}_$r.log \
      || { tail -20 gpurun_out/r05_ai_p${p}_$r.log; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r05_ai_p${p}_$r.json')); print(json.dumps({'grp_pair': $p, 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'mfu_pct': d['mfu_pct'], 'loss_last': d['loss_last']}))" >> gpurun_out/r05_ai_step.jsonl
  done
done
cat gpurun_out/r05_ai_step.jsonl
