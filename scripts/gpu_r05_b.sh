#!/bin/bash
# Round 5, box b: one-round block groups in the attention backward (PICO_ATTN_GROUPS) — numerics, the attention
# GPU tests, then a same-box A/B of the attention micro-bench (groups off / on, 3 interleaved rounds); the
# AccumulateGrad stream probe; the loss-overlay curves (PICO_LOSS_OUT).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/attn_check.py --cases c2,grp_ragged,grp_10,odd,ragged,gqa4,s4096,full,d128,d128_b2,d128_ragged,d128_full \
  > gpurun_out/r05_b_check.jsonl 2> gpurun_out/r05_b_check.log || { tail -20 gpurun_out/r05_b_check.log; exit 1; }
cat gpurun_out/r05_b_check.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_configs_gpu.py \
  tests/test_cp_ring_gpu.py -k "attn or attention or ring or C4 or C2" > gpurun_out/r05_b_tests.log 2>&1 || { tail -30 gpurun_out/r05_b_tests.log; exit 1; }
tail -2 gpurun_out/r05_b_tests.log
rm -f gpurun_out/r05_b_ab.jsonl
for r in 1 2 3; do
  for g in 0 1; do
    PICO_ATTN_GROUPS=$g timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs c2,gqa4,d128,d128_b2,s4096 \
      2>> gpurun_out/r05_b_ab.log | sed "s/^{/{\"groups\": $g, \"round\": $r, /" >> gpurun_out/r05_b_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_b_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["groups"])].append((r["attn_bwd_q_us"], r["attn_bwd_kv_us"], r["bwd_wall_us"]))
for (c, g), v in sorted(agg.items()):
    print(c, "groups", g, "dQ", [x[0] for x in v], "dKdV", [x[1] for x in v], "wall", [x[2] for x in v])
PY
timeout -k 10 300 python -u scripts/dbg_accgrad_stream.py > gpurun_out/r05_b_accgrad.log 2>&1 || { tail -20 gpurun_out/r05_b_accgrad.log; exit 1; }
tail -20 gpurun_out/r05_b_accgrad.log
PICO_LOSS_OUT=gpurun_out/r05_loss.json timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread \
  "tests/test_model_gpu.py::test_loss_curve_shipped_path_overlays_reference" > gpurun_out/r05_b_overlay.log 2>&1
grep loss-overlay gpurun_out/r05_b_overlay.log
exit 0
