#!/bin/bash
# Round 5, box q: 8 micro-batches per weight-gradient GEMM against 4 (plain and DataParallelBucket, 2 alternating
# rounds), then the RMSNorm backward with 16 waves per workgroup (one row per wave) in eager micro-batches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r05_q_ab.jsonl gpurun_out/r05_q_hbm.jsonl
for r in 1 2; do
  for v in "plain_g4 4" "plain_g8 8" "dp_g4 4 --dp-bucket" "dp_g8 8 --dp-bucket"; do
    set -- $v
    PICO_WGRAD_GROUP=$2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-kernel-timing ${3:-} > gpurun_out/r05_q_$1_$r.json 2> gpurun_out/r05_q_$1_$r.log \
      || { tail -20 gpurun_out/r05_q_$1_$r.log; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r05_q_$1_$r.json')); print(json.dumps({'variant': '$1', 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'mfu_pct': d['mfu_pct'], 'loss_last': d['loss_last']}))" >> gpurun_out/r05_q_ab.jsonl
  done
done
cat gpurun_out/r05_q_ab.jsonl
for r in 1 2 3; do
  for lib in "" picotron_amd/lib/variants/rms_nw16.so; do
    PICO_LIB_PATH=$lib timeout -k 10 200 python -u scripts/hbm_instep.py 2>> gpurun_out/r05_q_hbm.log | sed "s#^{#{\"lib\": \"$lib\", #" >> gpurun_out/r05_q_hbm.jsonl || exit $?
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r05_q_hbm.jsonl"):
    d = json.loads(l)
    print(d["lib"][-16:], {k: (v["avg_us"], v["frac"]) for k, v in d["kernels"].items() if k in ("rmsnorm_bwd", "rope")})
PY
