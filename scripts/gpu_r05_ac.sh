#!/bin/bash
# Round 5, box ac: TunableOp on the round-5 step's own GEMM signatures (grouped wgrads at K = 4T, the grouped LM
# head): tune once inside a bench run, then the step with the tuned selections vs hipBLASLt's heuristic, 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r05_ac_ab.jsonl gpurun_out/r05_ac_tunableop.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/r05_ac_tunableop.csv \
  timeout -k 10 900 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > gpurun_out/r05_ac_tune.json 2> gpurun_out/r05_ac_tune.log \
  || { tail -20 gpurun_out/r05_ac_tune.log; exit 1; }
ls -la gpurun_out/ | grep tunable
for r in 1 2 3; do
  for t in 0 1; do
    PYTORCH_TUNABLEOP_ENABLED=$t PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/r05_ac_tunableop.csv \
      timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-kernel-timing > gpurun_out/r05_ac_t${t}_$r.json 2> gpurun_out/r05_ac_t${t}_$r.log \
      || { tail -20 gpurun_out/r05_ac_t${t}_$r.log; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r05_ac_t${t}_$r.json')); print(json.dumps({'tunableop': $t, 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'mfu_pct': d['mfu_pct'], 'loss_last': d['loss_last']}))" >> gpurun_out/r05_ac_ab.jsonl
  done
done
cat gpurun_out/r05_ac_ab.jsonl
