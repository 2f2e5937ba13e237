#!/bin/bash
# Round 5, box ak: rocBLAS instead of hipBLASLt for the step's GEMMs (TORCH_BLAS_PREFER_HIPBLASLT=0), 3 alternating rounds.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r05_ak_ab.jsonl
for r in 1 2 3; do
  for v in 1 0; do
    TORCH_BLAS_PREFER_HIPBLASLT=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-kernel-timing > gpurun_out/r05_ak_v${v}_$r.json 2> gpurun_out/r05_ak_v${v}_$r.log \
      || { tail -20 gpurun_out/r05_ak_v${v}_$r.log; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r05_ak_v${v}_$r.json')); print(json.dumps({'prefer_hipblaslt': $v, 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'mfu_pct': d['mfu_pct'], 'loss_last': d['loss_last']}))" >> gpurun_out/r05_ak_ab.jsonl
  done
done
cat gpurun_out/r05_ak_ab.jsonl
