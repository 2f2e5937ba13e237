#!/bin/bash
# Round 5, box ah: the forward's rescale threshold (PICO_FWD_RESCALE_THR, log2 units: 8 shipped vs 12 / 16) —
# numerics of each variant, then 3 interleaved rounds of the attention micro-bench.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r05_ah_check.jsonl gpurun_out/r05_ah_ab.jsonl
for v in thr12 thr16; do
  PICO_LIB_PATH=picotron_amd/lib/variants/$v.so timeout -k 10 300 python -u scripts/attn_check.py --cases c2,odd,ragged,gqa4,full \
    >> gpurun_out/r05_ah_check.jsonl 2>> gpurun_out/r05_ah_check.log || { tail -20 gpurun_out/r05_ah_check.log; exit 1; }
done
cat gpurun_out/r05_ah_check.jsonl
for r in 1 2 3; do
  for v in base thr12 thr16; do
    lib=""; [ "$v" != base ] && lib=picotron_amd/lib/variants/$v.so
    PICO_LIB_PATH=$lib timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs c2,c2_full,gqa4,d128 \
      2>> gpurun_out/r05_ah_ab.log | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> gpurun_out/r05_ah_ab.jsonl || exit $?
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05_ah_ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["config"], r["variant"])].append(r["attn_fwd_us"])
for k, v in sorted(agg.items()):
    print(k, "fwd", v)
PY
