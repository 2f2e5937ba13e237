#!/bin/bash
# D = 128 dK/dV with 16 keys per wave (PICO_KV16=1) against the shipped 32-key kernel: numerics (attn_check d128
# cases, the attention GPU tests) with the variant on, then interleaved attn_bench rounds of both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/kv16d128_ab.jsonl
PICO_KV16=1 timeout -k 10 300 python -u scripts/attn_check.py --cases d128,d128_ragged,d128_full,d128_s4096 \
  > gpurun_out/kv16d128_check.jsonl 2> gpurun_out/kv16d128_check.log || { cat gpurun_out/kv16d128_check.jsonl; tail -20 gpurun_out/kv16d128_check.log; exit 1; }
cat gpurun_out/kv16d128_check.jsonl
PICO_KV16=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_configs_gpu.py -k "attention or attn or C4" > gpurun_out/kv16d128_tests.log 2>&1 \
  || { tail -30 gpurun_out/kv16d128_tests.log; exit 1; }
tail -2 gpurun_out/kv16d128_tests.log
for r in 1 2 3; do
  for v in 0 1; do
    PICO_KV16=$v timeout -k 10 240 python -u scripts/attn_bench.py --iters 50 --configs ${KV16_CONFIGS:-d128,d128_s4096} \
      2>> gpurun_out/kv16d128_ab.log | sed "s/^{/{\"kv16\": $v, \"round\": $r, /" >> gpurun_out/kv16d128_ab.jsonl
    rc=${PIPESTATUS[0]}
    if [ "$rc" -ne 0 ]; then echo "attn_bench kv16=$v failed rc=$rc"; tail -20 gpurun_out/kv16d128_ab.log; exit $rc; fi
  done
done
python - <<'EOF'
import json
for l in open("gpurun_out/kv16d128_ab.jsonl"):
    d = json.loads(l)
    print(d["kv16"], d["round"], d["config"], "kv", d["attn_bwd_kv_us"], "q", d["attn_bwd_q_us"], "wall", d["bwd_wall_us"])
EOF
