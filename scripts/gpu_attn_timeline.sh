#!/bin/bash
# Attention timelines on the box: micro-bench of the shipped kernels, then the workgroup-stamp variants
# (built beforehand with scripts/build_variants.py: wgkv / wgq / wgfwd).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 180 python scripts/attn_bench.py --configs ${ATTN_CONFIGS:-c2,d128} > gpurun_out/attn_base.jsonl 2> gpurun_out/attn_base.log || exit $?
for v in wgkv:bwd_kv_wgstamps wgq:bwd_q_wgstamps wgfwd:fwd_wgstamps; do
  lib=${v%%:*}; scr=${v##*:}
  if [ -f picotron_amd/lib/variants/$lib.so ]; then
    PICO_LIB_PATH=picotron_amd/lib/variants/$lib.so timeout -k 10 120 python scripts/$scr.py > gpurun_out/$lib.json 2> gpurun_out/$lib.log || exit $?
  fi
done
echo "== timeline done"
