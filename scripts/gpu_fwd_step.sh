#!/bin/bash
# Forward in the training step's form (rope_q fused, O^T written) vs the plain forward, for the 128-row kernel
# and the D = 64 ping-pong kernel (PICO_ATTN_FWD64), interleaved rounds; plus the attn_bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in 0 1; do
    PICO_ATTN_FWD64=$v timeout -k 10 120 python scripts/rope_q_fwd_bench.py | sed "s/^{/{\"round\": $r, /" >> gpurun_out/fwd_step.jsonl || exit $?
    PICO_ATTN_FWD64=$v timeout -k 10 300 python scripts/attn_bench.py --configs c2,c2_full | sed "s/^{/{\"fwd64\": $v, \"round\": $r, /" >> gpurun_out/fwd64_bench.jsonl || exit $?
  done
done
echo "== fwd_step done"
