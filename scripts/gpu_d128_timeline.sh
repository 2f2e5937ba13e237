#!/bin/bash
# C4 (D = 128) attention backward: workgroup timelines of the dK/dV and dQ kernels (stamp variants), then the
# A/B of library variants (VARIANTS, numerics first).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PICO_TL_SHAPE=${PICO_TL_SHAPE:-2,1024,16,128} QFRONT=${QFRONT:-0}
PICO_LIB_PATH=picotron_amd/lib/variants/wgkv.so timeout -k 10 120 python scripts/bwd_kv_wgstamps.py > gpurun_out/wgkv_c4.json 2> gpurun_out/wgkv_c4.log || exit $?
PICO_LIB_PATH=picotron_amd/lib/variants/wgq.so timeout -k 10 120 python scripts/bwd_q_wgstamps.py > gpurun_out/wgq_c4.json 2> gpurun_out/wgq_c4.log || exit $?
VARIANTS="${VARIANTS:-base pipe}" CHECK_CASES=${CHECK_CASES:-d128,d128_ragged,d128_full,d128_s4096} ROUNDS=${ROUNDS:-2} ATTN_CONFIGS=${ATTN_CONFIGS:-d128,d128_full,d128_s4096,d128_gqa4} bash scripts/gpu_ab_attn.sh
