// head_dim 128 instantiation of the split flash-attention backward (attn_bwd_split.hip): the same dQ and
// dK / dV kernels, compiled in their own translation unit without -amdgpu-mfma-vgpr-form, so their
// accumulators may use the AGPR half of the register file (dQ 248 VGPRs at two workgroups per CU; dK / dV
// ≈ 370 registers per lane at one workgroup of 4 waves per CU, its M2 operands read ahead). Serves the Llama-2-7B per-rank shapes of
// config C4 (ref picotron/model.py:36 at head_dim 128).
#define PICO_SPLIT_D128_TU 1
#include "attn_bwd_split.hip"
