"""Llama model whose hot path runs on the gfx950 kernels — same module API as the reference
picotron/model.py (class names, constructor arguments, attribute names, parameter registration
order and reset_parameters semantics), so tensor/pipeline/context-parallel wrappers that replace
submodules by attribute name, and the DP bucket layout (which follows parameter order), see the
same model.

Hot-path mapping (reference -> here):
  TritonRMSNorm / LlamaRMSNorm (ref :38-85)       -> RMSNorm on pico_rmsnorm_fwd/_bwd
  apply_rotary_emb (ref :135-136)                 -> ops.apply_rotary_emb on pico_rope
  flash_attn_func / SDPA (ref :153-156)           -> ops.flash_attn_func on pico_attn_fwd/_bwd (native
                                                      GQA: no repeat_interleave copies, ref :141-142)
  ring_attention (ref :147-150)                   -> context_parallel.ring_attention on the same kernels
  F.silu(gate) * up (ref :185)                    -> ops.swiglu on pico_swiglu_fwd/_bwd
There is no eager/CPU fallback: modules raise if the HIP library or a HIP device is missing.
The GEMMs (q/k/v/out/up/gate/down/final projections) stay torch (hipBLASLt).
"""
import math
import os
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from . import wgrad_pair as WP
from . import process_group_manager as pgm


@dataclass
class LlamaConfig:
    """Geometry of a Llama model (the fields picotron reads from HF AutoConfig, ref train.py:152-165)."""
    hidden_size: int = 2048
    intermediate_size: int = 8192
    num_attention_heads: int = 32
    num_key_value_heads: int = 32
    num_hidden_layers: int = 24
    vocab_size: int = 49152
    max_position_embeddings: int = 2048
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0


def smollm_1_7b(num_hidden_layers=24, seq_length=2048):
    """HuggingFaceTB/SmolLM-1.7B geometry (restated; checkpoints are not available offline)."""
    return LlamaConfig(hidden_size=2048, intermediate_size=8192, num_attention_heads=32, num_key_value_heads=32,
                       num_hidden_layers=num_hidden_layers, vocab_size=49152, max_position_embeddings=seq_length,
                       rms_norm_eps=1e-5, rope_theta=10000.0)


def llama2_7b(num_hidden_layers=32, seq_length=4096):
    """meta-llama/Llama-2-7b-hf geometry (restated)."""
    return LlamaConfig(hidden_size=4096, intermediate_size=11008, num_attention_heads=32, num_key_value_heads=32,
                       num_hidden_layers=num_hidden_layers, vocab_size=32000, max_position_embeddings=seq_length,
                       rms_norm_eps=1e-5, rope_theta=10000.0)


def require_kernel_path():
    """The reference's FLASH_ATTEN switch (ref picotron/model.py:126,151,191,247; set from the config's
    environment block, ref train.py:67): "1" (its default) runs the fused kernels, anything else the eager
    LlamaRMSNorm / apply_rotary_pos_emb / SDPA path. This package is the kernel path only — there is no eager
    path by design (north_star: no dual dispatch) — so FLASH_ATTEN != "1" is refused here instead of silently
    running the gfx950 kernels. Checked where the reference reads it: at module construction (:191, :247) and
    in Attention.forward (:126, :151)."""
    v = os.getenv("FLASH_ATTEN", "1")
    if v != "1":
        raise RuntimeError(f"FLASH_ATTEN={v!r}: picotron_amd runs the gfx950 kernel path only (the reference's eager "
                           "FLASH_ATTEN=0 path is not provided); unset FLASH_ATTEN or set it to 1")


def _table_device():
    if os.getenv("DEVICE", "cuda") == "cuda" and torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def get_cos_sin(seq_length, head_dim, base=500000.0):
    """RoPE tables [seq_length, head_dim] (freqs repeated twice), ref picotron/model.py:21-30:
    theta on CPU in fp32, position * theta and cos/sin on DEVICE, cast to DTYPE (bf16 default)."""
    assert head_dim % 2 == 0
    theta = 1.0 / (base ** (torch.arange(0, head_dim, 2, dtype=torch.int64, device="cpu").float() / head_dim))
    dtype = torch.bfloat16 if os.getenv("DTYPE", "bfloat16") == "bfloat16" else torch.float32
    device = _table_device()
    position = torch.arange(seq_length, device="cpu").to(device).unsqueeze(1).float()
    theta = theta.to(device)
    ang = position.float() * theta.float()
    return torch.cos(ang).to(dtype).repeat(1, 2), torch.sin(ang).to(dtype).repeat(1, 2)


def apply_rotary_pos_emb(x, cos, sin):
    """Rotate-half RoPE on x [B, H, S, D] with tables [S, D] (ref picotron/model.py:12-19), on the kernel."""
    S, D = x.shape[2], x.shape[3]
    out = ops.apply_rotary_emb(x.transpose(1, 2), cos[:S, : D // 2], sin[:S, : D // 2])
    return out.transpose(1, 2)


def flash_attention(q, k, v, causal=True):
    """q, k, v [B, H, S, D] -> [B, S, H, D] (ref picotron/model.py:32-36)."""
    return ops.flash_attn_func(q.permute(0, 2, 1, 3), k.permute(0, 2, 1, 3), v.permute(0, 2, 1, 3), causal=causal)


def _col_parallel(mods):
    """'tp' if every module is a bias-free ColumnParallelLinear shard the fused ops can take (its f region
    — the input-gradient all-reduce — applied once by the caller), 'plain' if every one is a bias-free
    nn.Linear, else None."""
    from .tensor_parallel.tensor_parallel import ColumnParallelLinear
    if all(type(m) is nn.Linear and m.bias is None for m in mods):
        return "plain"
    if all(type(m) is ColumnParallelLinear and m.bias is None and not m.gather_output and not m.async_all_reduce
           for m in mods):
        return "tp"
    return None


def _tp_input(kind, x):
    if kind == "tp" and pgm.process_group_manager is not None and pgm.process_group_manager.tp_world_size > 1:
        from .tensor_parallel.tp_communications import CopyToModelParallelRegion
        return CopyToModelParallelRegion.apply(x)
    return x


def _proj(mod, x):
    """A projection: bias-free nn.Linear runs ops.linear (gradient-accumulation fusion); anything
    else (TP-parallel layers, biases) runs as is."""
    if type(mod) is nn.Linear and mod.bias is None and os.getenv("PICO_UNFUSED", "0") != "1":
        return ops.linear(x, mod.weight)
    return mod(x)


class RMSNorm(nn.Module):
    """Fused RMSNorm (ref TritonRMSNorm, picotron/model.py:38-64): same constructor, weight init
    (ones) and forward signature; `residual`/`prenorm` fuse the residual add into the kernel."""

    def __init__(self, hidden_size, eps=1e-5, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.variance_epsilon = eps  # LlamaRMSNorm attribute name (ref :73)
        self.weight = nn.Parameter(torch.empty(hidden_size, device=device, dtype=dtype))
        self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.ones_(self.weight)

    def forward(self, hidden_states, residual=None, dropout_p=0.0, prenorm=False, residual_in_fp32=False,
                return_dropout_mask=False, _pair=None):
        # the norm outputs of this model feed projections (qkv, gate|up, LM head) whose weight-gradient
        # GEMM reads y^T: the kernel writes it alongside y (ops._wgrad_input picks it up). _pair: paired
        # weight-gradient hints (wgrad_pair; DecoderLayer._pair_hints)
        return ops.layer_norm_fn(hidden_states, self.weight, None, residual=residual, eps=self.eps,
                                 dropout_p=dropout_p, prenorm=prenorm, residual_in_fp32=residual_in_fp32,
                                 is_rms_norm=True, return_dropout_mask=return_dropout_mask, _emit_transposed=True,
                                 _pair=_pair)


TritonRMSNorm = RMSNorm
LlamaRMSNorm = RMSNorm


class Attention(nn.Module):
    """ref picotron/model.py:87-161. q/k/v/out projections keep their names so TP can replace them."""

    def __init__(self, config, layer_idx):
        super().__init__()
        tp = pgm.tp_world_size()
        self.hidden_size = config.hidden_size
        self.num_heads = config.num_attention_heads
        self.num_key_values = config.num_key_value_heads
        self.head_dim = self.hidden_size // self.num_heads
        assert config.num_attention_heads % tp == 0, "num_attention_heads should be divisible by tp world size"
        assert config.num_key_value_heads % tp == 0, "num_key_value_heads should be divisible by tp world size"
        self.num_local_heads = config.num_attention_heads // tp
        self.num_local_kv_heads = config.num_key_value_heads // tp
        self.q_proj = nn.Linear(config.hidden_size, self.num_heads * self.head_dim, bias=False)
        self.k_proj = nn.Linear(config.hidden_size, self.num_key_values * self.head_dim, bias=False)
        self.v_proj = nn.Linear(config.hidden_size, self.num_key_values * self.head_dim, bias=False)
        self.out_proj = nn.Linear(config.hidden_size, config.hidden_size, bias=False)
        self.layer_idx = layer_idx
        self.reset_parameters()

    def reset_parameters(self):
        for w in (self.q_proj.weight, self.k_proj.weight, self.v_proj.weight, self.out_proj.weight):
            bound = math.sqrt(1 / w.size(1))
            torch.nn.init.uniform_(w, -bound, bound)

    def _fusable(self):
        if os.getenv("CONTEXT_PARALLEL", "0") == "1" or os.getenv("PICO_UNFUSED", "0") == "1":
            return None
        return _col_parallel((self.q_proj, self.k_proj, self.v_proj))

    def forward(self, x, cos, sin, attention_mask=None, position_ids=None, out_hint=None):
        require_kernel_path()
        B, S, _ = x.size()
        D = self.head_dim
        kind = self._fusable()
        if kind is not None:
            # one q|k|v GEMM, RoPE in place on q|k, attention on strided views (ops._QKVRopeAttentionFn);
            # under TP the local shards, with one f region (input-gradient all-reduce) for all three
            x = _tp_input(kind, x)
            out = ops.qkv_rope_attention(x, self.q_proj.weight, self.k_proj.weight, self.v_proj.weight, cos, sin,
                                         self.num_local_heads, self.num_local_kv_heads, True, out_hint=out_hint)
            return _proj(self.out_proj, out)
        q = self.q_proj(x).view(B, S, self.num_local_heads, D)
        k = self.k_proj(x).view(B, S, self.num_local_kv_heads, D)
        v = self.v_proj(x).view(B, S, self.num_local_kv_heads, D)
        q = ops.apply_rotary_emb(q, cos[:, : D // 2], sin[:, : D // 2])
        k = ops.apply_rotary_emb(k, cos[:, : D // 2], sin[:, : D // 2])
        causal = q.size(1) == k.size(1)
        if os.getenv("CONTEXT_PARALLEL", "0") == "1":
            # the reference's call: [B, H, S, D] in, [B, H, S, D] out, transposed back (ref :139-150)
            from .context_parallel import context_parallel
            out = context_parallel.ring_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                                  1.0 / math.sqrt(D), causal).transpose(1, 2)
        else:
            out = ops.flash_attn_func(q, k, v, causal=causal)
        out = out.reshape(B, S, self.num_local_heads * D)
        return self.out_proj(out)


class MLP(nn.Module):
    """ref picotron/model.py:163-185."""

    def __init__(self, config) -> None:
        super().__init__()
        self.up_proj = nn.Linear(config.hidden_size, config.intermediate_size, bias=False)
        self.gate_proj = nn.Linear(config.hidden_size, config.intermediate_size, bias=False)
        self.down_proj = nn.Linear(config.intermediate_size, config.hidden_size, bias=False)
        self.reset_parameters()

    def reset_parameters(self):
        for w in (self.up_proj.weight, self.gate_proj.weight, self.down_proj.weight):
            bound = math.sqrt(1 / w.size(1))
            torch.nn.init.uniform_(w, -bound, bound)

    def forward(self, x, down_hint=None):
        kind = _col_parallel((self.gate_proj, self.up_proj)) if os.getenv("PICO_UNFUSED", "0") != "1" else None
        if kind is not None:
            # one gate|up GEMM + strided SwiGLU (ops._GateUpSwiGLUFn); under TP on the local shards, one f region
            x = _tp_input(kind, x)
            return _proj(self.down_proj, ops.gate_up_swiglu(x, self.gate_proj.weight, self.up_proj.weight,
                                                            down_hint=down_hint))
        return self.down_proj(ops.swiglu(self.gate_proj(x), self.up_proj(x)))


class DecoderLayer(nn.Module):
    """RMSNorm -> Attention -> Residual -> RMSNorm -> MLP -> Residual (ref picotron/model.py:187-208)."""

    def __init__(self, config, layer_idx):
        super().__init__()
        require_kernel_path()  # ref :191 picks the RMSNorm class from FLASH_ATTEN here
        self.input_layernorm = RMSNorm(config.hidden_size, eps=config.rms_norm_eps)
        self.post_attention_layernorm = RMSNorm(config.hidden_size, eps=config.rms_norm_eps)
        self.attention = Attention(config, layer_idx=layer_idx)
        self.mlp = MLP(config)
        self.layer_idx = layer_idx
        self._rope_geometry = (config.max_position_embeddings, config.hidden_size // config.num_attention_heads,
                               config.rope_theta)
        self.refresh_rope()

    def refresh_rope(self):
        """(Re)build this layer's cos/sin tables for the current context-parallel layout (ref
        picotron/model.py:198-201): the cp rank's contiguous slice, or its two zig-zag chunks. Built at
        construction like the reference; apply_context_parallel calls it again when it switches the layout
        of an already built model (the reference's order: model first, then CP, ref train.py:175-188)."""
        seq, head_dim, base = self._rope_geometry
        cos, sin = get_cos_sin(seq, head_dim=head_dim, base=base)
        from .context_parallel.context_parallel import update_rope_for_context_parallel
        self.cos, self.sin = update_rope_for_context_parallel(cos, sin)

    def forward(self, x, attention_mask=None, position_ids=None):
        cos, sin = self.cos, self.sin
        x = x + self.attention(self.input_layernorm(x), cos, sin, attention_mask, position_ids)
        x = x + self.mlp(self.post_attention_layernorm(x))
        return x

    def _pair_hints(self):
        """Paired weight-gradient hints (wgrad_pair) of this layer's four projections, (weight, N, K) each — the
        weight keys its pair buffers — or None when the pairing is off or a projection is not a plain bias-free
        nn.Linear on the fused paths (TP / CP layers, PICO_UNFUSED)."""
        if not WP.active() or os.getenv("PICO_UNFUSED", "0") == "1" or os.getenv("CONTEXT_PARALLEL", "0") == "1":
            return None
        a, m = self.attention, self.mlp
        lins = (a.q_proj, a.k_proj, a.v_proj, a.out_proj, m.gate_proj, m.up_proj, m.down_proj)
        if any(type(t) is not nn.Linear or t.bias is not None for t in lins) or pgm.tp_world_size() > 1:
            return None
        hd, inter = a.out_proj.weight.shape[0], m.down_proj.weight.shape[1]
        nqkv = a.q_proj.weight.shape[0] + a.k_proj.weight.shape[0] + a.v_proj.weight.shape[0]
        return {"qkv": (a.q_proj.weight, nqkv, a.q_proj.weight.shape[1]),
                "out": (a.out_proj.weight, hd, a.out_proj.weight.shape[1]),
                "gu": (m.gate_proj.weight, 2 * m.gate_proj.weight.shape[0], m.gate_proj.weight.shape[1]),
                "down": (m.down_proj.weight, hd, inter)}

    def forward_fused(self, delta, residual, prev_down=None):
        """Same layer with the residual adds fused into the norms (layer_norm_fn prenorm form):
        the layer input is residual + delta (residual None for the first layer). Returns the
        (delta, residual) pair whose sum is this layer's output; every sum is rounded to bf16 exactly
        like the reference's `x + f(x)`. prev_down: the previous layer's down-projection pair hint (delta is its
        output, so the input norm's dx is that projection's dy)."""
        hints = self._pair_hints()
        p_in = (hints["qkv"], prev_down) if hints else None
        p_post = (hints["gu"], hints["out"]) if hints else None
        if residual is None:  # prenorm form without a residual: x is the norm's second output, so the
            # embedding output has one consumer and its gradient needs no separate add
            h_in, x = self.input_layernorm(delta, residual=None, prenorm=True, _pair=p_in)
        else:
            h_in, x = self.input_layernorm(delta, residual=residual, prenorm=True, _pair=p_in)
        attn = self.attention(h_in, self.cos, self.sin, out_hint=hints["out"] if hints else None)
        h2, x = self.post_attention_layernorm(attn, residual=x, prenorm=True, _pair=p_post)
        return self.mlp(h2, down_hint=hints["down"] if hints else None), x


class Embedding(nn.Module):
    """ref picotron/model.py:210-224."""

    def __init__(self, num_embeddings, embedding_dim, padding_idx=None):
        super().__init__()
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self.padding_idx = padding_idx
        self.weight = nn.Parameter(torch.empty(num_embeddings, embedding_dim))
        self.reset_parameters()

    def reset_parameters(self):
        torch.nn.init.normal_(self.weight, mean=0.0, std=1.0)

    def forward(self, x):
        if self.padding_idx is None and x.is_cuda:
            return ops.embedding(x, self.weight)  # deterministic, graph-safe backward
        return F.embedding(x, self.weight, self.padding_idx)


class Llama(nn.Module):
    """ref picotron/model.py:226-271 (parameter order: embedding, layers (input_ln, post_attn_ln,
    q, k, v, out, up, gate, down), final_proj, final_norm)."""

    def __init__(self, config) -> None:
        super().__init__()
        require_kernel_path()  # ref :247
        assert config.hidden_size % config.num_attention_heads == 0
        assert config.num_attention_heads % config.num_key_value_heads == 0
        self.vocab_size = config.vocab_size
        self.hidden_size = config.hidden_size
        self.num_heads = config.num_attention_heads
        self.num_key_values = config.num_key_value_heads
        self.head_dim = self.hidden_size // self.num_heads
        self.max_position_embeddings = config.max_position_embeddings
        self.num_layers = config.num_hidden_layers
        self.model_config = config
        self.embedding = Embedding(self.vocab_size, self.hidden_size)
        self.decoder_layers = nn.ModuleList([DecoderLayer(config, layer_idx=i) for i in range(self.num_layers)])
        self.final_proj = nn.Linear(self.hidden_size, self.vocab_size, bias=False)
        self.final_norm = RMSNorm(self.hidden_size, eps=config.rms_norm_eps)
        self.reset_parameters()

    def reset_parameters(self):
        self.embedding.reset_parameters()
        for layer in self.decoder_layers:
            layer.input_layernorm.reset_parameters()
            layer.attention.reset_parameters()
            layer.post_attention_layernorm.reset_parameters()
            layer.mlp.reset_parameters()
        self.final_norm.reset_parameters()
        # NB: the reference never re-initialises final_proj here (ref :262 lacks the call); it is
        # zero-initialised by init_model_with_materialized_weights (ref picotron/checkpoint.py:88-91).

    def forward(self, input_ids, attention_mask=None, position_ids: torch.Tensor = None, return_hidden=False):
        """Logits [B, S, V] (ref :264-271); return_hidden=True stops after the final norm (the fused LM
        head + cross-entropy of train._micro_batch consumes it)."""
        x = self.embedding(input_ids)
        if os.getenv("PICO_UNFUSED", "0") == "1":
            for layer in self.decoder_layers:
                x = layer(x)
            return self.final_proj(self.final_norm(x))
        delta, residual = x, None
        down = None  # the previous layer's down-projection pair hint (wgrad_pair)
        for b, layer in enumerate(self.decoder_layers):
            delta, residual = layer.forward_fused(delta, residual, prev_down=down)
            hints = layer._pair_hints()
            down = hints["down"] if hints else None
        # the fused LM head + CE (return_hidden) groups its weight gradient too: the final norm's y^T goes into the
        # head's x^T group slot (wgrad_pair)
        head = getattr(self, "final_proj", None)
        lm = (head.weight, head.weight.shape[0], head.weight.shape[1]) if (
            return_hidden and down is not None and type(head) is nn.Linear and head.bias is None) else None
        pair = (lm, down) if down is not None else None
        h = self.final_norm(delta, _pair=pair) if residual is None else \
            self.final_norm(delta, residual=residual, _pair=pair)
        if return_hidden:
            return h
        return _proj(self.final_proj, h)


def build_llama(config, device="cuda", dtype=torch.bfloat16):
    """Materialise a Llama exactly as the reference's non-PP init path does
    (ref train.py:174-190, picotron/checkpoint.py:50-102): modules built without consuming RNG, params
    materialised in fp32 on CPU, a fresh CPU nn.Linear LM head (kaiming draw) zero-filled, then
    `reset_parameters()` draws from the CPU generator in module order (so set the seed first), then
    cast to `dtype` and move to `device`."""
    with torch.device("meta"):
        model = Llama(config)
    model.to_empty(device="cpu")
    for p in model.parameters():
        p.data = p.data.float()
    # ref checkpoint.py:90: a fresh CPU nn.Linear for the LM head (its kaiming init draws from the
    # CPU generator before reset_parameters), loaded with zeros (:91); registration order unchanged
    model.final_proj = nn.Linear(config.hidden_size, config.vocab_size, bias=False)
    with torch.no_grad():
        model.final_proj.weight.zero_()
    model.reset_parameters()
    return model.to(dtype).to(device)
