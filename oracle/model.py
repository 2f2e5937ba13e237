"""ORACLE — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference's eager Llama
(FLASH_ATTEN=0 path, ref picotron/model.py:12-271) plus its train_step (ref train.py:29-55) and
non-PP init path (ref train.py:174-190, picotron/checkpoint.py:50-102).

Used as (a) the checker for loss-curve parity of the gfx950 model and (b) bench.py's cpu_baseline
("port" of the reference CPU/gloo path timed on the GPU box's host cores).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import hotpath


class RMSNorm(nn.Module):
    """LlamaRMSNorm, ref picotron/model.py:66-85."""

    def __init__(self, hidden_size, eps=1e-5):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(hidden_size))
        self.eps = eps

    def reset_parameters(self):
        nn.init.ones_(self.weight)

    def forward(self, x):
        return hotpath.rmsnorm_eager(x, self.weight, self.eps)


def _uniform_init(w):
    bound = math.sqrt(1 / w.size(1))
    torch.nn.init.uniform_(w, -bound, bound)


class Attention(nn.Module):
    """ref picotron/model.py:87-161, eager branch (SDPA + eager rotary). cfg.tp_size (default 1): local
    head counts of a tensor-parallel rank (ref :95-96), once apply_tensor_parallel has sharded q/k/v/out."""

    def __init__(self, cfg):
        super().__init__()
        tp = getattr(cfg, "tp_size", 1)
        self.num_heads = cfg.num_attention_heads
        self.num_kv = cfg.num_key_value_heads
        self.head_dim = cfg.hidden_size // self.num_heads
        self.num_local_heads = self.num_heads // tp
        self.num_local_kv = self.num_kv // tp
        self.q_proj = nn.Linear(cfg.hidden_size, self.num_heads * self.head_dim, bias=False)
        self.k_proj = nn.Linear(cfg.hidden_size, self.num_kv * self.head_dim, bias=False)
        self.v_proj = nn.Linear(cfg.hidden_size, self.num_kv * self.head_dim, bias=False)
        self.out_proj = nn.Linear(cfg.hidden_size, cfg.hidden_size, bias=False)

    def reset_parameters(self):
        for w in (self.q_proj.weight, self.k_proj.weight, self.v_proj.weight, self.out_proj.weight):
            _uniform_init(w)

    def forward(self, x, cos, sin):
        B, S, _ = x.shape
        D = self.head_dim
        q = self.q_proj(x).view(B, S, self.num_local_heads, D).transpose(1, 2)
        k = self.k_proj(x).view(B, S, self.num_local_kv, D).transpose(1, 2)
        v = self.v_proj(x).view(B, S, self.num_local_kv, D).transpose(1, 2)
        q = hotpath.rope_eager(q, cos, sin)
        k = hotpath.rope_eager(k, cos, sin)
        g = self.num_local_heads // self.num_local_kv
        k = k.repeat_interleave(g, dim=1)
        v = v.repeat_interleave(g, dim=1)
        out = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        return self.out_proj(out.transpose(1, 2).reshape(B, S, self.num_local_heads * D))


class MLP(nn.Module):
    """ref picotron/model.py:163-185."""

    def __init__(self, cfg):
        super().__init__()
        self.up_proj = nn.Linear(cfg.hidden_size, cfg.intermediate_size, bias=False)
        self.gate_proj = nn.Linear(cfg.hidden_size, cfg.intermediate_size, bias=False)
        self.down_proj = nn.Linear(cfg.intermediate_size, cfg.hidden_size, bias=False)

    def reset_parameters(self):
        for w in (self.up_proj.weight, self.gate_proj.weight, self.down_proj.weight):
            _uniform_init(w)

    def forward(self, x):
        return self.down_proj(F.silu(self.gate_proj(x)) * self.up_proj(x))


class DecoderLayer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.attention = Attention(cfg)
        self.mlp = MLP(cfg)
        D = cfg.hidden_size // cfg.num_attention_heads
        self.cos, self.sin = hotpath.get_cos_sin(cfg.max_position_embeddings, D, cfg.rope_theta)

    def forward(self, x):
        S = x.size(1)
        cos, sin = self.cos[:S].to(x.dtype), self.sin[:S].to(x.dtype)
        x = x + self.attention(self.input_layernorm(x), cos, sin)
        return x + self.mlp(self.post_attention_layernorm(x))


class Embedding(nn.Module):
    def __init__(self, n, d):
        super().__init__()
        self.num_embeddings, self.embedding_dim = n, d
        self.weight = nn.Parameter(torch.empty(n, d))

    def reset_parameters(self):
        torch.nn.init.normal_(self.weight, mean=0.0, std=1.0)

    def forward(self, x):
        return F.embedding(x, self.weight)


class Llama(nn.Module):
    """Parameter order as ref picotron/model.py:244-248."""

    def __init__(self, cfg):
        super().__init__()
        self.embedding = Embedding(cfg.vocab_size, cfg.hidden_size)
        self.decoder_layers = nn.ModuleList([DecoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        self.final_proj = nn.Linear(cfg.hidden_size, cfg.vocab_size, bias=False)
        self.final_norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)

    def reset_parameters(self):
        """ref :252-262 — note final_proj is NOT re-initialised (missing call at :262)."""
        self.embedding.reset_parameters()
        for layer in self.decoder_layers:
            layer.input_layernorm.reset_parameters()
            layer.attention.reset_parameters()
            layer.post_attention_layernorm.reset_parameters()
            layer.mlp.reset_parameters()
        self.final_norm.reset_parameters()

    def forward(self, input_ids):
        x = self.embedding(input_ids)
        for layer in self.decoder_layers:
            x = layer(x)
        return self.final_proj(self.final_norm(x))


def build(cfg, dtype=torch.float32):
    """Reference non-PP init: modules on meta (no RNG), fp32 CPU params, a fresh CPU nn.Linear LM
    head zero-filled (ref checkpoint.py:88-91), reset_parameters() from the CPU generator (ref :100)."""
    with torch.device("meta"):
        m = Llama(cfg)
    m.to_empty(device="cpu")
    for layer in m.decoder_layers:  # tables are not parameters: rebuild them on CPU
        D = cfg.hidden_size // cfg.num_attention_heads
        layer.cos, layer.sin = hotpath.get_cos_sin(cfg.max_position_embeddings, D, cfg.rope_theta)
    with torch.no_grad():
        for p in m.parameters():
            p.zero_()
    # ref checkpoint.py:90 builds a fresh nn.Linear for the LM head on CPU (its kaiming init draws
    # from the CPU generator before reset_parameters), then loads zeros into it (:91)
    m.final_proj = nn.Linear(cfg.hidden_size, cfg.vocab_size, bias=False)
    with torch.no_grad():
        m.final_proj.weight.zero_()
    m.reset_parameters()
    return m.to(dtype)


def train_step(model, batches, grad_acc_steps):
    """ref train.py:29-55 (non-PP, single process): mean CE / grad_acc per micro-batch."""
    acc = 0.0
    for input_ids, target_ids in batches:
        logits = model(input_ids)
        B, S = input_ids.shape
        loss = F.cross_entropy(logits.view(B * S, -1), target_ids.reshape(-1), reduction="mean") / grad_acc_steps
        loss.backward()
        acc += loss.item()
    return acc
