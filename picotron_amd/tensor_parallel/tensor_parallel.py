"""Tensor parallelism (API of ref picotron/tensor_parallel/tensor_parallel.py:9-270): apply_tensor_parallel
replaces the decoder layers' projections by attribute name with column / row parallel layers and the
embedding / LM head with vocab-parallel ones, exactly as the reference does; the layers keep the
reference's constructor arguments, parameter shapes and initialisation (a master weight drawn whole,
then this rank's split).

MI355X-native differences (same numbers):
  * the GEMMs are picotron_amd.ops (hipBLASLt; weight-gradient accumulation fused into the GEMM epilogue,
    dgrad against a cached W^T), the collectives RCCL over xGMI (tp_communications);
  * picotron_amd.model keeps its fused paths under TP: with column-parallel q/k/v (gate/up) the layer runs
    ONE f region (all-reduce of the input gradient) around the fused q|k|v + RoPE + attention (gate|up +
    SwiGLU) op on the local shards, instead of one per projection — one collective instead of three
    (two) per layer backward, the same sum;
  * apply_tensor_parallel(model, shard_weights=True) converts an already initialised model in place
    (each new layer takes its rank's shard of the existing weight) — the reference re-initialises.
"""
import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .. import process_group_manager as pgm
from .tp_communications import (GatherFromModelParallelRegion, ReduceFromModelParallelRegion, linear_with_all_reduce,
                                linear_with_async_all_reduce)


def apply_tensor_parallel(model, shard_weights=False):
    """ref :9-51. shard_weights: take each rank's shard of the existing weights instead of re-initialising."""
    m = pgm.process_group_manager

    def _replace_module(_module, _linear_proj_name, _style, args={}):
        assert _style in ["column", "row", "vocab"]
        old = getattr(_module, _linear_proj_name)
        dev, dt = old.weight.device, old.weight.dtype
        if _style == "column":
            new = ColumnParallelLinear(in_features=old.in_features, out_features=old.out_features,
                                       bias=old.bias is not None, gather_output=args.get("gather_output", False))
        elif _style == "row":
            new = RowParallelLinear(in_features=old.in_features, out_features=old.out_features, bias=old.bias is not None)
        else:
            new = VocabParallelEmbedding(num_embeddings=old.num_embeddings, embedding_dim=old.embedding_dim)
        new = new.to(device=dev, dtype=dt) if dev.type != "meta" else new
        if shard_weights:
            with torch.no_grad():
                w = old.weight
                if _style == "row":
                    n = new.input_size_per_partition
                    new.weight.copy_(w[:, m.tp_rank * n:(m.tp_rank + 1) * n])
                    if old.bias is not None:
                        new.bias.copy_(old.bias)
                else:
                    n = new.weight.shape[0]
                    new.weight.copy_(w[m.tp_rank * n:(m.tp_rank + 1) * n])
                    if getattr(old, "bias", None) is not None:
                        new.bias.copy_(old.bias[m.tp_rank * n:(m.tp_rank + 1) * n])
        setattr(_module, _linear_proj_name, new)

    mapping = [
        ("attention", "q_proj", "column"),
        ("attention", "k_proj", "column"),
        ("attention", "v_proj", "column"),
        ("attention", "out_proj", "row"),
        ("mlp", "up_proj", "column"),
        ("mlp", "gate_proj", "column"),
        ("mlp", "down_proj", "row"),
    ]
    for layer in model.decoder_layers:
        for module_name, proj, style in mapping:
            _replace_module(getattr(layer, module_name), proj, style)
    _replace_module(model, "embedding", "vocab")
    _replace_module(model, "final_proj", "column", args={"gather_output": True})
    return model


class ColumnParallelLinear(nn.Module):
    """Y_i = X W_i^T (+ b_i), W split along its output rows (ref :53-129)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = False, gather_output: bool = False,
                 async_all_reduce: bool = False) -> None:
        super().__init__()
        self.tp_world_size = pgm.process_group_manager.tp_world_size
        self.tp_rank = pgm.process_group_manager.tp_rank
        self.in_features = in_features
        self.out_features = out_features
        assert out_features % self.tp_world_size == 0, "Hidden dimension must be divisible by the tensor parallel world size"
        self.output_size_per_partition = out_features // self.tp_world_size
        self.gather_output = gather_output
        self.async_all_reduce = async_all_reduce
        self.weight = nn.Parameter(torch.empty(self.output_size_per_partition, self.in_features))
        if bias:
            self.bias = nn.Parameter(torch.zeros(self.output_size_per_partition))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        """ref :104-120: nn.Linear's default bound on the whole master weight, then this rank's rows."""
        if self.weight.device.type == "meta":
            return
        master = torch.empty(self.out_features, self.in_features, dtype=self.weight.dtype, device=self.weight.device)
        bound = math.sqrt(1 / master.size(1))
        torch.nn.init.uniform_(master, -bound, bound)
        self.weight.data = torch.split(master, self.output_size_per_partition, dim=0)[self.tp_rank].contiguous()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.async_all_reduce:
            output = linear_with_async_all_reduce(x, self.weight, self.bias)
        else:
            output = linear_with_all_reduce(x, self.weight, self.bias)
        if self.gather_output:
            output = GatherFromModelParallelRegion.apply(output)
        return output


class RowParallelLinear(nn.Module):
    """Y = sum_i X_i W_i^T (+ b), W split along its input columns, X already split (ref :131-188)."""

    def __init__(self, in_features: int, out_features: int, bias: bool):
        super().__init__()
        self.tp_world_size = pgm.process_group_manager.tp_world_size
        self.tp_rank = pgm.process_group_manager.tp_rank
        self.in_features = in_features
        self.out_features = out_features
        assert in_features % self.tp_world_size == 0, "Hidden dimension must be divisible by the tensor parallel world size"
        self.input_size_per_partition = in_features // self.tp_world_size
        self.weight = nn.Parameter(torch.empty(self.out_features, self.input_size_per_partition))
        if bias:
            self.bias = nn.Parameter(torch.zeros(self.out_features))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        """ref :164-180."""
        if self.weight.device.type == "meta":
            return
        master = torch.empty(self.out_features, self.in_features, dtype=self.weight.dtype, device=self.weight.device)
        bound = math.sqrt(1 / master.size(1))
        torch.nn.init.uniform_(master, -bound, bound)
        self.weight.data = torch.split(master, self.input_size_per_partition, dim=1)[self.tp_rank].contiguous()

    def forward(self, x):
        out = ops.linear(x, self.weight) if x.is_cuda else F.linear(x, self.weight)
        out = ReduceFromModelParallelRegion.apply(out)
        return out if self.bias is None else out + self.bias


class VocabParallelEmbedding(nn.Module):
    """Embedding with the vocabulary split over the tp ranks (ref :190-270): masked local lookup,
    zero rows for ids outside this rank's range, all-reduce."""

    def __init__(self, num_embeddings: int, embedding_dim: int, padding_idx: Optional[int] = None,
                 max_norm: Optional[float] = None, norm_type: float = 2.0, scale_grad_by_freq: bool = False,
                 sparse: bool = False):
        super().__init__()
        self.tp_world_size = pgm.process_group_manager.tp_world_size
        self.tp_rank = pgm.process_group_manager.tp_rank
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self.padding_idx = padding_idx
        self.max_norm = max_norm
        self.norm_type = norm_type
        self.scale_grad_by_freq = scale_grad_by_freq
        self.sparse = sparse
        self.vocab_start_index, self.vocab_end_index = self._vocab_range_from_global_vocab_size(
            num_embeddings, self.tp_rank, self.tp_world_size)
        self.num_embeddings_per_partition = self.vocab_end_index - self.vocab_start_index
        self.weight = nn.Parameter(torch.empty(self.num_embeddings_per_partition, self.embedding_dim))
        self.reset_parameters()

    def _vocab_range_from_global_vocab_size(self, global_vocab_size: int, rank: int, world_size: int):
        assert global_vocab_size % world_size == 0, f"{global_vocab_size} is not divisible by {world_size}"
        per = global_vocab_size // world_size
        return rank * per, rank * per + per

    def reset_parameters(self):
        """ref :236-247."""
        if self.weight.device.type == "meta":
            return
        master = torch.empty(self.num_embeddings, self.embedding_dim, dtype=self.weight.dtype, device=self.weight.device)
        torch.nn.init.normal_(master, mean=0.0, std=1.0)
        self.weight.data = torch.split(master, self.num_embeddings_per_partition, dim=0)[self.tp_rank].contiguous()

    def forward(self, x):
        input_mask = (x < self.vocab_start_index) | (x >= self.vocab_end_index)
        masked_input = x.clone() - self.vocab_start_index
        masked_input[input_mask] = 0
        plain = (self.padding_idx is None and self.max_norm is None and not self.scale_grad_by_freq
                 and not self.sparse and x.is_cuda)
        if plain:
            output_parallel = ops.embedding(masked_input, self.weight)
        else:
            output_parallel = F.embedding(masked_input, self.weight, self.padding_idx, self.max_norm, self.norm_type,
                                          self.scale_grad_by_freq, self.sparse)
        output_parallel = output_parallel.masked_fill(input_mask.unsqueeze(-1), 0.0)
        return ReduceFromModelParallelRegion.apply(output_parallel)
