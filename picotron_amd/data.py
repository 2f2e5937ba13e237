"""Synthetic micro-batch loader with the interface of the reference's MicroBatchDataLoader
(ref picotron/data.py:12-137): `micro_batch_size`, `seq_length`, `grad_acc_steps`,
`global_batch_size`, `seq_length_per_gpu`, and `next(loader)` -> dict(input_ids, target_ids,
position_ids, hidden_states) with the same context-parallel slicing as its collate_batch (:102-116).

There is no network here (no HF datasets/tokenizers), so sequences of length S+1 are synthesised
deterministically per (seed, dp_rank, step):
  * "uniform": token ids ~ U[0, vocab) (throughput benchmarks);
  * "arith":   tok[t] = (start + stride * t) mod vocab with random start/stride per row — a learnable
               stream for loss-curve overlays.
"""
import os

import torch

from . import process_group_manager as pgm


def synth_tokens(n_rows, seq_plus_one, vocab, generator, kind="uniform"):
    if kind == "uniform":
        return torch.randint(0, vocab, (n_rows, seq_plus_one), generator=generator, dtype=torch.long)
    if kind == "arith":
        start = torch.randint(0, vocab, (n_rows, 1), generator=generator, dtype=torch.long)
        stride = torch.randint(1, 17, (n_rows, 1), generator=generator, dtype=torch.long)
        t = torch.arange(seq_plus_one, dtype=torch.long).unsqueeze(0)
        return (start + stride * t) % vocab
    raise ValueError(f"unknown synthetic data kind {kind!r}")


class SyntheticDataLoader:
    def __init__(self, micro_batch_size, seq_length, grad_acc_steps, vocab_size, seed=1234, kind="uniform",
                 num_batches=None, device="cpu", dp_rank=None):
        """dp_rank: the data-parallel rank whose stream to produce (default: this process's, from the process
        group manager) — a one-process check can replay every rank's micro-batches."""
        m = pgm.process_group_manager
        self.dp_world_size = m.dp_world_size if m is not None else 1
        self.dp_rank = dp_rank if dp_rank is not None else (m.dp_rank if m is not None else 0)
        self.cp_world_size = m.cp_world_size if m is not None else 1
        self.cp_rank = m.cp_rank if m is not None else 0
        self.micro_batch_size = micro_batch_size
        self.seq_length = seq_length
        self.grad_acc_steps = grad_acc_steps
        self.global_batch_size = micro_batch_size * grad_acc_steps * self.dp_world_size
        assert seq_length % self.cp_world_size == 0
        self.seq_length_per_gpu = seq_length // self.cp_world_size
        self.vocab_size = vocab_size
        self.kind = kind
        self.num_batches = num_batches  # cycle over this many distinct micro-batches (None = endless fresh)
        self.device = device
        self.seed = seed
        self._gen = torch.Generator().manual_seed(seed + self.dp_rank)
        self._cache = []
        self._i = 0

    def _make(self):
        return synth_tokens(self.micro_batch_size, self.seq_length + 1, self.vocab_size, self._gen, self.kind)

    def collate(self, tokens):
        """CP slicing of ref picotron/data.py:102-116 (zig-zag chunks with PICO_CP_ZIGZAG=1)."""
        if self.cp_world_size > 1 and os.getenv("PICO_CP_ZIGZAG", "0") == "1":
            from .context_parallel.context_parallel import zigzag_positions
            pos = zigzag_positions(self.seq_length, self.cp_rank, self.cp_world_size)
            B = tokens.size(0)
            return {
                "input_ids": tokens[:, pos].contiguous(),
                "target_ids": tokens[:, pos + 1].contiguous(),
                "position_ids": pos.unsqueeze(0).expand(B, -1).contiguous(),
                "hidden_states": None,
            }
        start = self.cp_rank * self.seq_length_per_gpu
        end = start + self.seq_length_per_gpu
        B = tokens.size(0)
        return {
            "input_ids": tokens[:, start:end].contiguous(),
            "target_ids": tokens[:, start + 1:end + 1].contiguous(),
            "position_ids": torch.arange(start, end, dtype=torch.long).unsqueeze(0).expand(B, -1).contiguous(),
            "hidden_states": None,
        }

    def __iter__(self):
        return self

    def _device_batch(self, toks):
        batch = self.collate(toks)
        if self.device != "cpu":
            for k in ("input_ids", "target_ids", "position_ids"):
                batch[k] = batch[k].to(self.device, non_blocking=True)
        return batch

    def __next__(self):
        self._i += 1
        if self.num_batches is None:
            return self._device_batch(self._make())
        # a fixed cycle of micro-batches: generated once and kept resident on the device
        if len(self._cache) < self.num_batches:
            self._cache.append(self._device_batch(self._make()))
        return dict(self._cache[(self._i - 1) % self.num_batches])
