"""Training step and loop — semantics of the reference train.py (train_step :29-55, loop :219-259),
on the gfx950 hot path. Data is synthetic (no network); the model is built by
picotron_amd.model.build_llama with the reference's init (seed first)."""
import time

import torch
import torch.nn.functional as F

from . import process_group_manager as pgm

# MI355X bf16 dense MFMA peak: 256 CUs x 4096 FLOP/clk x 2.4 GHz (MI355X_MICROARCH.md; the H100
# constant of ref picotron/utils.py:42 is 989.5e12)
MI355X_BF16_PEAK = 256 * 4096 * 2.4e9


def train_step(model, data_loader, device):
    """ref train.py:29-55: grad-accumulation loop, DP sync only on the last micro-batch,
    mean CE / grad_acc_steps, returns the accumulated (python float) loss."""
    acc_loss = 0.0
    m = pgm.process_group_manager
    requires_grad_sync = m is not None and m.cp_dp_world_size > 1
    losses = []
    for i in range(data_loader.grad_acc_steps):
        batch = next(data_loader)
        input_ids = batch["input_ids"].to(device)
        target_ids = batch["target_ids"].to(device)
        if requires_grad_sync:
            model.require_backward_grad_sync = (i == data_loader.grad_acc_steps - 1)
        outputs = model(input_ids=input_ids)
        batch_size, seq_len = input_ids.shape
        outputs = outputs.view(seq_len * batch_size, -1)
        loss = F.cross_entropy(outputs, target_ids.reshape(-1), reduction="mean") / data_loader.grad_acc_steps
        loss.backward()
        losses.append(loss.detach())
    # one host sync per step instead of one per micro-batch (ref :53 calls .item() each time)
    acc_loss = float(torch.stack(losses).float().sum().item()) if losses else 0.0
    return acc_loss


def get_mfu(tokens_per_second_per_gpu, num_params, model_config, theoretical_flops=MI355X_BF16_PEAK):
    """ref picotron/utils.py:42-48 with the MI355X peak: 6N + 12*L*H*S FLOP per token."""
    flops_per_token = (6 * num_params + 12 * model_config.num_hidden_layers * model_config.hidden_size *
                       model_config.max_position_embeddings)
    return tokens_per_second_per_gpu * flops_per_token / theoretical_flops * 100


def get_num_params(model):
    """Parameter count (tp = 1, single pipeline stage; ref picotron/utils.py:50-79)."""
    return sum(p.numel() for p in model.parameters())
