"""ORACLE — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference's pipeline parallelism for the
CPU baseline (config C1: dp2 tp2 pp2 1F1B) — nothing here runs on, or is used by, the GPU product:
  * Stage: the layer split of ref picotron/pipeline_parallel/pipeline_parallel.py:8-52 (embedding on the
    first stage, final norm + LM head on the last, contiguous decoder layers per stage);
  * p2p: ref picotron/pipeline_parallel/pp_communications.py (recv/send forward/backward and the
    bidirectional pairs) over gloo;
  * train_step_1f1b: ref pipeline_parallel.py:85-145 — warm-up forwards, one-forward-one-backward steady
    state, cool-down backwards, DP gradient sync on the last backward only.
"""
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


class Stage(nn.Module):
    def __init__(self, model, num_layers, m):
        super().__init__()
        per = [num_layers // m.pp_world_size + (1 if i < num_layers % m.pp_world_size else 0)
               for i in range(m.pp_world_size)]
        start = sum(per[:m.pp_rank])
        self.layers = list(range(start, start + per[m.pp_rank]))
        self.embedding = model.embedding if m.pp_is_first_stage else nn.Identity()
        self.decoder_layers = nn.ModuleDict({str(i): model.decoder_layers[i] for i in self.layers})
        self.final_norm = model.final_norm if m.pp_is_last_stage else nn.Identity()
        self.final_proj = model.final_proj if m.pp_is_last_stage else nn.Identity()

    def forward(self, input_ids, position_ids, hidden_states):
        x = hidden_states if hidden_states is not None else input_ids
        x = self.embedding(x)
        for layer in self.decoder_layers.values():
            x = layer(x)
        return self.final_proj(self.final_norm(x))

    def backward(self, input_tensor, output_tensor, output_tensor_grad):
        if input_tensor is not None:
            input_tensor.retain_grad()
        if output_tensor_grad is None:
            output_tensor_grad = torch.ones_like(output_tensor, memory_format=torch.preserve_format)
        torch.autograd.backward(output_tensor, grad_tensors=output_tensor_grad, retain_graph=False, create_graph=False)
        return input_tensor.grad if input_tensor is not None else None


def p2p(m, operation, tensor=None, shape=None):
    """ref pp_communications.py pipeline_communicate: one-directional stage-to-stage transfer."""
    if operation == "recv_forward":
        if m.pp_is_first_stage:
            return None
        t = torch.empty(shape, requires_grad=True)
        dist.recv(t.data, src=m.pp_prev_rank)
        return t
    if operation == "send_forward":
        if not m.pp_is_last_stage:
            dist.send(tensor.detach().contiguous(), dst=m.pp_next_rank)
        return None
    if operation == "recv_backward":
        if m.pp_is_last_stage:
            return None
        t = torch.empty(shape)
        dist.recv(t, src=m.pp_next_rank)
        return t
    if operation == "send_backward":
        if not m.pp_is_first_stage:
            dist.send(tensor.contiguous(), dst=m.pp_prev_rank)
        return None
    raise ValueError(operation)


def p2p_bidirectional(m, operation, send_tensor, shape):
    """ref pp_communications.py bidirectional_pipeline_communicate: send one way, receive the other."""
    is_fwd = operation == "send_fwd_recv_bwd"
    if (is_fwd and m.pp_is_last_stage) or (not is_fwd and m.pp_is_first_stage):
        return None
    peer = m.pp_next_rank if is_fwd else m.pp_prev_rank
    recv = torch.empty(shape, requires_grad=not is_fwd)
    reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, send_tensor.detach().contiguous(), peer),
                                   dist.P2POp(dist.irecv, recv.data if not is_fwd else recv, peer)])
    for r in reqs:
        r.wait()
    return recv


def train_step_1f1b(model, batches, shape, m):
    """ref pipeline_parallel.py:85-145. `model` is the DP-wrapped Stage; batches: grad_acc (input, target)."""
    n = len(batches)
    warm = min(m.pp_world_size - m.pp_rank - 1, n)
    remaining = n - warm
    logging_loss = 0.0
    ins, outs = [], []
    requires_grad_sync = m.cp_dp_world_size > 1
    it = iter(batches)

    def forward_step(inp):
        nonlocal logging_loss
        ids, tgt = next(it)
        out = model.forward(input_ids=ids, position_ids=None, hidden_states=inp)
        if m.pp_is_last_stage:
            out = F.cross_entropy(out.transpose(1, 2), tgt, reduction="mean")
            logging_loss += out.item() / n
        return out

    for _ in range(warm):
        inp = p2p(m, "recv_forward", shape=shape)
        out = forward_step(inp)
        p2p(m, "send_forward", tensor=out)
        ins.append(inp)
        outs.append(out)
    inp = p2p(m, "recv_forward", shape=shape) if remaining > 0 else None
    if requires_grad_sync:
        model.require_backward_grad_sync = False
    for i in range(remaining):
        is_last = i == remaining - 1
        out = forward_step(inp)
        out_grad = p2p_bidirectional(m, "send_fwd_recv_bwd", out, shape)
        ins.append(inp)
        outs.append(out)
        inp, out = ins.pop(0), outs.pop(0)
        if warm == 0 and is_last and requires_grad_sync:
            model.require_backward_grad_sync = True
        in_grad = model.backward(inp, out, out_grad)
        if is_last:
            inp = None
            p2p(m, "send_backward", tensor=in_grad)
        else:
            inp = p2p_bidirectional(m, "send_bwd_recv_fwd", in_grad, shape)
    for j in range(warm):
        if requires_grad_sync:
            model.require_backward_grad_sync = j == warm - 1
        inp, out = ins.pop(0), outs.pop(0)
        out_grad = p2p(m, "recv_backward", shape=shape)
        in_grad = model.backward(inp, out, out_grad)
        p2p(m, "send_backward", tensor=in_grad)
    return logging_loss
