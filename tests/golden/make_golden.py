"""Generate the golden fixtures in tests/golden/ by running the REFERENCE (rkinas/picotron at
/root/reference) on CPU in the build container. The reference never travels to the GPU box; only
the data written here (safetensors / JSON) is committed.

The reference's model module imports three flash-attn entry points at module load
(ref picotron/model.py:7-9). flash-attn is not installed here; with FLASH_ATTEN=0 the reference
never calls them, so they are registered as stubs that raise if called. Everything computed below
is the reference's own eager / data-parallel code.

Usage (build container only):  python tests/golden/make_golden.py
"""
import json
import math
import os
import sys
import types
from types import SimpleNamespace

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from safetensors.torch import save_file

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(OUT))


def _import_reference():
    os.environ["FLASH_ATTEN"] = "0"
    os.environ["DEVICE"] = "cpu"
    os.environ.setdefault("CONTEXT_PARALLEL", "0")
    if REF not in sys.path:
        sys.path.insert(0, REF)

    def _not_available(*a, **k):
        raise NotImplementedError("flash-attn is not installed; the eager path must not call it")

    for name in ["flash_attn", "flash_attn.flash_attn_interface", "flash_attn.layers", "flash_attn.layers.rotary",
                 "flash_attn.ops", "flash_attn.ops.triton", "flash_attn.ops.triton.layer_norm"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["flash_attn.flash_attn_interface"].flash_attn_func = _not_available
    sys.modules["flash_attn.layers.rotary"].apply_rotary_emb = _not_available
    sys.modules["flash_attn.ops.triton.layer_norm"].layer_norm_fn = _not_available
    import picotron.model as M  # noqa
    return M


TINY = dict(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
            num_hidden_layers=2, vocab_size=512, max_position_embeddings=128, rms_norm_eps=1e-5, rope_theta=10000.0)
SMOL15 = dict(hidden_size=2048, intermediate_size=8192, num_attention_heads=32, num_key_value_heads=32,
              num_hidden_layers=15, vocab_size=49152, max_position_embeddings=1024, rms_norm_eps=1e-5,
              rope_theta=10000.0)
TINY_DP = dict(hidden_size=128, intermediate_size=256, num_attention_heads=2, num_key_value_heads=1,
               num_hidden_layers=2, vocab_size=256, max_position_embeddings=64, rms_norm_eps=1e-5, rope_theta=10000.0)
LLAMA2_7B = dict(hidden_size=4096, intermediate_size=11008, num_attention_heads=32, num_key_value_heads=32,
                 num_hidden_layers=32, vocab_size=32000, max_position_embeddings=1024, rms_norm_eps=1e-5,
                 rope_theta=10000.0)


def _init_dist_single(port):
    if not dist.is_initialized():
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=0, world_size=1)


def gen_kernels(M):
    from picotron.context_parallel import context_parallel as CP
    g = torch.Generator().manual_seed(0)
    t = {}
    # (i) RMSNorm — LlamaRMSNorm (ref model.py:66-85)
    x = torch.randn(3, 37, 2048, generator=g).to(torch.bfloat16)
    w = (1.0 + 0.1 * torch.randn(2048, generator=g)).to(torch.bfloat16)
    dy = torch.randn(3, 37, 2048, generator=g)
    norm = M.LlamaRMSNorm(2048, eps=1e-5)
    with torch.no_grad():
        norm.weight.copy_(w.float())
    norm_bf = norm.to(torch.bfloat16)
    with torch.no_grad():
        t["rms.x"], t["rms.w"], t["rms.y_eager_bf16"] = x, w, norm_bf(x)
    norm64 = M.LlamaRMSNorm(2048, eps=1e-5).double()
    with torch.no_grad():
        norm64.weight.copy_(w.double())
    x64 = x.double().requires_grad_(True)
    y64 = norm64(x64)
    y64.backward(dy.double())
    t["rms.dy"], t["rms.y_f64"], t["rms.dx_f64"], t["rms.dw_f64"] = dy, y64.detach(), x64.grad, norm64.weight.grad

    # (ii) RoPE — get_cos_sin (DEVICE=cpu) + apply_rotary_pos_emb (ref model.py:12-30)
    cos, sin = M.get_cos_sin(64, 64, base=10000.0)
    q = torch.randn(2, 4, 64, 64, generator=g).to(torch.bfloat16)  # [B, H, S, D]
    dyr = torch.randn(2, 4, 64, 64, generator=g)
    t["rope.cos"], t["rope.sin"], t["rope.q"] = cos, sin, q
    t["rope.out_eager_bf16"] = M.apply_rotary_pos_emb(q, cos, sin)
    q64 = q.double().requires_grad_(True)
    o64 = M.apply_rotary_pos_emb(q64, cos.double(), sin.double())
    o64.backward(dyr.double())
    t["rope.out_f64"], t["rope.dy"], t["rope.dx_f64"] = o64.detach(), dyr, q64.grad
    cos_l, sin_l = M.get_cos_sin(1024, 64, base=10000.0)  # C2 tables
    t["rope.cos_1024"], t["rope.sin_1024"] = cos_l, sin_l

    # (iii) attention — ring_attention_forward/backward + SDPA (ref context_parallel.py:112-155, model.py:156)
    for causal in (True, False):
        tag = "causal" if causal else "full"
        qa = torch.randn(1, 4, 128, 64, generator=g)
        ka = torch.randn(1, 4, 128, 64, generator=g)
        va = torch.randn(1, 4, 128, 64, generator=g)
        doa = torch.randn(1, 4, 128, 64, generator=g)
        sc = 1.0 / math.sqrt(64)
        O, L = CP.ring_attention_forward(qa, ka, va, sc, causal)
        dq, dk, dv = CP.ring_attention_backward(doa, qa, ka, va, O, L, sc, causal)
        sdpa = torch.nn.functional.scaled_dot_product_attention(qa, ka, va, is_causal=causal)
        for k_, v_ in dict(q=qa, k=ka, v=va, do=doa, o=O, lse=L, dq=dq, dk=dk, dv=dv, sdpa=sdpa).items():
            t[f"attn.{tag}.{k_}"] = v_.contiguous()

    # (iv) update_out_and_lse (ref context_parallel.py:157-187) over 3 blocks
    out, lse = None, None
    for i in range(3):
        bo = torch.randn(1, 4, 32, 64, generator=g)
        bl = torch.randn(1, 4, 32, generator=g) * 3
        t[f"merge.block_out{i}"], t[f"merge.block_lse{i}"] = bo, bl
        out, lse = CP.update_out_and_lse(out, lse, bo, bl)
    t["merge.out"], t["merge.lse"] = out, lse.squeeze(-1)

    # (v) SwiGLU epilogue (ref model.py:185)
    gg = (2 * torch.randn(16, 4096, generator=g)).to(torch.bfloat16)
    uu = torch.randn(16, 4096, generator=g).to(torch.bfloat16)
    dh = torch.randn(16, 4096, generator=g)
    t["swiglu.g"], t["swiglu.u"], t["swiglu.dh"] = gg, uu, dh
    t["swiglu.h_eager_bf16"] = torch.nn.functional.silu(gg) * uu
    g64 = gg.double().requires_grad_(True)
    u64 = uu.double().requires_grad_(True)
    h64 = torch.nn.functional.silu(g64) * u64
    h64.backward(dh.double())
    t["swiglu.h_f64"], t["swiglu.dg_f64"], t["swiglu.du_f64"] = h64.detach(), g64.grad, u64.grad
    save_file({k: v.contiguous() for k, v in t.items()}, os.path.join(OUT, "kernels.safetensors"))
    print("kernels.safetensors:", len(t), "tensors")


def _fake_pgm(tp=1, pp=1, pp_rank=0):
    return SimpleNamespace(tp_world_size=tp, tp_rank=0, pp_world_size=pp, pp_rank=pp_rank,
                           pp_is_first_stage=pp_rank == 0, pp_is_last_stage=pp_rank == pp - 1, cp_world_size=1,
                           cp_rank=0, dp_world_size=1, dp_rank=0, cp_dp_world_size=1, cp_dp_group=None,
                           tp_group=None, pp_group=None)


def gen_bucket_layouts(M):
    import picotron.process_group_manager as pgm
    from picotron.checkpoint import init_model_with_dematerialized_weights
    from picotron.data_parallel.bucket import BucketManager
    from picotron.pipeline_parallel.pipeline_parallel import PipelineParallel
    from picotron.tensor_parallel.tensor_parallel import apply_tensor_parallel
    _init_dist_single(29511)
    layouts = {}

    def run(name, cfg, tp=1, pp=1, pp_rank=0, cap_mb=25):
        pgm.process_group_manager = _fake_pgm(tp, pp, pp_rank)
        c = SimpleNamespace(**cfg)
        with init_model_with_dematerialized_weights():
            model = M.Llama(config=c)
            if tp > 1:
                model = apply_tensor_parallel(model)
            if pp > 1:
                model = PipelineParallel(model, c)
        if pp_rank == pp - 1 or pp == 1:  # ref checkpoint.py:89-90 (on meta: no allocation)
            with torch.device("meta"):
                model.final_proj = torch.nn.Linear(c.hidden_size, c.vocab_size, bias=False)
        names = [n for n, _ in model.named_parameters()]
        params = list(model.parameters())
        bucket_size = cap_mb * 1024 * 1024 // 4
        bm = BucketManager(params, None, bucket_size, torch.float32)
        layouts[name] = {
            "bucket_size": bucket_size,
            "names": names,
            "numels": [p.numel() for p in params],
            "locations": [list(bm.params_to_bucket_location[p]) for p in params],
            "bucket_sizes": [int(x.numel()) for x in bm.grad_data_list],
        }
        print(f"layout {name}: {len(params)} params, {len(bm.buckets)} buckets, "
              f"{sum(layouts[name]['numels'])} elems")
        del bm

    run("smollm_1.7b_15l", SMOL15)
    run("tiny_cap0.05", TINY, cap_mb=0.05)
    run("tiny_cap25", TINY)
    run("llama2_7b_tp2_pp2_stage0", LLAMA2_7B, tp=2, pp=2, pp_rank=0)
    run("llama2_7b_tp2_pp2_stage1", LLAMA2_7B, tp=2, pp=2, pp_rank=1)
    with open(os.path.join(OUT, "bucket_layouts.json"), "w") as f:
        json.dump(layouts, f)
    pgm.process_group_manager = None


def _dp_worker(rank, world, port):
    M = _import_reference()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import picotron.process_group_manager as pgm
    from picotron.data_parallel.data_parallel import DataParallelBucket
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    sys.path.insert(0, REPO)
    from picotron_amd.data import synth_tokens
    torch.manual_seed(42)
    cfg = SimpleNamespace(**TINY_DP)
    model = M.Llama(cfg)
    init_state = {k: v.detach().clone() for k, v in model.state_dict().items()}
    ddp = DataParallelBucket(model, bucket_cap_mb=0.05)
    gen = torch.Generator().manual_seed(7 + rank)
    grad_acc = 3
    losses = []
    for i in range(grad_acc):
        toks = synth_tokens(2, cfg.max_position_embeddings + 1, cfg.vocab_size, gen, "arith")
        ddp.require_backward_grad_sync = i == grad_acc - 1
        logits = ddp(input_ids=toks[:, :-1])
        loss = torch.nn.functional.cross_entropy(logits.reshape(-1, cfg.vocab_size), toks[:, 1:].reshape(-1)) / grad_acc
        loss.backward()
        losses.append(loss.item())
    out = {"main_grad." + n: p.main_grad.clone() for n, p in model.named_parameters()}
    for n, p in model.named_parameters():  # fp32 params: .grad == main_grad.to(fp32) exactly
        assert torch.equal(p.grad, p.main_grad)
    if rank == 0:
        out.update({"init." + k: v for k, v in init_state.items()})
        save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(OUT, "dp_w2_tiny.safetensors"))
        print("dp_w2_tiny.safetensors:", len(out), "tensors", flush=True)
    dist.barrier()
    dist.destroy_process_group()


def gen_dp():
    mp.start_processes(_dp_worker, args=(2, 29522), nprocs=2, join=True, start_method="spawn")


def gen_loss_curve(M, steps=200):
    """Reference non-PP init path + train_step semantics (ref train.py:29-55, :209-240), fp32 CPU."""
    import picotron.process_group_manager as pgm
    from picotron.checkpoint import init_model_with_dematerialized_weights, init_model_with_materialized_weights
    _init_dist_single(29533)
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=1)
    sys.path.insert(0, REPO)
    from picotron_amd.data import synth_tokens
    cfg = SimpleNamespace(**TINY)
    # synthetic safetensors with HF names (values are discarded by the re-init, shapes matter)
    sft_dir = "/tmp/pico_golden_sft"
    os.makedirs(sft_dir, exist_ok=True)
    H, I, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
    D = H // cfg.num_attention_heads
    sd = {"model.embed_tokens.weight": torch.zeros(V, H), "model.norm.weight": torch.zeros(H)}
    for l in range(cfg.num_hidden_layers):
        p = f"model.layers.{l}."
        sd.update({p + "input_layernorm.weight": torch.zeros(H), p + "post_attention_layernorm.weight": torch.zeros(H),
                   p + "mlp.down_proj.weight": torch.zeros(H, I), p + "mlp.gate_proj.weight": torch.zeros(I, H),
                   p + "mlp.up_proj.weight": torch.zeros(I, H),
                   p + "self_attn.q_proj.weight": torch.zeros(H, H),
                   p + "self_attn.k_proj.weight": torch.zeros(cfg.num_key_value_heads * D, H),
                   p + "self_attn.v_proj.weight": torch.zeros(cfg.num_key_value_heads * D, H),
                   p + "self_attn.o_proj.weight": torch.zeros(H, H)})
    save_file(sd, os.path.join(sft_dir, "model.safetensors"))
    # ref train.py:103 seeds before building; nothing else draws from the CPU generator in between here
    torch.manual_seed(42)
    with init_model_with_dematerialized_weights():
        model = M.Llama(config=cfg)
    model = init_model_with_materialized_weights(model, cfg, save_dir=sft_dir)
    model.to(torch.float32)
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    gen = torch.Generator().manual_seed(1234)
    mbs, seq, grad_acc = 4, 128, 2
    batches = [synth_tokens(mbs, seq + 1, V, gen, "arith") for _ in range(16)]

    def train(model, dtype):
        # ref train.py:190 casts the model to the run dtype; the loss is F.cross_entropy on the
        # model's logits (ref train.py:46-49) in that dtype
        model.to(dtype)
        opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
        losses, k = [], 0
        for step in range(steps):
            opt.zero_grad()
            acc = 0.0
            for _ in range(grad_acc):
                toks = batches[k % len(batches)]
                k += 1
                logits = model(input_ids=toks[:, :-1])
                loss = torch.nn.functional.cross_entropy(logits.reshape(-1, V), toks[:, 1:].reshape(-1),
                                                         reduction="mean") / grad_acc
                loss.backward()
                acc += loss.item()
            opt.step()
            losses.append(acc)
        return losses

    losses = train(model, torch.float32)
    # the reference's bf16 dtype policy (its GPU path: bf16 params, bf16 AdamW states), same init
    model.load_state_dict(init)
    losses_bf16 = train(model, torch.bfloat16)
    fp = {k_: {"sum": float(v.double().sum()), "abs_sum": float(v.double().abs().sum()),
               "head": [float(x) for x in v.flatten()[:16]]} for k_, v in init.items()}
    with open(os.path.join(OUT, "tiny_init_fingerprint.json"), "w") as f:
        json.dump(fp, f)
    with open(os.path.join(OUT, "loss_curve_tiny.json"), "w") as f:
        json.dump({"config": TINY, "mbs": mbs, "seq": seq, "grad_acc": grad_acc, "lr": 1e-3, "seed": 42,
                   "data": "arith, torch.Generator seed 1234, 16 cycled micro-batches", "losses": losses,
                   "losses_bf16": losses_bf16}, f)
    print(f"loss curve: step0 {losses[0]:.5f} (ln V = {math.log(V):.5f}) -> step{steps - 1} {losses[-1]:.5f}; "
          f"bf16 {losses_bf16[0]:.5f} -> {losses_bf16[-1]:.5f}")
    pgm.process_group_manager = None


if __name__ == "__main__":
    torch.set_num_threads(8)
    which = sys.argv[1:] or ["kernels", "buckets", "loss", "dp"]
    M = _import_reference()
    if "kernels" in which:
        gen_kernels(M)
    if "buckets" in which:
        gen_bucket_layouts(M)
    if "loss" in which:
        gen_loss_curve(M)
    if dist.is_initialized():
        dist.destroy_process_group()
    if "dp" in which:
        gen_dp()
