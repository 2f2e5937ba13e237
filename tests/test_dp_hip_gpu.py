"""DataParallelBucket on the HIP path at world size 2: two gloo
ranks share one GPU and run the product model — fused LM-head CE, fused wgrad accumulation into the fp32
main_grad with 1/W folded into the syncing GEMMs, RMSNorm dw mode 2, embedding backward into main_grad,
the bucket all-reduce and the bf16 cast on the side stream — over grad_acc = 3 micro-batches
(ref picotron/data_parallel/data_parallel.py:62-171, bucket.py:6-57; ref train.py:29-55 micro-batch loop).

  * same data on both ranks: main_grad and .grad must equal, bit for bit, a one-rank run of the same
    micro-batches (the average of two identical sums is the sum: /2 and x/2 + x/2 are exact in fp32);
  * different data per rank: main_grad must equal (within fp32 summation order, rel-L2 2e-6) half the
    gradient sum of a one-rank run over both ranks' micro-batches, and .grad its bf16 cast bit for bit;
  * PICO_WGRAD_FUSION flipped between micro-batches (fused -> plain -> fused): no micro-batch may be
    dropped (the sticky per-param flag of round 1 could drop one).
"""
import math
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

GRAD_ACC = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(seed, n):
    g = torch.Generator().manual_seed(seed)
    toks = torch.randint(0, 512, (n, 2, 65), generator=g)
    return [(t[:, :-1].contiguous(), t[:, 1:].contiguous()) for t in toks]


def _worker(rank, world, port, seeds, toggle, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.model import LlamaConfig, build_llama
    from picotron_amd.train import _micro_batch

    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
                      num_hidden_layers=2, vocab_size=512, max_position_embeddings=64)
    torch.manual_seed(42)
    model = build_llama(cfg, device="cuda:0")
    with torch.no_grad():  # the reference init zeroes the LM head (no gradient below it at step 0)
        g = torch.Generator().manual_seed(7)
        model.final_proj.weight.copy_(torch.randn(model.final_proj.weight.shape, generator=g) * 0.02)
    model = DataParallelBucket(model)
    batches = [b for s in seeds[rank] for b in _batches(s, GRAD_ACC)]
    n = len(batches)
    for i, (x, y) in enumerate(batches):
        if toggle:
            os.environ["PICO_WGRAD_FUSION"] = "0" if i % 3 == 1 else "1"
        model.require_backward_grad_sync = i == n - 1
        _micro_batch(model, x.cuda(), y.cuda(), GRAD_ACC)
    torch.cuda.synchronize()
    res = {name: (p.main_grad.detach().cpu().clone(), p.grad.detach().cpu().clone())
           for name, p in model.module.named_parameters()}
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _run(world, seeds, toggle, tmp_path):
    d = tmp_path / f"w{world}_{'t' if toggle else 'f'}_{abs(hash(str(seeds))) % 1000}"
    d.mkdir()
    mp.start_processes(_worker, args=(world, _free_port(), seeds, toggle, str(d)), nprocs=world, join=True,
                       start_method="spawn")
    return [torch.load(d / f"r{r}.pt", weights_only=True) for r in range(world)]


def test_dp_w2_same_data_bit_exact(tmp_path):
    w2 = _run(2, [[11], [11]], False, tmp_path)
    w1 = _run(1, [[11]], False, tmp_path)[0]
    for r in range(2):
        for name, (mg, g) in w2[r].items():
            assert torch.equal(mg, w1[name][0]), name
            assert torch.equal(g, w1[name][1]), name
    nz = sum(int((mg != 0).any()) for mg, _ in w1.values())
    assert nz == len(w1)  # every parameter got a gradient


def test_dp_w2_rank_data_matches_single_process_sum(tmp_path):
    w2 = _run(2, [[21], [22]], False, tmp_path)
    w1 = _run(1, [[21, 22]], False, tmp_path)[0]  # both ranks' micro-batches in one process: the sum
    for r in range(2):
        for name, (mg, g) in w2[r].items():
            ref = w1[name][0] / 2
            err = float((mg - ref).norm() / ref.norm().clamp_min(1e-30))
            assert err < 2e-6, (name, err)
            assert torch.equal(g, mg.to(torch.bfloat16)), name  # .grad = the bf16 cast of the averaged main_grad
    for name in w2[0]:  # the all-reduce leaves both replicas identical
        assert torch.equal(w2[0][name][0], w2[1][name][0])


def test_dp_w2_fusion_toggled_between_micro_batches(tmp_path):
    fused = _run(2, [[31], [32]], False, tmp_path)
    mixed = _run(2, [[31], [32]], True, tmp_path)
    for name, (mg, _) in fused[0].items():
        err = float((mixed[0][name][0] - mg).norm() / mg.norm().clamp_min(1e-30))
        # the plain path rounds each micro-batch's dW to bf16 before the fp32 accumulate: ~1e-3; a dropped
        # micro-batch would be ~0.3
        assert err < 2e-2, (name, err)


def test_dp_w8_rank_data_matches_single_process_sum(tmp_path):
    """C3 rehearsal at its real world size: eight gloo ranks on one GPU, the product
    model with fused wgrad into main_grad and the 1/8 pre-scale folded into the syncing GEMMs / norm dw /
    embedding backward; main_grad must equal 1/8 of a one-process sum over the eight ranks' micro-batches
    (fp32 summation order only), .grad its bf16 cast bit for bit, and all eight replicas identical."""
    seeds = [[60 + r] for r in range(8)]
    w8 = _run(8, seeds, False, tmp_path)
    w1 = _run(1, [[60 + r for r in range(8)]], False, tmp_path)[0]
    for r in range(8):
        for name, (mg, g) in w8[r].items():
            ref = w1[name][0] / 8
            err = float((mg - ref).norm() / ref.norm().clamp_min(1e-30))
            assert err < 4e-6, (r, name, err)
            assert torch.equal(g, mg.to(torch.bfloat16)), name
    for r in range(1, 8):
        for name in w8[0]:
            assert torch.equal(w8[0][name][0], w8[r][name][0]), (r, name)


def _adam_worker(rank, world, port, defer, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.model import LlamaConfig, build_llama
    from picotron_amd.optim import AdamW
    from picotron_amd.train import _micro_batch

    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
                      num_hidden_layers=2, vocab_size=512, max_position_embeddings=64)
    torch.manual_seed(42)
    model = build_llama(cfg, device="cuda:0")
    with torch.no_grad():
        g = torch.Generator().manual_seed(7)
        model.final_proj.weight.copy_(torch.randn(model.final_proj.weight.shape, generator=g) * 0.02)
    model = DataParallelBucket(model, defer_grad_cast=defer)
    opt = AdamW(model.parameters(), lr=1e-3)
    for step in range(2):
        opt.zero_grad()
        batches = _batches(70 + 10 * step + rank, GRAD_ACC)
        for i, (x, y) in enumerate(batches):
            model.require_backward_grad_sync = i == len(batches) - 1
            _micro_batch(model, x.cuda(), y.cuda(), GRAD_ACC)
        if defer:
            assert all(p._pico_grad_deferred for p in model.module.parameters())
        opt.step()
        model.reset()
    torch.cuda.synchronize()
    res = {name: (p.detach().cpu().clone(), opt.state[p]["exp_avg"].cpu().clone(), opt.state[p]["exp_avg_sq"].cpu().clone())
           for name, p in model.module.named_parameters()}
    if defer:  # materialize_grads() gives the .grad the eager cast would have written
        for i, (x, y) in enumerate(_batches(99 + rank, 1)):
            model.require_backward_grad_sync = True
            _micro_batch(model, x.cuda(), y.cuda(), 1)
        model.materialize_grads()
        torch.cuda.synchronize()
        for p in model.module.parameters():
            assert torch.equal(p.grad, p.main_grad.to(torch.bfloat16))
    torch.save(res, os.path.join(out_dir, f"{'d' if defer else 'c'}{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_adamw_reads_deferred_fp32_grads_bit_exact(tmp_path):
    """DataParallelBucket(defer_grad_cast=True) skips the fp32 -> bf16
    .grad cast (ref picotron/data_parallel/data_parallel.py:165) and pico_adamw_bf16 reads the averaged fp32
    main_grad, rounding in register: two AdamW steps at W = 2 (gloo) leave parameters and both moments bit for
    bit equal to the eager cast + step."""
    for defer in (False, True):
        mp.start_processes(_adam_worker, args=(2, _free_port(), defer, str(tmp_path)), nprocs=2, join=True,
                           start_method="spawn")
    for r in range(2):
        c = torch.load(tmp_path / f"c{r}.pt", weights_only=True)
        d = torch.load(tmp_path / f"d{r}.pt", weights_only=True)
        for name in c:
            for a, b in zip(c[name], d[name]):
                assert torch.equal(a, b), name


# ------------------------------------------------------------------------------------------------------------
# C3 at its workload: SmolLM-1.7B geometry, DP = 8, the bench's own step
# ------------------------------------------------------------------------------------------------------------
C3_GA = 2
C3_LAYERS = 2


def _c3_head(model):
    """A non-zero LM head (the reference init zeroes it, ref picotron/checkpoint.py:88-91, which would leave every
    gradient below the head zero at step 0): the same values in every process."""
    with torch.no_grad():
        g = torch.Generator().manual_seed(7)
        w = model.final_proj.weight
        w.copy_((torch.randn(w.shape, generator=g) * 0.02).to(w.dtype))


def _c3_ref_worker(rank, world, port, out_path):
    """One process, W = 1: the eight ranks' micro-batches (each rank's SyntheticDataLoader stream) accumulated
    eagerly into fp32 main_grad — the sum the all-reduced buckets must equal 8x of."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    import bench
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data import SyntheticDataLoader
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.train import _micro_batch
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=1)
    dev = torch.device("cuda", 0)
    cfg, model, _, _, _ = bench.setup(C3_LAYERS, C3_GA, 1, dev, "pico", True, post_build=_c3_head)
    model = DataParallelBucket(model)
    batches = []
    for r in range(8):
        ld = SyntheticDataLoader(bench.MBS, bench.SEQ, C3_GA, cfg.vocab_size, seed=1234, kind="uniform",
                                 num_batches=C3_GA, device=dev, dp_rank=r)
        batches += [next(ld) for _ in range(C3_GA)]
    from picotron_amd import wgrad_pair as WP
    for i, b in enumerate(batches):
        model.require_backward_grad_sync = i == len(batches) - 1
        # each rank's grad_acc micro-batches announced as its train_step does, so their weight gradients pair the
        # same way (wgrad_pair: one GEMM, one bf16 rounding of a multi-parameter projection's dW per pair)
        with WP.micro_batch(i % C3_GA, C3_GA):
            _micro_batch(model, b["input_ids"], b["target_ids"], C3_GA)
    torch.cuda.synchronize()
    torch.save([g.cpu() for g in model.bucket_manager.grad_data_list], out_path)
    print("[c3 ref] one-process sum over 8 x 2 micro-batches saved", file=sys.stderr, flush=True)
    dist.destroy_process_group()


def _c3_worker(rank, world, port, ref_path, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import hashlib
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.optim import AdamW
    from picotron_amd.train import TrainingStep
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    dev = torch.device("cuda", 0)
    # exactly bench.py --gpus 8's objects and step (DataParallelBucket(defer_grad_cast=True), pico AdamW, graphs)
    cfg, model, opt, loader, _ = bench.setup(C3_LAYERS, C3_GA, world, dev, "pico", True, post_build=_c3_head)
    step = TrainingStep(model, opt, loader, dev, graphs=True)
    res = {"rank": rank, "buckets": len(model.bucket_manager.buckets),
           "bucket_mb": [round(g.numel() * 4 / 2**20, 1) for g in model.bucket_manager.grad_data_list]}
    print(f"[c3 rank {rank}] model built, {res['buckets']} buckets", file=sys.stderr, flush=True)
    step.zero()
    loss = step.micro_batches(sync_loss=True)  # micro-batch 0 from the graph, 1 eager + bucket all-reduces
    print(f"[c3 rank {rank}] micro-batches done, loss {loss:.4f}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    res["loss"] = loss
    res["replayed"] = step.graphs.graph is not None
    # (1) every bucket == 1/8 of the one-process fp32 sum (fp32 summation order only)
    ref = torch.load(ref_path, weights_only=True)
    errs = []
    for g, gr in zip(model.bucket_manager.grad_data_list, ref):
        r = gr.to(dev) / world
        errs.append(float((g - r).double().norm() / r.double().norm().clamp_min(1e-30)))
    res["bucket_rel_err"] = errs
    h = hashlib.sha1()
    for g in model.bucket_manager.grad_data_list:
        h.update(g.cpu().numpy())
    res["sha"] = h.hexdigest()
    params = list(model.module.parameters())
    res["deferred"] = all(getattr(p, "_pico_grad_deferred", False) for p in params)
    # (2) AdamW on the deferred fp32 main_grad == cast-then-step, bit for bit (params and both moments)
    shadow = [torch.nn.Parameter(p.detach().clone()) for p in params]
    for s_, p in zip(shadow, params):
        s_.grad = p.main_grad.to(torch.bfloat16)
    ref_opt = AdamW(shadow, lr=3e-4)
    ref_opt.step()
    step.optimizer_step()
    torch.cuda.synchronize()
    res["adam_equal"] = all(torch.equal(p, s_) and torch.equal(opt.state[p]["exp_avg"], ref_opt.state[s_]["exp_avg"])
                            and torch.equal(opt.state[p]["exp_avg_sq"], ref_opt.state[s_]["exp_avg_sq"])
                            for p, s_ in zip(params, shadow))
    # (3) the deferred cast, when asked for, writes exactly the bf16 .grad of the eager path
    model.materialize_grads()
    res["grad_equal"] = all(torch.equal(p.grad, p.main_grad.to(torch.bfloat16)) for p in params)
    step.reset()
    torch.save(res, os.path.join(out_dir, f"c3_r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_c3_smollm_dp8_bench_step(tmp_path):
    """C3 (SmolLM-1.7B DP = 8, ref picotron/data_parallel/bucket.py:25-31,84-129, data_parallel.py:122-165) at its
    real bucket layout: eight gloo ranks share this GPU (RCCL refuses several ranks on one device) and run
    bench.py's own setup and TrainingStep — SmolLM-1.7B geometry with 2 layers (so the 402 MB embedding and LM-head
    buckets are present), micro-batch 4, seq 1024, grad_acc 2 (one graph replay + the syncing eager micro-batch),
    DataParallelBucket(defer_grad_cast=True) and the pico AdamW. Checks: every bucket equals 1/8 of a one-process
    fp32 sum over the eight ranks' micro-batches (rel-L2 <= 4e-6: summation order only), the eight replicas are
    bit-identical, AdamW on the deferred fp32 main_grad equals cast-then-step bit for bit, and the materialised
    .grad equals the bf16 cast bit for bit."""
    ref_path = str(tmp_path / "c3_ref.pt")
    mp.start_processes(_c3_ref_worker, args=(1, _free_port(), ref_path), nprocs=1, join=True, start_method="spawn")
    world = 8
    mp.start_processes(_c3_worker, args=(world, _free_port(), ref_path, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = [torch.load(tmp_path / f"c3_r{r}.pt", weights_only=True) for r in range(world)]
    r0 = res[0]
    assert r0["buckets"] == 17  # embedding, 2 x (q + 2 norms, k, v, out, up, gate, down), final_proj, final_norm
    assert max(r0["bucket_mb"]) > 380  # the 402 MB embedding / LM-head buckets
    for r in res:
        assert r["replayed"] and r["deferred"], r["rank"]
        assert max(r["bucket_rel_err"]) <= 4e-6, (r["rank"], max(r["bucket_rel_err"]))
        assert r["sha"] == r0["sha"], r["rank"]  # identical replicas
        assert r["adam_equal"] and r["grad_equal"], r["rank"]
        assert math.isfinite(r["loss"])
