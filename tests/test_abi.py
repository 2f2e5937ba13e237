"""The C-ABI library builds, loads without a GPU, exports every symbol include/picotron_hip.h
declares, and rejects bad arguments with a status + message (no compute calls: CPU only)."""
import ctypes
import os
import re

import pytest
import torch

from conftest import ROOT


@pytest.fixture(scope="module")
def lib():
    from picotron_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from picotron_amd.build import build
        build()
    return _lib.load()


def _declared():
    src = open(os.path.join(ROOT, "include", "picotron_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pico_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol(lib):
    from picotron_amd import _lib
    names = _declared()
    assert len(names) >= 17
    for n in names:
        assert hasattr(lib, n), n
        assert n in _lib.EXPORTED_SYMBOLS, f"{n} has no ctypes signature"
    assert lib.pico_abi_version() == 2  # 2: pico_attn_args gained the RoPE-backward table fields


def test_struct_layout_matches(lib):
    from picotron_amd import _lib
    assert lib.pico_attn_args_size() == ctypes.sizeof(_lib.AttnArgs)


def test_argument_errors_return_status(lib):
    from picotron_amd import _lib
    rc = lib.pico_rmsnorm_fwd(None, None, None, None, None, None, 4, 64, 1e-5, None)
    assert rc == 1000 and b"null" in lib.pico_last_error()
    rc = lib.pico_rmsnorm_fwd(ctypes.c_void_p(16), None, ctypes.c_void_p(16), ctypes.c_void_p(16), None,
                              ctypes.c_void_p(16), 4, 12, 1e-5, None)
    assert rc == 1000 and b"multiple of 8" in lib.pico_last_error()
    a = _lib.AttnArgs()
    a.q = a.k = a.v = ctypes.c_void_p(64)
    a.batch, a.seqlen_q, a.seqlen_k, a.heads_q, a.heads_kv, a.head_dim = 1, 8, 8, 2, 2, 96
    assert lib.pico_attn_fwd(ctypes.byref(a), None) == 1000
    assert b"head_dim" in lib.pico_last_error()
    a.head_dim, a.heads_kv = 64, 3
    assert lib.pico_attn_fwd(ctypes.byref(a), None) == 1000
    a.heads_kv, a.causal, a.seqlen_k = 2, 1, 9
    assert lib.pico_attn_fwd(ctypes.byref(a), None) == 1000
    assert b"causal" in lib.pico_last_error()
    assert lib.pico_grad_accum(None, None, 10, 1.0, None) == 1000
    assert lib.pico_prof_collect(7, ctypes.byref(ctypes.c_double()), ctypes.byref(ctypes.c_int64())) == 1000


def test_workspace_sizes(lib):
    assert lib.pico_rmsnorm_bwd_workspace_bytes(4096, 2048) == 256 * 2048 * 4
    assert lib.pico_rmsnorm_bwd_workspace_bytes(3, 2048) == 1 * 2048 * 4
    from picotron_amd import _lib
    a = _lib.AttnArgs()
    a.batch, a.seqlen_q, a.seqlen_k, a.heads_q, a.heads_kv, a.head_dim = 4, 1024, 1024, 32, 32, 64
    # head_dim 64 (split backward): LSE*log2e + delta, each [B*Hq][Sq padded to 32] fp32 — nothing else
    assert lib.pico_attn_bwd_workspace_bytes(ctypes.byref(a)) == 2 * 4 * 32 * 1024 * 4
    a.seqlen_q = a.seqlen_k = 1000
    pad = ((4 * 32 * 1024 + 63) // 64) * 64
    assert lib.pico_attn_bwd_workspace_bytes(ctypes.byref(a)) == 2 * pad * 4
    # GQA 32/8 at S 1024: 4 key blocks x B 4 x 8 kv heads = 128 workgroups -> tile lists split 2 ways,
    # + fp32 dK/dV partials [2][2][B, S, Hkv, D]
    a.seqlen_q = a.seqlen_k = 1024
    a.heads_kv = 8
    assert lib.pico_attn_bwd_workspace_bytes(ctypes.byref(a)) == 2 * 4 * 32 * 1024 * 4 + 2 * 2 * 4 * 1024 * 8 * 64 * 4
    # O(S) at long sequences (the fused form's dQ slabs grew with S^2): 16K tokens, MHA
    a.heads_kv = 32
    a.batch, a.seqlen_q, a.seqlen_k = 1, 16384, 16384
    assert lib.pico_attn_bwd_workspace_bytes(ctypes.byref(a)) == 2 * 32 * 16384 * 4
    # head_dim 128 runs the split backward too: O(S) LSE / delta, no dQ slabs. C4 per-rank
    # shape: 8 key blocks x B 2 x 16 heads = 256 workgroups (one per CU at D = 128) -> no tile-list split
    a.batch, a.seqlen_q, a.seqlen_k, a.heads_q, a.heads_kv, a.head_dim = 2, 1024, 1024, 16, 16, 128
    assert lib.pico_attn_bwd_workspace_bytes(ctypes.byref(a)) == 2 * 2 * 16 * 1024 * 4
    # GQA 32/8: 128 workgroups -> tile lists split 2 ways, + fp32 dK/dV partials [2][2][B, S, Hkv, D]
    a.heads_q, a.heads_kv = 32, 8
    assert lib.pico_attn_bwd_workspace_bytes(ctypes.byref(a)) == 2 * 2 * 32 * 1024 * 4 + 2 * 2 * 2 * 1024 * 8 * 128 * 4
    # O(S) at long sequences
    a.batch, a.seqlen_q, a.seqlen_k, a.heads_q, a.heads_kv = 1, 16384, 16384, 32, 32
    assert lib.pico_attn_bwd_workspace_bytes(ctypes.byref(a)) == 2 * 32 * 16384 * 4


def test_ops_fail_loudly_without_hip_tensors(lib):
    from picotron_amd import ops
    x = torch.randn(2, 8, 2, 64, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        ops.flash_attn_func(x, x, x, causal=True)
    with pytest.raises(RuntimeError):
        ops.rms_norm(torch.randn(4, 64, dtype=torch.bfloat16), torch.ones(64, dtype=torch.bfloat16))
    with pytest.raises(RuntimeError):
        ops.swiglu(torch.randn(8, dtype=torch.bfloat16), torch.randn(8, dtype=torch.bfloat16))
    with pytest.raises(NotImplementedError):
        ops.flash_attn_func(x, x, x, dropout_p=0.1)
    with pytest.raises(NotImplementedError):
        ops.layer_norm_fn(x, None, None, is_rms_norm=False)


def test_weight_transpose_cache_host_logic(monkeypatch):
    """ops.weight_t's cache: one entry per weight storage, reused across the fresh stacked views each call
    builds. In-place writes through the parameter (version counter), `.data` rebinds (storage key),
    load_state_dict and optimizer steps (step post-hook) make the next use re-transpose by themselves; reading
    `.data` does not (no torch class is patched: VERDICT r03 item 6); a write through a `.data`
    alias is the documented case for invalidate_weight_transposes(). Entries hold their parameters only weakly
    and die with them. (CPU tensors: the transpose falls back to a strided copy; the cache logic is the same.)"""
    import gc
    from picotron_amd import ops
    monkeypatch.setattr(ops, "_WT_CACHE", {})
    monkeypatch.setattr(ops, "_WT_HOOK", [])
    assert not isinstance(torch.nn.Parameter.__dict__.get("data"), property)  # torch itself is left alone
    a = torch.nn.Parameter(torch.randn(8, 16))
    b = torch.nn.Parameter(torch.randn(8, 16))

    def fresh():
        return torch.equal(ops.weight_t(ops.stacked_weight((a, b)), (a, b)), torch.cat([a, b]).t())

    t1 = ops.weight_t(ops.stacked_weight((a, b)), (a, b))
    assert torch.equal(t1, torch.cat([a, b]).t())
    assert ops.weight_t(ops.stacked_weight((a, b)), (a, b)) is t1 and len(ops._WT_CACHE) == 1
    gen, n0 = ops._WT_GEN[0], ops._WT_STATS["transposes"]
    assert ops.weight_t(ops.stacked_weight((a, b)), (a, b)) is t1 and ops._WT_GEN[0] == gen  # no spurious bumps
    # reads of .data (logging, weight norms, EMA, deepcopy) neither bump the generation nor re-transpose
    _ = float(a.data.norm()) + float(b.data.abs().max())
    import copy
    copy.deepcopy(a)
    assert ops._WT_GEN[0] == gen
    assert ops.weight_t(ops.stacked_weight((a, b)), (a, b)) is t1 and ops._WT_STATS["transposes"] == n0
    with torch.no_grad():
        a.data.mul_(2)  # a `.data` alias has its own version counter: the documented explicit invalidation
    ops.invalidate_weight_transposes()
    assert fresh()
    a.data = torch.randn(8, 16)  # rebind: new storage
    assert fresh()
    with torch.no_grad():
        a.add_(1.0)  # version counter
    assert fresh()
    opt = torch.optim.SGD([a, b], lr=0.5)
    a.grad, b.grad = torch.ones_like(a), torch.ones_like(b)
    opt.step()  # step post-hook
    assert fresh()
    m = torch.nn.Linear(16, 8, bias=False)
    tm = ops.weight_t(m.weight.detach(), (m.weight,))
    m.load_state_dict({"weight": torch.randn(8, 16)})
    assert torch.equal(ops.weight_t(m.weight.detach(), (m.weight,)), m.weight.t())
    assert tm is ops.weight_t(m.weight.detach(), (m.weight,))  # same entry, refreshed in place
    ops.invalidate_weight_transposes()  # still available for raw writes by foreign code
    assert fresh()
    del a, b, t1, m, tm, opt
    gc.collect()
    ops._wt_purge()
    assert len(ops._WT_CACHE) == 0


def test_build_tracks_included_sources():
    """A translation unit that #includes another .hip source is rebuilt when that source changes (a stale
    attn_bwd_split_d128.o once sized its dK/dV partial writes for another split count than the workspace)."""
    import os
    from picotron_amd import build as B
    d128 = os.path.join(B.CSRC, "attn_bwd_split_d128.hip")
    deps = B.deps(d128)
    assert os.path.join(B.CSRC, "attn_bwd_split.hip") in deps
    assert os.path.abspath(B.__file__) in deps


def test_flash_atten_0_is_refused(monkeypatch):
    """The reference's FLASH_ATTEN switch (ref picotron/model.py:126,151,191,247): this package has no eager path,
    so FLASH_ATTEN=0 raises a clear error at model construction (where the reference picks its RMSNorm class) and
    in Attention.forward, instead of silently running the kernels."""
    from picotron_amd import model as M
    cfg = M.LlamaConfig(hidden_size=64, intermediate_size=128, num_attention_heads=2, num_key_value_heads=2,
                        num_hidden_layers=1, vocab_size=64, max_position_embeddings=16)
    monkeypatch.delenv("FLASH_ATTEN", raising=False)
    with torch.device("meta"):
        m = M.Llama(cfg)  # default (unset) and "1": the kernel path
    monkeypatch.setenv("FLASH_ATTEN", "1")
    with torch.device("meta"):
        M.Llama(cfg)
    monkeypatch.setenv("FLASH_ATTEN", "0")
    for build in (lambda: M.Llama(cfg), lambda: M.DecoderLayer(cfg, 0)):
        with pytest.raises(RuntimeError, match="FLASH_ATTEN"):
            with torch.device("meta"):
                build()
    x = torch.empty(1, 4, 64, device="meta")
    with pytest.raises(RuntimeError, match="FLASH_ATTEN"):
        m.decoder_layers[0].attention(x, None, None)


def test_train_step_groups_non_syncing_micro_batches():
    """train_step with a grouped graph object (PipelinedMicroBatchGraph's interface): the non-syncing
    micro-batches are handed over together, in loader order and with the DP sync flag off, BEFORE the syncing
    micro-batch runs eagerly with the flag on (host logic; a CPU stand-in model and graph object)."""
    from picotron_amd.data import SyntheticDataLoader
    from picotron_amd.train import train_step

    class Tiny(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.emb = torch.nn.Embedding(64, 8)
            self.out = torch.nn.Linear(8, 64, bias=False)
            self.require_backward_grad_sync = True
            self.log = []

        def forward(self, input_ids):
            self.log.append(("eager", self.require_backward_grad_sync, input_ids[0, 0].item()))
            return self.out(self.emb(input_ids))

    class Grouped:
        grouped = True

        def __init__(self, model):
            self.model = model

        def run(self, batches):
            self.model.log.append(("group", self.model.require_backward_grad_sync,
                                   [b[0][0, 0].item() for b in batches]))

        def take_loss(self):
            return torch.zeros(())

    m = Tiny()
    loader = SyntheticDataLoader(2, 16, 4, 64, seed=3, num_batches=4)
    firsts = [next(loader)["input_ids"][0, 0].item() for _ in range(4)]
    loader = SyntheticDataLoader(2, 16, 4, 64, seed=3, num_batches=4)
    train_step(m, loader, "cpu", graphs=Grouped(m))
    assert m.log == [("group", False, firsts[:3]), ("eager", True, firsts[3])], m.log


def test_train_step_syncing_forward_beside_graph_tail():
    """train_step with a grouped graph object that takes `between` (PipelinedMicroBatchGraph.tail_overlap): the
    non-syncing micro-batches replay with the DP sync flag off, the syncing micro-batch's forward is issued through
    `between` (inside the replay, beside the graph's last backward) with the flag on, and its backward runs after
    the replay returns (host logic; a CPU stand-in model and graph object)."""
    from picotron_amd.data import SyntheticDataLoader
    from picotron_amd.train import train_step

    class Tiny(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.emb = torch.nn.Embedding(64, 8)
            self.out = torch.nn.Linear(8, 64, bias=False)
            self.require_backward_grad_sync = True
            self.log = []
            self.out.weight.register_hook(lambda g: self.log.append(("backward", self.require_backward_grad_sync)))

        def forward(self, input_ids):
            self.log.append(("eager", self.require_backward_grad_sync, input_ids[0, 0].item()))
            return self.out(self.emb(input_ids))

    class Grouped:
        grouped = True
        tail_overlap = True

        def __init__(self, model):
            self.model = model

        def run(self, batches, between=None):
            self.model.log.append(("group", self.model.require_backward_grad_sync,
                                   [b[0][0, 0].item() for b in batches]))
            out = between() if between is not None else None
            self.model.log.append(("tail done",))
            return out

        def take_loss(self):
            return torch.zeros(())

    m = Tiny()
    loader = SyntheticDataLoader(2, 16, 4, 64, seed=3, num_batches=4)
    firsts = [next(loader)["input_ids"][0, 0].item() for _ in range(4)]
    loader = SyntheticDataLoader(2, 16, 4, 64, seed=3, num_batches=4)
    loss = train_step(m, loader, "cpu", graphs=Grouped(m))
    assert m.log == [("group", False, firsts[:3]), ("eager", True, firsts[3]), ("tail done",), ("backward", True)], \
        m.log
    assert loss > 0


def test_wgrad_pair_plan(monkeypatch):
    """wgrad_pair's decisions (host logic, CPU tensors): the first micro-batch of a pair whose operands sit in the
    pair buffers defers, the second runs one GEMM over both halves; no partner (odd grad_acc) or operands elsewhere
    -> its own GEMM; a second half not in place while its first half is pending is copied in; pairing off outside
    an announced micro-batch; a shape change with a first half pending raises."""
    from picotron_amd import wgrad_pair as WP
    monkeypatch.setenv("PICO_WGRAD_GROUP", "2")
    w = torch.nn.Parameter(torch.zeros(6, 4))
    N, K, T = 6, 4, 8

    def operands(i):
        dy = WP.dy_out(w, N, K, T, torch.float32, torch.device("cpu"))
        xt = WP.xt_out(w, N, K, T, torch.float32, torch.device("cpu"))
        dy.copy_(torch.full_like(dy, float(i + 1)))
        xt.copy_(torch.full_like(xt, float(10 * (i + 1))))
        return dy, xt.t()

    WP.begin_step()
    with WP.micro_batch(0, 3):
        dy, x = operands(0)
        assert WP.plan(w, dy, x) == ("skip",)
    with WP.micro_batch(1, 3):
        dy, x = operands(1)
        kind, dyp, xp = WP.plan(w, dy, x)
        assert kind == "gemm" and dyp.shape == (2 * T, N) and xp.shape == (2 * T, K)
        assert torch.equal(dyp[:T], torch.full((T, N), 1.0)) and torch.equal(dyp[T:], torch.full((T, N), 2.0))
        assert torch.equal(xp[:T], torch.full((T, K), 10.0)) and torch.equal(xp[T:], torch.full((T, K), 20.0))
    with WP.micro_batch(2, 3):  # no partner: its own GEMM
        dy, x = operands(2)
        kind, dyp, xp = WP.plan(w, dy, x)
        assert kind == "gemm" and dyp.data_ptr() == dy.data_ptr() and xp.shape == (T, K)
    # a second half whose operands are elsewhere: copied into the pair buffers, one GEMM over both
    WP.begin_step()
    with WP.micro_batch(0, 2):
        dy, x = operands(0)
        assert WP.plan(w, dy, x) == ("skip",)
    with WP.micro_batch(1, 2):
        dy2, x2 = torch.full((T, N), 7.0), torch.full((T, K), 70.0)
        kind, dyp, xp = WP.plan(w, dy2, x2)
        assert kind == "gemm" and torch.equal(dyp[T:], dy2) and torch.equal(xp[T:], x2)
        assert torch.equal(dyp[:T], torch.full((T, N), 1.0))
    # outside an announced micro-batch: no pairing
    assert not WP.active() and WP.xt_out(w, N, K, T, torch.float32, torch.device("cpu")) is None
    dy3, x3 = torch.ones(T, N), torch.ones(T, K)
    assert WP.plan(w, dy3, x3)[1] is dy3
    # a pending first half, then buffers of another shape for the same weight: refused loudly
    WP.begin_step()
    with WP.micro_batch(0, 2):
        dy, x = operands(0)
        assert WP.plan(w, dy, x) == ("skip",)
    with WP.micro_batch(1, 2):
        import pytest
        with pytest.raises(RuntimeError, match="one shape"):
            WP.dy_out(w, N, K, 2 * T, torch.float32, torch.device("cpu"))
    WP.begin_step()


def test_wgrad_group_plan(monkeypatch):
    """Groups of four (PICO_WGRAD_GROUP=4, the default): micro-batches 0-2 of a group defer, the fourth runs one
    GEMM over the four slots (K = 4T, slot order = micro-batch order); a last partial group of r runs over its r
    slots (r = 1: its own GEMM); x^T sets alternate per group; a group left pending when a new one starts raises
    (its deferred weight gradients would be lost)."""
    import pytest
    from picotron_amd import wgrad_pair as WP
    monkeypatch.setenv("PICO_WGRAD_GROUP", "4")
    w = torch.nn.Parameter(torch.zeros(6, 4))
    N, K, T = 6, 4, 8
    cpu = torch.device("cpu")

    def operands(i):
        dy = WP.dy_out(w, N, K, T, torch.float32, cpu)
        xt = WP.xt_out(w, N, K, T, torch.float32, cpu)
        dy.copy_(torch.full_like(dy, float(i + 1)))
        xt.copy_(torch.full_like(xt, float(10 * (i + 1))))
        return dy, xt.t()

    for n, tail in ((5, 1), (6, 2)):
        WP.begin_step()
        for i in range(n):
            with WP.micro_batch(i, n):
                dy, x = operands(i)
                res = WP.plan(w, dy, x)
                if i in (3, n - 1) and not (i == n - 1 and tail == 1):
                    r = 4 if i == 3 else tail
                    assert res[0] == "gemm" and res[1].shape == (r * T, N) and res[2].shape == (r * T, K), (n, i)
                    g0 = i - (r - 1)
                    for j in range(r):
                        assert torch.equal(res[1][j * T:(j + 1) * T], torch.full((T, N), float(g0 + j + 1)))
                        assert torch.equal(res[2][j * T:(j + 1) * T], torch.full((T, K), float(10 * (g0 + j + 1))))
                    assert res[2].stride() == (1, 4 * T)
                elif i == n - 1:  # a group of one: its own operands
                    assert res[0] == "gemm" and res[1].data_ptr() == dy.data_ptr()
                else:
                    assert res == ("skip",), (n, i)
        assert not WP.pending_state()
    b = WP._get(w)
    assert b.xt_slot(0).data_ptr() != b.xt_slot(4).data_ptr()  # groups 0 and 1 in different x^T sets
    assert b.xt_slot(0).data_ptr() == b.xt_slot(8).data_ptr()
    WP.begin_step()
    with WP.micro_batch(0, 8):
        dy, x = operands(0)
        assert WP.plan(w, dy, x) == ("skip",)
    with WP.micro_batch(0, 8), pytest.raises(RuntimeError, match=r"would be\s+lost"):
        dy, x = operands(0)
        WP.plan(w, dy, x)
    WP.begin_step()


def test_train_step_announces_micro_batches():
    """train_step announces each eager micro-batch's index to wgrad_pair (the pairing's only source of truth), and
    none under a per-micro-batch graph object (MicroBatchGraph cannot pair); PICO_WGRAD_PAIR=0 announces nothing."""
    import os
    from picotron_amd import wgrad_pair as WP
    from picotron_amd.data import SyntheticDataLoader
    from picotron_amd.train import train_step

    class Tiny(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.emb = torch.nn.Embedding(64, 8)
            self.out = torch.nn.Linear(8, 64, bias=False)
            self.seen = []

        def forward(self, input_ids):
            self.seen.append((WP._CTX["i"], WP._CTX["n"]))
            return self.out(self.emb(input_ids))

    m = Tiny()
    train_step(m, SyntheticDataLoader(2, 16, 3, 64, seed=3, num_batches=3), "cpu")
    assert m.seen == [(0, 3), (1, 3), (2, 3)], m.seen
    assert WP._CTX["i"] is None

    class PerMB:
        def replay(self, x, y):
            m(input_ids=x)

        def take_loss(self):
            return torch.zeros(())

    m.seen.clear()
    train_step(m, SyntheticDataLoader(2, 16, 2, 64, seed=3, num_batches=2), "cpu", graphs=PerMB())
    assert m.seen == [(None, None), (None, None)], m.seen
    old = os.environ.get("PICO_WGRAD_PAIR")
    os.environ["PICO_WGRAD_PAIR"] = "0"
    try:
        m.seen.clear()
        train_step(m, SyntheticDataLoader(2, 16, 2, 64, seed=3, num_batches=2), "cpu")
        assert m.seen == [(None, None), (None, None)], m.seen
    finally:
        if old is None:
            del os.environ["PICO_WGRAD_PAIR"]
        else:
            os.environ["PICO_WGRAD_PAIR"] = old


def test_kernel_selection_knobs(lib):
    """pico_select (include/picotron_hip.h): every knob starts at its environment value or PICO_SEL_AUTO, is set
    and restored through the ABI (returning the previous value), and an unknown knob is rejected — no launch reads
    the process environment. CPU only: selection touches no device."""
    from picotron_amd import _lib
    for knob in (_lib.SEL_ATTN_KVP, _lib.SEL_KVP_WAVES, _lib.SEL_ATTN_GROUPS, _lib.SEL_ATTN_FWD):
        env = os.environ.get(("PICO_ATTN_KVP", "PICO_KVP_WAVES", "PICO_ATTN_GROUPS", "PICO_ATTN_FWD")[knob])
        start = _lib.select(knob, 1)
        assert start == (int(env) if env else _lib.SEL_AUTO)
        assert _lib.select(knob, 0) == 1
        assert _lib.select(knob, start) == 0
    assert lib.pico_select(99, 0) == -2 and lib.pico_select(-1, 0) == -2
    with pytest.raises(ValueError):
        _lib.select(99, 0)
