"""m0 discipline of the LDS-DMA kernels, checked on CPU from the gfx950 assembly.

`dma_piece` (csrc/attn_common.h) writes m0 inside inline asm (`s_mov_b32 m0, ...; global_load_lds_dwordx4`) without
declaring it: hipcc rejects m0 in an asm clobber list. The compiler therefore does not know an asm block may have
replaced m0. Its own LDS-DMA instructions read m0 as the LDS destination. This test requires, per BASIC BLOCK,
that every compiler-emitted LDS-DMA (`global_load_lds_*` / `buffer_load_* ... lds` outside an asm block) is
preceded in the same block by a compiler write of m0, with no asm block writing m0 in between. That is stricter
than the hazard: an m0 value set in a dominating block with no asm write on any path would also be safe. Blocks
start at labels and after branches, so a loop back-edge or a join can never carry an asm-written m0 into a
compiler DMA unseen.
"""
import os
import re
import subprocess

import pytest

from picotron_amd import build

SOURCES = ["attn_fwd.hip", "attn_bwd_split.hip", "attn_bwd_split_d128.hip"]
_DMA = re.compile(r"(global_load_lds_|buffer_load_\w+ .*\blds\b)")
_M0_WRITE = re.compile(r"^s_\w+\s+m0\b")
_BRANCH = re.compile(r"^s_(c?branch|setpc|endpgm)")


def _asm(src, out_dir):
    out = os.path.join(out_dir, os.path.basename(src)[:-4] + ".s")
    cmd = [build.HIPCC, *build.CFLAGS, *build.FILE_FLAGS.get(os.path.basename(src), []), "--cuda-device-only", "-S",
           "-o", out, src]
    subprocess.run(cmd, check=True, cwd=os.path.dirname(src), stderr=subprocess.DEVNULL)
    with open(out) as f:
        return f.read()


def check_m0(asm_text):
    """(compiler LDS-DMAs, violations): per basic block, a compiler DMA needs a compiler m0 write before it in the
    block with no asm m0 write after that write."""
    n_dma, bad = 0, []
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n", asm_text, re.M):
        body = asm_text[m.end():asm_text.index(".Lfunc_end", m.end())].split("\n")
        in_asm = False
        m0_ok = False  # the block has set m0 itself since its start / the last asm m0 write
        for line in body:
            t = line.strip()
            if t.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if t.startswith(";;#ASMEND"):
                in_asm = False
                continue
            if not in_asm and (re.match(r"^\.?L\w*:", t) or re.match(r"^\.LBB\w*:", t)):
                m0_ok = False  # a new basic block: m0 may arrive from any predecessor
                continue
            writes_m0 = _M0_WRITE.match(t) is not None
            if in_asm:
                if writes_m0:
                    m0_ok = False
                continue
            if writes_m0:
                m0_ok = True
            if _DMA.search(t):
                n_dma += 1
                if not m0_ok:
                    bad.append((m.group(1)[:60], t))
            if _BRANCH.match(t):
                m0_ok = False
    return n_dma, bad


def test_checker_flags_a_stale_m0():
    """The checker itself: an asm m0 write between the compiler's m0 write and its DMA, and a DMA in a block that
    inherits m0 across a label, are both flagged; an in-block write is accepted."""
    good = "_Zk:\n s_mov_b32 m0, s4\n global_load_lds_dwordx4 v1, s[2:3]\n.Lfunc_end0:\n"
    stale = ("_Zk:\n s_mov_b32 m0, s4\n ;;#ASMSTART\n s_mov_b32 m0, s5\n global_load_lds_dwordx4 v2, s[6:7]\n"
             " ;;#ASMEND\n global_load_lds_dwordx4 v1, s[2:3]\n.Lfunc_end0:\n")
    joined = "_Zk:\n s_mov_b32 m0, s4\n.LBB0_1:\n global_load_lds_dwordx4 v1, s[2:3]\n.Lfunc_end0:\n"
    assert check_m0(good) == (1, [])
    assert len(check_m0(stale)[1]) == 1
    assert len(check_m0(joined)[1]) == 1


@pytest.mark.parametrize("src", SOURCES)
def test_compiler_dma_sets_m0_in_block(src, tmp_path):
    path = os.path.join(build.CSRC, src)
    n_dma, bad = check_m0(_asm(path, str(tmp_path)))
    if src == "attn_fwd.hip":  # its partial-tile path uses the compiler's LDS-DMA builtin: the check is not vacuous
        assert n_dma > 0
    assert not bad, f"{src}: {len(bad)} of {n_dma} compiler LDS-DMAs rely on an m0 set outside their block: {bad[:4]}"
