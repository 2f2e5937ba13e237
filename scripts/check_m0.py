"""dma_piece's inline asm writes m0 (`s_mov_b32 m0, ...`) without declaring it (hipcc rejects m0 in an
asm clobber list: "reserved register ... may not be preserved"). This checks, in the gfx950 assembly of every
kernel source that uses it, that each compiler-emitted LDS-DMA (`global_load_lds_*` / `buffer_load_* ... lds`
outside an inline-asm block) has its own m0 write after the last inline-asm block that wrote m0 — i.e. the
compiler never relies on an m0 value an asm block may have replaced. Exit status 1 on a violation.

  python scripts/check_m0.py [picotron_amd/csrc/attn_fwd.hip ...]
"""
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import build  # noqa: E402

DEFAULT = ["attn_fwd.hip", "attn_bwd_split.hip", "attn_bwd_split_d128.hip"]


def asm(src):
    out = "/tmp/check_m0.s"
    cmd = [build.HIPCC, *build.CFLAGS, *build.FILE_FLAGS.get(os.path.basename(src), []), "--cuda-device-only", "-S",
           "-o", out, os.path.abspath(src)]
    subprocess.run(cmd, check=True, cwd=os.path.dirname(os.path.abspath(src)), stderr=subprocess.DEVNULL)
    return open(out).read()


def check(src):
    bad, n_dma = 0, 0
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n", asm(src), re.M):
        pass
    s = asm(src)
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n", s, re.M):
        body = s[m.end():s.index(".Lfunc_end", m.end())].split("\n")
        in_asm = False
        asm_m0 = False      # an asm block wrote m0 since the compiler's last m0 write
        for line in body:
            t = line.strip()
            if t.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if t.startswith(";;#ASMEND"):
                in_asm = False
                continue
            if re.match(r"^\.LBB", t):  # a new basic block: the compiler cannot assume m0 from a predecessor's asm
                pass
            writes_m0 = re.match(r"s_\w+\s+m0\b", t) is not None
            if in_asm:
                asm_m0 = asm_m0 or writes_m0
                continue
            if writes_m0:
                asm_m0 = False
            if re.search(r"(global_load_lds_|buffer_load_\w+ .*\blds\b)", t):
                n_dma += 1
                if asm_m0:
                    bad += 1
                    print(f"{os.path.basename(src)} {m.group(1)[:60]}: compiler LDS-DMA after an asm m0 write: {t}")
    print(f"{os.path.basename(src)}: {n_dma} compiler-emitted LDS-DMA instructions, {bad} relying on a stale m0")
    return bad


def main():
    srcs = sys.argv[1:] or [os.path.join(build.CSRC, f) for f in DEFAULT]
    sys.exit(1 if sum(check(s) for s in srcs) else 0)


if __name__ == "__main__":
    main()
