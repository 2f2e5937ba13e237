"""Instruction mix per basic block of one kernel in the gfx950 assembly of a csrc/ source (CPU only: hipcc -S):

  python scripts/isa_mix.py attn_fwd.hip attn_fwd_kernelILi64ELb1E
  python scripts/isa_mix.py attn_bwd_split.hip attn_bwd_q_kernelILi64ELb1E

Prints every block with an MFMA or more than 40 vector instructions: its size, MFMA and VALU counts and the most
frequent vector / LDS / wait instructions — the tile bodies of an attention loop are the blocks with MFMAs.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import build as B  # noqa: E402


def main():
    src, pat = sys.argv[1], sys.argv[2]
    out = os.path.join(tempfile.mkdtemp(), "k.s")
    cmd = [B.HIPCC, *B.CFLAGS, *B.FILE_FLAGS.get(src, []), f"-I{B.CSRC}", "-S", "--cuda-device-only",
           f"--offload-arch={B.ARCH}", os.path.join(B.CSRC, src), "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)
    lines = open(out).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(pat) + r"\S*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    print(lines[start].split(":")[0])
    blocks, cur = [], None
    for line in lines[start + 1:end]:
        t = line.strip()
        if re.match(r"^\.LBB\d+_\d+:", t) or cur is None:
            cur = [t.split(":")[0] if t.startswith(".LBB") else "(entry)", []]
            blocks.append(cur)
            if t.startswith(".LBB"):
                continue
        if not t or t.startswith(";") or t.startswith("."):
            continue
        cur[1].append(t.split()[0])
    for name, ins in blocks:
        c = collections.Counter(ins)
        mf = sum(v for k, v in c.items() if k.startswith("v_mfma"))
        valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
        if mf or valu > 40:
            top = sorted(((v, k) for k, v in c.items() if k.startswith(("v_", "ds_", "s_waitcnt", "s_nop", "scratch_"))),
                         reverse=True)[:10]
            print(f"{name:10s} n {len(ins):4d}  mfma {mf:3d}  valu {valu:4d}  " + ", ".join(f"{k} {v}" for v, k in top))


if __name__ == "__main__":
    main()
