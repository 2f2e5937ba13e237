"""Where a kernel's scratch spills / reloads sit, by loop depth, from hipcc's gfx950 assembly (a reload inside the
tile loop costs a vmcnt(0) that drains the LDS-DMA ring every tile).

  python scripts/spill_depth.py picotron_amd/csrc/attn_bwd_split.hip [kernel-substring ...]
"""
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import build  # noqa: E402


def asm(src):
    out = "/tmp/spill_depth.s"
    cmd = [build.HIPCC, *build.CFLAGS, *build.FILE_FLAGS.get(os.path.basename(src), []), "--cuda-device-only", "-S",
           "-o", out, os.path.abspath(src)]
    subprocess.run(cmd, check=True, cwd=os.path.dirname(os.path.abspath(src)))
    return open(out).read()


def main():
    src, subs = sys.argv[1], sys.argv[2:]
    s = asm(src)
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n", s, re.M):
        name = m.group(1)
        if subs and not any(x in name for x in subs):
            continue
        body = s[m.end():s.index(".Lfunc_end", m.end())].split("\n")
        depth = 0
        rows = {}
        for line in body:
            d = re.search(r"Depth=(\d+)", line)
            if re.match(r"^\.LBB\d+_\d+:", line):
                depth = int(d.group(1)) if d else 0
            if "scratch_load" in line or "scratch_store" in line:
                kind = "reload" if "scratch_load" in line else "spill"
                rows[(kind, depth)] = rows.get((kind, depth), 0) + 1
        print(name, {f"{k}@depth{d}": n for (k, d), n in sorted(rows.items())} or "no scratch")


if __name__ == "__main__":
    main()
