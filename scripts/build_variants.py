"""Build A/B variants of the HIP library: each variant recompiles ONE source with extra -D flags
and relinks a full library to picotron_amd/lib/variants/<name>.so (select with PICO_LIB_PATH).

  python scripts/build_variants.py attn_bwd.hip base: unroll:-DPICO_BWD_DQ_UNROLL=1 prev:file=/tmp/old.hip
A `file=PATH` token compiles PATH (e.g. an older revision of the source) in place of csrc/<src>. Sources that
must agree on a define (attn_bwd_split.hip and attn_bwd_split_d128.hip, which #includes it) are given
together: `attn_bwd_split.hip,attn_bwd_split_d128.hip`.
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import build as B  # noqa: E402


def main():
    srcs = sys.argv[1].split(",")  # one source, or several that must share the flags (a.hip,b.hip)
    B.build()
    out_dir = os.path.join(B.HERE, "lib", "variants")
    os.makedirs(out_dir, exist_ok=True)
    objs = [os.path.join(B.OBJ, f[:-4] + ".o") for f in sorted(os.listdir(B.CSRC)) if f.endswith(".hip")]
    for spec in sys.argv[2:]:
        name, _, flags = spec.partition(":")
        replace = {}
        for src in srcs:
            vobj = os.path.join(out_dir, f"{name}_{src[:-4]}.o")
            path = os.path.join(B.CSRC, src)
            extra = []
            for tok in flags.split():
                if tok.startswith("file="):
                    path = tok[5:]
                else:
                    extra.append(tok)
            cmd = [B.HIPCC, *B.CFLAGS, *B.FILE_FLAGS.get(src, []), *extra, f"-I{B.CSRC}", "-c", path, "-o", vobj]
            subprocess.run(cmd, check=True)
            replace[os.path.join(B.OBJ, src[:-4] + ".o")] = vobj
        lib = os.path.join(out_dir, f"{name}.so")
        link = [B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib,
                *[replace.get(o, o) for o in objs]]
        subprocess.run(link, check=True)
        print(lib)


if __name__ == "__main__":
    main()
