#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a hipcc -save-temps .s file.

    python tools/isa_blocks.py <file.s> <kernel-symbol-substring>

Prints, for each block: instructions, VALU, packed VALU, transcendental VALU,
LDS and global-store counts -- the static issue budget behind the PMC numbers.
"""
import collections
import sys

TRANS = {"v_exp_f32", "v_rsq_f32", "v_rcp_f32", "v_sqrt_f32", "v_log_f32", "v_sin_f32", "v_cos_f32"}


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l.split(":")[0])
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks = [["entry", collections.Counter(), 0]]
    for raw in lines[start + 1:end]:
        l = raw.split(";")[0].strip()
        if not l:
            continue
        if l.startswith(".LBB") and l.endswith(":"):
            blocks.append([l[:-1], collections.Counter(), 0])
            continue
        if l.startswith("."):
            continue
        op = l.split()[0]
        blocks[-1][1][op] += 1
        blocks[-1][2] += 1
    for name, c, n in blocks:
        v = sum(x for o, x in c.items() if o.startswith("v_"))
        pk = sum(x for o, x in c.items() if o.startswith("v_pk"))
        tr = sum(x for o, x in c.items() if o in TRANS)
        ds = sum(x for o, x in c.items() if o.startswith("ds_"))
        gs = sum(x for o, x in c.items() if o.startswith("global_store") or o.startswith("buffer_store"))
        print(f"{name:12s} insts {n:5d}  valu {v:5d}  pk {pk:4d}  trans {tr:3d}  lds {ds:3d}  store {gs:3d}")
        if len(sys.argv) > 3 and n > 200:
            print("   ", ", ".join(f"{o}:{x}" for o, x in c.most_common(25)))


if __name__ == "__main__":
    main()
