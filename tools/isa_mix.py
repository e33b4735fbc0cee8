#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -S (gfx950) listing.
usage: isa_mix.py <file.s> <kernel-symbol-substring> [--lines A B]"""
import collections
import re
import sys


def kernel_body(lines, key):
    start = None
    for i, ln in enumerate(lines):
        if start is None and ln.startswith("_Z") and key in ln and ln.rstrip().endswith(":") is False and ":" in ln:
            start = i
        elif start is not None and (ln.startswith("\t.section") or ln.startswith(".Lfunc_end")):
            return lines[start:i]
    return lines[start:] if start is not None else []


def main():
    lines = open(sys.argv[1]).read().split("\n")
    body = kernel_body(lines, sys.argv[2])
    mix = collections.Counter()
    cls = collections.Counter()
    for ln in body:
        t = ln.strip()
        if not t or t.startswith((";", ".", "_")) or t.endswith(":"):
            continue
        op = t.split()[0]
        mix[op] += 1
        if op.startswith("v_pk_"):
            cls["valu_pk"] += 1
        elif op.startswith(("v_rcp", "v_rsq", "v_sqrt", "v_exp", "v_log", "v_sin", "v_cos")):
            cls["valu_trans"] += 1
        elif op.startswith("v_div"):
            cls["valu_div"] += 1
        elif op.startswith("v_"):
            cls["valu"] += 1
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            cls["smem"] += 1
        elif op.startswith("s_waitcnt"):
            cls["waitcnt"] += 1
        elif op.startswith("s_nop"):
            cls["nop"] += 1
        elif op.startswith("s_cbranch") or op.startswith("s_branch"):
            cls["branch"] += 1
        elif op.startswith("s_"):
            cls["salu"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            cls["vmem"] += 1
        elif op.startswith("ds_"):
            cls["lds"] += 1
        else:
            cls["other"] += 1
    print(f"{len(body)} lines; static instruction classes:", dict(cls))
    print("top:", mix.most_common(40))


if __name__ == "__main__":
    main()
