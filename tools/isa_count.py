#!/usr/bin/env python3
"""Instruction mix of a kernel's main time loop, per time step.

    python tools/isa_count.py <file.s> <mangled-name-substring> <steps-per-iteration>
Takes the innermost loop with the most instructions in the kernel's body.
"""
import collections
import re
import sys


def main(path, name, steps):
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l)]
    k = [i for i in starts if name in lines[i]][0]
    end = min([i for i in starts if i > k] + [len(lines)])
    body = lines[k:end]
    best = None
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\d+_\d+):.*Loop Header", l)
        if not m:
            continue
        lab = m.group(1)
        js = [j for j, l2 in enumerate(body) if re.search(r"s_c?branch\w* " + re.escape(lab) + r"$", l2)]
        if js and (best is None or js[-1] - i > best[1] - best[0]):
            best = (i, js[-1])
    ins = [l.strip() for l in body[best[0]:best[1] + 1] if l.strip() and not l.strip().startswith((".", ";"))]
    c = collections.Counter()
    for l in ins:
        op = l.split()[0]
        if op.startswith("v_"):
            if "row_" in l or "quad_perm" in l:
                key = "v_dpp"
            elif re.match(r"v_(sqrt|rsq|rcp|exp|log|sin|cos)", op):
                key = "v_trans"
            elif op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
                key = "v_lane"
            elif op.startswith(("v_cndmask", "v_cmp", "v_mov", "v_pk")):
                key = op.split("_e")[0][:9]
            else:
                key = "v_other"
        elif op.startswith("s_nop"):
            key = "s_nop"
        elif op.startswith("s_waitcnt"):
            key = "s_waitcnt"
        elif op.startswith(("buffer_load", "global_load")):
            key = "vmem_load"
        elif op.startswith(("buffer_store", "global_store")):
            key = "vmem_store"
        elif op.startswith("s_"):
            key = "salu/branch"
        else:
            key = op
        c[key] += 1
    print(f"{len(ins)} instructions, {len(ins) / steps:.1f} per step")
    for key, v in sorted(c.items(), key=lambda x: -x[1]):
        print(f"  {key:14s} {v:5d} {v / steps:6.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]))
