#!/usr/bin/env python3
"""Bitwise comparison of two tools/probe_bptt.py --dump files (two builds of the same kernels).

    python tools/cmp_dumps.py a.pt b.pt    -> exit 1 if any tensor differs in a single bit
"""
import sys

import torch

_INT = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}


def bits(t):
    return t.contiguous().view(_INT[t.element_size()])


def main():
    a, b = (torch.load(f, weights_only=True) for f in sys.argv[1:3])
    bad = 0
    for k in a:
        same = a[k].shape == b[k].shape and torch.equal(bits(a[k]), bits(b[k]))
        print(f"{k:6s} {tuple(a[k].shape)} {'bitwise equal' if same else 'DIFFERS'}")
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
