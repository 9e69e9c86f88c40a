#!/usr/bin/env python3
"""HBM yardstick on this box: torch device-to-device copy bandwidth."""
import json, torch
for mb in (64, 256, 1024):
    n = mb * 2**20 // 4
    a = torch.empty(n, device="cuda"); b = torch.empty(n, device="cuda")
    for _ in range(3): b.copy_(a)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20): b.copy_(a)
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    print(json.dumps({"MB": mb, "us": ms * 1e3, "GBps_rw": 2 * n * 4 / ms / 1e6}))
