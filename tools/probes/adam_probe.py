"""Which Adam sub-step differs between dpac_adam_apply, torch GPU ops and torch CPU ops."""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from deeppde_actorcritic_amd import ops
for dt in (torch.float64, torch.float32):
    gen = torch.Generator().manual_seed(5)
    v = torch.randn(40000, generator=gen, dtype=dt); g = torch.randn(40000, generator=gen, dtype=dt)
    b1, b2, eps = 0.9, 0.999, 1e-8
    alpha = 1e-3 * np.sqrt(1 - b2) / (1 - b1)
    def torch_path(v, g):
        m = torch.zeros_like(v); s = torch.zeros_like(v)
        m = m + (g - m) * (1 - b1); s = s + (g * g - s) * (1 - b2)
        den = torch.sqrt(s) + eps
        return v - (m * alpha) / den, m, s, den, (m * alpha)
    cpu = torch_path(v.clone(), g)
    gpu = [t.cpu() for t in torch_path(v.cuda(), g.cuda())]
    vd, md, sd = v.cuda(), torch.zeros(40000, dtype=dt, device="cuda"), torch.zeros(40000, dtype=dt, device="cuda")
    ops.adam_apply([vd], [g.cuda()], [md], [sd], alpha, b1, b2, eps)
    k = [vd.cpu(), md.cpu(), sd.cpu()]
    names = ["var", "m", "s", "den", "m*alpha"]
    for i in range(5):
        print(dt, names[i], "cpu!=gpu", int((cpu[i] != gpu[i]).sum()), end=" ")
        if i < 3:
            print("kernel!=cpu", int((k[i] != cpu[i]).sum()), "kernel!=gpu", int((k[i] != gpu[i]).sum()), end="")
        print()
    q = (cpu[4] / cpu[3]); print(" div cpu vs gpu", int((q != (gpu[4].cuda() / gpu[3].cuda()).cpu()).sum()))
    sq = torch.sqrt(cpu[2]); print(" sqrt cpu vs gpu", int((sq != torch.sqrt(cpu[2].cuda()).cpu()).sum()))
