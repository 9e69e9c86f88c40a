import torch, sys
sys.path.insert(0, "/root/repo")
from deeppde_actorcritic_amd import ops
from deeppde_actorcritic_amd import solver as psol
from deeppde_actorcritic_amd.config import set_floatx
from tests.helpers import full_config
set_floatx("float32")
for AC, hid, d in [("critic", (200, 200, 200), 20), ("critic_grad", (48, 130, 33), 10)]:
    cfg = full_config("LQR", d, hidden=hid, dtype="float32")
    net = psol.DeepNN(cfg, AC, torch.Generator().manual_seed(4), torch.float32, "cuda")
    R = 100
    x = torch.randn(R, d, device="cuda") * 0.5
    params = [p.detach() for p in net.trainable_variables()]
    res = {}
    for m in ("f32", "x3"):
        ops.MLP_MATH = m
        out, z = ops.mlp_rows(net.mlp_view(), x, save=True)
        g = torch.randn(R, out.shape[1], device="cuda", generator=torch.Generator("cuda").manual_seed(1))
        L, gam, bet, Ws, b = ops._split_params(params)
        view, wt, wt_km = ops.mlp_prepare(gam, bet, Ws, b, False, True)
        G = torch.full((R, sum(view.widths)), 7.0, device="cuda")
        gx = torch.full((R, d), 7.0, device="cuda")
        import ctypes
        from deeppde_actorcritic_amd import _lib
        _lib.call("dpac_mlp_rows_bwd", _lib.F32, R, ctypes.byref(view.struct), ops._ptr_array(wt), ops._ptr_array(wt_km),
                  ops._ptr(z), ops._ptr(g), ops._ptr(G), ops._ptr(gx), ops._stream(x))
        res[m] = (out, z, G, gx)
    w = [d] + list(hid) + [out.shape[1]]
    o = 0
    print(AC, "out", float((res['f32'][0]-res['x3'][0]).abs().max()), "z", float((res['f32'][1]-res['x3'][1]).abs().max()))
    for i, wi in enumerate(w):
        a, bb = res['f32'][2][:, o:o+wi], res['x3'][2][:, o:o+wi]
        print(" G block", i, wi, float((a-bb).abs().max()), float(a.abs().max()), "n7", int((bb == 7.0).sum()))
        o += wi
    print(" gx", float((res['f32'][3]-res['x3'][3]).abs().max()))
