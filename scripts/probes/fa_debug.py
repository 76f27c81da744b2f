"""Isolate a flash-attention NaN: run fwd/bwd variant combinations on one config and report
where the gradient is non-finite or off."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import lumen.ops.attention as att  # noqa: E402

nh, nkv, lens = int(sys.argv[1]), int(sys.argv[2]), [int(x) for x in sys.argv[3].split(",")]
D = 128
cu = [0]
for L in lens:
    cu.append(cu[-1] + L)
T = cu[-1]
torch.manual_seed(0)
qkv0 = (torch.randn(T, (nh + 2 * nkv) * D, device="cuda") * 0.5).to(torch.bfloat16)
q2 = qkv0.detach().float().requires_grad_(True)
o2 = att.flash_attention_ref(q2, tuple(cu), nh, nkv, D, True)
do = torch.randn_like(o2).to(torch.bfloat16)
o2.backward(do.float())
for fwd, bwd in [("v32", "ds"), ("v32", "recompute")]:
    att.FA_DS_MB = 2048 if bwd == "ds" else 0
    x = qkv0.clone().requires_grad_(True)
    o = att.flash_attention_qkv(x, cu, nh, nkv, D, True)
    o.backward(do)
    g = x.grad.float()
    qs, ks = nh * D, nkv * D
    out = [fwd, bwd]
    for name, sl in (("dq", slice(0, qs)), ("dk", slice(qs, qs + ks)), ("dv", slice(qs + ks, None))):
        a, b = g[:, sl], q2.grad[:, sl]
        bad = (~torch.isfinite(a)).any(1).nonzero().flatten()
        err = ((a - b).norm() / b.norm()).item()
        out.append(f"{name}: rel {err:.3g} nonfinite rows {bad[:8].tolist()} (n={bad.numel()})")
    print(" | ".join(out), flush=True)
