"""Numerics of every HIP kernel against a plain PyTorch f32 reference of the same op (GPU)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(autouse=True)
def _native():
    from lumen.ops._native import native, native_error

    assert native() is not None, f"native extension must load on the GPU box: {native_error()!r}"
    torch.manual_seed(0)


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("H", [128, 768, 4096, 8192])
def test_rmsnorm_fwd_bwd(dtype, H):
    """(fp32: the backward once held 8 elements per lane in a 16-byte register pack -- half of
    every f32 row vector was lost; fp32 tolerances are 1e-5.)"""
    from lumen.ops.norm import rms_norm, rms_norm_ref

    tf, tb = (1e-5, 1e-5) if dtype == torch.float32 else (1e-2, 2e-2)

    T = 300
    x = torch.randn(T, H, device=DEV, dtype=dtype, requires_grad=True)
    r = torch.randn(T, H, device=DEV, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(dtype)
    y, s = rms_norm(x, w, 1e-5, r)
    x2 = x.detach().float().requires_grad_(True)
    r2 = r.detach().float().requires_grad_(True)
    y2, s2 = rms_norm_ref(x2, w.float(), 1e-5, r2)
    assert rel(s, s2) < tf and rel(y, y2) < tf
    dy = torch.randn_like(y)
    ds = torch.randn_like(s)
    torch.autograd.backward([y, s], [dy, ds])
    torch.autograd.backward([y2, s2], [dy.float(), ds.float()])
    assert rel(x.grad, x2.grad) < tb
    assert rel(r.grad, r2.grad) < tb
    # no-residual variant
    x3 = x.detach().clone().requires_grad_(True)
    y3, s3 = rms_norm(x3, w, 1e-5)
    x4 = x.detach().float().requires_grad_(True)
    y4, _ = rms_norm_ref(x4, w.float(), 1e-5)
    assert rel(y3, y4) < tf
    y3.backward(dy)
    y4.backward(dy.float())
    assert rel(x3.grad, x4.grad) < tb


@pytest.mark.parametrize("nh,nkv,D", [(32, 32, 128), (8, 2, 128), (4, 2, 32), (4, 4, 64)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_qkv_rope_split(nh, nkv, D, dtype):
    """Split + rotate of the fused QKV buffer (the portable-attention path, head_dim != 128 and
    --dtype fp32 models) vs the fp32 reference, v included (an fp32 v copy once moved only half
    of each 16-element chunk)."""
    from lumen.ops.rope import qkv_rope_split, qkv_rope_split_ref, rope_tables

    B, S = 2, 64
    cos, sin = rope_tables(D, 4096, 10000.0, DEV)
    qkv = torch.randn(B * S, (nh + 2 * nkv) * D, device=DEV, dtype=dtype,
                      requires_grad=True)
    q, k, v = qkv_rope_split(qkv, B, S, nh, nkv, D, cos, sin)
    qkv2 = qkv.detach().float().requires_grad_(True)
    q2, k2, v2 = qkv_rope_split_ref(qkv2, B, S, nh, nkv, D, cos, sin)
    for a, b in ((q, q2), (k, k2), (v, v2)):
        assert a.shape == b.shape and rel(a, b) < (1e-5 if dtype == torch.float32 else 1e-2)
    g = [torch.randn_like(t) for t in (q, k, v)]
    torch.autograd.backward([q, k, v], g)
    torch.autograd.backward([q2, k2, v2], [t.float() for t in g])
    assert rel(qkv.grad, qkv2.grad) < 1e-2
    # explicit positions
    pos = torch.randint(0, 4000, (B * S,), device=DEV)
    qp, kp, _ = qkv_rope_split(qkv.detach(), B, S, nh, nkv, D, cos, sin, pos)
    qr, kr, _ = qkv_rope_split_ref(qkv.detach().float(), B, S, nh, nkv, D, cos, sin, pos)
    assert rel(qp, qr) < 1e-2 and rel(kp, kr) < 1e-2


@pytest.mark.parametrize("nh", [4, 16])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_rope_inplace(dtype, nh):
    from lumen.ops.rope import rope_inplace, rope_tables, _rotate_ref

    T, D = 37, 128
    cos, sin = rope_tables(D, 4096, 10000.0, DEV)
    x = torch.randn(T, 3 * nh * D, device=DEV, dtype=dtype)
    pos = torch.randint(0, 2000, (T,), device=DEV)
    ref = x.clone().float()
    view = ref[:, nh * D: 2 * nh * D].view(T, nh, D)
    view.copy_(_rotate_ref(view, cos[pos][:, None], sin[pos][:, None]))
    rope_inplace(x, pos, nh, D, cos, sin, col_offset=nh * D)
    assert rel(x, ref) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_swiglu(dtype):
    from lumen.ops.activation import swiglu, swiglu_ref

    gu = torch.randn(333, 2 * 1024, device=DEV, dtype=dtype, requires_grad=True)
    y = swiglu(gu)
    gu2 = gu.detach().float().requires_grad_(True)
    y2 = swiglu_ref(gu2)
    assert rel(y, y2) < 1e-2
    d = torch.randn_like(y)
    y.backward(d)
    y2.backward(d.float())
    assert rel(gu.grad, gu2.grad) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_swiglu_column_ranges(dtype):
    """The column-range entry (used beside a split GEMM's tail): two ranges == the whole row,
    forward and backward, and columns outside the range stay untouched."""
    from lumen.ops._native import native

    T, F, c = 129, 1024, 392
    gu = torch.randn(T, 2 * F, device=DEV, dtype=dtype)
    d = torch.randn(T, F, device=DEV, dtype=dtype)
    whole, parts = torch.empty(T, F, device=DEV, dtype=dtype), torch.full((T, F), 7.0, device=DEV, dtype=dtype)
    native().swiglu(False, gu, None, whole)
    native().swiglu(False, gu, None, parts, 0, c)
    assert torch.equal(parts[:, :c], whole[:, :c]) and bool((parts[:, c:] == 7).all())
    native().swiglu(False, gu, None, parts, c, F)
    assert torch.equal(parts, whole)
    dw, dp = torch.empty_like(gu), torch.empty_like(gu)
    native().swiglu(True, gu, d, dw)
    native().swiglu(True, gu, d, dp, 0, c)
    native().swiglu(True, gu, d, dp, c, F)
    assert torch.equal(dp, dw)


@pytest.mark.parametrize("mode", [1, 2])
def test_overlap_mlp(mode, monkeypatch):
    """The frozen MLP with its split GEMMs' tails on a side stream beside the SwiGLU of the
    columns already produced (``_OverlapMLP``, both issue orders) vs the fp32 reference and the
    unfused path: output and input gradient."""
    import lumen.ops.activation as act
    import lumen.ops.gemm as G
    from lumen.models.layers import Linear

    T, H, F = 512, 512, 1376
    monkeypatch.setattr(act, "MLP_OVERLAP", mode)
    monkeypatch.setattr(G, "_split_plan", lambda x, w: 1024 if w.shape[0] == F else 0)
    gu_l = Linear(H, 2 * F, dtype=torch.bfloat16, device=DEV)
    dn_l = Linear(F, H, dtype=torch.bfloat16, device=DEV)
    for m in (gu_l, dn_l):
        m.weight.requires_grad_(False)
        m.weight.copy_(torch.randn_like(m.weight) * 0.05)
        m.transpose_bwd = True
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    out = act.overlap_mlp(x, gu_l, dn_l, F + 256)
    g = torch.randn_like(out)
    out.backward(g)
    x2 = x.detach().clone().requires_grad_(True)
    out2 = dn_l(act.swiglu(gu_l(x2)))
    out2.backward(g)
    x3 = x.detach().float().requires_grad_(True)
    out3 = act.swiglu_ref(x3 @ gu_l.weight.float().t()) @ dn_l.weight.float().t()
    out3.backward(g.float())
    assert rel(out, out2) < 2e-3 and rel(x.grad, x2.grad) < 2e-3
    assert rel(out, out3) < 1e-2 and rel(x.grad, x3.grad) < 1e-2
    assert act.overlap_mlp_plan(x.cpu(), gu_l, dn_l) == 0  # CPU: never


@pytest.mark.parametrize("V", [32000, 50272])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_lm_head_cross_entropy(V, dtype):
    from lumen.ops.loss import lm_head_cross_entropy

    T, H = 257, 256
    h = torch.randn(T, H, device=DEV, dtype=dtype, requires_grad=True)
    W = (torch.randn(V, H, device=DEV) * 0.05).to(dtype)
    labels = torch.randint(0, V, (T,), device=DEV)
    labels[::7] = -100
    n_valid = int((labels != -100).sum())
    loss = lm_head_cross_entropy(h, labels, lambda: W, n_valid)
    h2 = h.detach().float().requires_grad_(True)
    logits = h2 @ W.float().t()
    loss2 = torch.nn.functional.cross_entropy(logits, labels, ignore_index=-100)
    assert abs(loss.item() - loss2.item()) < 2e-2 * max(1, abs(loss2.item()))
    (loss * 3).backward()
    (loss2 * 3).backward()
    assert rel(h.grad, h2.grad) < 3e-2
    # TN input gradient against a cached W^T (the frozen head's weight_t_fn)
    Wt = W.t().contiguous()
    h3 = h.detach().clone().requires_grad_(True)
    (lm_head_cross_entropy(h3, labels, lambda: W, n_valid, None, lambda: Wt) * 3).backward()
    assert rel(h3.grad, h2.grad) < 3e-2 and rel(h3.grad, h.grad) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_scale_dev(dtype):
    """x *= num / den with device f32 scalars (the LM head's dH times the upstream gradient and
    the fp16 loss-scale hint), f32 math, vs torch."""
    from lumen.ops._native import native

    x = torch.randn(1000, 24, device=DEV).to(dtype)
    num = torch.tensor([65536.0 * 3], device=DEV)
    den = torch.tensor([65536.0], device=DEV)
    ref = (x.float() * 3).to(dtype)
    y = x.clone()
    native().scale_dev(y, num, den)
    assert torch.equal(y, ref)
    y = x.clone()
    native().scale_dev(y, torch.tensor([0.37], device=DEV), None)
    assert torch.equal(y, (x.float() * 0.37).to(dtype))


@pytest.mark.parametrize("n", [1, 7, 8, 1000003, 16777216 + 5])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_grad_norm_sq_sizes(n, dtype):
    """Sum of squares (the global grad-norm pass): ragged tails and the LoRA-set size, vs torch
    in f64 (it accumulates into a pre-zeroed scalar)."""
    from lumen.ops._native import native

    g = (torch.randn(n, device=DEV) * 3).to(dtype)
    out = torch.zeros(1, device=DEV)
    native().grad_norm_sq(g, out)
    ref = (g.double() ** 2).sum().item()
    assert abs(out.item() - ref) <= 1e-4 * ref + 1e-6


def test_grad_norm_and_adamw():
    from lumen.ops._native import native
    from lumen.parallel.zero import _adamw_torch

    C = native()
    n = 1_000_003
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV) * 3
    m = torch.randn(n, device=DEV).abs() * 0.1
    v = torch.rand(n, device=DEV) * 0.1
    ns = torch.zeros(1, device=DEV)
    C.grad_norm_sq(g, ns)
    assert abs(ns.item() - g.double().pow(2).sum().item()) / g.double().pow(2).sum().item() < 1e-5
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    lr, b1, b2, eps, wd, inv = 1e-3, 0.9, 0.999, 1e-8, 0.01, 0.5
    maxn = 1.0
    copy = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    C.adamw(p, g, m, v, copy, lr, b1, b2, eps, wd, 1 - b1 ** 3, 1 - b2 ** 3, inv, ns, maxn, None,
            [])
    gn = math.sqrt(ns.item()) * inv
    coef = inv * (maxn / (gn + 1e-6) if gn > maxn else 1.0)
    _adamw_torch(p2, g, m2, v2, lr, b1, b2, eps, wd, 1 - b1 ** 3, 1 - b2 ** 3, coef)
    assert (p - p2).abs().max().item() < 1e-5
    assert (m - m2).abs().max().item() < 1e-6
    assert rel(copy, p2) < 1e-2
    # overflow -> no update
    p3 = p.clone()
    bad = torch.tensor([float("inf")], device=DEV)
    C.adamw(p, g, m, v, None, lr, b1, b2, eps, wd, 0.1, 0.1, 1.0, bad, 1.0, None, [])
    assert torch.equal(p, p3)


def test_adamw_device_step_counter():
    """Device Adam step counter: bias corrections from [applied, skipped]; a non-finite norm
    skips the update and counts as skipped without advancing t (bf16 NaN steps)."""
    from lumen.ops._native import native
    from lumen.parallel.zero import _adamw_torch

    C = native()
    n = 4096 * 3 + 5
    p = torch.randn(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    st = torch.zeros(8, device=DEV)
    st[2] = 1.0                      # loss scale
    lr, b1, b2 = 1e-2, 0.9, 0.999
    # lr_min, lr_max, warm_n, warm_linear, inv_world, dynamic, window, hysteresis, min_scale
    sched = [lr, lr, 0, 0, 1.0, 0, 1000, 2, 1.0]
    g = torch.randn(n, device=DEV)
    good = torch.zeros(1, device=DEV)
    C.grad_norm_sq(g, good)
    bad = torch.tensor([float("nan")], device=DEV)
    t = 0
    for norm in (good, bad, good, good, bad):
        C.adamw(p, g, m, v, None, 0.0, b1, b2, 1e-8, 0.0, 1.0, 1.0, 0.0, norm, 0.0, st, sched)
        if norm is good:
            t += 1
            _adamw_torch(p2, g, m2, v2, lr, b1, b2, 1e-8, 0.0, 1 - b1 ** t, 1 - b2 ** t, 1.0)
    assert st[:2].tolist() == [3.0, 2.0]
    assert (p - p2).abs().max().item() < 1e-5
    assert (v - v2).abs().max().item() < 1e-6


def test_adamw_device_hf_linear_schedule():
    """Device LR schedule with decay_total (HF linear warm-up + decay, the no-DeepSpeed
    baseline): each applied step uses lr_max * sched(t), same as the host ``warmup_lr``."""
    from lumen.ops._native import native
    from lumen.parallel.zero import _adamw_torch
    from lumen.train.config import load_ds_config, warmup_lr

    C = native()
    n = 4096 + 7
    p = torch.randn(n, device=DEV)
    m, v = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    st = torch.zeros(8, device=DEV)
    st[2] = 1.0
    c = load_ds_config(None, 1, 1, 1, 1e-2, warmup_steps=2)
    c.decay_total_steps = 6
    b1, b2 = 0.9, 0.999
    sched = [0.0, 1e-2, 2, 0, 1.0, 0, 1000, 2, 1.0, 6]
    g = torch.randn(n, device=DEV)
    norm = torch.zeros(1, device=DEV)
    C.grad_norm_sq(g, norm)
    for t in range(1, 7):
        C.adamw(p, g, m, v, None, 0.0, b1, b2, 1e-8, 0.0, 1.0, 1.0, 0.0, norm, 0.0, st, sched)
        _adamw_torch(p2, g, m2, v2, warmup_lr(t - 1, c), b1, b2, 1e-8, 0.0, 1 - b1 ** t,
                     1 - b2 ** t, 1.0)
        assert (p - p2).abs().max().item() < 1e-5, t


@pytest.mark.parametrize("segs_kind", ["qkv", "o", "gqa_sparse"])
@pytest.mark.parametrize("p_drop", [0.0, 0.1])
@pytest.mark.parametrize("impl", ["v3", "v3_overlap", "v2", "f32"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_lora_linear_fwd_bwd(segs_kind, p_drop, impl, monkeypatch, dtype):
    """impl v3 (shipped default): one-shot DOWN / fused dY pass / fused dA + dx (lora_v3.hip)
    with the v2 UP write-back; v3_overlap: the same with the dY pass on a side stream beside
    the input-gradient GEMM (LUMEN_LORA_BWD_OVERLAP); v2: 16-bit MFMA kernels (lora_v2.hip, the
    fallback for unaligned segments); f32: exact-f32 MFMA kernel (lora.hip, other ranks)."""
    import lumen.ops.lora as lora_mod
    from lumen.ops.lora import lora_linear, lora_linear_ref

    monkeypatch.setattr(lora_mod, "USE_V2", impl != "f32")
    monkeypatch.setattr(lora_mod, "USE_V3", impl.startswith("v3"))
    monkeypatch.setattr(lora_mod, "BWD_OVERLAP", impl == "v3_overlap")

    T, K, r = 512 + 64, 1024, 16
    if segs_kind == "qkv":
        sizes = [1024, 1024, 1024]
        segs = [(0, 1024, 0, 0), (1024, 1024, 16, 1024), (2048, 1024, 32, 2048)]
    elif segs_kind == "o":
        sizes = [1024]
        segs = [(0, 1024, 0, 0)]
    else:  # GQA q|k|v with adapters on q and v only
        sizes = [1024, 256, 256]
        segs = [(0, 1024, 0, 0), (1280, 256, 16, 1024)]
    N = sum(sizes)
    R = r * len(segs)
    nb = sum(s[1] for s in segs)
    x = torch.randn(T, K, device=DEV, dtype=dtype, requires_grad=True)
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(dtype)
    A = (torch.randn(R, K, device=DEV) / math.sqrt(K)).requires_grad_(True)
    B = (torch.randn(nb, r, device=DEV) * 0.1).requires_grad_(True)
    seed = 1234567
    y = lora_linear(x, lambda: W, None, A, B, segs, r, 2.0, p_drop, seed)
    x2 = x.detach().float().requires_grad_(True)
    A2 = A.detach().clone().requires_grad_(True)
    B2 = B.detach().clone().requires_grad_(True)
    y2 = lora_linear_ref(x2.to(dtype).float(), W.float(), None, A2, B2, segs, r, 2.0,
                         p_drop, seed)
    assert rel(y, y2) < 1e-2
    dy = torch.randn_like(y)
    y.backward(dy)
    y2.backward(dy.float())
    assert rel(x.grad, x2.grad) < 2e-2
    assert rel(A.grad, A2.grad) < 1e-2
    assert rel(B.grad, B2.grad) < 1e-2


@pytest.mark.parametrize("nh,nkv,D", [(32, 32, 128), (64, 8, 128), (12, 12, 64)])
@pytest.mark.parametrize("ctx_max", [37, 700, 2100])
def test_paged_decode(nh, nkv, D, ctx_max):
    from lumen.ops.attention import paged_decode, paged_decode_ref, write_kv_cache

    bs, nseq = 16, 5
    lens = torch.randint(1, ctx_max + 1, (nseq,))
    lens[0] = ctx_max
    max_blocks = (ctx_max + bs - 1) // bs
    nblocks = nseq * max_blocks + 3
    kc = torch.zeros(nblocks, nkv, bs, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    perm = torch.randperm(nblocks)[: nseq * max_blocks].view(nseq, max_blocks).int()
    # fill caches through the cache-write kernel
    for i in range(nseq):
        L = int(lens[i])
        k = torch.randn(L, nkv, D, device=DEV, dtype=torch.bfloat16)
        v = torch.randn(L, nkv, D, device=DEV, dtype=torch.bfloat16)
        t = torch.arange(L)
        slots = (perm[i, t // bs].long() * bs + t % bs).to(DEV)
        write_kv_cache(k, v, kc, vc, slots)
    q = torch.randn(nseq, nh, D, device=DEV, dtype=torch.bfloat16)
    bt = perm.to(DEV)
    cl = lens.int().to(DEV)
    scale = 1 / math.sqrt(D)
    o2 = paged_decode_ref(q, kc, vc, bt, cl, scale)
    for part in (512, 64):
        o = paged_decode(q, kc, vc, bt, cl, int(lens.max()), scale, part)
        assert rel(o, o2) < 1e-2
        # two-pass (0), single-pass (1), single-pass with uniform block ids + nt loads (2),
        # and its software-pipelined form (3); 2 / 3 fall back to 1 where block size != 16
        for one in (0, 1, 2, 3):
            assert rel(paged_decode(q, kc, vc, bt, cl, int(lens.max()), scale, part,
                                    one_pass=one), o2) < 1e-2, (one, part)
        # fused merge (arrival counters, last partition merges) == two-kernel merge, and the
        # counters reset themselves: a repeat call gives the same bits
        o_f = paged_decode(q, kc, vc, bt, cl, int(lens.max()), scale, part, fused_merge=True,
                           one_pass=False)
        o_sep = paged_decode(q, kc, vc, bt, cl, int(lens.max()), scale, part, fused_merge=False,
                             one_pass=False)
        assert torch.equal(o_f, o_sep)
        assert torch.equal(paged_decode(q, kc, vc, bt, cl, int(lens.max()), scale, part,
                                        fused_merge=True, one_pass=False), o_f)
    from lumen.ops.attention import _merge_counters

    assert all(int(c.abs().sum()) == 0 for c in _merge_counters.values())


def test_sampling_greedy_and_topk():
    from lumen.ops._native import native

    C = native()
    R, V = 6, 32000
    logits = torch.randn(R, V, device=DEV)
    temp = torch.zeros(R, device=DEV)
    top_p = torch.ones(R, device=DEV)
    top_k = torch.zeros(R, device=DEV, dtype=torch.int32)
    out = torch.empty(R, device=DEV, dtype=torch.int64)
    C.sample(logits, temp, top_p, top_k, 1, 0, out, None)
    assert torch.equal(out, logits.argmax(-1))
    # top-k = 1 with temperature must also be the argmax
    temp.fill_(0.7)
    top_k.fill_(1)
    C.sample(logits, temp, top_p, top_k, 7, 3, out, None)
    assert torch.equal(out, logits.argmax(-1))
    # top-p tiny -> argmax
    top_k.zero_()
    top_p.fill_(1e-6)
    C.sample(logits, temp, top_p, top_k, 7, 4, out, None)
    assert torch.equal(out, logits.argmax(-1))
    # distribution check: 2-token vocab-like logits
    V2 = 1024
    lg = torch.full((4096, V2), -30.0, device=DEV)
    lg[:, 0] = 0.0
    lg[:, 1] = math.log(3.0)
    t2 = torch.ones(4096, device=DEV)
    o2 = torch.empty(4096, device=DEV, dtype=torch.int64)
    C.sample(lg, t2, torch.ones(4096, device=DEV), torch.zeros(4096, device=DEV, dtype=torch.int32),
             11, 0, o2, None)
    frac1 = (o2 == 1).float().mean().item()
    assert 0.70 < frac1 < 0.80


def _kept_matches(zs, kept, ref, p):
    """Kernel kept set vs the sort-based reference: equal, or different only in the tokens at
    the top-p boundary where the reference's cumulative mass sits within 1e-5 of p (the
    kernel's fast exp / fixed-point masses vs torch's f32 softmax)."""
    if torch.equal(kept, ref):
        return True
    if p >= 1.0:
        return False
    # exact ties at the top-p boundary (bf16 logits): the value threshold keeps every tied
    # token, the sort keeps the ones its order put first
    if torch.equal(kept, zs >= zs[ref].min()):
        return True
    diff = (kept ^ ref).nonzero().flatten()
    zk = torch.where(ref | kept, zs, torch.full_like(zs, -float("inf")))
    pr = torch.softmax(zs.double(), -1)
    for j in diff.tolist():
        above = pr[zs > zs[j]].sum().item()  # mass strictly above token j (untruncated)
        tot = pr[zk > -float("inf")].sum().item()
        if min(abs(above / tot - p), abs((above + pr[j].item()) / tot - p)) > 1e-5:
            return False
    return True


@pytest.mark.parametrize("k,p", [(1, 1.0), (50, 1.0), (1000, 1.0), (0, 0.5), (0, 0.9), (0, 0.99),
                                 (50, 0.9), (1000, 0.5), (1000, 0.99), (31999, 0.9)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sampling_kept_set_vs_sort(k, p, dtype):
    """Radix-select top-k / top-p (kernels/sampling.hip) against vLLM 0.6.0's sort-based
    ``_apply_top_k_top_p`` (lumen.serve.model_runner.topk_topp_keep), V = 32000: the kept set
    (the kernel reports its threshold) and every sampled token inside it.  bf16 logits have
    exact ties, which top-k keeps (value threshold) like the reference."""
    from lumen.ops._native import native
    from lumen.serve.model_runner import topk_topp_keep

    C = native()
    R, V = 8, 32000
    g = torch.Generator(device="cpu").manual_seed(k * 7 + int(p * 100))
    logits = (torch.randn(R, V, generator=g) * 3.0).to(dtype).to(DEV)
    temp = torch.tensor([1.0, 0.5] * (R // 2), device=DEV)   # 1/T exact: same z as torch
    out = torch.empty(R, device=DEV, dtype=torch.int64)
    tau = torch.empty(R, device=DEV, dtype=torch.float32)
    C.sample(logits, temp, torch.full((R,), p, device=DEV),
             torch.full((R,), k, device=DEV, dtype=torch.int32), 5, 1, out, None, tau)
    for i in range(R):
        zs = logits[i].float() * (1.0 / temp[i])
        kept = zs >= tau[i]
        ref = topk_topp_keep(zs, k, p)
        assert _kept_matches(zs, kept, ref, p), (i, int(kept.sum()), int(ref.sum()))
        assert kept[out[i]], i
        if 0 < k < V and p >= 1.0:
            assert int(kept.sum()) >= k


def test_sampling_distribution_chi2():
    """65,536 draws (one row each: the Gumbel noise is hashed per row) from one V = 200
    distribution with top-k 50 and top-p 0.9 at temperature 0.8: nothing outside the kept set,
    and a chi-square test of the counts against the renormalised truncated distribution."""
    from scipy.stats import chisquare

    from lumen.ops._native import native
    from lumen.serve.model_runner import topk_topp_keep

    C = native()
    R, V = 65536, 200
    g = torch.Generator(device="cpu").manual_seed(3)
    row = torch.randn(V, generator=g) * 2.0
    logits = row.expand(R, V).contiguous().to(DEV)
    T = 0.8
    temp = torch.full((R,), T, device=DEV)
    out = torch.empty(R, device=DEV, dtype=torch.int64)
    C.sample(logits, temp, torch.full((R,), 0.9, device=DEV),
             torch.full((R,), 50, device=DEV, dtype=torch.int32), 1234, 9, out, None)
    zs = row.float() * (1.0 / torch.tensor(T, dtype=torch.float32))
    keep = topk_topp_keep(zs, 50, 0.9)
    cnt = torch.bincount(out.cpu(), minlength=V).double()
    assert cnt[~keep].sum() == 0
    pr = torch.softmax(zs.double(), -1)[keep]
    exp = pr / pr.sum() * R
    res = chisquare(cnt[keep].numpy(), exp.numpy())
    assert res.pvalue > 1e-4, (res, int(keep.sum()))


def test_sampling_speed_256_rows():
    """The decode-step sampler with both filters (256 rows x 32000, top-k 50, top-p 0.95,
    temperature 0.8): radix select replaced the 30-pass bisections (VERDICT r5 Weak #6).
    A loose regression bound; the measured time goes in the bench record."""
    from lumen.ops._native import native

    C = native()
    R, V = 256, 32000
    logits = torch.randn(R, V, device=DEV) * 3
    args = (logits, torch.full((R,), 0.8, device=DEV), torch.full((R,), 0.95, device=DEV),
            torch.full((R,), 50, device=DEV, dtype=torch.int32))
    out = torch.empty(R, device=DEV, dtype=torch.int64)
    for _ in range(3):
        C.sample(*args, 1, 0, out, None)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(20):
        C.sample(*args, 1, i, out, None)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1000 / 20
    print(f"sampler 256 x 32000, top-k 50 + top-p 0.95: {us:.1f} us")
    assert us < 300, us


@pytest.mark.parametrize("nh,nkv,lens", [(8, 8, [512, 512]), (8, 2, [512, 300, 77]),
                                         (4, 4, [1000, 64, 129])])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_flash_attention_fwd_bwd(nh, nkv, lens, monkeypatch, dtype):
    """Forward kernel and the recompute backward (dK/dV + 32x32 dQ: the path when the dS
    hand-off buffer does not fit) vs the f32 reference."""
    import lumen.ops.attention as att
    from lumen.ops.attention import flash_attention_qkv, flash_attention_ref

    monkeypatch.setattr(att, "FA_DS_MB", 0)  # the recompute dQ kernels (dS hand-off: below)

    D = 128
    cu = [0]
    for L in lens:
        cu.append(cu[-1] + L)
    T = cu[-1]
    qkv = (torch.randn(T, (nh + 2 * nkv) * D, device=DEV) * 0.5).to(dtype)
    qkv.requires_grad_(True)
    o = flash_attention_qkv(qkv, cu, nh, nkv, D, True)
    q2 = qkv.detach().float().requires_grad_(True)
    o2 = flash_attention_ref(q2, tuple(cu), nh, nkv, D, True)
    assert rel(o, o2) < 2e-2
    do = torch.randn_like(o)
    o.backward(do)
    o2.backward(do.float())
    g, g2 = qkv.grad.float(), q2.grad
    qs, ks = nh * D, nkv * D
    assert rel(g[:, :qs], g2[:, :qs]) < 3e-2, "dq"
    assert rel(g[:, qs:qs + ks], g2[:, qs:qs + ks]) < 3e-2, "dk"
    assert rel(g[:, qs + ks:], g2[:, qs + ks:]) < 3e-2, "dv"


@pytest.mark.parametrize("nh,nkv,lens", [(8, 8, [512, 512]), (8, 2, [512, 300, 77]),
                                         (4, 4, [1000, 64, 129])])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_flash_attention_ds_handoff(nh, nkv, lens, causal, monkeypatch, dtype):
    """dS hand-off backward (dK/dV kernel stores dS tiles, dQ = dS K from them) vs the fp32
    reference, and dQ vs the recompute kernel (same bf16 dS operand: near-identical)."""
    import lumen.ops.attention as att
    from lumen.ops.attention import flash_attention_qkv, flash_attention_ref

    D = 128
    cu = [0]
    for L in lens:
        cu.append(cu[-1] + L)
    T = cu[-1]
    qkv = (torch.randn(T, (nh + 2 * nkv) * D, device=DEV) * 0.5).to(dtype)
    do = torch.randn(T, nh * D, device=DEV).to(dtype)
    grads = {}
    for mb in (2048, 0):
        monkeypatch.setattr(att, "FA_DS_MB", mb)
        x = qkv.clone().requires_grad_(True)
        o = flash_attention_qkv(x, cu, nh, nkv, D, causal)
        (grads[mb],) = torch.autograd.grad(o, x, do)
    q2 = qkv.float().requires_grad_(True)
    o2 = flash_attention_ref(q2, tuple(cu), nh, nkv, D, causal)
    (g2,) = torch.autograd.grad(o2, q2, do.float())
    g = grads[2048].float()
    qs, ks = nh * D, nkv * D
    assert rel(g[:, :qs], g2[:, :qs]) < 3e-2, "dq"
    assert rel(g[:, qs:qs + ks], g2[:, qs:qs + ks]) < 3e-2, "dk"
    assert rel(g[:, qs + ks:], g2[:, qs + ks:]) < 3e-2, "dv"
    assert rel(g[:, :qs], grads[0][:, :qs].float()) < 1e-2, "dq vs recompute"
    # same dK/dV kernel with and without the dS store
    assert torch.equal(grads[2048][:, qs:], grads[0][:, qs:]), "dk/dv unchanged"


@pytest.mark.parametrize("nh,nkv", [(8, 8), (8, 2)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_flash_backward_fused_inverse_rope(nh, nkv, dtype):
    """dQ / dK epilogues with the inverse RoPE (FA backward given the rotation) == plain FA
    backward followed by the separate inverse-rotation pass; dV untouched.  (The skip of the
    producer's own inverse pass is checked end to end by test_llama_fused_rope_backward_matches.)"""
    from lumen.ops.attention import flash_attention_qkv
    from lumen.ops.rope import _neg, rope_tables

    D = 128
    cu = [0, 300, 812, 1000]
    T = cu[-1]
    cos, sin = rope_tables(D, 4096, 10000.0, DEV)
    pos = torch.randint(0, 4096, (T,), device=DEV, dtype=torch.int32)
    qkv = (torch.randn(T, (nh + 2 * nkv) * D, device=DEV) * 0.5).to(dtype)
    do = torch.randn(T, nh * D, device=DEV).to(dtype)
    grads = []
    for fused in (True, False):
        x = qkv.clone().requires_grad_(True)
        o = flash_attention_qkv(x, cu, nh, nkv, D, True, rope=(pos, cos, sin) if fused else None)
        (g,) = torch.autograd.grad(o, x, do)
        if not fused:
            g = g.clone()
            from lumen.ops._native import native

            native().rope_inplace(g, pos, cos, _neg(sin), T, g.stride(0), nh + nkv, D)
        grads.append(g.float())
    qk = (nh + nkv) * D
    assert rel(grads[0][:, :qk], grads[1][:, :qk]) < 1e-2
    assert torch.equal(grads[0][:, qk:], grads[1][:, qk:])


def test_llama_fused_rope_backward_matches():
    """Full model step: inverse RoPE in the flash-attention epilogues vs in the q|k|v adapter
    backward -- same loss, same adapter gradients."""
    import lumen.models.llama as L
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model

    torch.manual_seed(0)
    m = build_model("llama2-7b", dtype=torch.bfloat16, device="meta")  # config only
    cfg = m.config
    cfg.num_hidden_layers = 2
    cfg.vocab_size = 1024
    model = L.LlamaForCausalLM(cfg, dtype=torch.bfloat16, device=DEV)
    model.init_weights(seed=1)
    apply_lora(model, LoraConfig(r=8, lora_dropout=0.0))
    for p in model.parameters():
        if p.requires_grad:
            p.data.normal_(0, 0.02)
    ids = torch.randint(3, 1024, (2, 256), device=DEV)
    labels = torch.full_like(ids, -100)
    labels[:, :-1] = ids[:, 1:]
    res = {}
    try:
        for fused in (True, False):
            L.FUSED_ROPE_BWD = fused
            model.zero_grad(set_to_none=True)
            loss = model(ids, labels, int((labels != -100).sum()))
            loss.backward()
            res[fused] = (loss.item(), [p.grad.clone() for p in model.parameters() if p.requires_grad])
    finally:
        L.FUSED_ROPE_BWD = True
    assert abs(res[True][0] - res[False][0]) < 1e-3  # LoRA split-K atomics: order-dependent
    for a, b in zip(res[True][1], res[False][1]):
        assert rel(a, b) < 1e-2


def test_llama_layer_flash_vs_sdpa_path():
    import lumen.models.llama as L
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model

    torch.manual_seed(0)
    m = build_model("llama2-7b", dtype=torch.bfloat16, device="meta")  # config only
    cfg = m.config
    cfg.num_hidden_layers = 2
    cfg.vocab_size = 1024
    model = L.LlamaForCausalLM(cfg, dtype=torch.bfloat16, device=DEV)
    model.init_weights(seed=1)
    apply_lora(model, LoraConfig(r=8, lora_dropout=0.0))
    for p in model.parameters():
        if p.requires_grad:
            p.data.normal_(0, 0.02)
    ids = torch.randint(3, 1024, (2, 256), device=DEV)
    labels = torch.full_like(ids, -100)
    labels[:, :-1] = ids[:, 1:]
    res = {}
    for flash in (True, False):
        L.USE_FLASH = flash
        model.zero_grad(set_to_none=True)
        loss = model(ids, labels, int((labels != -100).sum()))
        loss.backward()
        res[flash] = (loss.item(), [p.grad.clone() for p in model.parameters() if p.requires_grad])
    L.USE_FLASH = True
    assert abs(res[True][0] - res[False][0]) < 1e-2
    for a, b in zip(res[True][1], res[False][1]):
        assert rel(a, b) < 5e-2


@pytest.mark.gpu
def test_transposed_weight_backward_matches():
    """TN input-gradient path (cached W^T) gives the same dX / adapter grads as the NN path."""
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model
    from lumen.models.layers import configure_backward_layout

    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = build_model("tiny-llama", dtype=torch.bfloat16, device=dev)
    apply_lora(m, LoraConfig(r=8, lora_dropout=0.0))
    m.train()
    ids = torch.randint(3, m.config.vocab_size, (2, 64), device=dev)
    labels = torch.roll(ids, -1, 1)
    grads = []
    import os

    head = int(os.environ.get("LUMEN_LMHEAD_WT", "1") != "0")  # the LM head's W^T (TN dH)
    for pol in ("none", "all"):
        assert configure_backward_layout(m, pol) == (0 if pol == "none" else 8 + head)
        for p in m.parameters():
            p.grad = None
        loss = m(ids, labels=labels)
        loss.backward()
        grads.append({n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None})
    assert grads[0].keys() == grads[1].keys() and len(grads[0]) > 0
    for k in grads[0]:
        torch.testing.assert_close(grads[1][k], grads[0][k], rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("shape", [(4096, 12288), (11008, 4096), (72, 200), (136, 64)])
def test_transpose_2d(shape):
    from lumen.ops.transpose import transpose_2d

    x = torch.randn(*shape, device=DEV).to(torch.bfloat16)
    torch.testing.assert_close(transpose_2d(x), x.t().contiguous(), rtol=0, atol=0)


@pytest.mark.parametrize("direct,arena,ckpt", [(False, False, False), (True, True, False),
                                               (True, True, "full"), (True, True, "selective")])
def test_engine_lora_grad_paths_match(direct, arena, ckpt, monkeypatch):
    """Direct .grad accumulation + zero arena give the same training trajectory as the plain
    path (adapter grads returned to autograd, torch.zeros scratch); so do full per-layer
    recompute and selective recompute (gate|up output recomputed in the backward)."""
    import lumen.ops.lora as lora_mod
    from lumen.lora import LoraConfig, adapter_state_dict, apply_lora
    from lumen.models import build_model
    from lumen.parallel.dist import init
    from lumen.train.config import load_ds_config
    from lumen.train.engine import ZeroEngine

    def run(direct_, arena_, ckpt_=False):
        monkeypatch.setattr(lora_mod, "DIRECT_GRAD", direct_)
        monkeypatch.setattr(lora_mod, "USE_ARENA", arena_)
        torch.manual_seed(0)
        m = build_model("small-llama", dtype=torch.bfloat16, device=torch.device("cuda"), seed=3)
        apply_lora(m, LoraConfig(r=16, lora_dropout=0.1))
        m.gradient_checkpointing = ckpt_
        assert m.gradient_checkpointing == (ckpt_ or "none")
        m.train()
        env = init()
        ds = load_ds_config({"zero_optimization": {"stage": 1}}, 2, 2, 1, 1e-3)
        eng = ZeroEngine(m, ds, env)
        g = torch.Generator(device="cpu").manual_seed(5)
        for _ in range(6):
            ids = torch.randint(3, m.config.vocab_size, (2, 64), generator=g).cuda()
            labels = torch.roll(ids, -1, 1)
            loss = eng.forward({"input_ids": ids, "labels": labels})
            eng.backward(loss)
            eng.step()
        return adapter_state_dict(m)

    ref = run(False, False)
    got = run(direct, arena, ckpt)
    # the adapter reductions land with f32 atomics (order not fixed), and Adam's early steps move
    # an element by ~lr * sign(g): an element whose gradient is ~0 can differ by one lr step.
    # Everything else must agree tightly.
    lr = 1e-3
    for k in ref:
        d = (got[k].float() - ref[k].float()).abs()
        loose = d > 1e-5 + 1e-3 * ref[k].float().abs()
        assert loose.float().mean().item() < 0.02, (k, loose.float().mean().item())
        assert d.max().item() <= 2 * lr, (k, d.max().item())


@pytest.mark.parametrize("nh,nkv", [(8, 8), (8, 2)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_lora_linear_fused_rope(nh, nkv, dtype):
    """RoPE fused into the q|k adapter write-back == lora_linear followed by RoPE (fwd + grads)."""
    from lumen.ops.lora import lora_linear
    from lumen.ops.rope import rope_qkv_, rope_tables

    D, K, T, r = 128, 512, 320, 16
    N = (nh + 2 * nkv) * D
    segs = [(0, nh * D, 0, 0), (nh * D, nkv * D, 16, nh * D), ((nh + nkv) * D, nkv * D, 32, (nh + nkv) * D)]
    torch.manual_seed(0)
    x = torch.randn(T, K, device=DEV, dtype=dtype, requires_grad=True)
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(dtype)
    A = (torch.randn(48, K, device=DEV) / math.sqrt(K)).requires_grad_(True)
    B = (torch.randn(N, r, device=DEV) * 0.1).requires_grad_(True)
    cos, sin = rope_tables(D, 4096, 10000.0, DEV)
    pos = (torch.arange(T, device=DEV, dtype=torch.int32) * 7) % 1000
    y1 = lora_linear(x, lambda: W, None, A, B, segs, r, 2.0, 0.0, 0, rope=(pos, cos, sin, (nh + nkv) * D))
    x2, A2, B2 = (t.detach().clone().requires_grad_(True) for t in (x, A, B))
    y2 = rope_qkv_(lora_linear(x2, lambda: W, None, A2, B2, segs, r, 2.0, 0.0, 0), pos, nh, nkv, D,
                   cos, sin)
    assert rel(y1, y2) < 1e-2
    dy = torch.randn_like(y1)
    y1.backward(dy)
    y2.backward(dy.clone())
    for a, b in ((x.grad, x2.grad), (A.grad, A2.grad), (B.grad, B2.grad)):
        assert rel(a, b) < 2e-2


@pytest.mark.parametrize("M", [1, 2, 3, 4, 8, 16])
@pytest.mark.parametrize("N,K", [(4096, 4096), (12288, 4096), (4096, 11008), (1024, 11008)])
def test_skinny_gemm(M, N, K):
    """Weight-streaming decode GEMM (kernels/skinny_gemm.hip) vs an f32 reference."""
    from lumen.ops.gemm import linear_nt, skinny_ok

    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.02).to(torch.bfloat16)
    from lumen.ops._native import native

    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ref = x.float() @ w.float().t()
    for form in (0, 1):  # M = 1: row-group / rows-per-lane forms; M <= 4 VALU, M > 4 MFMA
        native().set_gemv_form(form)
        native().skinny_gemm(x, w, y)
        assert rel(y, ref) < 1e-2
    native().set_gemv_form(1)
    assert skinny_ok(x, w) == (M <= 2 or (M <= 4 and N <= 4096))
    y = linear_nt(x, w)
    ref = x.float() @ w.float().t()
    assert y.shape == (M, N) and rel(y, ref) < 1e-2
    # strided activation rows (a view into a wider buffer)
    xb = torch.randn(M, K + 128, device=DEV).to(torch.bfloat16)
    xv = xb[:, :K]
    yv = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    native().skinny_gemm(xv, w, yv)
    assert rel(yv, xv.float() @ w.float().t()) < 1e-2


@pytest.mark.parametrize("bm", [64, 128, 192, 256])
def test_decode_gemm_variants(bm):
    """Decode-batch MFMA GEMM (kernels/decode_gemm.hip) vs an f32 matmul: every compiled (BM, BN)
    variant, split-K 1 / 2 / 3 (in-launch slab reduction, counters left zeroed for the next
    launch), a ragged last column tile, M below the block height, strided x rows, fp16."""
    from lumen.ops._native import native
    from lumen.ops.gemm import DG_BNS, DG_BNS8, decode_gemm, dg_workspace

    g = torch.Generator(device="cpu").manual_seed(bm)
    K = 640
    for bn, nw in [(b, 4) for b in DG_BNS[bm]] + [(b, 8) for b in DG_BNS8.get(bm, ())]:
        for N in (3 * bn + 4 * 3, 2 * bn):        # ragged (N % BN != 0) and whole tiles
            w = (torch.randn(N, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
            for M in sorted({bm, bm - 11, 5 if bm == 64 else bm // 2 + 3}):
                xb = torch.randn(M, K + 64, generator=g).to(DEV, torch.bfloat16)
                x = xb[:, :K]                      # row stride K + 64
                ref = x.float() @ w.float().t()
                for s in (1, 2, 3):
                    y = decode_gemm(x, w, bm, bn, s, nw)
                    assert y.shape == (M, N)
                    assert rel(y, ref) < 1e-2, (bm, bn, nw, N, M, s, rel(y, ref))
                    if s > 1:  # the tile counters are zero again after the launch
                        assert int(dg_workspace(x.device)[1].abs().sum()) == 0
    # fp16 operands
    w = (torch.randn(256, K, generator=g) * 0.05).to(DEV, torch.float16)
    x = torch.randn(bm - 3, K, generator=g).to(DEV, torch.float16)
    y = decode_gemm(x, w, bm, DG_BNS[bm][0], 2)
    assert rel(y, x.float() @ w.float().t()) < 1e-2
    # a split-K GEMM on a side stream gets a workspace of its own
    main_ws = dg_workspace(x.device)[0].data_ptr()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        y2 = decode_gemm(x, w, bm, DG_BNS[bm][0], 2)
        assert dg_workspace(x.device)[0].data_ptr() != main_ws
    torch.cuda.current_stream().wait_stream(side)
    assert torch.equal(y2, y)
    # argument checks fail loudly (M above the block height)
    with pytest.raises(Exception):
        native().decode_gemm(torch.randn(bm + 1, K, device=DEV).to(torch.bfloat16),
                             w.to(torch.bfloat16), torch.empty(bm + 1, 256, device=DEV,
                                                               dtype=torch.bfloat16),
                             None, None, bm, DG_BNS[bm][0], 1, 4, 0)
    # k-rotated loop (flags 1) and the k-tiled x layout (flags 2, BM 256): same products
    from lumen.ops.gemm import x_ktiled

    w = (torch.randn(3 * 64 + 8, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
    for M in sorted({bm, bm - 11}):
        x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
        ref = x.float() @ w.float().t()
        for s in (1, 3):
            assert rel(decode_gemm(x, w, bm, DG_BNS[bm][0], s, 4, flags=1), ref) < 1e-2
            if bm == 256:
                xt = x_ktiled(x)
                for fl in (2, 3):
                    for bn, nw in ((64, 4), (128, 4), (64, 8), (128, 8)):
                        y = decode_gemm(xt, w, bm, bn, s, nw, flags=fl, m=M)
                        assert y.shape == (M, w.shape[0])
                        assert rel(y, ref) < 1e-2, (fl, bn, nw, s, M, rel(y, ref))


@pytest.mark.parametrize("N,K", [(12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008),
                                 (32000, 4096)])
@pytest.mark.parametrize("M", [64, 100, 200, 256])
def test_decode_gemm_planned_shapes(N, K, M):
    """linear_nt on the serving shapes of Llama-2-7B: the planned decode GEMM (or hipBLASLt where
    the plan table has no win) matches an f32 matmul."""
    from lumen.ops.gemm import dg_plan, linear_nt

    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.02).to(torch.bfloat16)
    y = linear_nt(x, w)
    assert rel(y, x.float() @ w.float().t()) < 1e-2, dg_plan(x, w)


@pytest.mark.parametrize("N,F", [(4096, 11008), (1024, 2752)])
def test_swiglu_down_projection(N, F):
    """Batch-1 MLP down projection of the serving path: SwiGLU kernel + weight-streaming GEMV ==
    the f32 reference (silu in f32, product rounded to bf16 as the kernel does)."""
    from lumen.ops.gemm import swiglu_linear_nt

    gu = torch.randn(1, 2 * F, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, F, device=DEV) * 0.02).to(torch.bfloat16)
    g, u = gu.float().chunk(2, -1)
    ref32 = (F_silu(g) * u).to(torch.bfloat16).float() @ w.float().t()
    assert rel(swiglu_linear_nt(gu, w), ref32) < 1e-2


def F_silu(x):
    return x * torch.sigmoid(x)


@pytest.mark.parametrize("nh,nkv", [(32, 32), (8, 2)])
def test_rope_write_kv_fused(nh, nkv):
    """Fused RoPE + paged KV-cache write == rope_inplace then write_kv_cache (bit-exact)."""
    from lumen.ops.attention import rope_write_kv, write_kv_cache
    from lumen.ops.rope import rope_inplace, rope_tables

    D, T, bs, nb = 128, 37, 16, 64
    qkv = torch.randn(T, (nh + 2 * nkv) * D + 8, device=DEV).to(torch.bfloat16)[:, :(nh + 2 * nkv) * D]
    pos = torch.randint(0, 900, (T,), device=DEV, dtype=torch.int32)
    cos, sin = rope_tables(D, 1024, 10000.0, DEV)
    slots = torch.randperm(nb * bs, device=DEV)[:T].to(torch.int64)
    slots[3] = -1  # padding row: no cache write
    kc = torch.zeros(nb, nkv, bs, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    q1 = qkv.clone()
    rope_write_kv(q1, pos, nh, nkv, D, cos, sin, kc, vc, slots)
    q2 = qkv.clone()
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
    rope_inplace(q2, pos, nh + nkv, D, cos, sin)
    qs, ks = nh * D, nkv * D
    write_kv_cache(q2[:, qs:qs + ks].view(T, nkv, D), q2[:, qs + ks:].view(T, nkv, D), kc2, vc2,
                   slots)
    assert torch.equal(q1, q2)
    assert torch.equal(kc, kc2) and torch.equal(vc, vc2)


@pytest.mark.parametrize("nh,nkv", [(32, 32), (16, 4)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_flash_attention_paged_prefill(nh, nkv, dtype):
    """Chunked / mixed prefill: queries of each chunk attend (causally, offset by the cached
    context) over K/V read from the paged cache through a shuffled block table."""
    from lumen.ops.attention import flash_attention_paged, flash_attention_paged_ref

    torch.manual_seed(0)
    D, bs = 128, 16
    # (cached context, chunk length): whole prompts, chunks after long contexts, 1-row chunks
    shapes = [(0, 512), (37, 100), (600, 200), (128, 1), (0, 7), (1000, 129)]
    nblocks = sum((c + n + bs - 1) // bs for c, n in shapes) + 8
    perm = torch.randperm(nblocks).tolist()
    kc = (torch.randn(nblocks, nkv, bs, D, device=DEV) * 0.5).to(dtype)
    vc = torch.randn(nblocks, nkv, bs, D, device=DEV).to(dtype)
    maxb = max((c + n + bs - 1) // bs for c, n in shapes)
    bt = torch.zeros(len(shapes), maxb, dtype=torch.int32, device=DEV)
    cu, kl, used = [0], [], 0
    for i, (c, n) in enumerate(shapes):
        nb = (c + n + bs - 1) // bs
        bt[i, :nb] = torch.tensor(perm[used:used + nb], dtype=torch.int32)
        used += nb
        cu.append(cu[-1] + n)
        kl.append(c + n)
    T = cu[-1]
    q = (torch.randn(T, (nh + 2 * nkv) * D, device=DEV) * 0.5).to(dtype)  # fused qkv rows
    got = flash_attention_paged(q, kc, vc, cu, kl, bt, nh, nkv, D)
    ref = flash_attention_paged_ref(q.float(), kc.float(), vc.float(), cu, kl, bt, nh, nkv, D)
    assert torch.isfinite(got.float()).all()
    assert rel(got, ref) < 1e-2


@pytest.mark.parametrize("D", [64, 96])
@pytest.mark.parametrize("nh,nkv", [(12, 12), (8, 2)])
def test_flash_attention_small_head_dim(D, nh, nkv):
    """Head dims below 128 (OPT-125m: 64) run the HIP kernels zero-padded to 128 with the true
    1/sqrt(D) scale: fwd + bwd vs the f32 reference."""
    from lumen.ops.attention import flash_attention_qkv, flash_attention_ref

    cu = [0, 77, 333, 512]
    T = cu[-1]
    qkv = (torch.randn(T, (nh + 2 * nkv) * D, device=DEV) * 0.5).to(torch.bfloat16)
    qkv.requires_grad_(True)
    o = flash_attention_qkv(qkv, cu, nh, nkv, D, True)
    q2 = qkv.detach().float().requires_grad_(True)
    o2 = flash_attention_ref(q2, tuple(cu), nh, nkv, D, True)
    assert o.shape == o2.shape and rel(o, o2) < 2e-2
    do = torch.randn_like(o)
    o.backward(do)
    o2.backward(do.float())
    assert rel(qkv.grad, q2.grad) < 3e-2


def test_opt_gpu_flash_matches_reference(monkeypatch):
    """OPT-125m (head dim 64) with the HIP flash attention == the same bf16 GPU model with the
    torch reference attention, for loss and LoRA gradients."""
    import lumen.models.opt as opt_mod
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model
    from lumen.ops.attention import flash_attention_qkv, flash_attention_ref

    torch.manual_seed(0)
    m = build_model("opt-125m", dtype=torch.bfloat16, device=torch.device("cuda"), init="random",
                    seed=4)
    apply_lora(m, LoraConfig(r=8, lora_dropout=0.0, target_modules=["q_proj", "v_proj"]))
    with torch.no_grad():
        for _, mod in m.lora_modules():
            mod.lora.lora_B.normal_(0, 0.02)
    m.train()
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(3, m.config.vocab_size, (2, 96), generator=g).cuda()
    labels = torch.roll(ids, -1, 1)
    outs = []
    for attn in (flash_attention_qkv, lambda qkv, cu, nh, nkv, D, c: flash_attention_ref(
            qkv.float(), tuple(cu), nh, nkv, D, c).to(qkv.dtype)):
        monkeypatch.setattr(opt_mod, "flash_attention_qkv", attn)
        m.zero_grad(set_to_none=True)
        loss = m(ids, labels)
        loss.backward()
        outs.append((loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters()
                                   if p.requires_grad}))
    (l1, g1), (l2, g2) = outs
    assert abs(l1 - l2) < 1e-2 * abs(l2)
    # bf16 attention-gradient rounding compounds through the backward: measured 2.3% at the last
    # layer growing smoothly to 8.5% at layer 0 of 12 (a kernel bug would show a step, not a ramp)
    rels = [rel(g1[n], g2[n]) for n in g1]
    assert rels[-1] < 3e-2 and max(rels) < 0.12, rels


@pytest.mark.parametrize("H", [768, 4096, 8192])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_embedding_gather(H, dtype):
    """HIP token-embedding gather == F.embedding (exact copy); out-of-range ids give zero rows."""
    import torch.nn.functional as F

    from lumen.ops._native import native
    from lumen.ops.embedding import embedding

    V = 1000
    W = torch.randn(V, H, device=DEV).to(dtype)
    ids = torch.randint(0, V, (3, 333), device=DEV)
    out = embedding(ids, W)
    assert out.shape == (3, 333, H)
    assert torch.equal(out, F.embedding(ids, W))
    bad = torch.tensor([0, V, -1, 5], device=DEV)
    o = torch.empty(4, H, device=DEV, dtype=dtype)
    native().embedding(W, bad, o)
    assert torch.equal(o[0], W[0]) and torch.equal(o[3], W[5])
    assert (o[1] == 0).all() and (o[2] == 0).all()


@pytest.mark.parametrize("nh,nkv,D", [(32, 32, 128), (64, 8, 128), (12, 12, 64)])
def test_fp8_kv_cache_kernels(nh, nkv, D):
    """fp8 (e4m3fn) KV cache: the cache-write kernels round like torch's float8_e4m3fn cast, and
    paged decode / chunked-prefill attention over the fp8 cache match the references computed
    on the same (dequantised) cache."""
    from lumen.ops.attention import (flash_attention_paged, flash_attention_paged_ref,
                                     paged_decode, paged_decode_ref, rope_write_kv,
                                     write_kv_cache)
    from lumen.ops.rope import rope_tables

    torch.manual_seed(0)
    f8 = torch.float8_e4m3fn
    bs, nseq, ctx = 16, 4, 300
    maxb = (ctx + bs - 1) // bs
    nblocks = nseq * maxb + 5
    kc = torch.zeros(nblocks, nkv, bs, D, device=DEV, dtype=f8)
    vc = torch.zeros_like(kc)
    perm = torch.randperm(nblocks)[: nseq * maxb].view(nseq, maxb).int().to(DEV)
    lens = torch.tensor([ctx, 17, 200, 129])
    for i in range(nseq):
        L = int(lens[i])
        k = torch.randn(L, nkv, D, device=DEV, dtype=torch.bfloat16) * 3
        v = torch.randn(L, nkv, D, device=DEV, dtype=torch.bfloat16)
        t = torch.arange(L, device=DEV)
        slots = perm[i, t // bs].long() * bs + t % bs
        write_kv_cache(k, v, kc, vc, slots)
        got_k = kc[perm[i, t // bs].long(), :, t % bs]
        assert (got_k.float() == k.to(f8).float()).float().mean().item() > 0.999
    q = torch.randn(nseq, nh, D, device=DEV, dtype=torch.bfloat16)
    cl = lens.int().to(DEV)
    scale = 1 / math.sqrt(D)
    o2 = paged_decode_ref(q, kc, vc, perm, cl, scale)
    for part in (512, 64):
        for one in (1, 2, 3):
            assert rel(paged_decode(q, kc, vc, perm, cl, ctx, scale, part, one_pass=one),
                       o2) < 1e-2, (one, part)
    if D == 128:  # chunked prefill over the fp8 cache (dequantised into the 16-bit scratch)
        cu, kl = [0, 20, 37, 137, 138], [300, 17, 200, 129]
        qr = (torch.randn(cu[-1], (nh + 2 * nkv) * D, device=DEV) * 0.5).to(torch.bfloat16)
        got = flash_attention_paged(qr, kc, vc, cu, kl, perm, nh, nkv, D)
        ref = flash_attention_paged_ref(qr.float(), kc, vc, cu, kl, perm, nh, nkv, D)
        assert rel(got, ref) < 1e-2
    # fused RoPE + fp8 cache write == RoPE + bf16 write, then cast
    T = 50
    qkv = torch.randn(T, (nh + 2 * nkv) * D, device=DEV, dtype=torch.bfloat16)
    pos = torch.randint(0, 400, (T,), device=DEV, dtype=torch.int32)
    slots = torch.arange(T, device=DEV, dtype=torch.int64) + 3 * bs
    cos, sin = rope_tables(D, 4096, 10000.0, DEV)
    k8, v8 = torch.zeros_like(kc), torch.zeros_like(vc)
    kb = torch.zeros(nblocks, nkv, bs, D, device=DEV, dtype=torch.bfloat16)
    vb = torch.zeros_like(kb)
    x1, x2 = qkv.clone(), qkv.clone()
    rope_write_kv(x1, pos, nh, nkv, D, cos, sin, k8, v8, slots)
    rope_write_kv(x2, pos, nh, nkv, D, cos, sin, kb, vb, slots)
    assert torch.equal(x1, x2)
    # rotated k goes f32 -> fp8 in the kernel, the reference f32 -> bf16 -> fp8: double rounding
    # moves ~0.1% of elements by one fp8 step
    assert (k8.float() == kb.to(f8).float()).float().mean().item() > 0.995
    assert (v8.float() == vb.to(f8).float()).float().mean().item() > 0.999


@pytest.mark.parametrize("p_drop", [0.0, 0.1])
def test_llama_lora_fold_matches_unfolded(p_drop, monkeypatch):
    """The K-extended forward ([x | Z | 0] [W | s B_bd | 0]^T GEMM, RMSNorm / flash attention
    writing into the extended operand, RoPE as its own pass) == the unfolded UP write-back:
    same loss and adapter gradients, and the folded path is really taken."""
    import lumen.ops.lora as lora_mod
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model

    torch.manual_seed(0)
    m = build_model("small-llama", dtype=torch.bfloat16, device=torch.device("cuda"), init="random",
                    seed=5)
    apply_lora(m, LoraConfig(r=16, lora_dropout=p_drop))
    with torch.no_grad():
        for _, mod in m.lora_modules():
            mod.lora.lora_B.normal_(0, 0.02)
    m.train()
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(3, m.config.vocab_size, (2, 200), generator=g).cuda()
    labels = torch.roll(ids, -1, 1)
    outs = []
    for fold in (True, False):
        monkeypatch.setattr(lora_mod, "FOLD", fold)
        m.zero_grad(set_to_none=True)
        torch.manual_seed(7)  # same dropout seeds on both passes
        loss = m(ids, labels)
        loss.backward()
        outs.append((loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters()
                                   if p.requires_grad}))
        if fold:
            assert all(mod._wext is not None for _, mod in m.lora_modules())
    (l1, g1), (l2, g2) = outs
    assert abs(l1 - l2) < 2e-3 * abs(l2)
    for n in g1:
        assert rel(g1[n], g2[n]) < 3e-2, n
    # an optimizer-style in-place update of lora_B refreshes the folded weight's tail
    monkeypatch.setattr(lora_mod, "FOLD", True)
    mod = next(mod for _, mod in m.lora_modules())
    w1 = mod.fold_weight().clone()
    with torch.no_grad():
        mod.lora.lora_B.add_(0.01)
    w2 = mod.fold_weight()
    K = mod.in_features
    assert torch.equal(w1[:, :K], w2[:, :K]) and not torch.equal(w1[:, K:], w2[:, K:])


@pytest.mark.parametrize("stage", [2, 3])
def test_engine_steps_refresh_fold_tail(stage):
    """The optimizer writes the adapters through the engine's flat buffer (views installed with
    ``p.data``, whose version counters do not see those writes): every publish must still
    refresh the folded weights' [s B] tail, so the forward after step k uses step k's lora_B
    (stage 2: the cached [W | s B] copy; stage 3 at world 1: the tail of the unit's own rows)."""
    import lumen.ops.lora as lora_mod
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model
    from lumen.parallel.dist import init
    from lumen.train.config import load_ds_config
    from lumen.train.engine import ZeroEngine

    assert lora_mod.FOLD
    torch.manual_seed(0)
    m = build_model("small-llama", dtype=torch.bfloat16, device=torch.device("cuda"), seed=3)
    apply_lora(m, LoraConfig(r=16, lora_dropout=0.0))
    m.train()
    eng = ZeroEngine(m, load_ds_config({"zero_optimization": {"stage": stage}}, 2, 1, 1, 1e-2),
                     init())
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(3, m.config.vocab_size, (2, 64), generator=g).cuda()
    for _ in range(3):
        loss = eng.forward({"input_ids": ids, "labels": torch.roll(ids, -1, 1)})
        eng.backward(loss)
        eng.step()
    loss = eng.forward({"input_ids": ids, "labels": torch.roll(ids, -1, 1)})
    eng.backward(loss)
    torch.cuda.synchronize()
    KP = lora_mod.FOLD_KP
    n = 0
    for _, mod in m.lora_modules():
        W, K = mod.weight, mod.in_features
        wext = (W.as_strided((W.shape[0], K + KP), (K + KP, 1)) if W.stride(0) == K + KP
                else mod._wext)
        if wext is None:
            continue
        want = torch.zeros(W.shape[0], K + KP, dtype=W.dtype, device=W.device)
        mod._fill_tail(want)
        assert want[:, K:].abs().sum() > 0  # lora_B moved off its zero init
        torch.testing.assert_close(wext[:, K:], want[:, K:], rtol=0, atol=0)
        n += 1
    assert n > 0
    # the engine's one-launch refresh (FoldTails, run at every publish) covers every folded linear
    assert eng.fold_tails.refresh() == n
    eng.close()


@pytest.mark.parametrize("p_drop", [0.0, 0.1])
def test_lora3_dxa_delta_handoff_kernel(p_drop):
    """The o_proj fused dA + dx kernel's delta output == rowsum(dO * O) per 128-column head,
    taken over the 16-bit dO it writes and the un-dropped O (fp32 reference)."""
    from lumen.ops import lora as L
    from lumen.ops._native import native

    dev = torch.device("cuda")
    T, K, R = 1000, 1024, 16
    g = torch.Generator(device=dev).manual_seed(11)
    ob = torch.randn(T, K + 64, device=dev, generator=g).bfloat16()  # fold operand buffer
    o = ob[:, :K]
    dx = torch.randn(T, K, device=dev, generator=g).bfloat16()
    dZ = torch.randn(T, R, device=dev, generator=g) * 0.1
    A = torch.randn(R, K, device=dev, generator=g) * 0.05
    dA = torch.zeros(R, K, device=dev)
    delta = torch.full((K // 128, T), float("nan"), device=dev)
    th = L.drop_threshold(p_drop)
    native().lora3_dxa(o, dx, dZ, A, dA, 128, 99, th, 1.0 / (1.0 - p_drop), K, 0, delta)
    torch.cuda.synchronize()
    ref = (dx.float() * o.float()).view(T, K // 128, 128).sum(-1).t()
    assert torch.allclose(delta, ref, atol=1e-3, rtol=1e-4), (delta - ref).abs().max()


@pytest.mark.gpu
def test_llama_delta_handoff_matches(monkeypatch):
    """Training step with the attention delta handed over by the o_proj backward == with the
    attention backward's own delta pass (loss and adapter gradients), and the hand-off is
    really taken in every layer."""
    import lumen.ops.attention as attn_mod
    import lumen.ops.lora as lora_mod
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model

    torch.manual_seed(0)
    m = build_model("small-llama", dtype=torch.bfloat16, device=torch.device("cuda"),
                    init="random", seed=5)
    apply_lora(m, LoraConfig(r=16, lora_dropout=0.05))
    with torch.no_grad():
        for _, mod in m.lora_modules():
            mod.lora.lora_B.normal_(0, 0.02)
    m.train()
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(3, m.config.vocab_size, (2, 256), generator=g).cuda()
    labels = torch.roll(ids, -1, 1)
    outs = []
    for on in (True, False):
        monkeypatch.setattr(lora_mod, "DELTA_HANDOFF", on)
        attn_mod.DELTA_HANDOFFS[0] = 0
        m.zero_grad(set_to_none=True)
        torch.manual_seed(7)
        loss = m(ids, labels)
        loss.backward()
        torch.cuda.synchronize()
        outs.append((loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters()
                                   if p.requires_grad}, attn_mod.DELTA_HANDOFFS[0]))
    (l1, g1, n1), (l2, g2, n2) = outs
    assert n1 == m.config.num_hidden_layers and n2 == 0
    assert abs(l1 - l2) <= 1e-6 * abs(l2)
    for n in g1:
        assert rel(g1[n], g2[n]) < 1e-2, n


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-llama-deep"])
def test_fp32_model_matches_cpu(name):
    """--dtype fp32 on the GPU (portable attention with the HIP split/RoPE kernel, head_dim 64 /
    32 with GQA; adapter products in torch) == the same weights on the CPU: loss and every
    adapter gradient to fp32 accuracy."""
    import copy

    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model

    cpu = build_model(name, dtype=torch.float32, device="cpu", init="random", seed=7)
    apply_lora(cpu, LoraConfig(r=4, lora_alpha=8, lora_dropout=0.0))
    for n, p in cpu.named_parameters():
        if "lora_B" in n:
            p.data.normal_(0, 0.02, generator=torch.Generator().manual_seed(len(n)))
    gpu = copy.deepcopy(cpu).to(DEV)
    ids = torch.randint(0, 500, (8, 16), generator=torch.Generator().manual_seed(3))
    lc = cpu(ids, labels=ids)
    lg = gpu(ids.to(DEV), labels=ids.to(DEV))
    lc, lg = (x[0] if isinstance(x, tuple) else x for x in (lc, lg))
    assert abs(float(lc) - float(lg)) < 1e-4 * abs(float(lc)), (float(lc), float(lg))
    lc.backward()
    lg.backward()
    gg = dict(gpu.named_parameters())
    n_checked = 0
    for n, p in cpu.named_parameters():
        if p.grad is None:
            continue
        assert rel(gg[n].grad, p.grad.to(DEV)) < 1e-3, n
        n_checked += 1
    assert n_checked > 0


def test_serving_prefill_projection_wave_split():
    """Serving prefill / mixed-step projections (``linear_nt`` at M = 2048 tokens) take the
    whole-wave column split where both parts are in the shipped TunableOp table (q|k|v 8192 +
    4096, gate|up 16384 + 5632 columns) and equal the single GEMM."""
    import lumen.ops.gemm as G
    from lumen.utils.gemm_tuning import load_tuned_gemms

    assert load_tuned_gemms(), "shipped TunableOp table did not load"
    G._plans.clear()
    for N, n1 in ((12288, 8192), (22016, 16384)):
        x = torch.randn(2048, 4096, device=DEV, dtype=torch.bfloat16)
        w = torch.randn(N, 4096, device=DEV, dtype=torch.bfloat16) * 0.02
        assert G._split_plan(x, w) == n1, N
        y = G.linear_nt(x, w)
        ref = x.float() @ w.float().t()
        assert rel(y, ref) < 1e-2
        assert torch.equal(y, G.mm_nt(x, w))


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("K", [11008, 1024])
def test_skinny_swiglu_gemm(M, K, monkeypatch):
    """Batch <= 4 decode down projection with SwiGLU formed inside the weight stream
    (kernels/skinny_gemm.hip, gemv_r4_kernel<SWIGLU>; opt-in LUMEN_SWIGLU_GEMV) vs an f32
    reference of swiglu + matmul."""
    import lumen.ops.gemm as G

    monkeypatch.setattr(G, "SWIGLU_GEMV", True)
    import torch.nn.functional as F
    from lumen.ops._native import native
    from lumen.ops.gemm import swiglu_linear_nt

    N = 4096
    gu = torch.randn(M, 2 * K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16)
    act = (F.silu(gu[:, :K].float()) * gu[:, K:].float()).to(torch.bfloat16).float()
    ref = act @ w.float().t()
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    native().skinny_swiglu_gemm(gu, w, y)
    assert rel(y, ref) < 1e-2
    assert rel(swiglu_linear_nt(gu, w), ref) < 1e-2


@pytest.mark.parametrize("M,N,K,dtype", [(4096, 22016, 4096, torch.bfloat16),
                                         (4096, 11008, 4096, torch.bfloat16),
                                         (300, 1024, 512, torch.bfloat16),
                                         (512, 2048, 1024, torch.float16)])
def test_mlp_gemm_plain_vs_fp32(M, N, K, dtype):
    """kernels/mlp_gemm.hip epi 0 (ping-pong LDS-DMA MFMA GEMM; the 22016 shape runs its last
    wave split in two k halves) against an fp32 matmul; partial last row tile at M = 300."""
    from lumen.ops.mlp_gemm import mlp_gemm

    g = torch.Generator(device="cpu").manual_seed(M + N)
    x = torch.randn(M, K, generator=g).to(dtype).to(DEV)
    w = (torch.randn(N, K, generator=g) * 0.02).to(dtype).to(DEV)
    c = torch.empty(M, N, device=DEV, dtype=dtype)
    mlp_gemm(0, x, w, c)
    ref = x.float() @ w.float().t()
    err = ((c.float() - ref).norm() / ref.norm()).item()
    assert err < 4e-3, err


@pytest.mark.parametrize("T,H,F", [(4096, 4096, 11008), (384, 512, 768)])
def test_mlp_gemm_swiglu_fwd_bwd_vs_fp32(T, H, F):
    """The fused SwiGLU epilogues against fp32 torch: forward gu = y @ [Wg | Wu]^T and
    act = silu(g) * u in one launch; backward dact = dout @ Wd (against Wd^T) with dg | du
    formed in the epilogue from the saved gu."""
    import torch.nn.functional as Fn

    from lumen.ops.mlp_gemm import mlp_gemm

    g = torch.Generator(device="cpu").manual_seed(T + F)
    y = torch.randn(T, H, generator=g).to(torch.bfloat16).to(DEV)
    wgu = (torch.randn(2 * F, H, generator=g) * 0.02).to(torch.bfloat16).to(DEV)
    gu = torch.empty(T, 2 * F, device=DEV, dtype=torch.bfloat16)
    act = torch.empty(T, F, device=DEV, dtype=torch.bfloat16)
    mlp_gemm(1, y, wgu, gu, act)
    ref = y.float() @ wgu.float().t()
    gr, ur = ref.chunk(2, dim=-1)
    assert ((gu.float() - ref).norm() / ref.norm()).item() < 4e-3
    ra = Fn.silu(gr) * ur
    assert ((act.float() - ra).norm() / ra.norm()).item() < 8e-3
    # backward from the kernel's own (bf16) gu, as training does
    dout = torch.randn(T, H, generator=g).to(torch.bfloat16).to(DEV)
    wdt = (torch.randn(F, H, generator=g) * 0.02).to(torch.bfloat16).to(DEV)   # Wd^T
    dgu = torch.empty(T, 2 * F, device=DEV, dtype=torch.bfloat16)
    mlp_gemm(2, dout, wdt, dgu, None, gu)
    g_ = gu.float()[:, :F].clone().requires_grad_(True)
    u_ = gu.float()[:, F:].clone().requires_grad_(True)
    (Fn.silu(g_) * u_).backward(dout.float() @ wdt.float().t())
    rd = torch.cat([g_.grad, u_.grad], dim=1)
    assert ((dgu.float() - rd).norm() / rd.norm()).item() < 8e-3


def test_mlp_gemm_split_tail_matches_unsplit():
    """The split last wave (two k halves, f32 slabs, last-arriver sum) gives the unsplit result
    up to f32 summation order, and leaves its ticket counters zeroed for the next launch."""
    from lumen.ops import mlp_gemm as mg

    M, N, K = 4096, 22016, 4096
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.02).to(torch.bfloat16)
    a = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    b = torch.empty_like(a)
    mg.mlp_gemm(0, x, w, a, split=True)
    mg.mlp_gemm(0, x, w, b, split=False)
    assert int(mg.native().mlp_gemm_split(M, N, K, 0, mg._cu_count(x.device))) > 0
    d = (a.float() - b.float()).abs().max().item()
    assert d <= 2e-2 * b.float().abs().max().item(), d
    for ws, cnt in mg._ws.values():
        assert int(cnt.abs().sum()) == 0


def test_fused_mlp_autograd_matches_unfused(monkeypatch):
    """LlamaMLP through _FusedMLP (LUMEN_FUSED_MLP=1: both fused GEMMs) against the default
    path (library GEMMs + SwiGLU passes): output and input gradient agree to bf16 rounding."""
    import dataclasses

    import lumen.ops.activation as act_mod
    import lumen.ops.mlp_gemm as mg
    from lumen.models.config import get_config
    from lumen.models.llama import LlamaMLP

    cfg = dataclasses.replace(get_config("small-llama"), intermediate_size=1536)
    torch.manual_seed(0)
    mlp = LlamaMLP(cfg, dtype=torch.bfloat16, device=DEV)
    for p in mlp.parameters():
        torch.nn.init.normal_(p, std=0.02)
    mlp.gate_up_proj.transpose_bwd = mlp.down_proj.transpose_bwd = True   # W^T, as in training
    x = torch.randn(512, cfg.hidden_size, device=DEV, dtype=torch.bfloat16)
    calls = []
    real = mg.mlp_gemm
    monkeypatch.setattr(mg, "mlp_gemm", lambda epi, *a, **k: (calls.append(epi), real(epi, *a, **k))[1])
    outs = {}
    for mode in ("0", "1"):
        monkeypatch.setattr(act_mod, "FUSED_MLP", mode)
        xi = x.clone().requires_grad_(True)
        y = mlp(xi)
        y.float().square().sum().backward()
        outs[mode] = (y.detach().float(), xi.grad.float())
    assert calls == [1, 2], calls   # both fused kernels ran in mode 1, none in mode 0
    for a, b in zip(outs["1"], outs["0"]):
        assert ((a - b).norm() / b.norm()).item() < 1e-2


@pytest.mark.parametrize("D", [32, 64, 128, 256])
@pytest.mark.parametrize("G", [1, 2, 4, 8])
def test_paged_decode_uniform_variants_all_shapes(D, G):
    """The uniform-block-id decode (LUMEN_PA_1PASS 2) and its pipelined inline-asm form (3) at
    the block size that enables them (256 / (D / 8) rows), every head size and GQA group: the
    pipelined form runs where scripts/tools/check_asm_loads.py passes (D = 128 or G = 1) and
    falls back to variant 2 elsewhere -- both must match the fp32 reference at several
    partition sizes."""
    from lumen.ops.attention import paged_decode, paged_decode_ref, write_kv_cache

    torch.manual_seed(D * 10 + G)
    bs = 256 // (D // 8)
    nkv = 2
    nh = nkv * G
    lens = torch.tensor([5 * bs + 3, 1, bs, 17 * bs - 1])
    nseq, ctx = len(lens), int(lens.max())
    maxb = (ctx + bs - 1) // bs
    nblocks = nseq * maxb + 2
    kc = torch.zeros(nblocks, nkv, bs, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    perm = torch.randperm(nblocks)[: nseq * maxb].view(nseq, maxb).int()
    for i in range(nseq):
        L = int(lens[i])
        t = torch.arange(L)
        slots = (perm[i, t // bs].long() * bs + t % bs).to(DEV)
        write_kv_cache(torch.randn(L, nkv, D, device=DEV, dtype=torch.bfloat16),
                       torch.randn(L, nkv, D, device=DEV, dtype=torch.bfloat16), kc, vc, slots)
    q = torch.randn(nseq, nh, D, device=DEV, dtype=torch.bfloat16)
    bt, cl = perm.to(DEV), lens.int().to(DEV)
    scale = 1 / math.sqrt(D)
    ref = paged_decode_ref(q, kc, vc, bt, cl, scale)
    for part in (bs, 4 * bs, 512 if 512 % bs == 0 else 8 * bs):
        for one in (2, 3):
            got = paged_decode(q, kc, vc, bt, cl, ctx, scale, part, one_pass=one)
            assert rel(got, ref) < 1e-2, (one, part)
