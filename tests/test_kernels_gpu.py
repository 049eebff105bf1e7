"""HIP kernel numerics vs the fp32 PyTorch reference of the same op (MI355X only)."""
import ctypes
import math

import numpy as np
import pytest
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.gguf import quants as Q
from nats_llm_studio_amd.gguf.constants import GGMLType

pytestmark = pytest.mark.gpu

TYPES = [GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K, GGMLType.Q8_0, GGMLType.F16, GGMLType.BF16, GGMLType.F32,
         # re-encoded at load (ops/transcode.py): Q51 device blocks, Q3_K -> Q6_K, Q2_K -> F16
         GGMLType.Q4_0, GGMLType.Q4_1, GGMLType.Q5_0, GGMLType.Q5_1, GGMLType.Q3_K, GGMLType.Q2_K]
NEW_TYPES = [GGMLType.Q4_0, GGMLType.Q4_1, GGMLType.Q5_0, GGMLType.Q5_1, GGMLType.Q3_K, GGMLType.Q2_K]


def _qw(rows, K, t, dev, seed=0):
    rng = np.random.default_rng(seed)
    raw = Q.random_blocks(t, rows * K, 0.05, rng)
    cpu = ops.QWeight(raw, t, rows, K, "cpu")
    return ops.QWeight(raw, t, rows, K, dev), cpu.dense()


def _x(M, K, dev, seed=1):
    g = torch.Generator().manual_seed(seed)
    pad = (M + 63) // 64 * 64
    x = torch.zeros(pad, K, dtype=ops.ACT_DTYPE)
    x[:M] = torch.randn(M, K, generator=g).to(ops.ACT_DTYPE)
    return x.to(dev)


def _close(a, b, rtol=2e-2):
    err = (a.float().cpu() - b.float().cpu()).abs().max().item()
    scale = b.float().abs().max().item() + 1e-6
    assert err <= rtol * scale, f"max err {err} vs scale {scale}"


CFGS = [(0, 8, 1, 1), (0, 4, 2, 1), (1, 8, 1, 1), (1, 4, 2, 2), (1, 8, 1, 4)]


@pytest.mark.parametrize("t", TYPES)
@pytest.mark.parametrize("M", [1, 7, 16, 33, 64])
@pytest.mark.parametrize("cfg", CFGS)
def test_qgemv_types(gpu, t, M, cfg):
    rows, K = 200, 1024
    w, Wd = _qw(rows, K, t, gpu)
    x = _x(M, K, gpu)
    y = torch.zeros(64, rows, device=gpu)
    mode, waves, rt, ks = cfg
    ops.qgemv([ops.Seg(w)], x, y, M, mode=mode, waves=waves, rt=rt, ks=ks)
    ref = x[:M].float().cpu() @ Wd.t()
    _close(y[:M], ref)


def test_dequant_kernel_exact(gpu):
    """Register dequant (f16 magic-number path) vs the numpy ggml codec: f16 rounding only
    (one rounding of d*sc*q - dmin*m; cancellation bounded by the row scale)."""
    for t in TYPES:
        w, Wd = _qw(48, 512, t, gpu, seed=3)
        d = w.dense().float().cpu()
        torch.testing.assert_close(d, Wd, rtol=2e-3, atol=2e-3 * Wd.abs().max().item())


@pytest.mark.parametrize("t", NEW_TYPES)
@pytest.mark.parametrize("M", [65, 300])
def test_new_types_large_m_and_dense(gpu, t, M):
    """The load-time re-encoded formats at prefill sizes: path-B GEMM (mode 1, split-K), and the dense
    f16 copy (the dequant kernel of the device format) through mode 10 -- vs the fp32 product of the
    numpy ggml decode of the ORIGINAL bytes."""
    rows, K = 200, 1024
    w, Wd = _qw(rows, K, t, gpu)
    x = _x(M, K, gpu)
    ref = x[:M].float().cpu() @ Wd.t()
    y = torch.zeros(x.shape[0], rows, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y, M, mode=1, waves=8, rt=1, ks=2)
    _close(y[:M], ref)
    y.zero_()
    ops.qgemv([ops.Seg(w)], x, y, M)                      # automatic launch config
    _close(y[:M], ref)
    w.expand_dense()
    y.zero_()
    ops.qgemv([ops.Seg(w)], x, y, M, mode=10, waves=8, rt=1, ks=1)
    _close(y[:M], ref)


def test_q51_mixed_with_q6k_q8_segments(gpu):
    """A Q4_0 model's fused launch: Q51 (re-encoded Q4_0 / Q5_1) segments next to Q6_K and Q8_0 ones in
    ONE launch (kernel type-set 3)."""
    K = 512
    a, Ad = _qw(64, K, GGMLType.Q4_0, gpu, 1)
    b, Bd = _qw(48, K, GGMLType.Q6_K, gpu, 2)
    c, Cd = _qw(32, K, GGMLType.Q5_1, gpu, 3)
    d, Dd = _qw(16, K, GGMLType.Q8_0, gpu, 4)
    assert ops.kernel_set([a.type, b.type, c.type, d.type]) == 3
    for M in (3, 40):
        x = _x(M, K, gpu)
        y = torch.zeros(64, 160, device=gpu)
        ops.qgemv([ops.Seg(a, 0), ops.Seg(b, 64), ops.Seg(c, 112), ops.Seg(d, 144)], x, y, M)
        _close(y[:M], x[:M].float().cpu() @ torch.cat([Ad, Bd, Cd, Dd]).t())


@pytest.mark.parametrize("cfg", CFGS)
def test_qgemv_multiseg_add_argmax(gpu, cfg):
    mode, waves, rt, ks = cfg
    K = 768
    a, Ad = _qw(64, K, GGMLType.Q4_K, gpu, 1)
    b, Bd = _qw(40, K, GGMLType.Q6_K, gpu, 2)     # rows not a multiple of 16
    c, Cd = _qw(32, K, GGMLType.Q8_0, gpu, 3)
    M = 5
    x = _x(M, K, gpu)
    base = torch.randn(64, 136, device=gpu)
    y = base.clone()
    ops.qgemv([ops.Seg(a, 0), ops.Seg(b, 64)], x, y, M, alpha=0.5, epi="add", waves=waves, rt=rt, mode=mode, ks=ks)
    ops.qgemv([ops.Seg(c, 104)], x, y, M, alpha=0.5, epi="add", waves=waves, rt=rt, mode=mode, ks=ks)
    W = torch.cat([Ad, Bd, Cd])
    ref = base[:M].cpu() + 0.5 * (x[:M].float().cpu() @ W.t())
    _close(y[:M], ref)
    # fused argmax on a single segment
    keys = torch.zeros(64, dtype=torch.int64, device=gpu)
    logits = torch.zeros(64, 40, device=gpu)
    ops.qgemv([ops.Seg(b)], x, logits, M, argmax=keys, waves=waves, rt=rt, mode=mode, ks=ks)
    ids = torch.zeros(64, dtype=torch.int32, device=gpu)
    ops.argmax_unpack(keys, M, ids)
    assert ids[:M].cpu().tolist() == logits[:M].argmax(1).cpu().tolist()


@pytest.mark.parametrize("cfg", CFGS)
def test_qgemv_swiglu(gpu, cfg):
    mode, waves, rt, ks = cfg
    K, F = 512, 256
    rng = np.random.default_rng(5)
    g_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    u_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    raw = ops.interleave_gate_up(g_raw, u_raw, GGMLType.Q4_K, F, K)
    w = ops.QWeight(raw, GGMLType.Q4_K, 2 * F, K, gpu)
    G = torch.from_numpy(Q.dequantize(g_raw, 12, (F, K)))
    U = torch.from_numpy(Q.dequantize(u_raw, 12, (F, K)))
    for M in (1, 20):
        x = _x(M, K, gpu)
        y = torch.zeros(64, F, dtype=ops.ACT_DTYPE, device=gpu)
        ops.qgemv([ops.Seg(w)], x, y, M, epi="swiglu", mode=mode, waves=waves, rt=rt, ks=ks)
        xf = x[:M].float().cpu()
        ref = torch.nn.functional.silu(xf @ G.t()) * (xf @ U.t())
        _close(y[:M], ref, 3e-2)


def test_qgemv_mapped_rows(gpu):
    """MoE-style: per-segment x/y row maps and a device row count (0 -> tile skipped)."""
    K = 512
    w0, W0 = _qw(32, K, GGMLType.Q4_K, gpu, 7)
    w1, W1 = _qw(32, K, GGMLType.Q4_K, gpu, 8)
    x = _x(6, K, gpu)
    xm0 = torch.tensor([4, 1, 0, 0], dtype=torch.int32, device=gpu)
    ym0 = torch.tensor([0, 3, 0, 0], dtype=torch.int32, device=gpu)
    c0 = torch.tensor([2], dtype=torch.int32, device=gpu)
    c1 = torch.tensor([0], dtype=torch.int32, device=gpu)
    y = torch.full((64, 32), 7.0, device=gpu)
    ops.qgemv([ops.Seg(w0, 0, xm0, ym0, c0), ops.Seg(w1, 0, xm0, ym0, c1)], x, y, 6)
    xf = x.float().cpu()
    _close(y[0], xf[4] @ W0.t())
    _close(y[3], xf[1] @ W0.t())
    assert (y[1].cpu() == 7.0).all()


@pytest.mark.parametrize("T,rt,qt,mode,waves", [(200, 2, GGMLType.Q4_K, 2, 8), (300, 4, GGMLType.Q5_K, 2, 8),
                                                (150, 1, GGMLType.Q6_K, 2, 8), (200, 2, GGMLType.Q4_K, 5, 8),
                                                (300, 4, GGMLType.Q5_K, 4, 16), (150, 2, GGMLType.Q6_K, 4, 8),
                                                (200, 2, GGMLType.Q4_K, 1, 8), (300, 2, GGMLType.Q5_K, 1, 8),
                                                (150, 1, GGMLType.Q6_K, 1, 4), (40, 2, GGMLType.Q5_K, 1, 8),
                                                (200, 6, GGMLType.Q4_K, 3, 4), (300, 4, GGMLType.Q5_K, 3, 4),
                                                (150, 6, GGMLType.Q6_K, 3, 4), (40, 4, GGMLType.Q5_K, 3, 4),
                                                (300, 8, GGMLType.Q5_K, 3, 4)])
def test_qgemm_mapped_moe(gpu, T, rt, qt, mode, waves):
    """Grouped MoE GEMM (mapped rows; mode 1 = path B register dequant with per-block active tiles,
    mode 2 = LDS dequant, mode 3 = LDS-DMA of the raw blocks with the DMA gathering the routed rows (rt 4 / 6: the
    64 / 96-row two-workgroups-per-CU blocks), modes 4/5 = dense DMA GEMM on the experts' f16 copies): one route over T tokens, SwiGLU
    gate/up and f32 down over every expert in one launch each, against the per-row fp32 reference."""
    E, k, K, F = 4, 2, 512, 256
    logits = torch.randn(T, E, device=gpu)
    cap = T
    topw = torch.zeros(T * k, device=gpu)
    counts = torch.zeros(E, dtype=torch.int32, device=gpu)
    xrows = torch.zeros(E * cap, dtype=torch.int32, device=gpu)
    yrows = torch.zeros(E * cap, dtype=torch.int32, device=gpu)
    ops.moe_route(logits, T, k, topw, counts, xrows, yrows, cap)
    rng = np.random.default_rng(9)
    gus, G, U = [], [], []
    for e in range(E):
        g_raw = Q.random_blocks(qt, F * K, 0.05, rng)
        u_raw = Q.random_blocks(qt, F * K, 0.05, rng)
        gus.append(ops.QWeight(ops.interleave_gate_up(g_raw, u_raw, qt, F, K), qt, 2 * F, K, gpu))
        G.append(ops.QWeight(g_raw, qt, F, K, "cpu").dense())
        U.append(ops.QWeight(u_raw, qt, F, K, "cpu").dense())
    dns = [_qw(K, F, qt, gpu, 40 + e) for e in range(E)]
    if mode >= 4:
        for w in gus + [d[0] for d in dns]:
            w.expand_dense()
    x = _x(T, K, gpu)
    act = torch.zeros(T * k, F, dtype=ops.ACT_DTYPE, device=gpu)
    yexp = torch.full((T * k, K), 5.0, device=gpu)
    cfg = dict(mode=mode, waves=waves, rt=rt, ks=1)
    segs = [ops.Seg(gus[e], 0, xrows[e * cap:], yrows[e * cap:], counts[e:e + 1]) for e in range(E)]
    ops.qgemv(segs, x, act, T, epi="swiglu", **cfg)
    segs = [ops.Seg(dns[e][0], 0, yrows[e * cap:], yrows[e * cap:], counts[e:e + 1]) for e in range(E)]
    ops.qgemv(segs, act, yexp, T, epi="f32", **cfg)
    # mapped split-K (the MoE down projection at many tokens): slabs by y row, launch M = T*k rows
    yks = torch.full((T * k, K), 7.0, device=gpu)
    ops.qgemv(segs, act, yks, T * k, epi="f32", mode=mode, waves=waves, rt=rt, ks=3)
    torch.cuda.synchronize()
    _close(yks, yexp, 1e-3)
    cnt, xr, yr = counts.cpu(), xrows.cpu(), yrows.cpu()
    assert int(cnt.sum()) == T * k and sorted(yr[e * cap + i].item() for e in range(E)
                                              for i in range(int(cnt[e]))) == list(range(T * k))
    xf = x.float().cpu()
    for e in range(E):
        n = int(cnt[e])
        xi, yi = xr[e * cap:e * cap + n].long(), yr[e * cap:e * cap + n].long()
        ref = torch.nn.functional.silu(xf[xi] @ G[e].t()) * (xf[xi] @ U[e].t())
        _close(act[yi], ref, 3e-2)
        _close(yexp[yi], act[yi].float().cpu() @ dns[e][1].t(), 3e-2)


def test_rmsnorm_embed(gpu):
    x = torch.randn(5, 1024, device=gpu)
    w = torch.randn(1024, device=gpu)
    out = torch.zeros(64, 1024, dtype=ops.ACT_DTYPE, device=gpu)
    ops.rmsnorm(x, w, out, 5, 1e-5)
    ref = x * torch.rsqrt(x.pow(2).mean(1, keepdim=True) + 1e-5) * w
    _close(out[:5], ref, 1e-2)
    for t in TYPES:
        raw = Q.random_blocks(t, 50 * 512, 0.05, np.random.default_rng(11))
        qw = ops.QWeight(raw, t, 50, 512, gpu, layout="rows")
        Wd = ops.QWeight(raw, t, 50, 512, "cpu").dense()
        ids = torch.tensor([0, 49, 7], dtype=torch.int32, device=gpu)
        e = torch.zeros(3, 512, device=gpu)
        ops.embed(ids, qw, e, 3, 2.0)
        # Q4_1 / Q5_1 / Q2_K embedding tables are kept as f16 rows (ops/transcode.py device_form, "rows"):
        # one f16 rounding of the exact value; every other type gathers exactly
        f16_rows = qw.type == int(GGMLType.F16) and t != GGMLType.F16
        torch.testing.assert_close(e.cpu(), 2.0 * Wd[[0, 49, 7]], rtol=1e-3 if f16_rows else 1e-5,
                                   atol=1e-5 if f16_rows else 1e-6)


@pytest.mark.parametrize("kvt", [torch.bfloat16, torch.float8_e4m3fn])
@pytest.mark.parametrize("neox", [False, True])
def test_rope_kv(gpu, neox, kvt):
    """RoPE + paged KV append (bf16 or fp8 e4m3 cache: the CPU path rounds the same values)."""
    T, Hq, Hkv, D = 3, 8, 2, 128
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=gpu)
    pos = torch.tensor([0, 5, 100], dtype=torch.int32, device=gpu)
    slot = torch.tensor([3, -1, 7], dtype=torch.int32, device=gpu)
    cs = ops.rope_table(256, D, 10000.0, gpu)
    outs = []
    for dev in (gpu, "cpu"):
        q = torch.zeros(T, Hq * D, dtype=torch.bfloat16, device=dev)
        kc = torch.zeros(16, Hkv, D, dtype=kvt, device=dev)
        vc = torch.zeros_like(kc)
        ops.rope_kv(qkv.to(dev), pos.to(dev), slot.to(dev), cs.to(dev), q, kc, vc, T, Hq, Hkv, D, neox)
        outs.append((q.cpu().float(), kc.cpu().float(), vc.cpu().float()))
    tol = 1e-2 if kvt == torch.bfloat16 else 7e-2      # e4m3: 3 mantissa bits (rounding may differ by 1 ulp)
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, rtol=tol, atol=tol)
    if kvt != torch.bfloat16:
        assert outs[0][1].abs().sum() > 0 and float(outs[0][1][[0, 1, 2, 4]].abs().max()) == 0.0


@pytest.mark.parametrize("D,G", [(128, 4), (64, 4), (128, 8), (128, 1), (128, 7), (64, 6), (128, 5)])
@pytest.mark.parametrize("n_split,chunk", [(1, 0), (4, 0), (32, 0), (8, -16), (3, 512)])
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("kvt", [torch.bfloat16, torch.float8_e4m3fn])
def test_attention_paged(gpu, D, G, n_split, chunk, fused, kvt):
    """fused: flash-decoding splits merged in-kernel by the last split (ticket counters), called twice
    to check the counters re-arm; else the separate combine kernel. kvt: bf16 or fp8 e4m3 cache (the
    fp32 reference reads the same rounded values)."""
    if kvt != torch.bfloat16 and (G not in (1, 4) or chunk == 512):
        pytest.skip("fp8 cache: a representative subset")
    Hkv = 2
    Hq = Hkv * G
    bs = 16
    ctx = [1, 17, 300, 0, 64, 1500]
    T = len(ctx)
    nblk = 256
    g = torch.Generator().manual_seed(0)
    kc = torch.randn(nblk * bs, Hkv, D, generator=g).to(kvt)
    vc = torch.randn(nblk * bs, Hkv, D, generator=g).to(kvt)
    bt = torch.zeros(T, 100, dtype=torch.int32)
    for i in range(T):
        bt[i] = torch.randperm(nblk, generator=g)[:100].to(torch.int32)
    q = torch.randn(T, Hq * D, generator=g).to(torch.bfloat16)
    ts = torch.arange(T, dtype=torch.int32)
    cl = torch.tensor(ctx, dtype=torch.int32)
    ref = torch.zeros(T, Hq * D, dtype=ops.ACT_DTYPE)
    ops.attention(q, kc, vc, bt, ts, cl, ref, T, Hq, Hkv, D, bs, D ** -0.5)
    cnt = torch.zeros(T * Hkv, dtype=torch.int32, device=gpu) if fused else None
    for _ in range(2 if fused else 1):
        out = torch.zeros(T, Hq * D, dtype=ops.ACT_DTYPE, device=gpu)
        ops.attention(q.to(gpu), kc.to(gpu), vc.to(gpu), bt.to(gpu), ts.to(gpu), cl.to(gpu), out, T, Hq, Hkv, D, bs,
                      D ** -0.5, chunk=chunk, n_split=n_split, counters=cnt)
        torch.testing.assert_close(out.cpu().float(), ref.float(), rtol=2e-2, atol=2e-2)
    if fused:
        assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("G", [4, 8, 1, 7])
@pytest.mark.parametrize("n_split,fused", [(1, False), (4, True), (3, False)])
@pytest.mark.parametrize("kvt", [torch.bfloat16, torch.float8_e4m3fn])
@pytest.mark.parametrize("D", [128, 64])
def test_attention_decode_mfma(gpu, G, n_split, fused, kvt, D):
    """The MFMA decode kernel (one wave per workgroup once batch x kv heads x splits >= 1K workgroups; D = 128,
    and since round 6 D = 64 -- Granite-3.0): G query heads as MFMA columns, V^T through transposed LDS reads;
    contexts around the 32-key groups (0, 1, 31, 32, 33, ...), flash-decoding splits with the fused or the
    separate combine, bf16 and fp8 caches."""
    if kvt != torch.bfloat16 and G not in (4, 1):
        pytest.skip("fp8 cache: a representative subset")
    Hkv, bs, nblk = 8, 16, 512
    Hq = Hkv * G
    ctx = [0, 1, 31, 32, 33, 100, 300, 777] * 16
    T = len(ctx)
    g = torch.Generator().manual_seed(1)
    kc = torch.randn(nblk * bs, Hkv, D, generator=g).to(kvt)
    vc = torch.randn(nblk * bs, Hkv, D, generator=g).to(kvt)
    bt = torch.stack([torch.randperm(nblk, generator=g)[:64] for _ in range(T)]).to(torch.int32)
    q = torch.randn(T, Hq * D, generator=g).to(torch.bfloat16)
    ts = torch.arange(T, dtype=torch.int32)
    cl = torch.tensor(ctx, dtype=torch.int32)
    ref = torch.zeros(T, Hq * D, dtype=ops.ACT_DTYPE)
    ops.attention(q, kc, vc, bt, ts, cl, ref, T, Hq, Hkv, D, bs, D ** -0.5)
    cnt = torch.zeros(T * Hkv, dtype=torch.int32, device=gpu) if fused else None
    for _ in range(2 if fused else 1):
        out = torch.zeros(T, Hq * D, dtype=ops.ACT_DTYPE, device=gpu)
        ops.attention(q.to(gpu), kc.to(gpu), vc.to(gpu), bt.to(gpu), ts.to(gpu), cl.to(gpu), out, T, Hq, Hkv, D, bs,
                      D ** -0.5, chunk=0, n_split=n_split, counters=cnt)
        torch.testing.assert_close(out.cpu().float(), ref.float(), rtol=2e-2, atol=2e-2)
    if fused:
        assert int(cnt.abs().sum()) == 0


def test_argmax_kernel(gpu):
    lg = torch.randn(3, 128256, device=gpu)
    lg[1, 777] = 100.0
    out = torch.zeros(3, dtype=torch.int32, device=gpu)
    ops.argmax(lg, 3, out)
    assert out.cpu().tolist() == lg.argmax(1).cpu().tolist()


def test_embed_prev_and_argmax_rearm(gpu):
    """Chained decode: the embedding launch picks next_ids[t] where use_prev[t] (and writes the choice back
    to ids); the arg-max unpack with rearm zeroes the keys it read (no reset launch before the next step)."""
    raw = Q.random_blocks(GGMLType.Q6_K, 40 * 256, 0.05, np.random.default_rng(3))
    qw = ops.QWeight(raw, GGMLType.Q6_K, 40, 256, gpu, layout="rows")
    Wd = ops.QWeight(raw, GGMLType.Q6_K, 40, 256, "cpu").dense()
    ids = torch.tensor([1, 2, 3, 4], dtype=torch.int32, device=gpu)
    nxt = torch.tensor([10, 20, 30, 39], dtype=torch.int32, device=gpu)
    use = torch.tensor([0, 1, 0, 1], dtype=torch.int32, device=gpu)
    e = torch.zeros(4, 256, device=gpu)
    ops.embed(ids, qw, e, 4, 1.0, prev=(nxt, use))
    assert ids.cpu().tolist() == [1, 20, 3, 39]
    torch.testing.assert_close(e.cpu(), Wd[[1, 20, 3, 39]], rtol=1e-5, atol=1e-6)
    lg = torch.randn(4, 4096)
    ref = lg.argmax(1)
    # the packed key the fused lm-head arg-max leaves for each row's winner (u32 order-preserving float bits
    # << 32 | ~index), written as int64 bit patterns
    u = lg.max(1).values.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    u = torch.where(u >= 2 ** 31, 0xFFFFFFFF - u, u + 2 ** 31)
    packed = [int(((int(a) << 32) | (0xFFFFFFFF - int(b))) - (1 << 64 if int(a) >= 2 ** 31 else 0))
              for a, b in zip(u, ref)]
    dk = torch.zeros(8, dtype=torch.int64, device=gpu)
    dk[:4] = torch.tensor(packed, dtype=torch.int64)
    out = torch.zeros(8, dtype=torch.int32, device=gpu)
    ops.argmax_unpack(dk, 4, out, rearm=True)
    assert out[:4].cpu().tolist() == ref.tolist()
    assert int(dk.abs().sum()) == 0


def test_moe_route(gpu):
    T, E, k = 10, 8, 2
    lg = torch.randn(T, E, device=gpu)
    topw = torch.zeros(T * k, device=gpu)
    counts = torch.zeros(E, dtype=torch.int32, device=gpu)
    xr = torch.zeros(E * 64, dtype=torch.int32, device=gpu)
    yr = torch.zeros(E * 64, dtype=torch.int32, device=gpu)
    ops.moe_route(lg, T, k, topw, counts, xr, yr, 64)
    p = torch.softmax(lg, -1)
    w, e = torch.topk(p, k, -1)
    w = w / w.sum(-1, keepdim=True)
    torch.testing.assert_close(topw.view(T, k), w, rtol=1e-5, atol=1e-6)
    assert counts.sum().item() == T * k
    c = counts.cpu()
    for ex in range(E):
        toks = sorted(xr[ex * 64:ex * 64 + c[ex]].cpu().tolist())
        assert toks == sorted([t for t in range(T) if ex in e[t].tolist()])


@pytest.mark.parametrize("T,E,D", [(1, 8, 4096), (3, 8, 4096), (4, 4, 1024), (2, 2, 768)])
def test_moe_norm_route_fused(gpu, T, E, D):
    """One launch = RMSNorm -> f16 h, router logits h . Wr[e], top-2 route; vs the fp32 oracle of each part
    and vs the unfused kernels' routing (the same experts, weights and row lists)."""
    k, cap = 2, 16
    g = torch.Generator().manual_seed(T * 100 + E)
    x = (torch.randn(cap, D, generator=g) * 3).to(gpu)
    nw = (torch.rand(D, generator=g) + 0.5).to(gpu)
    wr = (torch.randn(E, D, generator=g) * 0.05).to(torch.float16).to(gpu)
    outs = []
    for fused in (True, False):
        h = torch.zeros(cap, D, dtype=ops.ACT_DTYPE, device=gpu)
        lg = torch.zeros(cap, E, device=gpu)
        topw = torch.zeros(cap * k, device=gpu)
        counts = torch.full((E,), 7, dtype=torch.int32, device=gpu)     # stale counts: zeroed in-kernel
        xr = torch.full((E * cap,), -1, dtype=torch.int32, device=gpu)
        yr = torch.full((E * cap,), -1, dtype=torch.int32, device=gpu)
        sel = torch.full((cap * k,), -1, dtype=torch.int32, device=gpu)
        if fused:
            assert ops.moe_norm_route(x, nw, 1e-5, wr, h, lg, T, k, topw, counts, xr, yr, cap, sel=sel)
        else:
            ops.rmsnorm(x, nw, h, T, 1e-5)
            lg[:T] = h[:T].float() @ wr.float().t()
            ops.moe_route(lg, T, k, topw, counts, xr, yr, cap, sel=sel)
        torch.cuda.synchronize()
        outs.append((h.cpu(), lg.cpu(), topw.cpu(), counts.cpu(), xr.cpu(), yr.cpu(), sel.cpu()))
    xs = x[:T].cpu()
    href = xs * torch.rsqrt(xs.pow(2).mean(1, keepdim=True) + 1e-5) * nw.cpu()
    _close(outs[0][0][:T], href, 1e-2)
    _close(outs[0][1][:T], outs[0][0][:T].float() @ wr.float().cpu().t(), 1e-3)
    assert (outs[0][0][T:] == 0).all()
    torch.testing.assert_close(outs[0][2], outs[1][2], rtol=1e-5, atol=1e-6)
    assert torch.equal(outs[0][3], outs[1][3]) and int(outs[0][3].sum()) == T * k
    assert torch.equal(outs[0][6], outs[1][6])
    for ex in range(E):
        c = int(outs[0][3][ex])
        assert sorted(outs[0][4][ex * cap:ex * cap + c].tolist()) == sorted(outs[1][4][ex * cap:ex * cap + c].tolist())
        assert sorted(outs[0][5][ex * cap:ex * cap + c].tolist()) == sorted(outs[1][5][ex * cap:ex * cap + c].tolist())
    lgs = torch.zeros(cap, E)
    assert not ops.moe_norm_route(x, nw, 1e-5, wr, torch.zeros(cap, D, dtype=ops.ACT_DTYPE, device=gpu),
                                  lgs.to(gpu), 5, k, topw, counts, xr, yr, cap)      # > 4 tokens: not taken


@pytest.mark.parametrize("T,E,D", [(1, 8, 4096), (5, 8, 4096), (257, 8, 4096), (2048, 8, 4096), (7, 4, 1024),
                                   (33, 2, 768)])
def test_router_logits(gpu, T, E, D):
    """ops.router_logits (the E-row router kernel of MoE prefill / large decode batches) vs the fp32 product of
    the same f16 operands; rows past T untouched."""
    g = torch.Generator().manual_seed(T + E)
    cap = T + 3
    h = (torch.randn(cap, D, generator=g)).to(ops.ACT_DTYPE).to(gpu)
    wr = (torch.randn(E, D, generator=g) * 0.05).to(torch.float16).to(gpu)
    lg = torch.full((cap, E), 7.0, device=gpu)
    counts = torch.full((E,), 5, dtype=torch.int32, device=gpu)
    ops.router_logits(h, wr, lg, T, zero=counts)          # the next route's expert counts, zeroed in-launch
    torch.cuda.synchronize()
    ref = h[:T].float().cpu() @ wr.float().cpu().t()
    _close(lg[:T], ref, 1e-3)
    assert (lg[T:] == 7.0).all()
    assert (counts.cpu() == 0).all()


def test_moe_route_nan_rows_stay_in_bounds(gpu):
    """A router row of NaN / inf logits must still pick k distinct valid experts (no index -1)."""
    T, E, k, cap = 6, 8, 2, 64
    lg = torch.randn(T, E, device=gpu)
    lg[1] = float("nan")
    lg[2, 3] = float("inf")
    lg[3, :4] = float("-inf")
    lg[4, 5] = float("nan")
    topw = torch.zeros(T * k, device=gpu)
    counts = torch.zeros(E, dtype=torch.int32, device=gpu)
    xr = torch.full((E * cap + 64,), -7, dtype=torch.int32, device=gpu)   # guard tail: never written
    yr = torch.full((E * cap + 64,), -7, dtype=torch.int32, device=gpu)
    ops.moe_route(lg, T, k, topw, counts, xr, yr, cap)
    torch.cuda.synchronize()
    c = counts.cpu()
    assert c.sum().item() == T * k and (c >= 0).all()
    assert (xr[E * cap:] == -7).all() and (yr[E * cap:] == -7).all()
    seen = {t: [] for t in range(T)}
    for ex in range(E):
        for t in xr[ex * cap:ex * cap + c[ex]].cpu().tolist():
            seen[t].append(ex)
    assert all(len(v) == k and len(set(v)) == k for v in seen.values()), seen


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2])
def test_oneshot_allreduce_simulated(gpu, world):
    """The one-shot IPC all-reduce protocol with W ranks as W concurrent streams on one GPU
    (W=2: with GPU_MAX_HW_QUEUES=4 more simulated ranks can share a hardware queue and then
    serialise, which the bounded spin reports as a timeout rather than a hang):
    every rank must get the rank-ordered fp32 sum (of values rounded to 30 bits: 2-bit epoch tags),
    bit-identical across ranks, over calls of varying size -- small calls skip most slot blocks, so a
    later call of the same parity must not take a stale granule (per-block epochs, blocks written whole)."""
    from nats_llm_studio_amd.parallel.oneshot import SimulatedGroup
    cap = 1 << 16
    g = SimulatedGroup(world, cap, gpu)
    try:
        for it, n in enumerate([4096, 100, 65536, 8, 4096 * 3, 4096, 64, 65536, 8, 65536, 4096]):
            xs = [torch.randn(n, device=gpu) for _ in range(world)]
            ref = xs[0].clone()
            for r in range(1, world):
                ref = ref + xs[r]
            g.all_reduce(xs)
            torch.cuda.synchronize()
            assert int(g.err.item()) == 0, f"timeout at call {it}"
            for r in range(world):
                assert torch.equal(xs[r], xs[0])
            torch.testing.assert_close(xs[0], ref, rtol=1e-6, atol=1e-5)
        assert not any(g.err_words())
    finally:
        g.close()


@pytest.mark.parametrize("world,rows,D", [(2, 1, 4096), (2, 3, 8192), (2, 16, 4096), (2, 5, 2048),
                                          (8, 1, 8192), (8, 16, 8192), (8, 64, 8192), (4, 7, 5120)])
def test_oneshot_allreduce_addnorm_simulated(gpu, world, rows, D):
    """Fused TP decode epilogue (one launch, each row over D/256 workgroups, the last to arrive at the
    row ticket normalises): x += sum of the ranks' partials in rank order, then h = f16(rmsnorm(x) * w)
    -- vs the fp32 reference, bit-identical x and h across ranks; repeated with a varying row count to
    exercise both epoch parities, per-slice epochs and the per-row ticket reset. World 8, D 8192, rows
    1/16/64 is the Llama-3-70B TP=8 decode regime."""
    from nats_llm_studio_amd.parallel.oneshot import SimulatedGroup
    g = SimulatedGroup(world, 1 << 20, gpu)
    try:
        nw = (1 + 0.1 * torch.randn(D, device=gpu)).float()
        for it, rr in enumerate([rows, max(1, rows // 2), rows, rows]):
            base = torch.randn(rr, D, device=gpu)
            parts = torch.randn(world, rr, D, device=gpu)
            xs = base.unsqueeze(0).repeat(world, 1, 1).contiguous()
            hs = torch.zeros(world, rr, D, dtype=ops.ACT_DTYPE, device=gpu)
            g.add_norm(parts, xs, nw, hs, rr, 1e-5)
            torch.cuda.synchronize()
            assert int(g.err.item()) == 0, f"timeout at call {it}"
            ref = base + parts.sum(0)
            href = ref * torch.rsqrt(ref.pow(2).mean(1, keepdim=True) + 1e-5) * nw
            for r in range(1, world):
                assert torch.equal(xs[0], xs[r]) and torch.equal(hs[0], hs[r])
            torch.testing.assert_close(xs[0], ref, rtol=1e-5, atol=1e-5)
            _close(hs[0], href, 1e-2)
        assert not any(g.err_words())
    finally:
        g.close()


def test_oneshot_timeout_raises_every_rank(gpu):
    """Fault injection: rank 0 runs its fused add+norm while its peer never arrives. The bounded spin
    gives up, the kernel returns (no GPU hang) and raises the error word of EVERY rank -- which the
    engine reads with each decode step's tokens -- and OneShot's local flag."""
    from nats_llm_studio_amd.parallel.oneshot import SimulatedGroup
    g = SimulatedGroup(2, 1 << 16, gpu)
    try:
        D = 4096
        x = torch.randn(2, D, device=gpu)
        h = torch.zeros(2, D, dtype=ops.ACT_DTYPE, device=gpu)
        g.add_norm_rank(0, torch.randn(2, D, device=gpu), x, torch.ones(D, device=gpu), h, 2, 1e-5, max_spins=2000)
        torch.cuda.synchronize()
        assert int(g.err.item()) == 1
        w = g.err_words()                   # [rank0 buf, rank0 nbuf, rank1 buf, rank1 nbuf]
        assert w[1] == 1 and w[3] == 1, w
    finally:
        g.close()


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q5_K, GGMLType.Q8_0, GGMLType.BF16])
@pytest.mark.parametrize("M", [65, 128, 200, 300])
@pytest.mark.parametrize("wr", [(8, 1, 1), (4, 2, 1), (8, 1, 3)])
def test_qgemm_large_m(gpu, t, M, wr):
    """Large-M MFMA GEMM (prefill / big decode batches): 128-row activation blocks, XCD-grouped
    weight tiles, partial last block; plain store, residual add and fused argmax."""
    rows, K = 264, 768
    w, Wd = _qw(rows, K, t, gpu)
    x = _x(M, K, gpu)
    pad = x.shape[0]
    y = torch.zeros(pad, rows, device=gpu)
    waves, rt, ks = wr
    keys = torch.zeros(pad, dtype=torch.int64, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y, M, mode=1, waves=waves, rt=rt, ks=ks, argmax=keys)
    ref = x[:M].float().cpu() @ Wd.t()
    _close(y[:M], ref)
    assert float(y[M:].abs().max().cpu()) == 0.0 if M < pad else True
    ids = torch.zeros(pad, dtype=torch.int32, device=gpu)
    ops.argmax_unpack(keys, M, ids)
    assert (ids[:M].cpu() == y[:M].argmax(1).cpu().to(torch.int32)).float().mean() > 0.99
    base = torch.randn(pad, rows, device=gpu)
    y2 = base.clone()
    ops.qgemv([ops.Seg(w)], x, y2, M, alpha=0.5, epi="add", mode=1, waves=waves, rt=rt, ks=ks)
    _close(y2[:M], base[:M].cpu() + 0.5 * ref)


def test_qgemm_large_m_swiglu(gpu):
    K, F = 512, 256
    rng = np.random.default_rng(9)
    g_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    u_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    w = ops.QWeight(ops.interleave_gate_up(g_raw, u_raw, GGMLType.Q4_K, F, K), GGMLType.Q4_K, 2 * F, K, gpu)
    G = torch.from_numpy(Q.dequantize(g_raw, 12, (F, K)))
    U = torch.from_numpy(Q.dequantize(u_raw, 12, (F, K)))
    M = 333
    x = _x(M, K, gpu)
    y = torch.zeros(x.shape[0], F, dtype=ops.ACT_DTYPE, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y, M, epi="swiglu", mode=1, waves=8, rt=1, ks=1)
    xf = x[:M].float().cpu()
    y3 = torch.zeros_like(y)
    ops.qgemv([ops.Seg(w)], x, y3, M, epi="swiglu", mode=1, waves=8, rt=1, ks=2)
    _close(y3[:M], y[:M].cpu(), 1e-2)
    _close(y[:M], torch.nn.functional.silu(xf @ G.t()) * (xf @ U.t()), 3e-2)


@pytest.mark.parametrize("kvt", [torch.bfloat16, torch.float8_e4m3fn])
@pytest.mark.parametrize("D,G", [(128, 4), (64, 4), (128, 8)])
def test_attention_prefill_paged(gpu, D, G, kvt):
    """MFMA flash-prefill vs the fp32 reference: 3 sequences, chunks that start mid-context
    (chunked prefill), partial 16-token blocks, scattered KV pages."""
    torch.manual_seed(0)
    Hkv, bs = 2, 16
    Hq = Hkv * G
    # (seq, pos0, n): seq 0 fresh 37 tokens, seq 1 continues at 100 for 20, seq 2 at 5 for 16
    chunks = [(0, 0, 37), (1, 100, 20), (2, 5, 16)]
    nblk = 16
    perm = torch.randperm(3 * nblk).view(3, nblk).int()
    slots = 3 * nblk * bs
    kc = (torch.randn(slots, Hkv, D) * 0.5).to(kvt)
    vc = torch.randn(slots, Hkv, D).to(kvt)
    T = sum(n for _, _, n in chunks)
    pos, tseq = [], []
    for s, p0, n in chunks:
        pos += list(range(p0, p0 + n))
        tseq += [s] * n
    pos = np.array(pos, np.int32)
    tseq = np.array(tseq, np.int32)
    q = (torch.randn(T, Hq * D)).to(torch.bfloat16)
    ctx = torch.from_numpy(pos + 1)
    ref = torch.zeros(T, Hq * D, dtype=ops.ACT_DTYPE)
    ops.attention(q, kc, vc, perm, torch.from_numpy(tseq), ctx, ref, T, Hq, Hkv, D, bs, D ** -0.5)
    qb = ops.prefill_blocks(tseq, pos, T)
    out = torch.zeros(T, Hq * D, dtype=ops.ACT_DTYPE, device=gpu)
    ops.attention_prefill(q.to(gpu), kc.to(gpu), vc.to(gpu), perm.to(gpu), torch.from_numpy(qb).to(gpu), len(qb),
                          None, None, out, T, Hq, Hkv, D, bs, D ** -0.5)
    _close(out.cpu(), ref, 2e-2)


def test_sample_kernel(gpu):
    """GPU sampler vs its definition: greedy == argmax, top_k=1 == argmax, draws stay inside
    top-k / top-p sets with the right frequencies, penalties applied on distinct history ids,
    seeded draws reproducible."""
    from nats_llm_studio_amd.engine.sampling import SamplingParams, sample_rows_gpu
    torch.manual_seed(0)
    V = 5000
    base = torch.randn(1, V)           # planted top-3 well above the rest (max of 5000 N(0,1) ~ 3.7)
    base[0, 123] = 9.0
    base[0, 456] = 8.5
    base[0, 789] = 8.0
    n = 2000
    lg = base.repeat(n, 1).to(gpu)
    greedy = sample_rows_gpu(lg[:4].clone(), [SamplingParams()] * 4, [[]] * 4, [None] * 4)
    assert greedy == [123] * 4
    k1 = sample_rows_gpu(lg[:4].clone(), [SamplingParams(temperature=1.0, top_k=1)] * 4, [[]] * 4, [None] * 4)
    assert k1 == [123] * 4
    p = SamplingParams(temperature=1.0, top_k=3)
    toks = sample_rows_gpu(lg.clone(), [p] * n, [[]] * n, [None] * n)
    assert set(toks) <= {123, 456, 789}
    pr = torch.softmax(torch.tensor([9.0, 8.5, 8.0]), 0)
    freq = torch.tensor([toks.count(t) for t in (123, 456, 789)], dtype=torch.float32) / n
    assert (freq - pr).abs().max() < 0.05, (freq, pr)
    tp = sample_rows_gpu(lg[:64].clone(), [SamplingParams(temperature=1.0, top_p=0.3)] * 64, [[]] * 64, [None] * 64)
    assert set(tp) == {123}
    pen = sample_rows_gpu(lg[:2].clone(), [SamplingParams(repeat_penalty=100.0)] * 2, [[123, 123], [5]],
                          [None] * 2)
    assert pen == [456, 123]
    g1 = [torch.Generator().manual_seed(7) for _ in range(8)]
    g2 = [torch.Generator().manual_seed(7) for _ in range(8)]
    pp = [SamplingParams(temperature=1.5)] * 8
    assert sample_rows_gpu(lg[:8].clone(), pp, [[]] * 8, g1) == sample_rows_gpu(lg[:8].clone(), pp, [[]] * 8, g2)


@pytest.mark.parametrize("params", [dict(temperature=0.7, top_p=0.95, top_k=40),       # the reference payload
                                    dict(temperature=1.0, top_k=5),
                                    dict(temperature=0.9, top_k=256, top_p=0.8, min_p=0.02),
                                    dict(temperature=1.1, top_k=40, repeat_penalty=1.3, presence_penalty=0.2),
                                    dict(temperature=0.8, top_k=300, top_p=0.9)])          # past the fast path
def test_sample_kernel_matches_cpu_twin(gpu, params):
    """GPU sampler (csrc/kernels/sample.hip; top_k <= 256 takes the compacted fast path) vs the CPU twin
    (engine/sampling.py sample_rows, float64 sort-based): same variate per row -> the same token, apart
    from rows whose variate lands within float rounding of a CDF step."""
    from nats_llm_studio_amd.engine.sampling import SamplingParams, sample_rows, sample_rows_gpu
    g = torch.Generator().manual_seed(3)
    n, V = 256, 32000
    lg = torch.randn(n, V, generator=g) * 2.5
    us = [float(u) for u in torch.rand(n, generator=g)]
    hist = [[int(t) for t in torch.randint(0, V, (12,), generator=g)] for _ in range(n)]
    ps = [SamplingParams(**params)] * n
    want = sample_rows(lg.clone(), ps, hist, us)
    got = sample_rows_gpu(lg.clone().to(gpu), ps, hist, us)
    same = sum(a == b for a, b in zip(want, got))
    assert same >= n - 2, (same, [(a, b) for a, b in zip(want, got) if a != b][:8])


def test_sample_top_k_with_masked_logits(gpu):
    """-inf entries (a logit-bias / grammar mask) do not widen top-k: the histogram search spans the
    finite logits only, so every draw stays inside the k largest finite logits."""
    from nats_llm_studio_amd.engine.sampling import SamplingParams, sample_rows_gpu
    torch.manual_seed(1)
    V = 6000
    base = torch.randn(1, V)
    base[0, ::2] = float("-inf")
    base[0, 101] = 7.0
    base[0, 303] = 6.8
    base[0, 505] = 6.6
    n = 512
    lg = base.repeat(n, 1).to(gpu)
    toks = sample_rows_gpu(lg, [SamplingParams(temperature=1.0, top_k=3)] * n, [[]] * n, [None] * n)
    assert set(toks) <= {101, 303, 505} and len(set(toks)) == 3, sorted(set(toks))


def test_sample_and_embed_never_emit_wild_ids(gpu):
    """A non-finite logit row (all NaN / -inf) still yields an id inside the vocabulary from both the
    greedy and the sampling branch, and the embedding gather clamps ids: chained decode feeds sampled
    ids back on the device, so neither may turn into an out-of-range address."""
    from nats_llm_studio_amd.engine.sampling import SamplingParams, sample_rows_gpu
    V = 3000
    lg = torch.full((4, V), float("nan"), device=gpu)
    lg[2:] = float("-inf")
    ps = [SamplingParams(), SamplingParams(temperature=0.7, top_p=0.95, top_k=40)] * 2
    toks = sample_rows_gpu(lg, ps, [[]] * 4, [None] * 4)
    assert all(0 <= t < V for t in toks), toks
    raw = Q.random_blocks(GGMLType.Q4_K, 50 * 512, 0.05, np.random.default_rng(11))
    qw = ops.QWeight(raw, GGMLType.Q4_K, 50, 512, gpu, layout="rows")
    Wd = ops.QWeight(raw, GGMLType.Q4_K, 50, 512, "cpu").dense()
    ids = torch.tensor([-1, 50, 1 << 30, 3], dtype=torch.int32, device=gpu)
    e = torch.zeros(4, 512, device=gpu)
    ops.embed(ids, qw, e, 4)
    torch.cuda.synchronize()
    torch.testing.assert_close(e.cpu(), Wd[[0, 49, 49, 3]], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("M,cfg", [(5, (1, 8, 1, 4)), (64, (1, 4, 1, 2)), (200, (1, 8, 1, 3)), (200, (1, 8, 1, 1)),
                                   (7, (0, 4, 1, 1)), (256, (2, 8, 4, 4)), (130, (2, 8, 2, 2)),
                                   (1, (0, 8, 1, 1)), (3, (0, 4, 2, 1)), (8, (0, 8, 2, 1))])
@pytest.mark.parametrize("ticket", [False, True])
def test_qgemv_add_rmsnorm_fused(gpu, M, cfg, ticket):
    """Row-parallel projection + residual + next RMSNorm (split-K slabs reduced by the fused kernel;
    few-row path A with `ticket`: the norm runs in the GEMV's last workgroup, repeated to check the
    counter re-arms)."""
    D, K = 512, 768
    w, Wd = _qw(D, K, GGMLType.Q4_K, gpu, 11)
    xin = _x(M, K, gpu)
    pad = xin.shape[0]
    base = torch.randn(pad, D, device=gpu)
    nw = (1 + 0.1 * torch.randn(D)).to(gpu)
    cnt = torch.zeros(4, dtype=torch.int32, device=gpu) if ticket else None
    xr = base[:M].cpu() + 0.7 * (xin[:M].float().cpu() @ Wd.t())
    hr = xr * torch.rsqrt(xr.pow(2).mean(1, keepdim=True) + 1e-5) * nw.cpu()
    for _ in range(3 if ticket else 1):
        x = base.clone()
        h = torch.zeros(pad, D, dtype=ops.ACT_DTYPE, device=gpu)
        ops.qgemv_add_rmsnorm(ops.Seg(w), xin, x, nw, h, M, 0.7, 1e-5, cfg=cfg, counter=cnt)
        _close(x[:M], xr)
        _close(h[:M], hr, 3e-2)
    if ticket:
        assert int(cnt.abs().sum()) == 0


def test_lm_head_argmax_only_epilogue(gpu):
    """Greedy decode: arg-max keys without writing logits."""
    K, V = 512, 1000
    w, Wd = _qw(V, K, GGMLType.Q6_K, gpu, 12)
    for M, cfg in ((3, (0, 4, 1, 1)), (40, (1, 8, 1, 2)), (150, (1, 8, 1, 1)), (256, (2, 8, 4, 1))):
        x = _x(M, K, gpu)
        y = torch.full((x.shape[0], V), 7.0, device=gpu)
        keys = torch.zeros(x.shape[0], dtype=torch.int64, device=gpu)
        mode, waves, rt, ks = cfg
        ops.qgemv([ops.Seg(w)], x, y, M, epi="argmax", argmax=keys, mode=mode, waves=waves, rt=rt, ks=ks)
        ids = torch.zeros(x.shape[0], dtype=torch.int32, device=gpu)
        ops.argmax_unpack(keys, M, ids)
        ref = (x[:M].float().cpu() @ Wd.t()).argmax(1)
        assert (ids[:M].cpu().long() == ref).float().mean() > 0.98
        assert bool((y == 7.0).all())


@pytest.mark.parametrize("cfg", [(1, 8, 1, 2), (1, 8, 1, 3), (0, 4, 1, 1), (2, 8, 4, 2), (2, 8, 2, 1), (0, 8, 2, 1),
                                 (0, 8, 1, 1)])
@pytest.mark.parametrize("M", [1, 3, 16, 70, 256])
@pytest.mark.parametrize("bias", [False, True])
def test_qkv_rope_kv_fused(gpu, cfg, M, bias):
    """QKV projection (3 segments) + RoPE + KV append: path A rotates in the GEMV epilogue, split-K
    launches sum their slabs inside the RoPE kernel. `bias`: Qwen2 QKV bias added before rotating."""
    _qkv_rope_case(gpu, cfg, M, bias, dense=False)


@pytest.mark.parametrize("cfg", [(4, 16, 2, 1), (4, 16, 4, 1), (5, 8, 4, 1), (10, 8, 1, 1), (10, 8, 1, 2), (10, 8, 2, 1),
                                 ])
@pytest.mark.parametrize("M", [70, 300, 520])
@pytest.mark.parametrize("bias", [False, True])
def test_qkv_rope_kv_dense(gpu, cfg, M, bias):
    """The dense GEMMs on the weights' f16 copies (modes 4/5/10) with the RoPE + KV-append epilogue (split-K 1:
    lane pairs rotated in registers; split-K 2: slabs summed by the RoPE kernel). M = 300: the Q|K|V copies as one
    buffer (QWeight.expand_dense_group: one merged launch segment, as the model loads them)."""
    _qkv_rope_case(gpu, cfg, M, bias, dense=True)


def _qkv_rope_case(gpu, cfg, M, bias, dense):
    Hq, Hkv, D, K = 4, 2, 128, 512
    wq, Wq = _qw(Hq * D, K, GGMLType.Q4_K, gpu, 21)
    wk, Wk = _qw(Hkv * D, K, GGMLType.Q4_K, gpu, 22)
    wv, Wv = _qw(Hkv * D, K, GGMLType.Q6_K, gpu, 23)
    if dense and M == 300:
        assert ops.QWeight.expand_dense_group([wq, wk, wv]) == (Hq + 2 * Hkv) * D * K * 2
        assert wk.d16.data_ptr() == wq.d16.data_ptr() + Hq * D * K * 2
    elif dense:        # the f16 copies ARE the dequantised values the references multiply with
        for w in (wq, wk, wv):
            w.expand_dense()
    segs = [ops.Seg(wq, 0), ops.Seg(wk, Hq * D), ops.Seg(wv, (Hq + Hkv) * D)]
    x = _x(M, K, gpu)
    pad = x.shape[0]
    cs = ops.rope_table(4 * pad, D, 10000.0, gpu)
    pos = torch.arange(pad, dtype=torch.int32, device=gpu) * 3
    slot = torch.arange(pad, dtype=torch.int32, device=gpu)
    qkv = torch.zeros(pad, (Hq + 2 * Hkv) * D, device=gpu)
    bv = torch.randn((Hq + 2 * Hkv) * D, device=gpu) if bias else None
    outs = []
    for c in (cfg, None):
        q = torch.zeros(pad, Hq * D, dtype=torch.bfloat16, device=gpu)
        kc = torch.zeros(pad, Hkv, D, dtype=torch.bfloat16, device=gpu)
        vc = torch.zeros_like(kc)
        if c is None:       # reference: plain GEMM then the rope kernel on the CPU path
            qkv_ref = x[:M].float().cpu() @ torch.cat([Wq, Wk, Wv]).t()
            qc, kcc, vcc = q.cpu(), kc.cpu(), vc.cpu()
            ops.rope_kv(qkv_ref, pos.cpu(), slot.cpu(), cs.cpu(), qc, kcc, vcc, M, Hq, Hkv, D,
                        bias=None if bv is None else bv.cpu())
            outs.append((qc, kcc, vcc))
        else:
            ops.qkv_rope_kv(segs, x, qkv, pos, slot, cs, q, kc, vc, M, Hq, Hkv, D, cfg=c, bias=bv)
            outs.append((q.cpu(), kc.cpu(), vc.cpu()))
    for a, b in zip(outs[0], outs[1]):
        _close(a[:M], b[:M], 3e-2)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q5_K, GGMLType.Q8_0])
@pytest.mark.parametrize("M", [65, 256, 300, 520])
@pytest.mark.parametrize("wm,ks", [(4, 1), (2, 1), (4, 3)])
def test_qgemm_lds(gpu, t, M, wm, ks):
    """Large-M LDS-dequant GEMM (mode 2): weight tile dequantised once into LDS and shared by
    8 waves; partial last 128-row weight tile and activation block; store, add, argmax."""
    rows, K = 264, 768
    w, Wd = _qw(rows, K, t, gpu)
    x = _x(M, K, gpu)
    pad = x.shape[0]
    y = torch.zeros(pad, rows, device=gpu)
    keys = torch.zeros(pad, dtype=torch.int64, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y, M, mode=2, waves=8, rt=wm, ks=ks, argmax=keys)
    ref = x[:M].float().cpu() @ Wd.t()
    _close(y[:M], ref)
    assert float(y[M:].abs().max().cpu()) == 0.0 if M < pad else True
    ids = torch.zeros(pad, dtype=torch.int32, device=gpu)
    ops.argmax_unpack(keys, M, ids)
    assert (ids[:M].cpu() == y[:M].argmax(1).cpu().to(torch.int32)).float().mean() > 0.99
    base = torch.randn(pad, rows, device=gpu)
    y2 = base.clone()
    ops.qgemv([ops.Seg(w)], x, y2, M, alpha=0.5, epi="add", mode=2, waves=8, rt=wm, ks=ks)
    _close(y2[:M], base[:M].cpu() + 0.5 * ref)


@pytest.mark.parametrize("ks", [1, 2])
def test_qgemm_lds_swiglu_multiseg(gpu, ks):
    """Mode 2 with the SwiGLU epilogue, and a Q|K|V-style multi-segment (Q4_K, Q4_K, Q6_K) launch."""
    K, F = 512, 256
    rng = np.random.default_rng(9)
    g_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    u_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    w = ops.QWeight(ops.interleave_gate_up(g_raw, u_raw, GGMLType.Q4_K, F, K), GGMLType.Q4_K, 2 * F, K, gpu)
    G = torch.from_numpy(Q.dequantize(g_raw, 12, (F, K)))
    U = torch.from_numpy(Q.dequantize(u_raw, 12, (F, K)))
    M = 333
    x = _x(M, K, gpu)
    y = torch.zeros(x.shape[0], F, dtype=ops.ACT_DTYPE, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y, M, epi="swiglu", mode=2, waves=8, rt=4, ks=ks)
    xf = x[:M].float().cpu()
    _close(y[:M], torch.nn.functional.silu(xf @ G.t()) * (xf @ U.t()), 3e-2)
    a, Ad = _qw(256, K, GGMLType.Q4_K, gpu, 1)
    b, Bd = _qw(128, K, GGMLType.Q4_K, gpu, 2)
    c, Cd = _qw(128, K, GGMLType.Q6_K, gpu, 3)
    yq = torch.zeros(x.shape[0], 512, device=gpu)
    ops.qgemv([ops.Seg(a, 0), ops.Seg(b, 256), ops.Seg(c, 384)], x, yq, M, mode=2, waves=8, rt=4, ks=ks)
    _close(yq[:M], xf @ torch.cat([Ad, Bd, Cd]).t())


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q5_K])
@pytest.mark.parametrize("M", [65, 256, 300, 520])
@pytest.mark.parametrize("mt,ks", [(16, 1), (8, 1), (16, 3), (8, 2), (6, 1), (6, 2), (4, 1), (4, 3)])
def test_qgemm_dma(gpu, t, M, mt, ks):
    """Large-M LDS-DMA GEMM (mode 3): activation quarters and raw weight tile-blocks arrive by
    global_load_lds, weights dequantised per wave in registers; partial last 128-row weight tile and
    activation block, K slices with 1..n super-blocks; store, add, argmax."""
    rows, K = 264, 768
    w, Wd = _qw(rows, K, t, gpu)
    x = _x(M, K, gpu)
    pad = x.shape[0]
    y = torch.zeros(pad, rows, device=gpu)
    keys = torch.zeros(pad, dtype=torch.int64, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y, M, mode=3, waves=4, rt=mt, ks=ks, argmax=keys)
    ref = x[:M].float().cpu() @ Wd.t()
    _close(y[:M], ref)
    assert float(y[M:].abs().max().cpu()) == 0.0 if M < pad else True
    ids = torch.zeros(pad, dtype=torch.int32, device=gpu)
    ops.argmax_unpack(keys, M, ids)
    assert (ids[:M].cpu() == y[:M].argmax(1).cpu().to(torch.int32)).float().mean() > 0.99
    base = torch.randn(pad, rows, device=gpu)
    y2 = base.clone()
    ops.qgemv([ops.Seg(w)], x, y2, M, alpha=0.5, epi="add", mode=3, waves=4, rt=mt, ks=ks)
    _close(y2[:M], base[:M].cpu() + 0.5 * ref)


@pytest.mark.parametrize("ks", [1, 2])
def test_qgemm_dma_swiglu_multiseg(gpu, ks):
    """Mode 3 with the SwiGLU epilogue, and a Q|K|V-style multi-segment (Q4_K, Q4_K, Q6_K) launch."""
    K, F = 1024, 384
    rng = np.random.default_rng(9)
    g_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    u_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    w = ops.QWeight(ops.interleave_gate_up(g_raw, u_raw, GGMLType.Q4_K, F, K), GGMLType.Q4_K, 2 * F, K, gpu)
    G = torch.from_numpy(Q.dequantize(g_raw, 12, (F, K)))
    U = torch.from_numpy(Q.dequantize(u_raw, 12, (F, K)))
    M = 256
    x = _x(M, K, gpu)
    y = torch.zeros(x.shape[0], F, dtype=ops.ACT_DTYPE, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y, M, epi="swiglu", mode=3, waves=4, rt=16, ks=ks)
    xf = x[:M].float().cpu()
    _close(y[:M], torch.nn.functional.silu(xf @ G.t()) * (xf @ U.t()), 3e-2)
    a, Ad = _qw(256, K, GGMLType.Q4_K, gpu, 1)
    b, Bd = _qw(128, K, GGMLType.Q4_K, gpu, 2)
    c, Cd = _qw(128, K, GGMLType.Q6_K, gpu, 3)
    yq = torch.zeros(x.shape[0], 512, device=gpu)
    ops.qgemv([ops.Seg(a, 0), ops.Seg(b, 256), ops.Seg(c, 384)], x, yq, M, mode=3, waves=4, rt=16, ks=ks)
    _close(yq[:M], xf @ torch.cat([Ad, Bd, Cd]).t())


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0])
@pytest.mark.parametrize("M", [1, 3, 6])
@pytest.mark.parametrize("epi", ["f32", "add", "swiglu", "argmax"])
def test_qgemv_fused_rmsnorm(gpu, t, M, epi):
    """Path A with the input RMSNorm folded into the staged activation rows == rmsnorm kernel + GEMV."""
    rows, K = 272, 2048
    w, Wd = _qw(rows, K, t, gpu)
    g = torch.Generator().manual_seed(5)
    xf = (torch.randn(16, K, generator=g) * 3).to(gpu)
    nw = (1 + 0.1 * torch.randn(K, generator=g)).to(gpu)
    h = torch.zeros(16, K, dtype=ops.ACT_DTYPE, device=gpu)
    ops.rmsnorm(xf, nw, h, M, 1e-5)
    ncol = rows // 2 if epi == "swiglu" else rows
    dt = ops.ACT_DTYPE if epi == "swiglu" else torch.float32
    base = torch.randn(16, ncol, device=gpu).to(dt)
    outs = []
    for fused in (False, True):
        y = base.clone()
        keys = torch.zeros(16, dtype=torch.int64, device=gpu)
        ops.qgemv([ops.Seg(w)], h, y, M, alpha=0.5, epi=epi, argmax=keys if epi == "argmax" else None,
                  norm=(xf, nw, 1e-5) if fused else None, mode=0 if not fused else -1, waves=4, rt=2)
        outs.append((y[:M].float().cpu(), keys[:M].cpu()))
    if epi == "argmax":     # same winning index (the value may differ in its last ulp: rms summation order)
        assert ((outs[0][1] & 0xFFFFFFFF) == (outs[1][1] & 0xFFFFFFFF)).all()
    else:
        _close(outs[1][0], outs[0][0], 5e-3)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0])
@pytest.mark.parametrize("M", [65, 128, 300, 520])
@pytest.mark.parametrize("mode,wm,ks,wv", [(4, 4, 1, 8), (4, 2, 1, 8), (4, 4, 3, 8), (4, 2, 5, 8), (5, 4, 1, 8),
                                           (5, 2, 1, 8), (5, 4, 3, 8), (5, 2, 2, 8), (4, 4, 2, 16), (4, 2, 1, 16),
                                           (5, 4, 1, 16), (5, 2, 3, 16), (6, 2, 1, 8), (6, 2, 3, 8)])
def test_hgemm_dense(gpu, t, M, mode, wm, ks, wv):
    """Dense f16 GEMM (mode 4) on the weights' f16 copy: both operands by LDS-DMA into a 3-deep ring;
    partial last 128-row weight tile and activation block, K slices of 2..12 steps; store, add, argmax."""
    rows, K = 264, 768
    w, Wd = _qw(rows, K, t, gpu)
    assert w.expand_dense() == rows * K * 2 and w.expand_dense() == 0
    x = _x(M, K, gpu)
    pad = x.shape[0]
    y = torch.zeros(pad, rows, device=gpu)
    keys = torch.zeros(pad, dtype=torch.int64, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y, M, mode=mode, waves=wv, rt=wm, ks=ks, argmax=keys)
    ref = x[:M].float().cpu() @ Wd.t()
    _close(y[:M], ref)
    assert float(y[M:].abs().max().cpu()) == 0.0 if M < pad else True
    ids = torch.zeros(pad, dtype=torch.int32, device=gpu)
    ops.argmax_unpack(keys, M, ids)
    assert (ids[:M].cpu() == y[:M].argmax(1).cpu().to(torch.int32)).float().mean() > 0.99
    base = torch.randn(pad, rows, device=gpu)
    y2 = base.clone()
    ops.qgemv([ops.Seg(w)], x, y2, M, alpha=0.5, epi="add", mode=mode, waves=wv, rt=wm, ks=ks)
    _close(y2[:M], base[:M].cpu() + 0.5 * ref)
    # the same launch through the quantised LDS GEMM agrees to accumulation order
    y3 = torch.zeros(pad, rows, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y3, M, mode=2, waves=8, rt=wm, ks=1)
    _close(y3[:M], y[:M], 1e-3)


@pytest.mark.parametrize("mode,ks,wv", [(4, 1, 8), (4, 2, 8), (5, 1, 8), (5, 2, 8), (5, 1, 16), (4, 2, 16)])
def test_hgemm_dense_swiglu_multiseg_auto(gpu, mode, ks, wv):
    """Mode 4 with the SwiGLU epilogue and a Q|K|V-style multi-segment launch; then the automatic
    selection (gemv_config) picks mode 4 exactly when every segment carries an f16 copy and M is large."""
    K, F = 512, 256
    rng = np.random.default_rng(9)
    g_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    u_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    w = ops.QWeight(ops.interleave_gate_up(g_raw, u_raw, GGMLType.Q4_K, F, K), GGMLType.Q4_K, 2 * F, K, gpu)
    w.expand_dense()
    G = torch.from_numpy(Q.dequantize(g_raw, 12, (F, K)))
    U = torch.from_numpy(Q.dequantize(u_raw, 12, (F, K)))
    M = 333
    x = _x(M, K, gpu)
    y = torch.zeros(x.shape[0], F, dtype=ops.ACT_DTYPE, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y, M, epi="swiglu", mode=mode, waves=wv, rt=4, ks=ks)
    xf = x[:M].float().cpu()
    _close(y[:M], torch.nn.functional.silu(xf @ G.t()) * (xf @ U.t()), 3e-2)
    a, Ad = _qw(256, K, GGMLType.Q4_K, gpu, 1)
    b, Bd = _qw(128, K, GGMLType.Q4_K, gpu, 2)
    c, Cd = _qw(128, K, GGMLType.Q6_K, gpu, 3)
    segs = [ops.Seg(a, 0), ops.Seg(b, 256), ops.Seg(c, 384)]
    assert ops.gemv_config(segs, M)[0] != 4
    for q in (a, b, c):
        q.expand_dense()
    assert ops.gemv_config(segs, M)[0] in (4, 5) and ops.gemv_config(segs, 8)[0] not in (4, 5)
    yq = torch.zeros(x.shape[0], 512, device=gpu)
    ops.qgemv(segs, x, yq, M, mode=mode, waves=wv, rt=4, ks=ks)
    _close(yq[:M], xf @ torch.cat([Ad, Bd, Cd]).t())
    yq.zero_()
    ops.qgemv(segs, x, yq, M)
    _close(yq[:M], xf @ torch.cat([Ad, Bd, Cd]).t())


@pytest.mark.parametrize("rt", [1, 2])
@pytest.mark.parametrize("M,ks", [(512, 1), (333, 1), (100, 2), (256, 3), (1024, 1), (64, 4)])
def test_hgemm10_dense(gpu, M, ks, rt):
    """Mode 10 (hgemm10.hip: 256 x 256 tiles, 4 phases per 64-deep K-tile, the two wave groups staggered by
    a barrier, one LDS-DMA unit per phase under a counted vmcnt): partial last weight tile (264 rows),
    partial / multiple activation blocks, k-slices of 1..12 K-tiles (the clamped tail units), split-K
    through the slab reduce; f32 store with arg-max keys, residual add with alpha."""
    rows, K = 264, 768
    w, Wd = _qw(rows, K, GGMLType.Q4_K, gpu)
    w.expand_dense()
    x = _x(M, K, gpu)
    pad = x.shape[0]
    y = torch.zeros(pad, rows, device=gpu)
    keys = torch.zeros(pad, dtype=torch.int64, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y, M, mode=10, waves=8, rt=rt, ks=ks, argmax=keys if ks == 1 else None)
    ref = x[:M].float().cpu() @ Wd.t()
    _close(y[:M], ref)
    if M < pad:
        assert float(y[M:].abs().max().cpu()) == 0.0
    if ks == 1:
        ids = torch.zeros(pad, dtype=torch.int32, device=gpu)
        ops.argmax_unpack(keys, M, ids)
        assert (ids[:M].cpu() == y[:M].argmax(1).cpu().to(torch.int32)).float().mean() > 0.99
    base = torch.randn(pad, rows, device=gpu)
    y2 = base.clone()
    ops.qgemv([ops.Seg(w)], x, y2, M, alpha=0.5, epi="add", mode=10, waves=8, rt=rt, ks=ks)
    _close(y2[:M], base[:M].cpu() + 0.5 * ref)
    # the same launch through the mode-4 dense GEMM agrees to accumulation order
    y3 = torch.zeros(pad, rows, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y3, M, mode=4, waves=8, rt=4, ks=1)
    _close(y3[:M], y[:M], 1e-3)


@pytest.mark.parametrize("rt", [1, 2])
@pytest.mark.parametrize("ks", [1, 2])
def test_hgemm10_swiglu_multiseg(gpu, ks, rt):
    """Mode 10 SwiGLU epilogue (interleaved gate/up rows: partner lane ^ 32) and a Q|K|V-style launch."""
    K, F = 512, 256
    rng = np.random.default_rng(9)
    g_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    u_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    w = ops.QWeight(ops.interleave_gate_up(g_raw, u_raw, GGMLType.Q4_K, F, K), GGMLType.Q4_K, 2 * F, K, gpu)
    w.expand_dense()
    G = torch.from_numpy(Q.dequantize(g_raw, 12, (F, K)))
    U = torch.from_numpy(Q.dequantize(u_raw, 12, (F, K)))
    M = 333
    x = _x(M, K, gpu)
    xf = x[:M].float().cpu()
    y = torch.zeros(x.shape[0], F, dtype=ops.ACT_DTYPE, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y, M, alpha=0.75, epi="swiglu", mode=10, waves=8, rt=rt, ks=ks)
    _close(y[:M], torch.nn.functional.silu(0.75 * xf @ G.t()) * (0.75 * xf @ U.t()), 3e-2)
    a, Ad = _qw(256, K, GGMLType.Q4_K, gpu, 1)
    b, Bd = _qw(256, K, GGMLType.Q4_K, gpu, 2)
    c, Cd = _qw(256, K, GGMLType.Q6_K, gpu, 3)
    for q in (a, b, c):
        q.expand_dense()
    segs = [ops.Seg(a, 0), ops.Seg(b, 256), ops.Seg(c, 512)]
    yq = torch.zeros(x.shape[0], 768, device=gpu)
    ops.qgemv(segs, x, yq, M, mode=10, waves=8, rt=rt, ks=ks)
    _close(yq[:M], xf @ torch.cat([Ad, Bd, Cd]).t())


Q9_TYPES = [GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K, GGMLType.Q8_0, GGMLType.Q4_0, GGMLType.Q5_1, GGMLType.Q3_K]


@pytest.mark.parametrize("t", Q9_TYPES)
@pytest.mark.parametrize("M,waves,rt,ks", [(256, 8, 2, 1), (300, 8, 1, 2), (100, 8, 2, 3), (512, 8, 1, 1), (512, 8, 2, 2),
                                           (300, 4, 2, 1), (512, 4, 2, 3)])
def test_qgemm9_types(gpu, t, M, waves, rt, ks):
    """Mode 9 (qgemm9.hip: raw tile-blocks DMA'd per super-block and dequantised in registers, activations
    through an NS-deep 32-k stage ring, weights as the MFMA A operand): every device format, a partial last
    weight tile (264 rows over 128 / 256-row tiles), partial activation blocks, k-slices of 1..3
    super-blocks (split-K through the slab reduce); f32 store with arg-max keys, residual add with alpha."""
    rows, K = 264, 768
    w, Wd = _qw(rows, K, t, gpu)
    x = _x(M, K, gpu)
    pad = x.shape[0]
    y = torch.zeros(pad, rows, device=gpu)
    keys = torch.zeros(pad, dtype=torch.int64, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y, M, mode=9, waves=waves, rt=rt, ks=ks, argmax=keys if ks == 1 else None)
    ref = x[:M].float().cpu() @ Wd.t()
    _close(y[:M], ref)
    if M < pad:
        assert float(y[M:].abs().max().cpu()) == 0.0
    if ks == 1:
        ids = torch.zeros(pad, dtype=torch.int32, device=gpu)
        ops.argmax_unpack(keys, M, ids)
        assert (ids[:M].cpu() == y[:M].argmax(1).cpu().to(torch.int32)).float().mean() > 0.99
    base = torch.randn(pad, rows, device=gpu)
    y2 = base.clone()
    ops.qgemv([ops.Seg(w)], x, y2, M, alpha=0.5, epi="add", mode=9, waves=waves, rt=rt, ks=ks)
    _close(y2[:M], base[:M].cpu() + 0.5 * ref)


@pytest.mark.parametrize("waves,rt,ks", [(8, 2, 1), (8, 1, 1), (8, 2, 2), (4, 2, 1)])
def test_qgemm9_swiglu_multiseg(gpu, waves, rt, ks):
    """Mode 9 SwiGLU epilogue on interleaved gate/up tile-blocks and a Q|K|V-style launch mixing Q4_K and
    Q6_K segments (each workgroup picks its segment's format) at column offsets; the mode-2 LDS-dequant
    GEMM agrees to accumulation order."""
    K, F = 512, 256
    rng = np.random.default_rng(9)
    g_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    u_raw = Q.random_blocks(GGMLType.Q4_K, F * K, 0.05, rng)
    w = ops.QWeight(ops.interleave_gate_up(g_raw, u_raw, GGMLType.Q4_K, F, K), GGMLType.Q4_K, 2 * F, K, gpu)
    G = torch.from_numpy(Q.dequantize(g_raw, 12, (F, K)))
    U = torch.from_numpy(Q.dequantize(u_raw, 12, (F, K)))
    M = 333
    x = _x(M, K, gpu)
    xf = x[:M].float().cpu()
    y = torch.zeros(x.shape[0], F, dtype=ops.ACT_DTYPE, device=gpu)
    ops.qgemv([ops.Seg(w)], x, y, M, alpha=0.75, epi="swiglu", mode=9, waves=waves, rt=rt, ks=ks)
    _close(y[:M], torch.nn.functional.silu(0.75 * xf @ G.t()) * (0.75 * xf @ U.t()), 3e-2)
    a, Ad = _qw(256, K, GGMLType.Q4_K, gpu, 1)
    b, Bd = _qw(256, K, GGMLType.Q4_K, gpu, 2)
    c, Cd = _qw(256, K, GGMLType.Q6_K, gpu, 3)
    segs = [ops.Seg(a, 0), ops.Seg(b, 256), ops.Seg(c, 512)]
    yq = torch.zeros(x.shape[0], 768, device=gpu)
    ops.qgemv(segs, x, yq, M, mode=9, waves=waves, rt=rt, ks=ks)
    _close(yq[:M], xf @ torch.cat([Ad, Bd, Cd]).t())
    y2 = torch.zeros(x.shape[0], 768, device=gpu)
    ops.qgemv(segs, x, y2, M, mode=2, waves=8, rt=4, ks=1)
    _close(yq[:M], y2[:M], 1e-3)


def test_hgemm_dense_add_rmsnorm_slabs(gpu):
    """Mode 4 split-K slabs feeding the fused reduce + residual + RMSNorm kernel (o / down projections)."""
    D, K, M = 512, 1024, 200
    w, Wd = _qw(D, K, GGMLType.Q4_K, gpu, 4)
    w.expand_dense()
    xin = _x(M, K, gpu)
    x = torch.randn(xin.shape[0], D, device=gpu)
    x0 = x.clone()
    nw = torch.rand(D, device=gpu) + 0.5
    h = torch.zeros(xin.shape[0], D, dtype=ops.ACT_DTYPE, device=gpu)
    ops.qgemv_add_rmsnorm(ops.Seg(w), xin, x, nw, h, M, 1.0, 1e-5, cfg=(5, 8, 4, 4))
    ref = x0[:M].cpu() + xin[:M].float().cpu() @ Wd.t()
    _close(x[:M], ref)
    hn = ref * torch.rsqrt(ref.pow(2).mean(1, keepdim=True) + 1e-5) * nw.cpu()
    _close(h[:M], hn, 2e-2)


@pytest.mark.parametrize("M", [1, 3, 16])
def test_split_rmsnorm_producer_consumer(gpu, M):
    """Split RMSNorm: a path-A residual-add GEMV leaves per-workgroup shares of sum(x^2); a fused-norm
    consumer (path A, path B XL, path B XL split-K) sums them instead of re-reading the row."""
    D, K2 = 1024, 512
    wo, Wo = _qw(D, K2, GGMLType.Q4_K, gpu, 21)
    xin = _x(M, K2, gpu, seed=5)
    x = (torch.randn(xin.shape[0], D) * 0.7).to(gpu)
    x0 = x.clone()
    ldss = D // 16
    ssq = torch.full((xin.shape[0] * ldss,), float("nan"), device=gpu)
    parts = ops.qgemv_add_ssq(ops.Seg(wo), xin, x, M, 0.5, ssq, ldss, cfg=(0, 8, 1, 1))
    assert parts == D // 16
    ref = x0[:M].cpu() + 0.5 * (xin[:M].float().cpu() @ Wo.t())
    _close(x[:M], ref)
    tot = ssq.view(-1, ldss)[:M, :parts].double().sum(1).cpu()
    assert torch.allclose(tot, ref.double().pow(2).sum(1), rtol=1e-4), (tot, ref.pow(2).sum(1))
    nw = (torch.rand(D) + 0.5).to(gpu)
    xn = ref * torch.rsqrt(ref.pow(2).mean(1, keepdim=True) + 1e-5) * nw.cpu()
    wc, Wc = _qw(768, D, GGMLType.Q4_K, gpu, 22)
    want = xn @ Wc.t()
    for cfg in [(0, 8, 1, 1), (0, 4, 2, 1), (1, 4, 2, 1), (1, 8, 1, 2)]:
        y = torch.zeros(xin.shape[0], 768, device=gpu)
        fz = ops._lib.NlsFuse(xf=x.data_ptr(), ldxf=x.stride(0), nw=nw.data_ptr(), eps=1e-5, ssq_in=ssq.data_ptr(),
                              ldss=ldss, nss_in=parts)
        mode, waves, rt, ks = cfg
        ws = ops._workspace(gpu, ks * M * 768).data_ptr() if ks > 1 else None
        rc = ops._lib.lib().nls_qgemv_ex(ops._segs([ops.Seg(wc)]), 1, x.data_ptr(), x.stride(0), y.data_ptr(),
                                         y.stride(0), M, 1.0, ops.EPI["f32"], None, waves, rt, mode, ks, ws,
                                         ops._stream_ptr(x), ctypes.byref(fz))
        assert rc == 0, (cfg, rc)
        _close(y[:M], want, 3e-2)
    # the public entry: tuned config, partials tuple
    y = torch.zeros(xin.shape[0], 768, device=gpu)
    ops.qgemv([ops.Seg(wc)], x, y, M, norm=(x, nw, 1e-5, ssq, ldss, parts))
    _close(y[:M], want, 3e-2)


@pytest.mark.parametrize("T", [1, 3, 10])
def test_moe_route_sel_and_selected_expert_launch(gpu, T):
    """The route kernel lists each (token, slot)'s expert (and zeroes stale counts itself for T <= 4);
    a device-selected launch over those slots equals the launch over every expert."""
    E, k, K, R = 8, 2, 512, 64
    lg = torch.randn(T, E, device=gpu)
    topw = torch.zeros(T * k, device=gpu)
    counts = torch.full((E,), 5 if T <= 4 else 0, dtype=torch.int32, device=gpu)   # stale counts: T<=4 zeroes
    cap = 64
    xr = torch.zeros(E * cap, dtype=torch.int32, device=gpu)
    yr = torch.zeros(E * cap, dtype=torch.int32, device=gpu)
    sel = torch.full((T * k,), -1, dtype=torch.int32, device=gpu)
    ops.moe_route(lg, T, k, topw, counts, xr, yr, cap, sel=sel)
    _, e = torch.topk(torch.softmax(lg, -1), k, -1)
    assert sorted(sel.view(T, k).cpu().tolist()[0]) == sorted(e.cpu().tolist()[0])
    assert set(sel.cpu().tolist()) == set(e.flatten().cpu().tolist())
    assert counts.sum().item() == T * k
    ws = [_qw(R, K, GGMLType.Q5_K, gpu, 30 + i)[0] for i in range(E)]
    x = _x(T, K, gpu)
    segs = [ops.Seg(ws[i], 0, xr[i * cap:], yr[i * cap:], counts[i:i + 1]) for i in range(E)]
    y_all = torch.zeros(64, R, device=gpu)
    ops.qgemv(segs, x, y_all, T)
    y_sel = torch.zeros(64, R, device=gpu)
    ops.qgemv(segs, x, y_sel, T, sel=(sel, T * k, 0))
    assert torch.equal(y_all[:T * k], y_sel[:T * k])
    # a base offset (expert group 4..7 of an EP rank / an 8-segment group): out-of-range slots exit
    y_hi = torch.zeros(64, R, device=gpu)
    ops.qgemv(segs[4:], x, y_hi, T, sel=(sel, T * k, 4))
    for t in range(T):
        for j in range(k):
            ex = int(e[t, j])
            row = t * k + j
            want = y_all[row] if ex >= 4 else torch.zeros(R, device=gpu)
            assert torch.equal(y_hi[row], want), (t, j, ex)


@pytest.mark.parametrize("T,k,D", [(1, 2, 4096), (3, 2, 1024), (2, 4, 4096), (5, 8, 8192)])
def test_moe_combine_norm(gpu, T, k, D):
    """Fused MoE combine + next RMSNorm vs the two-step fp32 reference."""
    g = torch.Generator().manual_seed(T * 100 + k)
    y = torch.randn(T * k, D, generator=g)
    w = torch.rand(T * k, generator=g)
    x = torch.randn(T, D, generator=g)
    nw = torch.rand(D, generator=g) + 0.5
    ref = x + 0.7 * (w.view(T, k, 1) * y.view(T, k, D)).sum(1)
    href = ref * torch.rsqrt(ref.pow(2).mean(1, keepdim=True) + 1e-5) * nw
    xg = x.to(gpu)
    h = torch.zeros(T, D, dtype=ops.ACT_DTYPE, device=gpu)
    ops.moe_combine_norm(y.to(gpu), w.to(gpu), T, k, xg, 0.7, nw.to(gpu), 1e-5, h)
    _close(xg, ref, 1e-5)
    _close(h, href, 1e-2)


@pytest.mark.parametrize("shards", [2, 8])
def test_candidate_sampling_matches_full_vocab(gpu, shards):
    """TP sampling draws from the per-rank top-128 candidates (ops.topc_candidates, vocabulary order): the
    GPU sampler on the concatenated candidate rows, with history ids mapped to candidate positions, gives
    the token the GPU sampler gives on the full [rows, vocab] logits (top_k <= 64, penalties, top-p, min-p)."""
    from nats_llm_studio_amd.engine.sampling import SamplingParams, sample_rows_gpu, uniform01
    V, n, C = 32000, 6, 128
    g = torch.Generator().manual_seed(5)
    lg = (torch.randn(n, V, generator=g) * 3.0).to(gpu)
    params = [SamplingParams(temperature=0.8, top_k=40, top_p=0.95, repeat_penalty=1.2, seed=3),
              SamplingParams(temperature=1.3, top_k=64, min_p=0.02, presence_penalty=0.5, seed=7),
              SamplingParams(temperature=0.5, top_k=5),
              SamplingParams(temperature=1.0, top_k=1),
              SamplingParams(temperature=0.0, repeat_penalty=1.5),           # penalised arg-max
              SamplingParams(temperature=0.9, top_k=60, top_p=0.5, frequency_penalty=0.3)]
    top = torch.topk(lg, 80, dim=1).indices.cpu()
    hist = [top[r, torch.randperm(80, generator=g)[:30]].tolist() * 2 for r in range(n)]   # repeats: counts
    us = [uniform01(100 + r, 7) for r in range(n)]
    ref = sample_rows_gpu(lg.clone(), params, hist, us)
    per = -(-V // shards)
    vals, ids = [], []
    for r in range(shards):
        lo = r * per
        cv_r, ci_r = ops.topc_candidates(lg[:, lo:lo + per].contiguous(), n, C, lo, min(per, V - lo))
        vals.append(cv_r)
        ids.append(ci_r)
    cv, ci = torch.cat(vals, 1), torch.cat(ids, 1)
    ixl = ci.cpu().tolist()
    mh = [[{t: j for j, t in enumerate(ixl[r])}[t] for t in hist[r][-64:] if t in set(ixl[r])] for r in range(n)]
    picks = sample_rows_gpu(cv.contiguous(), params, mh, us)
    assert [ixl[r][j] for r, j in enumerate(picks)] == ref


def _prefill_ref_gpu(q, kc, vc, bt, chunks, Hq, Hkv, D, bs, scale):
    """Plain fp32 PyTorch causal attention over the paged cache, per chunk (seq, pos0, n): the reference of
    attn_prefill at long offsets (the CPU per-token reference is too slow for 32K contexts)."""
    out, t = [], 0
    G = Hq // Hkv
    for s, p0, n in chunks:
        nk = p0 + n
        keys = torch.arange(nk, device=q.device)
        slots = bt[s, keys // bs].long() * bs + keys % bs
        K = kc[slots].float()                     # [nk, Hkv, D]
        V = vc[slots].float()
        Q = q[t:t + n].float().view(n, Hkv, G, D)
        S = torch.einsum("nhgd,khd->hgnk", Q, K) * scale
        qpos = torch.arange(p0, p0 + n, device=q.device)
        S = S.masked_fill(keys[None, None, None, :] > qpos[None, None, :, None], float("-inf"))
        P = torch.softmax(S, dim=-1)
        O = torch.einsum("hgnk,khd->nhgd", P, V).reshape(n, Hq * D)
        out.append(O)
        t += n
    return torch.cat(out)


@pytest.mark.parametrize("kvt", [torch.bfloat16, torch.float8_e4m3fn])
@pytest.mark.parametrize("D,G,Hkv", [(128, 4, 2), (128, 8, 1), (64, 4, 2)])
def test_attention_prefill_long_offsets(gpu, D, G, Hkv, kvt):
    """attn_prefill at production shapes: a 2048-token chunk continuing a 30K-token prefix (the last chunk of
    a 32K prompt), next to short chunks of two other sequences (one fresh, one mid-context), pages scattered
    over the pool; fp32 PyTorch reference."""
    torch.manual_seed(1)
    bs = 16
    Hq = Hkv * G
    chunks = [(0, 30720, 2048), (1, 5000, 100), (2, 0, 70)]
    nblk = (32768 + bs - 1) // bs
    nseq = 3
    perm = torch.randperm(nseq * nblk, device=gpu).view(nseq, nblk).int()
    slots = nseq * nblk * bs
    kc = (torch.randn(slots, Hkv, D, device=gpu) * 0.5).to(kvt)
    vc = torch.randn(slots, Hkv, D, device=gpu).to(kvt)
    T = sum(n for _, _, n in chunks)
    pos, tseq = [], []
    for s, p0, n in chunks:
        pos += list(range(p0, p0 + n))
        tseq += [s] * n
    pos = np.array(pos, np.int32)
    tseq = np.array(tseq, np.int32)
    q = torch.randn(T, Hq * D, device=gpu).to(torch.bfloat16)
    ref = _prefill_ref_gpu(q, kc, vc, perm, chunks, Hq, Hkv, D, bs, D ** -0.5)
    qb = ops.prefill_blocks(tseq, pos, T)
    out = torch.zeros(T, Hq * D, dtype=ops.ACT_DTYPE, device=gpu)
    ops.attention_prefill(q, kc, vc, perm, torch.from_numpy(qb).to(gpu), len(qb), None, None, out, T, Hq, Hkv, D, bs,
                          D ** -0.5)
    torch.cuda.synchronize()
    err = (out.float() - ref).abs().max().item()
    assert err < 2e-2, err


@pytest.mark.parametrize("n,valid,C,lo", [(1, 16032, 128, 16032), (8, 16032, 128, 0), (5, 64128, 128, 64128),
                                          (3, 100, 128, 7), (4, 4000, 64, 4000), (2, 129, 128, 0)])
def test_topc_candidates_kernel(gpu, n, valid, C, lo):
    """sample.hip topc_kernel (tensor-parallel candidate selection) against torch.topk + sort on the CPU: the same
    C largest logits of the shard, in vocabulary order, global ids, (-inf, -1) padding of short shards; ties at the
    threshold (quantised logits) resolved to the lowest indices; both planes of the gather's source block."""
    g = torch.Generator().manual_seed(valid + n)
    lg = torch.randn(n, valid + 32, generator=g)
    lg[1::2] = (lg[1::2] * 4).round() / 4             # many exact ties on odd rows
    lg[:, valid:] = 1e9                                # padding columns past `valid` must never be picked
    v, i = ops.topc_candidates(lg.to(gpu), n, C, lo, valid)
    assert v._packed is i._packed and v._packed.shape == (2, n, C)
    vr, ir = ops.topc_candidates(lg, n, C, lo, valid)
    k = min(C, valid)
    v, i = v.cpu(), i.cpu()
    assert torch.equal(i[:, k:], torch.full((n, C - k), -1, dtype=torch.int32))
    assert torch.isinf(v[:, k:]).all()
    for r in range(n):
        # the selected set has the reference's values (a tie at the threshold may pick other equal entries)
        assert torch.equal(torch.sort(v[r, :k]).values, torch.sort(vr[r, :k]).values), r
        ids = i[r, :k]
        assert bool((ids[1:] > ids[:-1]).all()), "vocabulary order"
        assert torch.equal(lg[r, (ids - lo).long()], v[r, :k])
        thr = v[r, :k].min()
        eq = (lg[r, :valid] == thr).nonzero().flatten()
        taken = set((ids - lo).tolist())
        want = [int(j) for j in eq[:sum(int(t) in taken for t in eq.tolist())]]
        assert all(j in taken for j in want), "ties resolved to the lowest indices"
