"""GPU parity of the individual HIP kernels (through the C ABI) against plain
PyTorch fp32 references of the same op / the CPU oracle's functions."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from oracle import vggt_oracle as O  # noqa: E402


@pytest.fixture(scope="module")
def N():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from aligned_vggt import _native
    _native.lib()
    return _native


def _bf(x):
    return x.to(torch.bfloat16)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


# (6592, 3072, 1024): the 154x518 sequence chunk's qkv, where the auto choice
# takes a 192-wide ping-pong tile (256 wide would be 1.22 rounds of CUs)
@pytest.mark.parametrize("M,Nn,K", [(128, 128, 64), (300, 256, 192), (1374, 1024, 1024), (77, 3072, 640),
                                    (6592, 3072, 1024)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
def test_gemm_epilogues(N, M, Nn, K, epi):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + epi)
    a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    # asymmetric operand (catches transposed C writes)
    w = (torch.randn(Nn, K, device="cuda", generator=g) + torch.arange(Nn, device="cuda")[:, None] * 1e-3).to(torch.bfloat16)
    b = torch.randn(Nn, device="cuda", generator=g).to(torch.bfloat16).float()
    ref = a.float() @ w.float().t() + b
    refb = ref.to(torch.bfloat16).float()
    if epi == N.EPI_BF16:
        out = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
        N.gemm_bf16(a, w, b, out, epi)
        assert _rel(out, refb) < 4e-3
    elif epi == N.EPI_GELU_BF16:
        out = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
        N.gemm_bf16(a, w, b, out, epi)
        assert _rel(out, F.gelu(refb)) < 6e-3
    elif epi == N.EPI_RESID_F32:
        x0 = torch.randn(M, Nn, device="cuda", generator=g)
        gam = torch.rand(Nn, device="cuda", generator=g)
        x = x0.clone()
        o2 = torch.zeros(M, 2 * Nn, device="cuda")
        N.gemm_bf16(a, w, b, x, epi, gamma=gam, out2=o2[:, Nn:])
        r = x0 + gam * refb
        assert _rel(x, r) < 4e-3
        torch.testing.assert_close(o2[:, Nn:], x)
        assert o2[:, :Nn].abs().max().item() == 0
    else:
        out = torch.empty(M, Nn, device="cuda")
        N.gemm_bf16(a, w, b, out, epi)
        assert _rel(out, refb) < 4e-3


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("M,Nn,K", [(300, 256, 96), (1000, 768, 1024), (2300, 1024, 4096), (21984, 1024, 1024),
                                    (5000, 3072, 1024)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_gemm_tile_variants(N, mode, M, Nn, K, epi):
    """Every tile form (vggt_tune VGGT_TUNE_GEMM_TILE) on shapes that exercise
    the ring's prologue/tail (K/32 = 3, 32, 128), ragged M and N % 256 != 0."""
    prev = N.tune(N.TUNE_GEMM_TILE, mode)
    try:
        g = torch.Generator(device="cuda").manual_seed(M + Nn + K + epi)
        a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        w = (torch.randn(Nn, K, device="cuda", generator=g) * K ** -0.5
             + torch.arange(Nn, device="cuda")[:, None] * 1e-3).to(torch.bfloat16)
        b = torch.randn(Nn, device="cuda", generator=g).to(torch.bfloat16).float()
        refb = (a.float() @ w.float().t() + b).to(torch.bfloat16).float()
        if epi == N.EPI_RESID_F32:
            x0 = torch.randn(M, Nn, device="cuda", generator=g)
            gam = torch.rand(Nn, device="cuda", generator=g)
            x = x0.clone()
            N.gemm_bf16(a, w, b, x, epi, gamma=gam)
            assert _rel(x, x0 + gam * refb) < 4e-3
        else:
            out = torch.full((M + 1, Nn), 7.0, device="cuda", dtype=torch.bfloat16)
            N.gemm_bf16(a, w, b, out[:M], epi)
            r = F.gelu(refb) if epi == N.EPI_GELU_BF16 else refb
            assert _rel(out[:M], r) < 6e-3
            assert (out[M] == 7.0).all()  # no write past row M
    finally:
        N.tune(N.TUNE_GEMM_TILE, prev)


def test_gemm_rejects_bad_shapes(N):
    a = torch.zeros(64, 80, device="cuda", dtype=torch.bfloat16)
    w = torch.zeros(128, 80, device="cuda", dtype=torch.bfloat16)
    b = torch.zeros(128, device="cuda")
    with pytest.raises(RuntimeError, match="shape"):
        N.gemm_bf16(a, w, b, torch.empty(64, 128, device="cuda", dtype=torch.bfloat16), 0)


@pytest.mark.parametrize("C", [512, 1024, 2048])
@pytest.mark.parametrize("ib,ob", [(False, True), (False, False), (True, False)])
def test_layernorm(N, C, ib, ob):
    x = torch.randn(301, C, device="cuda") * 3 + 1
    if ib:
        x = x.to(torch.bfloat16)
    w = torch.randn(C, device="cuda")
    b = torch.randn(C, device="cuda")
    out = torch.empty(301, C, device="cuda", dtype=torch.bfloat16 if ob else torch.float32)
    N.layernorm(x, w, b, 1e-6, out)
    ref = F.layer_norm(x.float(), (C,), w, b, 1e-6)
    assert _rel(out, ref) < (4e-3 if ob else 1e-5)


@pytest.mark.parametrize("C", [256, 1024, 2048])
@pytest.mark.parametrize("ln,mirror,affine", [(True, True, True), (True, False, False), (False, True, True)])
def test_resid_add_layernorm(N, C, ln, mirror, affine):
    """x += gamma * y; out2 = x; xn = LayerNorm(x) (bf16) vs fp32 torch, on a
    strided residual (ld > C) and a ragged row count."""
    g = torch.Generator().manual_seed(C)
    M = 301
    xb = (torch.randn(M, C + 64, generator=g) * 3 + 1).cuda()
    x = xb[:, :C]
    pad = xb[:, C:].clone()
    y = (torch.randn(M, C, generator=g)).to(torch.bfloat16).cuda()
    gamma = (torch.rand(C, generator=g) * 0.5).cuda()
    w = torch.randn(C, generator=g).cuda() if affine else None
    b = torch.randn(C, generator=g).cuda() if affine else None
    ref_x = x.clone() + gamma * y.float()
    ref_n = F.layer_norm(ref_x, (C,), w, b, 1e-5)
    o2 = torch.zeros(M, 2 * C, device="cuda")[:, C:] if mirror else None
    xn = torch.empty(M, C, device="cuda", dtype=torch.bfloat16) if ln else None
    N.resid_add_layernorm(x, y, gamma, o2, w, b, 1e-5, xn)
    torch.cuda.synchronize()
    assert _rel(x, ref_x) < 1e-6
    assert torch.equal(xb[:, C:], pad)  # columns past C untouched
    if mirror:
        assert torch.equal(o2, x)
    if ln:
        assert _rel(xn, ref_n) < 4e-3


def test_resid_add_layernorm_rejects(N):
    x = torch.zeros(4, 768, device="cuda")
    y = torch.zeros(4, 768, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="shape"):
        N.resid_add_layernorm(x, y, torch.ones(768, device="cuda"), None, None, None, 1e-5, None)


@pytest.mark.parametrize("D,mode", [(64, 1), (128, 1), (64, 0), (128, 2), (64, 2)])
def test_headnorm_rope(N, D, mode):
    H = 1024 // D
    M = 3 * 21
    g = torch.Generator().manual_seed(D + mode)
    qkv = (torch.randn(M, 3 * 1024, generator=g) * 2).to(torch.bfloat16)
    w = torch.randn(D, generator=g)
    b = torch.randn(D, generator=g)
    if mode == 1:
        pos = O.position_grid(1, 4, 4, 5)[0]
        period = pos.shape[0]
        from aligned_vggt.backbone.layers import RopeTables
        rt = RopeTables(pos, D, 100.0, "cuda")
    elif mode == 2:
        pos = torch.randint(0, 30, (7,), generator=g)
        period = 7
        from aligned_vggt.backbone.layers import RopeTables
        rt = RopeTables(pos, D, 100.0, "cuda", mode=2)
    buf = qkv.cuda()
    N.headnorm_rope(buf, 1024, H, D, w.cuda(), b.cuda(), 1e-5, mode, rt.pos if mode else None, period if mode else 1,
                    rt.cos if mode else None, rt.sin if mode else None)
    # oracle: (B=1, heads, N, D)
    k = qkv[:, 1024:2048].float().reshape(M, H, D).permute(1, 0, 2)[None]
    k = O.layer_norm(k, w, b, 1e-5)
    if mode == 1:
        pfull = pos.repeat(M // period, 1)[None]
        k = O.rope2d(k, pfull)
    elif mode == 2:
        pfull = pos.repeat(M // period)[None]
        k = O.rope1d(k, pfull)
    ref = k[0].permute(1, 0, 2).reshape(M, 1024)
    got = buf[:, 1024:2048].float().cpu()
    assert _rel(got, ref) < 4e-3
    # q/v columns untouched
    assert torch.equal(buf[:, 2048:].cpu(), qkv[:, 2048:])
    assert torch.equal(buf[:, :1024].cpu(), qkv[:, :1024])


@pytest.mark.parametrize("D,mode", [(64, 1), (128, 2), (64, 0)])
def test_norm_rope_out_of_place_matches_in_place(N, D, mode):
    """vggt_qknorm_rope_out / vggt_headnorm_rope_out (training recompute) are
    bit-identical to the in-place forms and leave the source untouched."""
    from aligned_vggt.backbone.layers import RopeTables
    H, M = 1024 // D, 3 * 21
    g = torch.Generator().manual_seed(7 + D + mode)
    src = (torch.randn(M, 3 * 1024, generator=g) * 2).to(torch.bfloat16).cuda()
    qw, qb, kw, kb = (torch.randn(D, generator=g).cuda() for _ in range(4))
    rt, period = None, 1
    if mode == 1:
        pos = O.position_grid(1, 4, 4, 5)[0]
        rt, period = RopeTables(pos, D, 100.0, "cuda"), pos.shape[0]
    elif mode == 2:
        pos = torch.randint(0, 30, (7,), generator=g)
        rt, period = RopeTables(pos, D, 100.0, "cuda", mode=2), 7
    tabs = (rt.pos, period, rt.cos, rt.sin) if rt else (None, 1, None, None)
    keep = src.clone()
    inplace = src.clone()
    N.qknorm_rope(inplace, H, D, qw, qb, kw, kb, 1e-5, mode, *tabs)
    dst = torch.zeros(M, 2 * 1024, device="cuda", dtype=torch.bfloat16)
    N.qknorm_rope_out(src, dst, H, D, qw, qb, kw, kb, 1e-5, mode, *tabs)
    assert torch.equal(dst, inplace[:, :2048])
    assert torch.equal(src, keep)
    inplace = src.clone()
    N.headnorm_rope(inplace, 1024, H, D, kw, kb, 1e-5, mode, *tabs)
    dst = torch.zeros(M, 1024, device="cuda", dtype=torch.bfloat16)
    N.headnorm_rope_out(src[:, 1024:], dst, H, D, kw, kb, 1e-5, mode, *tabs)
    assert torch.equal(dst, inplace[:, 1024:2048])
    assert torch.equal(src, keep)


def test_gemm_gelu_pre(N):
    """vggt_gemm_bf16_gelu_pre = the plain GEMM (pre) and the GELU epilogue (out), both bit-identical to the
    separate launches, on the 128x128 (small M) and the persistent (M >= 4096: 192- and 256-row tiles) forms."""
    g = torch.Generator(device="cuda").manual_seed(11)
    for M in (300, 4200, 22000):
        a = (torch.randn(M, 1024, device="cuda", generator=g)).to(torch.bfloat16)
        w = (torch.randn(4096, 1024, device="cuda", generator=g) * 0.03).to(torch.bfloat16)
        b = torch.randn(4096, device="cuda", generator=g) * 0.1
        out = torch.empty(M, 4096, device="cuda", dtype=torch.bfloat16)
        pre = torch.empty_like(out)
        N.gemm_bf16_gelu_pre(a, w, b, out, pre)
        ref_pre = torch.empty_like(out)
        N.gemm_bf16(a, w, b, ref_pre, N.EPI_BF16)
        ref_out = torch.empty_like(out)
        N.gemm_bf16(a, w, b, ref_out, N.EPI_GELU_BF16)
        assert torch.equal(pre, ref_pre)
        assert torch.equal(out, ref_out)
        assert _rel(out, F.gelu(ref_pre.float())) < 4e-3


def test_resid_scale_add_from(N):
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(77, 1024, device="cuda", generator=g)
    br = torch.randn(77, 1024, device="cuda", generator=g).to(torch.bfloat16)
    gamma = torch.rand(1024, device="cuda", generator=g)
    out = torch.empty_like(x)
    keep = x.clone()
    N.resid_scale_add_from(out, x, br, gamma)
    assert torch.equal(x, keep)
    assert torch.allclose(out, x + gamma * br.float(), rtol=1e-6, atol=1e-6)
    N.resid_scale_add(x, br, gamma)
    assert torch.equal(x, out)


def _ref_attn(q, k, v, scale):
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    return torch.softmax(s, -1) @ v.float()


@pytest.mark.parametrize("variant", [3, 11, 15, 19, 23, 32, 97, 161, 289, 545, 2081, 4129])
@pytest.mark.parametrize("D,H,batch,n", [(64, 16, 3, 21), (64, 16, 2, 1374), (128, 8, 2, 1375), (64, 2, 1, 4100),
                                         (128, 2, 1, 64), (64, 1, 1, 1)])
def test_attention_vs_torch(N, D, H, batch, n, variant):
    prev = N.tune(N.TUNE_ATTN_VARIANT, variant)
    try:
        _attention_vs_torch(N, D, H, batch, n)
    finally:
        N.tune(N.TUNE_ATTN_VARIANT, prev)


def _attention_vs_torch(N, D, H, batch, n):
    C = H * D
    g = torch.Generator(device="cuda").manual_seed(n + D)
    qkv = (torch.randn(batch * n, 3 * C, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
    o = torch.zeros(batch * n, C, device="cuda", dtype=torch.bfloat16)
    N.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, batch, H, n, n, D, n, n, n)
    t = qkv.float().view(batch, n, 3, H, D).permute(2, 0, 3, 1, 4)
    ref = _ref_attn(t[0], t[1], t[2], D ** -0.5).permute(0, 2, 1, 3).reshape(batch * n, C)
    e = _rel(o, ref)
    print(f"attention D={D} H={H} batch={batch} n={n}: rel-L2 vs fp32 {e:.2e}")
    # bf16 P and bf16 output: ~2-3e-3 (round 4); the bar is about 2x that
    assert e < 6e-3, e


@pytest.mark.parametrize("waves,n,D", [(8, 4100, 64), (8, 5000, 64), (8, 8191, 64), (8, 4100, 128), (2, 65, 64), (2, 1374, 64),
                                        (2, 6592, 64), (2, 1375, 128), (2, 33, 128)])
def test_attention_eight_wave_form(N, waves, n, D):
    """8-wave (256-query-row) workgroups, used for nq >= 4096, and 2-wave
    (64-row) workgroups (VGGT_TUNE_ATTN_WAVES 2)."""
    prev = N.tune(N.TUNE_ATTN_WAVES, waves)
    try:
        H = 2
        C = H * D
        g = torch.Generator(device="cuda").manual_seed(n)
        qkv = (torch.randn(n, 3 * C, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
        o = torch.zeros(n, C, device="cuda", dtype=torch.bfloat16)
        N.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, 1, H, n, n, D, n, n, n)
        t = qkv.float().view(1, n, 3, H, D).permute(2, 0, 3, 1, 4)
        ref = _ref_attn(t[0], t[1], t[2], D ** -0.5).permute(0, 2, 1, 3).reshape(n, C)
        e = _rel(o, ref)
        print(f"attention {waves}-wave D={D} n={n}: rel-L2 vs fp32 {e:.2e}")
        assert e < 6e-3, e
    finally:
        N.tune(N.TUNE_ATTN_WAVES, prev)


def test_attention_global_shape_rows(N):
    """Full BASELINE global-attention shape (1 x 16 heads x 21984 x 64):
    spot-check 256 query rows of every head against an fp32 reference."""
    n, H, D = 16 * 1374, 16, 64
    C = H * D
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(n, 3 * C, device="cuda", generator=g).to(torch.bfloat16)
    o = torch.empty(n, C, device="cuda", dtype=torch.bfloat16)
    N.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, 1, H, n, n, D, n, n, n)
    rows = torch.randperm(n, generator=torch.Generator().manual_seed(1))[:256].cuda()
    q = qkv[rows, :C].float().view(-1, H, D).transpose(0, 1)
    k = qkv[:, C:2 * C].float().view(n, H, D).transpose(0, 1)
    v = qkv[:, 2 * C:].float().view(n, H, D).transpose(0, 1)
    ref = _ref_attn(q, k, v, D ** -0.5).transpose(0, 1).reshape(-1, C)
    assert _rel(o[rows], ref) < 1e-2


@pytest.mark.parametrize("M,Nn,K,epi", [(21984, 4096, 1024, 1), (21984, 1024, 4096, 2), (21984, 3072, 1024, 0),
                                        (21984, 1024, 4096, 0), (19776, 4096, 1024, 1), (13500, 4096, 1024, 3)])
def test_gemm_balance_split_bitwise(N, M, Nn, K, epi):
    """VGGT_TUNE_GEMM_BALANCE: a persistent GEMM whose last round of tiles would be
    under 60 % full runs as whole rounds + the remaining rows on the 128x128 form;
    the output (and the residual mirror / the GELU pre-activation) equals the one
    launch bitwise."""
    g = torch.Generator(device="cuda").manual_seed(M + Nn + K + epi)
    a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(Nn, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(Nn, device="cuda", generator=g).to(torch.bfloat16).float()
    gam = torch.rand(Nn, device="cuda", generator=g)
    x0 = torch.randn(M, Nn, device="cuda", generator=g)
    outs = []
    for bal in (0, 1):
        prev = N.tune(N.TUNE_GEMM_BALANCE, bal)
        try:
            if epi == N.EPI_RESID_F32:
                out = x0.clone()
                o2 = torch.zeros(M, Nn, device="cuda")
                N.gemm_bf16(a, w, b, out, epi, gamma=gam, out2=o2)
                outs.append((out, o2))
            elif epi == N.EPI_GELU_BF16:
                out = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
                pre = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
                N.gemm_bf16(a, w, b, out, epi)
                N.gemm_bf16_gelu_pre(a, w, b, out.clone(), pre)
                outs.append((out, pre))
            else:
                out = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16 if epi == 0 else torch.float32)
                N.gemm_bf16(a, w, b, out, epi)
                outs.append((out,))
        finally:
            N.tune(N.TUNE_GEMM_BALANCE, prev)
    torch.cuda.synchronize()
    for x, y in zip(outs[0], outs[1]):
        assert torch.equal(x, y), (x.float() - y.float()).abs().max().item()


@pytest.mark.parametrize("variant", [3, 11, 19, 32, 96, 161])
def test_attention_online_softmax_rescale(N, variant):
    """Force the running max to jump late (rule 26): one key with a huge score
    in the last tile for some rows."""
    prev = N.tune(N.TUNE_ATTN_VARIANT, variant)
    try:
        _online_softmax_rescale(N)
    finally:
        N.tune(N.TUNE_ATTN_VARIANT, prev)


@pytest.mark.parametrize("variant", [32, 33, 96, 97, 161, 289, 545, 2081, 4129])
@pytest.mark.parametrize("case", ["overflow_late", "all_negative", "huge_first_tile", "mixed_rows"])
@pytest.mark.parametrize("waves,n", [(4, 700), (8, 4200)])
def test_attention_offset_free_extremes(N, variant, case, waves, n):
    """Offset-free softmax (VAR & 32): every branch of its range guard against
    an fp64 host reference of the whole tensor (cdna_hip_programming.md §5.4
    rule 26) -- rows whose scores overflow 2^60 only in a late tile, rows whose
    first-tile max is below -60 or above +60 (offset rows), and a mix of offset
    and zero-offset rows inside one wave.  Run on the 4-wave form and on the
    8-wave form (nq >= 4096, the default there: static priority for waves 4-7)."""
    H, D = 2, 64
    C = H * D
    g = torch.Generator().manual_seed(7)
    q = torch.randn(n, C, generator=g) * 0.3
    k = torch.randn(n, C, generator=g) * 0.3
    v = torch.randn(n, C, generator=g)
    if case == "overflow_late":      # score ~ +1100 (log2 units ~ +200) at key n - 50
        q[:40] = 4.0
        k[n - 50] = 4.0
    elif case == "all_negative":     # every score ~ -900 for the first rows
        q[:64] = 4.0
        k[:] = -3.5 + 0.05 * torch.randn(n, C, generator=g)
    elif case == "huge_first_tile":  # key 3 dominates from the first tile on
        q[:64] = 4.0
        k[3] = 4.0
    else:                            # alternate rows: offset / zero-offset in one wave
        q[0:128:2] = 4.0
        q[n - 256:n - 128:2] = 4.0  # rows of the second half of an 8-wave group
        k[10] = 4.0
        k[n - 100] = 4.5
    qkv = torch.cat([q, k, v], 1).to(torch.bfloat16)
    prev = N.tune(N.TUNE_ATTN_VARIANT, variant)
    prev_w = N.tune(N.TUNE_ATTN_WAVES, waves)
    try:
        qkv_d = qkv.cuda()
        o = torch.empty(n, C, device="cuda", dtype=torch.bfloat16)
        N.attention(qkv_d[:, :C], qkv_d[:, C:2 * C], qkv_d[:, 2 * C:], o, 1, H, n, n, D, n, n, n)
        torch.cuda.synchronize()
    finally:
        N.tune(N.TUNE_ATTN_VARIANT, prev)
        N.tune(N.TUNE_ATTN_WAVES, prev_w)
    t = qkv.double().view(1, n, 3, H, D).permute(2, 0, 3, 1, 4)
    ref = _ref_attn(t[0], t[1], t[2], D ** -0.5).permute(0, 2, 1, 3).reshape(n, C)
    got = o.double().cpu()
    assert torch.isfinite(got).all()
    assert _rel(got, ref) < 1e-2, _rel(got, ref)
    # per-row check: no row may be silently wrong (a bad rescale hits whole rows)
    row_err = (got - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-6)
    assert row_err.max() < 5e-2, row_err.max()


def _online_softmax_rescale(N):
    n, H, D = 700, 2, 64
    C = H * D
    q = torch.randn(n, C, device="cuda") * 0.1
    k = torch.randn(n, C, device="cuda") * 0.1
    v = torch.randn(n, C, device="cuda")
    k[650] = 3.0
    q[:50] = 3.0
    qkv = torch.cat([q, k, v], 1).to(torch.bfloat16)
    o = torch.empty(n, C, device="cuda", dtype=torch.bfloat16)
    N.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, 1, H, n, n, D, n, n, n)
    t = qkv.float().view(1, n, 3, H, D).permute(2, 0, 3, 1, 4)
    ref = _ref_attn(t[0], t[1], t[2], D ** -0.5).permute(0, 2, 1, 3).reshape(n, C)
    assert _rel(o, ref) < 1e-2


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("D,H,mode,norm", [(64, 16, 1, True), (64, 16, 0, True), (128, 8, 1, True), (128, 8, 2, True),
                                           (64, 4, 1, False)])
def test_gemm_qkv_fused_matches_two_pass(N, tile, D, H, mode, norm):
    """vggt_gemm_qkv (q/k LayerNorm + RoPE in the GEMM epilogue) against the
    parity-tested two-launch path (gemm_bf16 + qknorm_rope)."""
    _qkv_fused_check(N, tile, D, H, mode, norm, 1500, 256)


@pytest.mark.parametrize("D,H,mode", [(64, 16, 1), (128, 8, 2)])
def test_gemm_qkv_fused_production_rows(N, D, H, mode):
    """Production row count (16 x 1374 tokens, auto tile: the 256x256 ping-pong
    form with a ragged last row panel)."""
    _qkv_fused_check(N, -1, D, H, mode, True, 21984, 1024)


@pytest.mark.parametrize("tile", [4, 8, 9])
@pytest.mark.parametrize("Nn,epi", [(3072, 0), (4096, 1), (4096, 0), (3072, 2), (3072, 3), (1024, 2)])
def test_gemm_production_rows(N, Nn, epi, tile):
    """Every epilogue at M = 21984 on the 256x256 ping-pong form and the
    two-per-CU 256x128 form (a partial last round of workgroups, ragged last
    panel)."""
    prev = N.tune(N.TUNE_GEMM_TILE, tile)
    try:
        test_gemm_epilogues(N, 21984, Nn, 1024, epi)
    finally:
        N.tune(N.TUNE_GEMM_TILE, prev)


def _qkv_fused_check(N, tile, D, H, mode, norm, M, K):
    from aligned_vggt.backbone.layers import RopeTables
    C = H * D
    g = torch.Generator(device="cuda").manual_seed(D + H + mode)
    a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(3 * C, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(3 * C, device="cuda", generator=g).to(torch.bfloat16).float()
    qw, qb, kw, kb = (torch.rand(D, device="cuda", generator=g) + 0.5 for _ in range(4))
    if not norm:
        qw = qb = kw = kb = None
    if mode == 1:
        yy, xx = torch.meshgrid(torch.arange(7), torch.arange(9), indexing="ij")
        pos = torch.cat([torch.zeros(5, 2, dtype=torch.long), torch.stack([yy.reshape(-1), xx.reshape(-1)], -1) + 1])
        rp = RopeTables(pos, D, 100.0, "cuda", N.ROPE_2D)
    elif mode == 2:
        rp = RopeTables(torch.arange(10), D, 100.0, "cuda", N.ROPE_1D)
    else:
        rp = None
    args = (qw, qb, kw, kb, 1e-5 if norm else 0.0, mode, rp.pos if rp else None, rp.period if rp else 1,
            rp.cos if rp else None, rp.sin if rp else None)
    ref = torch.empty(M, 3 * C, device="cuda", dtype=torch.bfloat16)
    N.gemm_bf16(a, w, b, ref, N.EPI_BF16)
    N.qknorm_rope(ref, H, D, *args)
    prev = N.tune(N.TUNE_GEMM_TILE, tile)
    try:
        out = torch.empty_like(ref)
        N.gemm_qkv(a, w, b, out, H, D, *args)
    finally:
        N.tune(N.TUNE_GEMM_TILE, prev)
    torch.cuda.synchronize()
    d = (out.float() - ref.float()).abs()
    # identical arithmetic up to fp32 contraction order: at most one bf16 ulp apart
    assert (d <= ref.float().abs() * 2 ** -7 + 1e-6).all(), d.max().item()
    assert torch.equal(out[:, 2 * C:], ref[:, 2 * C:])  # v block untouched


@pytest.mark.parametrize("tile", [-1, 0, 2, 8])
@pytest.mark.parametrize("M,kv,norm", [(6608, False, True), (2065, True, True), (300, True, False),
                                       (6608, True, True)])
def test_gemm_headnorm_matches_two_pass(N, tile, M, kv, norm):
    """vggt_gemm_headnorm (the temporal cross-attention blocks' q / packed kv
    projection with q_norm / k_norm + 1-D RoPE in the epilogue) against the
    two-pass path it replaces (gemm_bf16, then headnorm_rope on the first H*D
    columns): within one bf16 ulp, the v block of a kv projection bitwise."""
    from aligned_vggt.backbone.layers import RopeTables
    H, D, K = 8, 128, 1024
    C = H * D
    Nn = 2 * C if kv else C
    g = torch.Generator(device="cuda").manual_seed(M + kv)
    a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(Nn, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(Nn, device="cuda", generator=g).to(torch.bfloat16).float()
    nw, nb = (torch.rand(D, device="cuda", generator=g) + 0.5 for _ in range(2))
    if not norm:
        nw = nb = None
    rp = RopeTables(torch.arange(5 if kv else 16) + 3, D, 100.0, "cuda", N.ROPE_1D)
    args = (nw, nb, 1e-6 if norm else 0.0, N.ROPE_1D, rp.pos, rp.period, rp.cos, rp.sin)
    ref = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
    N.gemm_bf16(a, w, b, ref, N.EPI_BF16)
    N.headnorm_rope(ref, 0, H, D, *args)
    prev = N.tune(N.TUNE_GEMM_TILE, tile)
    try:
        out = torch.empty_like(ref)
        N.gemm_headnorm(a, w, b, out, H, D, *args)
    finally:
        N.tune(N.TUNE_GEMM_TILE, prev)
    torch.cuda.synchronize()
    d = (out.float() - ref.float()).abs()
    assert (d <= ref.float().abs() * 2 ** -7 + 1e-6).all(), d.max().item()
    if kv:
        assert torch.equal(out[:, C:], ref[:, C:])  # v block untouched


@pytest.mark.parametrize("tile", [0, 4, 8, 9])
@pytest.mark.parametrize("scale", [1.0, 40.0, 1e-6])
def test_gemm_gelu_lut_exact(N, scale, tile):
    """fc1 epilogue of every GEMM form: GELU from the table of torch's float32
    GELU (LDS copy in the persistent form, global memory in the others) is
    bit-exact against torch (CPU) applied to the same bf16 Linear output --
    including pre-activations outside the table (|x| < 2^-16 and |x| >= 64,
    the scale 1e-6 / 40 cases) that take the limit rules."""
    prev = N.tune(N.TUNE_GEMM_TILE, tile)
    try:
        g = torch.Generator(device="cuda").manual_seed(5)
        M, K, Nn = 4100, 1024, 1024
        a = (torch.randn(M, K, device="cuda", generator=g) * scale).to(torch.bfloat16)
        w = (torch.randn(Nn, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
        b = torch.zeros(Nn, device="cuda")
        pre = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
        out = torch.empty_like(pre)
        N.gemm_bf16(a, w, b, pre, N.EPI_BF16)
        N.gemm_bf16(a, w, b, out, N.EPI_GELU_BF16)
        ref = F.gelu(pre.float().cpu()).to(torch.bfloat16)
        assert torch.equal(out.cpu().view(torch.int16), ref.view(torch.int16))
    finally:
        N.tune(N.TUNE_GEMM_TILE, prev)


@pytest.mark.parametrize("batch,n,H", [(1, 21984, 2), (16, 1374, 4), (3, 51, 16), (3, 17, 16), (1, 6592, 2)])
def test_attention16_accuracy_matches_32x32(N, batch, n, H):
    """The 16x16x32 form (variant 161) against the 32x32x16 form (33) on the
    same inputs, both against an fp64 host reference: the matrix-core shape
    and the exact-restart softmax must not cost accuracy (rel-L2 within 10 %
    of the 32x32 form's, and either form < 5e-3)."""
    D = 64
    C = H * D
    g = torch.Generator().manual_seed(n + H)
    qkv = (torch.randn(batch * n, 3 * C, generator=g) * 1.2).to(torch.bfloat16)
    qkv_d = qkv.cuda()
    outs = {}
    for var in (33, 161):
        prev = N.tune(N.TUNE_ATTN_VARIANT, var)
        prev16 = N.tune(N.TUNE_ATTN16, 0)
        try:
            o = torch.empty(batch * n, C, device="cuda", dtype=torch.bfloat16)
            N.attention(qkv_d[:, :C], qkv_d[:, C:2 * C], qkv_d[:, 2 * C:], o, batch, H, n, n, D, n, n, n)
            outs[var] = o.double().cpu()
        finally:
            N.tune(N.TUNE_ATTN_VARIANT, prev)
            N.tune(N.TUNE_ATTN16, prev16)
    rows = torch.arange(batch * n) if batch * n <= 4096 else torch.randperm(batch * n, generator=g)[:2048]
    t = qkv.double().view(batch, n, 3, H, D)
    errs = {}
    for var, o in outs.items():
        num, den = 0.0, 0.0
        for r in rows.tolist()[:2048]:
            bi, qi = divmod(r, n)
            q = t[bi, qi, 0]                      # (H, D)
            k, v = t[bi, :, 1], t[bi, :, 2]       # (n, H, D)
            s = torch.einsum("hd,nhd->hn", q, k) * D ** -0.5
            ref = torch.einsum("hn,nhd->hd", torch.softmax(s, -1), v).reshape(C)
            num += float(((o[r] - ref) ** 2).sum())
            den += float((ref ** 2).sum())
        errs[var] = (num / den) ** 0.5
    print("rel-L2 vs fp64:", errs)
    assert errs[161] < 5e-3 and errs[33] < 5e-3, errs
    assert errs[161] <= 1.1 * errs[33] + 1e-5, errs


@pytest.mark.parametrize("Nn,K,epi,M", [(4096, 1024, 1, 5000), (1024, 4096, 0, 21984), (3072, 1024, 0, 1000),
                                        (1024, 1024, 2, 6592)])
def test_gemm_persistent_whole_k_loop(N, Nn, K, epi, M):
    """The persistent GEMM's whole-K-tile loop (half 0 stages every W piece, no READ segment
    waits on DMA) at ragged M with the bf16 / GELU / residual epilogues: bitwise run-to-run, and within bf16
    output rounding of an fp32 torch reference of the same op."""
    torch.manual_seed(7)
    dev = torch.device("cuda:0")
    a = ((torch.rand(M, K, device=dev) * 2 - 1)).bfloat16()
    w = ((torch.rand(Nn, K, device=dev) * 2 - 1) * K ** -0.5).bfloat16()
    b = torch.randn(Nn, device=dev) * 0.1
    g = torch.rand(Nn, device=dev)
    x0 = torch.randn(M, Nn, device=dev)

    def run():
        if epi == 2:
            out = x0.clone()
            N.gemm_bf16(a, w, b, out, epi, gamma=g)
        else:
            out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
            N.gemm_bf16(a, w, b, out, epi)
        torch.cuda.synchronize()
        return out

    got = run()
    assert torch.equal(run(), got)
    y = a.float() @ w.float().t() + b
    if epi == 1:
        y = torch.nn.functional.gelu(y)
    elif epi == 2:
        y = x0 + g * y.bfloat16().float()
    e = ((got.float() - y).norm() / y.norm()).item()
    assert e < 4e-3, e
