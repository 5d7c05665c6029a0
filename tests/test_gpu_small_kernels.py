"""GPU parity of the fp32 / small-window HIP kernels (heads, decoder) against
plain PyTorch fp32 references of the same op."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def N():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from aligned_vggt import _native
    _native.lib()
    return _native


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("M,Nn,K", [(1, 8, 512), (16, 6144, 2048), (15, 9, 9), (75, 1024, 2048), (23, 100, 36),
                                    (16, 2048, 8192), (3, 64, 1000), (40, 300, 1040), (130, 72, 4160)])
@pytest.mark.parametrize("epi,act", [(3, 0), (1, 0), (2, 0), (3, 1)])
def test_linear_f32(N, M, Nn, K, epi, act):
    g = torch.Generator(device="cuda").manual_seed(M + Nn)
    a = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(Nn, K, device="cuda", generator=g) / K ** 0.5
    b = torch.randn(Nn, device="cuda", generator=g)
    x = F.silu(a) if act else a
    ref = x @ w.t() + b
    if epi == 1:
        ref = F.gelu(ref)
    out = torch.randn(M, Nn, device="cuda", generator=g)
    gam = None
    if epi == 2:
        gam = torch.rand(Nn, device="cuda", generator=g)
        ref = out + gam * ref
    N.linear_f32(a, w, b, out, epi, act_in=act, gamma=gam)
    assert _rel(out, ref) < 2e-6


@pytest.mark.parametrize("M,Nn,K,epi,act", [(16, 512, 512, 3, 0), (16, 2048, 512, 1, 0), (1, 512, 2048, 2, 0),
                                             (130, 1536, 1024, 3, 0), (16, 7, 256, 3, 0), (256, 4096, 4096, 1, 0),
                                             (16, 6144, 2048, 3, 1), (16, 512, 1024, 2, 1)])
@pytest.mark.parametrize("split_k", [128, 32])
def test_linear_f32_split_k_one_launch(N, M, Nn, K, epi, act, split_k):
    """Skinny-M split-K (vggt_linear_f32_ws): the last split block of each output
    tile combines the partials in split order in the same launch.  Bitwise
    run-to-run (fixed order) AND bitwise equal to the two-launch form (partials,
    then a reduce launch in the same split order; VGGT_TUNE_LINEAR_ONE_LAUNCH 0),
    within fp32 rounding of an fp64 reference, incl. the SiLU-on-input form
    (act_in = 1: the camera head's adaLN modulation), and the scratch's tile
    counters are left zero for the next call.  split_k: the smallest k range a
    split keeps (VGGT_TUNE_LINEAR_SPLIT_K; 32: up to 32 splits)."""
    import torch.nn.functional as F_
    g = torch.Generator(device="cuda").manual_seed(M * Nn + K)
    a = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(Nn, K, device="cuda", generator=g) / K ** 0.5
    b = torch.randn(Nn, device="cuda", generator=g)
    gam = torch.rand(Nn, device="cuda", generator=g) if epi == 2 else None
    base = torch.randn(M, Nn, device="cuda", generator=g)
    outs = []
    prev_k = N.tune(N.TUNE_LINEAR_SPLIT_K, split_k)
    prev_wk = N.tune(N.TUNE_LINEAR_WK, 0)  # the cross-workgroup split form
    try:
        for one in (1, 1, 1, 0):
            prev = N.tune(N.TUNE_LINEAR_ONE_LAUNCH, one)
            try:
                out = base.clone()
                N.linear_f32(a, w, b, out, epi, act_in=act, gamma=gam)
            finally:
                N.tune(N.TUNE_LINEAR_ONE_LAUNCH, prev)
            outs.append(out)
    finally:
        N.tune(N.TUNE_LINEAR_SPLIT_K, prev_k)
        N.tune(N.TUNE_LINEAR_WK, prev_wk)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert torch.equal(outs[0], outs[3]), (outs[0] - outs[3]).abs().max()  # one launch == two launches, bitwise
    x = F_.silu(a.double()) if act else a.double()
    ref = x @ w.double().t() + b.double()
    if epi == 1:
        ref = F.gelu(ref)
    if epi == 2:
        ref = base.double() + gam.double() * ref
    assert _rel(outs[0].double(), ref) < 2e-6, _rel(outs[0].double(), ref)
    ws = N._split_ws(a.device, 0)
    assert int(ws[:N.LINEAR_F32_WS_COUNTERS].view(torch.int32).count_nonzero()) == 0


@pytest.mark.parametrize("wk", [64, 128, 512])
@pytest.mark.parametrize("M,Nn,K,epi,act", [(1, 512, 512, 3, 0), (15, 2048, 512, 1, 0), (1, 512, 2048, 2, 0),
                                             (24, 1024, 512, 3, 0), (16, 7, 1000, 3, 0), (64, 512, 4096, 1, 0),
                                             (16, 6144, 2048, 3, 1), (40, 512, 1024, 2, 1), (17, 96, 200, 3, 0),
                                             (130, 1024, 2048, 2, 0)])
def test_linear_f32_in_workgroup_split(N, M, Nn, K, epi, act, wk):
    """M <= 64 on the in-workgroup split-K form (VGGT_TUNE_LINEAR_WK: 2..8
    waves on 16 columns, partials summed in LDS in wave order): bitwise run to
    run, within fp32 rounding of an fp64 reference (ragged K and N, the SiLU
    input, the GELU / LayerScale-residual epilogues), and close to the
    cross-workgroup split form it replaces."""
    import torch.nn.functional as F_
    g = torch.Generator(device="cuda").manual_seed(M * Nn + K + wk)
    a = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(Nn, K, device="cuda", generator=g) / K ** 0.5
    b = torch.randn(Nn, device="cuda", generator=g)
    gam = torch.rand(Nn, device="cuda", generator=g) if epi == 2 else None
    base = torch.randn(M, Nn, device="cuda", generator=g)
    outs = []
    for v in (wk, wk, 0):
        prev = N.tune(N.TUNE_LINEAR_WK, v)
        try:
            out = base.clone()
            N.linear_f32(a, w, b, out, epi, act_in=act, gamma=gam)
        finally:
            N.tune(N.TUNE_LINEAR_WK, prev)
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    x = F_.silu(a.double()) if act else a.double()
    ref = x @ w.double().t() + b.double()
    if epi == 1:
        ref = F.gelu(ref)
    if epi == 2:
        ref = base.double() + gam.double() * ref
    assert _rel(outs[0].double(), ref) < 2e-6, _rel(outs[0].double(), ref)
    assert _rel(outs[0].double(), outs[2].double()) < 2e-6
    # each row's bits do not depend on M: the first 16 rows alone (a chunk's
    # camera-trunk rows) equal their rows of the batched call (a grouped encode)
    if M > 16:
        prev = N.tune(N.TUNE_LINEAR_WK, wk)
        try:
            part = base[:16].clone()
            N.linear_f32(a[:16], w, b, part, epi, act_in=act, gamma=gam)
        finally:
            N.tune(N.TUNE_LINEAR_WK, prev)
        assert torch.equal(part, outs[0][:16])


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("G,H,nq,nk,D", [(1375, 8, 16, 5, 128), (2, 8, 1, 24, 64), (1, 16, 75, 75, 128),
                                          (3, 2, 7, 130 - 2, 32), (413, 8, 16, 16, 128), (5, 3, 9, 11, 48),
                                          (7, 2, 1, 1, 16)])
@pytest.mark.parametrize("exact", [False, True])
def test_attention_small(N, dt, G, H, nq, nk, D, exact):
    C = H * D
    g = torch.Generator(device="cuda").manual_seed(nq * nk)
    q = torch.randn(G * nq, C, device="cuda", generator=g).to(dt)
    kv = torch.randn(G * nk, 2 * C, device="cuda", generator=g).to(dt)
    o = torch.empty(G * nq, C, device="cuda", dtype=dt)
    N.attention_small(q, kv[:, :C], kv[:, C:], o, G, H, nq, nk, D, nq, nk, nq, exact=exact)
    qq = q.float().view(G, nq, H, D).transpose(1, 2)
    kk = kv[:, :C].float().view(G, nk, H, D).transpose(1, 2)
    vv = kv[:, C:].float().view(G, nk, H, D).transpose(1, 2)
    ref = torch.softmax(qq @ kk.transpose(-1, -2) * D ** -0.5, -1) @ vv
    ref = ref.transpose(1, 2).reshape(G * nq, C)
    assert _rel(o, ref) < (4e-3 if dt == torch.bfloat16 else 1e-5)


def test_headnorm_rope_f32_matches_oracle(N):
    from oracle import vggt_oracle as O
    from aligned_vggt.layers.rope import RotaryPositionEmbedding
    H, D, M = 8, 64, 24
    x = torch.randn(M, H * D)
    w, b = torch.randn(D), torch.randn(D)
    pos = torch.arange(M) * 2
    cos, sin = RotaryPositionEmbedding().tables(D, int(pos.max()), "cuda")
    buf = x.clone().cuda()
    N.headnorm_rope_any(buf, 0, H, D, w.cuda(), b.cuda(), 1e-5, N.ROPE_1D, pos.to(torch.int32).cuda(), M, cos, sin)
    ref = O.rope1d(O.layer_norm(x.view(M, H, D).transpose(0, 1)[None], w, b, 1e-5), pos[None])
    ref = ref[0].transpose(0, 1).reshape(M, H * D)
    assert _rel(buf.cpu(), ref) < 1e-6


def test_rope_module_matches_reference_fixture(N, golden):
    from aligned_vggt.layers.rope import RotaryPositionEmbedding
    g = golden("rope1d")
    for i in range(3):
        y = RotaryPositionEmbedding()(torch.from_numpy(g[f"x{i}"]).cuda(), torch.from_numpy(g[f"pos{i}"]).cuda())
        torch.testing.assert_close(y.cpu(), torch.from_numpy(g[f"y{i}"]), atol=2e-6, rtol=0)


def test_gated_update_matches_reference_fixture(N, golden):
    from aligned_vggt.layers.gated_update import GatedUpdate
    for tag in ("d64", "d32"):
        g = golden("gated_update_" + tag)
        D, Nt = g["memory"].shape[2], g["memory"].shape[1]
        m = GatedUpdate(D, Nt)
        m.load_state_dict({k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("p.")})
        m = m.cuda()
        out = m(torch.from_numpy(g["memory"]).cuda(), torch.from_numpy(g["update"]).cuda())
        torch.testing.assert_close(out.cpu(), torch.from_numpy(g["out"]), atol=2e-5, rtol=0)


@pytest.mark.parametrize("B,Nt,D", [(1, 8, 512), (2, 8, 512), (3, 5, 96)])
def test_gated_update_fused_matches_torch_form(N, B, Nt, D):
    """The inference GatedUpdate (prep / grouped delta MLPs / diff / gate MLP /
    tail kernels) against its fp32 torch form (forward_train under no_grad:
    the reference's algebra, gated_update.py:43-79) at the decoder's shape and
    a batch; the grouped linears equal per-token linear_f32 calls bitwise."""
    from aligned_vggt.layers.gated_update import GatedUpdate
    torch.manual_seed(B * Nt + D)
    m = GatedUpdate(D, Nt).cuda()
    mem = F.normalize(torch.randn(B, Nt, D, device="cuda"), dim=-1)
    upd = torch.randn(B, 1, D, device="cuda") * 3
    out = m(mem, upd)
    with torch.no_grad():
        ref = m.forward_train(mem, upd)
    torch.testing.assert_close(out, ref, atol=2e-5, rtol=0)
    # grouped == per token, bitwise
    scale = upd.norm(dim=-1, keepdim=True)
    inp = torch.cat([upd.expand_as(mem), mem * scale, mem.mean(1, keepdim=True).expand_as(mem) * scale], -1)
    w1, b1, w2, b2 = m._packed()
    hid = torch.empty(Nt, B, D, device="cuda")
    N.linear_f32_grouped(inp.transpose(0, 1), w1, b1, hid, N.EPI_GELU_BF16)
    for i, mlp in enumerate(m.delta_mlps):
        h1 = torch.empty(B, D, device="cuda")
        N.linear_f32(inp[:, i], mlp[0].weight, mlp[0].bias, h1, N.EPI_GELU_BF16)
        assert torch.equal(h1, hid[i])


def test_layernorm_grouped_and_cast(N):
    F_, P, C, skip = 3, 21, 1024, 5
    x = torch.randn(F_ * P, C, device="cuda")
    w, b = torch.randn(C, device="cuda"), torch.randn(C, device="cuda")
    hw = P - skip
    y = torch.zeros(F_ * hw, C, device="cuda")
    N.layernorm_grouped(x, w, b, 1e-5, y, F_ * hw, C, hw, P, skip, hw, 0)
    ref = F.layer_norm(x.view(F_, P, C)[:, skip:], (C,), w, b, 1e-5).reshape(-1, C)
    assert _rel(y, ref) < 1e-6
    z = torch.zeros(F_ * (hw + 1), C, device="cuda")
    N.layernorm_grouped(y, w, b, 1e-5, z, F_ * hw, C, hw, hw, 0, hw + 1, 1)
    assert z.view(F_, hw + 1, C)[:, 0].abs().max() == 0
    xb = torch.empty(F_ * P, C, device="cuda", dtype=torch.bfloat16)
    N.cast_f32_bf16(x, xb)
    assert torch.equal(xb, x.to(torch.bfloat16))


def _conv_call(N, prec, xr, n, hi, wi, ci, wp, b, co, k, s, p, y, **kw):
    if prec == "fp32":
        return N.conv2d_f32(xr, n, hi, wi, ci, wp, b, co, k, k, s, p, y, **kw)
    w_hi, w_lo = N.split_bf16x2(wp)
    if prec == "bf16x3pre":
        # pre-split activation (LDS-DMA gather): bitwise equal to the register-staged form
        relu_in = kw.pop("relu_in", False)
        x_hi, x_lo = N.split_act_bf16x2(xr, relu_in)
        N.conv2d_bf16x3_pre(x_hi, x_lo, n, hi, wi, ci, w_hi, w_lo, b, co, k, k, s, p, y, **kw)
        y2 = torch.empty_like(y)
        N.conv2d_bf16x3(xr, n, hi, wi, ci, w_hi, w_lo, b, co, k, k, s, p, y2, relu_in=relu_in, **kw)
        assert torch.equal(y, y2)
        return y
    return N.conv2d_bf16x3(xr, n, hi, wi, ci, w_hi, w_lo, b, co, k, k, s, p, y, **kw)


@pytest.mark.parametrize("prec,tol", [("fp32", 2e-6), ("bf16x3", 3e-5), ("bf16x3pre", 3e-5)])
@pytest.mark.parametrize("case", ["3x3", "3x3s2", "1x1pos", "rcu", "shuffle4", "shuffle2", "co2", "co256", "co192"])
def test_conv2d_f32(N, case, prec, tol):
    """fp32 implicit-GEMM conv (exact f32 MFMA) and its split-bf16 form
    against torch fp32; the split form's tolerance is its 2^-16 operand split."""
    g = torch.Generator(device="cuda").manual_seed(hash(case) % 1000)
    n, hi, wi = 2, 13, 11
    ci, co, k, s, p = 64, 64, 3, 1, 1
    if case == "3x3s2":
        s = 2
    if case == "1x1pos":
        k, p, co = 1, 0, 128
    if case == "co2":
        k, p, ci, co = 1, 0, 32, 2
    if case == "co256":
        co = 256
    if case == "co192":  # partial 128-wide N tile
        co, k, p = 192, 1, 0
    if case.startswith("shuffle"):
        f = int(case[-1])
        x = torch.randn(n, ci, hi, wi, device="cuda", generator=g)
        wt = torch.randn(ci, co, f, f, device="cuda", generator=g) / ci ** 0.5
        bt = torch.randn(co, device="cuda", generator=g)
        ref = F.conv_transpose2d(x, wt, bt, stride=f)
        wp = wt.permute(2, 3, 1, 0).reshape(f * f * co, ci)
        wp = torch.cat([wp, wp.new_zeros((-wp.shape[0]) % 128, ci)])
        xr = x.permute(0, 2, 3, 1).reshape(-1, ci).contiguous()
        y = torch.empty(n * hi * f * wi * f, co, device="cuda")
        _conv_call(N, prec, xr, n, hi, wi, ci, wp.contiguous(), bt, co, 1, 1, 0, y, shuffle=f)
        got = y.view(n, hi * f, wi * f, co).permute(0, 3, 1, 2)
        assert _rel(got, ref) < tol
        return
    x = torch.randn(n, ci, hi, wi, device="cuda", generator=g)
    w = torch.randn(co, ci, k, k, device="cuda", generator=g) / (ci * k * k) ** 0.5
    b = torch.randn(co, device="cuda", generator=g)
    ho, wo = (hi + 2 * p - k) // s + 1, (wi + 2 * p - k) // s + 1
    xr = x.permute(0, 2, 3, 1).reshape(-1, ci).contiguous()
    wp = w.permute(0, 2, 3, 1).reshape(co, -1)
    wp = torch.cat([wp, wp.new_zeros((-co) % 128, wp.shape[1])]).contiguous()
    y = torch.empty(n * ho * wo, co, device="cuda")
    kw = {}
    ref_in = x
    if case == "rcu":
        kw = dict(relu_in=True, relu_out=True)
        ref_in = F.relu(x)
    pos = None
    if case == "1x1pos":
        pos = torch.randn(ho * wo, co, device="cuda", generator=g)
    r1 = r2 = None
    if case == "3x3":
        r1 = torch.randn(n * ho * wo, co, device="cuda", generator=g)
        r2 = torch.randn(n * ho * wo, co, device="cuda", generator=g)
    _conv_call(N, prec, xr, n, hi, wi, ci, wp, b, co, k, s, p, y, res1=r1, res1_relu=True, res2=r2, pos=pos, **kw)
    ref = F.conv2d(ref_in, w, b, stride=s, padding=p)
    if case == "rcu":
        ref = F.relu(ref)
    ref = ref.permute(0, 2, 3, 1).reshape(-1, co)
    if pos is not None:
        ref = ref + pos.repeat(n, 1)
    if r1 is not None:
        ref = ref + F.relu(r1) + r2
    assert _rel(y, ref) < tol


def test_upsample_and_activate(N):
    n, hi, wi, C = 2, 7, 9, 8
    x = torch.randn(n, C, hi, wi, device="cuda")
    ref = F.interpolate(x, size=(20, 13), mode="bilinear", align_corners=True)
    y = torch.empty(n * 20 * 13, C, device="cuda")
    N.upsample_bilinear_f32(x.permute(0, 2, 3, 1).reshape(-1, C).contiguous(), n, hi, wi, C, y, 20, 13)
    assert _rel(y.view(n, 20, 13, C).permute(0, 3, 1, 2), ref) < 1e-6
    z = torch.randn(100, 4, device="cuda")
    pts = torch.empty(100, 3, device="cuda")
    conf = torch.empty(100, device="cuda")
    sc = torch.tensor([2.0, 3.0], device="cuda")
    N.dpt_activate(z, 100, 50, 4, 1, sc, pts, conf)
    ref = torch.sign(z[:, :3]) * torch.expm1(z[:, :3].abs()) * sc.repeat_interleave(50)[:, None]
    assert _rel(pts, ref) < 1e-6
    assert _rel(conf, 1 + z[:, 3].exp()) < 1e-6


def _rand_quat(g, *shape):
    """Unit quaternions spread over the whole sphere (every mat_to_quat branch)."""
    return F.normalize(torch.randn(*shape, 4, generator=g), dim=-1)


@pytest.mark.parametrize("B,S,S_prev,ov,mode", [(1, 16, 16, 4, "markley"), (2, 5, 5, 2, "markley"),
                                                (3, 8, 16, 7, "markley"), (2, 6, 6, 1, "single"),
                                                (2, 4, 4, 2, "gt"), (2, 9, 0, 0, "first"), (1, 1, 0, 0, "first")])
def test_pose_compose_matches_oracle(N, B, S, S_prev, ov, mode):
    """vggt_pose_compose (featureAligned_vggt.py:96-143, :187-196) against the
    oracle's torch restatement: first chunk, Markley mean (ov > 1), single
    overlap transform, chunk_gt; large rotations.  The Markley eigenvector's
    sign is arbitrary but enters only through quat_to_mat, so outputs agree."""
    from oracle import vggt_oracle as O
    g = torch.Generator().manual_seed(B * 100 + S)
    H, W = 154, 518
    cs = torch.cat([torch.randn(B, 1, 3, generator=g), _rand_quat(g, B, 1), 0.5 + torch.rand(B, 1, 1, generator=g)], -1)
    fs = torch.cat([torch.randn(B, S - 1, 3, generator=g), _rand_quat(g, B, S - 1) * 1.3], -1)
    cam = torch.cat([torch.randn(B, S, 3, generator=g), _rand_quat(g, B, S) * 0.9,
                     0.8 + 0.4 * torch.rand(B, S, 2, generator=g)], -1)
    ctx = gt = None
    if mode != "first":
        ctx = torch.cat([torch.randn(B, S_prev, 3, generator=g), _rand_quat(g, B, S_prev),
                         torch.rand(B, S_prev, 2, generator=g)], -1)
    if mode == "gt":
        gt = O.pose_encoding_to_extri(torch.cat([torch.randn(B, 1, 3, generator=g), _rand_quat(g, B, 1)], -1))[:, 0]
    ref, ref_pt = O.compose_poses(cs, fs, cam, ctx, gt, ov, (H, W))
    out, pt = N.pose_compose(cs.cuda(), fs.cuda(), cam.cuda(), ctx.cuda() if ctx is not None else None,
                             gt.cuda() if gt is not None else None, ov, (H, W))
    torch.cuda.synchronize()
    out, pt = out.cpu(), pt.cpu()
    assert _rel(out[..., :3], ref[..., :3]) < 2e-5, _rel(out[..., :3], ref[..., :3])
    assert float((1 - (out[..., 3:7] * ref[..., 3:7]).sum(-1).abs()).abs().max()) < 1e-5  # w >= 0 in both
    assert _rel(out[..., 7:], ref[..., 7:]) < 1e-6
    assert _rel(pt, ref_pt) < 2e-5


def test_upsample_separable_pos_bitwise(N):
    """The final DPT upsample with the separable [w + h, C/2] positional table
    equals the full [h*w, C] table form bitwise (same floats, same adds)."""
    from aligned_vggt.backbone.dpt_head import pos_table, pos_table_sep
    n, hi, wi, C, ho, wo = 2, 9, 13, 16, 22, 31
    x = torch.randn(n * hi * wi, C, device="cuda")
    full = pos_table(C, ho, wo, wo, ho).cuda()
    sep = pos_table_sep(C, ho, wo, wo, ho).cuda()
    outs = []
    for kind in ("full", "sep"):
        y = torch.empty(n * ho * wo, C, device="cuda")
        ys = (torch.empty(n * ho * wo, C, device="cuda", dtype=torch.bfloat16),
              torch.empty(n * ho * wo, C, device="cuda", dtype=torch.bfloat16))
        if kind == "full":
            N.upsample_bilinear_split(x, n, hi, wi, C, y, ho, wo, full, y_split=ys)
        else:
            N.upsample_bilinear_split_sep(x, n, hi, wi, C, y, ho, wo, sep, y_split=ys)
        outs.append((y, ys))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1][0], outs[1][1][0]) and torch.equal(outs[0][1][1], outs[1][1][1])


@pytest.mark.parametrize("n,hi,wi,C,ho,wo,co", [(2, 9, 13, 64, 22, 37, 32), (1, 17, 17, 128, 30, 30, 17),
                                                (3, 8, 6, 32, 8, 6, 32), (16, 74, 74, 128, 130, 130, 32)])
def test_conv_upsample_fused(N, n, hi, wi, C, ho, wo, co):
    """vggt_conv2d_upsample_bf16x3 (resize + separable pos + split + 3x3 conv in one
    launch) against the unfused upsample_split_sep + conv2d_bf16x3_pre (same
    products: equal to fp32 round-off) and against torch fp32 (F.interpolate,
    align_corners=True, + pos, F.conv2d) at the split-bf16 tolerance; ragged
    4 x 32 output tiles at the image edges, co < 32."""
    from aligned_vggt.backbone.dpt_head import pos_table, pos_table_sep
    g = torch.Generator(device="cuda").manual_seed(n * 1000 + ho)
    x = torch.randn(n * hi * wi, C, device="cuda", generator=g)
    w = torch.randn(co, C, 3, 3, device="cuda", generator=g) * 0.05
    b = torch.randn(co, device="cuda", generator=g) * 0.1
    wp = torch.zeros(128, 9 * C, device="cuda")
    wp[:co] = w.permute(0, 2, 3, 1).reshape(co, 9 * C)
    whi, wlo = N.split_bf16x2(wp)
    sep = pos_table_sep(C, ho, wo, wo, ho).cuda()
    y = torch.empty(n * ho * wo, co, device="cuda")
    ys = (torch.empty(n * ho * wo, co, device="cuda", dtype=torch.bfloat16),
          torch.empty(n * ho * wo, co, device="cuda", dtype=torch.bfloat16))
    N.conv2d_upsample_bf16x3(x, n, hi, wi, C, sep, ho, wo, whi, wlo, b, co, y, relu_out=True, y_split=ys)
    # unfused form
    uh = torch.empty(n * ho * wo, C, device="cuda", dtype=torch.bfloat16)
    ul = torch.empty_like(uh)
    N.upsample_bilinear_split_sep(x, n, hi, wi, C, None, ho, wo, sep, y_split=(uh, ul))
    y2 = torch.empty_like(y)
    N.conv2d_bf16x3_pre(uh, ul, n, ho, wo, C, whi, wlo, b, co, 3, 3, 1, 1, y2, relu_out=True)
    # torch fp32
    xi = x.view(n, hi, wi, C).permute(0, 3, 1, 2)
    up = F.interpolate(xi, size=(ho, wo), mode="bilinear", align_corners=True)
    up = up + pos_table(C, ho, wo, wo, ho).cuda().view(ho, wo, C).permute(2, 0, 1)[None]
    ref = F.relu(F.conv2d(up, w, b, padding=1)).permute(0, 2, 3, 1).reshape(-1, co)
    torch.cuda.synchronize()
    assert _rel(y, y2) < 1e-6, _rel(y, y2)
    assert _rel(y, ref) < 3e-5, _rel(y, ref)
    hv = y.to(torch.bfloat16)
    assert torch.equal(ys[0], hv) and _rel(ys[0].float() + ys[1].float(), y) < 1e-5
