"""The fc forward on 128x128 tiles with split K (csrc/conv_mfma.hip fc_gemm128_kernel +
fc_splitk_epilogue_kernel, ``ops.conv.dense_fwd128``) against an fp64 reference of the
same op: online rows [0, r) on the first weight set, target rows [r, M) on the second,
bias + ReLU, in bf16 and in split (hi / lo planes, fp32-accurate) mode, for every K
split and with / without the loader waves; a row count that is not a tile multiple
exercises the clamped rows.  Also the step's default path (the fused learner's
``fc_fwd`` routes here) against the 64x64-tile kernel it replaced."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _sp(t):
    hi = t.to(torch.bfloat16)
    return hi, (t - hi.float()).to(torch.bfloat16)


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("ksplit,lw", [(1, False), (2, True), (3, True), (4, False), (10, True), (49, True)])
def test_fc128_matches_fp64(split, ksplit, lw):
    from apex_dqn_amd.ops import _lib as L, conv as C
    lib = L.require_kernels()
    g = torch.Generator(device="cpu").manual_seed(5)
    M, r, N, K = 1000, 640, 256, 3136
    x = torch.relu(torch.randn(M, K, generator=g)).to(DEV)
    w = (torch.randn(N, K, generator=g) * 0.02).to(DEV)
    w2 = (torch.randn(N, K, generator=g) * 0.02).to(DEV)
    b, b2 = (torch.randn(N, generator=g) * 0.1).to(DEV), (torch.randn(N, generator=g) * 0.1).to(DEV)
    (xh, xl), (wh, wl), (w2h, w2l) = _sp(x), _sp(w), _sp(w2)
    out = torch.full((M, N), 7.0, device=DEV, dtype=torch.bfloat16)
    out_lo = torch.full_like(out, 7.0)
    kw = dict(x_lo=xl, w_lo=wl, w2_lo=w2l, out_lo=out_lo) if split else {}
    ws = C.Workspace()
    C.dense_fwd128(lib, ws, xh, wh, b, out, True, w2h, b2, r, ksplit, lw, **kw)
    torch.cuda.synchronize()
    if split:   # the operands the kernel sees are exactly hi + lo
        xs, ws_, w2s = (xh.double() + xl.double()), (wh.double() + wl.double()), (w2h.double() + w2l.double())
        got = out.double() + out_lo.double()
        tol = 1e-4
    else:
        xs, ws_, w2s = xh.double(), wh.double(), w2h.double()
        got = out.double()
        tol = 8e-3
    ref = torch.cat([xs[:r] @ ws_.T + b.double(), xs[r:] @ w2s.T + b2.double()]).clamp_min(0)
    err = ((got - ref).abs() / (ref.abs() + 1e-1)).max().item()
    assert err < tol, err


@pytest.mark.parametrize("split", [False, True])
def test_backend_fc_fwd_routes_to_fc128(split):
    """HipBackend.fc_fwd at the learner shape (3B = 1536 rows, N = 1024) uses the split-K
    128-tile kernel and agrees with the 64x64-tile kernel to fp32 summation order."""
    from apex_dqn_amd.ops import _lib as L, conv as C
    from apex_dqn_amd.ops.fused_ops import HipBackend
    lib = L.require_kernels()
    be = HipBackend()
    g = torch.Generator(device="cpu").manual_seed(9)
    B = 512
    x = torch.relu(torch.randn(3 * B, 7, 7, 64, generator=g)).to(DEV)
    w = (torch.randn(1024, 3136, generator=g) * 0.02).to(DEV)
    w2 = (torch.randn(1024, 3136, generator=g) * 0.02).to(DEV)
    b, b2 = (torch.randn(1024, generator=g) * 0.1).to(DEV), (torch.randn(1024, generator=g) * 0.1).to(DEV)
    (xh, xl), (wh, wl), (w2h, w2l) = _sp(x), _sp(w), _sp(w2)
    outs = [torch.zeros(3 * B, 1024, device=DEV, dtype=torch.bfloat16) for _ in range(4)]
    lo = lambda o: dict(x_lo=xl, w_lo=wl, w2_lo=w2l, out_lo=o) if split else {}
    calls = []
    orig = C.dense_fwd128
    C.dense_fwd128 = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
    try:
        be.fc_fwd(xh, wh, b, outs[0], w2h, b2, 2 * B, **lo(outs[1]))
    finally:
        C.dense_fwd128 = orig
    assert calls, "fc_fwd did not take the 128-tile path"
    C.dense_fwd(lib, xh.reshape(3 * B, -1), wh, b, outs[2], True, None, w2h, b2, 2 * B,
                **({} if not split else dict(x_lo=xl.reshape(3 * B, -1), w_lo=wl, w2_lo=w2l, out_lo=outs[3])))
    torch.cuda.synchronize()
    a = outs[0].double() + (outs[1].double() if split else 0)
    c = outs[2].double() + (outs[3].double() if split else 0)
    err = ((a - c).abs() / (c.abs() + 1e-1)).max().item()
    assert err < (1e-4 if split else 8e-3), err


@pytest.mark.parametrize("split", [False, True])
def test_c2d_pack_in_fc_epilogue_matches_own_pack(split):
    """The conv2 weight-fragment pack that rides on the fc epilogue launch gives the
    conv2 data gradient bit-identical results to the launcher's own pack."""
    from apex_dqn_amd.ops import _lib as L, conv as C
    lib = L.require_kernels()
    g = torch.Generator(device="cpu").manual_seed(11)
    ws = C.Workspace()
    B = 64
    (xh, xl) = _sp(torch.relu(torch.randn(256, 3136, generator=g)).to(DEV))
    (wh, wl) = _sp((torch.randn(128, 3136, generator=g) * 0.02).to(DEV))
    b = torch.zeros(128, device=DEV)
    fo = [torch.zeros(256, 128, device=DEV, dtype=torch.bfloat16) for _ in range(2)]
    (c2h, c2l) = _sp((torch.randn(64, 4, 4, 64, generator=g) * 0.03).to(DEV))
    (dyh, dyl) = _sp(torch.randn(B, 9, 9, 64, generator=g).to(DEV))
    y1 = torch.relu(torch.randn(B, 20, 20, 64, generator=g)).to(DEV).to(torch.bfloat16)
    outs = [torch.zeros(B, 20, 20, 64, device=DEV, dtype=torch.bfloat16) for _ in range(4)]
    lo = lambda o: dict(dy_lo=dyl, w_lo=c2l, out_lo=o) if split else {}
    C.conv2_dgrad_img(lib, dyh, c2h, y1, outs[0], ws=ws, **lo(outs[1]))
    C.c2d_wfrag_buffer(ws, DEV).fill_(3.0)     # stale contents must be overwritten by the fc launch
    C.dense_fwd128(lib, ws, xh, wh, b, fo[0], True, ksplit=2, loader_waves=True,
                   c2d_pack=(c2h, c2l if split else None),
                   **(dict(x_lo=xl, w_lo=wl, out_lo=fo[1]) if split else {}))
    C.conv2_dgrad_img(lib, dyh, c2h, y1, outs[2], ws=ws, packed=True, **lo(outs[3]))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[2])
    if split:
        assert torch.equal(outs[1], outs[3])
