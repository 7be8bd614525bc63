"""The LDS-DMA staged implicit GEMM (csrc/conv_mfma.hip igemm_dma_kernel) against the
register-staged kernel on every operand mode the learner uses: dense rows (fc forward
with the online/target weight switch, fc dgrad with the K-major B and the ReLU mask),
NHWC im2col (conv3 forward) and the padded K-major dgrad GEMMs (conv3, conv2 per
stride-parity class).  Both kernels run the same MFMA sequence per accumulator, so
the outputs must be identical, in bf16 and in split (hi / lo planes) mode; row counts
that are not tile multiples exercise the clamped rows."""
import pytest
import torch

from apex_dqn_amd.ops.switches import SW

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _sp(t):
    hi = t.to(torch.bfloat16)
    return hi, (t - hi.float()).to(torch.bfloat16)


def _run(C, hint, fn, outs):
    C._HINTS["tile"], C._HINTS["order"] = hint, 0
    try:
        for o in outs:
            o.fill_(7.0)
        fn()
        torch.cuda.synchronize()
        return [o.clone() for o in outs]
    finally:
        C._HINTS["tile"] = C._HINTS["order"] = 0


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("op", ["fc_fwd", "fc_dgrad", "conv3_fwd", "conv3_dgrad", "conv2_dgrad"])
def test_dma_kernel_matches_register_staged(op, split, monkeypatch):
    from apex_dqn_amd.ops import _lib as L, conv as C
    lib = L.require_kernels()
    monkeypatch.setattr(SW, "conv3_dgrad_img", False)
    monkeypatch.setattr(SW, "conv2_dgrad_img", False)
    g = torch.Generator(device="cpu").manual_seed(3)

    def rnd(*shape, s=1.0, relu=False):
        t = torch.randn(*shape, generator=g) * s
        return (torch.relu(t) if relu else t).to(DEV)

    def bfo(*shape):
        return [torch.empty(*shape, device=DEV, dtype=torch.bfloat16) for _ in range(2 if split else 1)]

    def lo(**kw):
        return kw if split else {}

    if op == "fc_fwd":
        M = 384
        (xh, xl), (wh, wl), (w2h, w2l) = _sp(rnd(M, 3136, relu=True)), _sp(rnd(512, 3136, s=0.02)), \
            _sp(rnd(512, 3136, s=0.02))
        b, b2 = rnd(512), rnd(512)
        outs = bfo(M, 512)
        fn = lambda: C.dense_fwd(lib, xh, wh, b, outs[0], True, None, w2h, b2, 256,
                                 **lo(x_lo=xl, w_lo=wl, w2_lo=w2l, out_lo=outs[-1]))
    elif op == "fc_dgrad":
        M = 200
        (dh, dhl), (wh, wl) = _sp(rnd(M, 1024, s=0.01)), _sp(rnd(1024, 3136, s=0.02))
        mask = rnd(M, 3136, relu=True).to(torch.bfloat16)
        outs = bfo(M, 3136)
        fn = lambda: C.dense_dgrad(lib, dh, wh, outs[0], mask, **lo(dh_lo=dhl, w_lo=wl, out_lo=outs[-1]))
    elif op == "conv3_fwd":
        N = 70
        (xh, xl), (wh, wl) = _sp(rnd(N, 9, 9, 64, relu=True)), _sp(rnd(64, 3, 3, 64, s=0.04))
        b = rnd(64)
        outs = bfo(N, 7, 7, 64)
        fn = lambda: C.conv_fwd(lib, xh, wh, b, 1, outs[0], **lo(x_lo=xl, w_lo=wl, out_lo=outs[-1]))
    elif op == "conv3_dgrad":
        N = 37
        (dy, dyl), (wh, wl) = _sp(rnd(N, 7, 7, 64)), _sp(rnd(64, 3, 3, 64, s=0.04))
        mask = rnd(N, 9, 9, 64, relu=True).to(torch.bfloat16)
        outs = bfo(N, 9, 9, 64)
        fn = lambda: C.conv3_dgrad(lib, dy, wh, mask, outs[0], **lo(dy_lo=dyl, w_lo=wl, out_lo=outs[-1]))
    else:
        N = 21
        (dy, dyl), (wh, wl) = _sp(rnd(N, 9, 9, 64)), _sp(rnd(64, 4, 4, 64, s=0.03))
        mask = rnd(N, 20, 20, 64, relu=True).to(torch.bfloat16)
        outs = bfo(N, 20, 20, 64)
        fn = lambda: C.conv2_dgrad(lib, dy, wh, mask, outs[0], **lo(dy_lo=dyl, w_lo=wl, out_lo=outs[-1]))

    ref = _run(C, 2, fn, outs)      # register-staged, 64-row tiles
    assert all(torch.isfinite(r.float()).all() for r in ref)
    # LDS-DMA ring: 128-row 3-stage, 64-row 2-stage, 64-row 3-stage
    for hint in (3, 4, 5):
        got = _run(C, hint, fn, outs)
        for r, o in zip(ref, got):
            assert torch.equal(r, o), (op, split, hint, float((r.float() - o.float()).abs().max()))
