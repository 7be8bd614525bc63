"""MFMA implicit-GEMM kernels (csrc/conv_mfma.hip) vs plain PyTorch fp32
references of the same ops, on bf16-rounded inputs."""
import pytest
import torch

from apex_dqn_amd.ops import reference as R

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _lib():
    from apex_dqn_amd.ops import _lib as L
    return L.require_kernels()


def _bf(x):
    return x.to(DEV, torch.bfloat16)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def _maxrel(a, b):
    return float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12))


@pytest.mark.parametrize("N", [3, 64])
def test_conv1_fwd_from_ring(N):
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(0)
    from apex_dqn_amd.replay.gpu_replay import to_s2d
    raw = torch.randint(0, 256, (50, 84, 84), generator=g, dtype=torch.uint8).to(DEV)
    ring = to_s2d(raw)
    slots = torch.randint(0, 50, (N, 4), generator=g, dtype=torch.int32).to(DEV)
    w = _bf(torch.randn(64, 4, 8, 8, generator=g) * 0.05)
    b = (torch.randn(64, generator=g) * 0.1).to(DEV)
    out = torch.empty(N, 20, 20, 64, dtype=torch.bfloat16, device=DEV)
    C.conv1_s2d_fwd(_lib(), C.Workspace(), ring, slots, w, b, 1 / 255.0, out)
    frames = raw[slots.long()]
    ref = R.conv1_fwd(frames, w.float(), b, 1 / 255.0)
    assert _rel(out, ref) < 1e-2 and _maxrel(out, ref) < 2e-2


@pytest.mark.parametrize("N,layer", [(5, 2), (64, 2), (7, 3), (64, 3)])
def test_conv_fwd_nhwc(N, layer):
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(layer * 100 + N)
    if layer == 2:
        x = _bf(torch.relu(torch.randn(N, 20, 20, 64, generator=g)))
        w = _bf(torch.randn(64, 4, 4, 64, generator=g) * 0.03)
        stride, oh = 2, 9
    else:
        x = _bf(torch.relu(torch.randn(N, 9, 9, 64, generator=g)))
        w = _bf(torch.randn(64, 3, 3, 64, generator=g) * 0.04)
        stride, oh = 1, 7
    b = (torch.randn(64, generator=g) * 0.1).to(DEV)
    out = torch.empty(N, oh, oh, 64, dtype=torch.bfloat16, device=DEV)
    C.conv_fwd(_lib(), x, w, b, stride, out)
    ref = R.conv_fwd(x.float(), w.float(), b, stride)
    assert _rel(out, ref) < 1e-2 and _maxrel(out, ref) < 2e-2


@pytest.mark.parametrize("M", [64, 200, 1024])
def test_dense_fwd_relu_and_mask(M):
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(M)
    x = _bf(torch.relu(torch.randn(M, 3136, generator=g)))
    w = _bf(torch.randn(1024, 3136, generator=g) * 0.02)
    b = (torch.randn(1024, generator=g) * 0.1).to(DEV)
    out = torch.empty(M, 1024, dtype=torch.bfloat16, device=DEV)
    C.dense_fwd(_lib(), x, w, b, out, relu=True)
    ref = R.fc_fwd(x.float(), w.float(), b)
    assert _rel(out, ref) < 1e-2
    # masked (fc dgrad form): out = (dh @ WfcT^T) * (mask > 0)
    dh = _bf(torch.randn(M, 1024, generator=g) * 0.01)
    wT = _bf(torch.randn(3136, 1024, generator=g) * 0.02)
    mask = _bf(torch.randn(M, 3136, generator=g))
    out2 = torch.empty(M, 3136, dtype=torch.bfloat16, device=DEV)
    C.dense_fwd(_lib(), dh, wT, None, out2, relu=False, mask=mask)
    ref2 = (dh.float() @ wT.float().t()) * (mask.float() > 0)
    assert _rel(out2, ref2) < 1e-2
    # K-major B operand (fc dgrad straight from the natural [1024][3136] weight)
    out3 = torch.empty(M, 3136, dtype=torch.bfloat16, device=DEV)
    C.dense_dgrad(_lib(), dh, w, out3, mask)
    ref3 = (dh.float() @ w.float()) * (mask.float() > 0)
    assert _rel(out3, ref3) < 1e-2


def test_pack_dgrad_weights():
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(3)
    wfc = _bf(torch.randn(1024, 3136, generator=g))
    w3 = _bf(torch.randn(64, 3, 3, 64, generator=g))
    w2 = _bf(torch.randn(64, 4, 4, 64, generator=g))
    wfcT = torch.empty(3136, 1024, dtype=torch.bfloat16, device=DEV)
    w3tf = torch.empty(64, 576, dtype=torch.bfloat16, device=DEV)
    w2t = torch.empty(4, 64, 256, dtype=torch.bfloat16, device=DEV)
    C.pack_dgrad_weights(_lib(), wfc, w3, w2, wfcT, w3tf, w2t)
    assert torch.equal(wfcT, wfc.t())
    ref3 = w3.flip(1, 2).permute(3, 1, 2, 0).reshape(64, 576)
    assert torch.equal(w3tf, ref3)
    for cls in range(4):
        p, q = cls >> 1, cls & 1
        sub = w2[:, p::2, q::2, :].flip(1, 2)  # [co][a'][b'][ci] with a' = 1 - a
        assert torch.equal(w2t[cls], sub.permute(3, 1, 2, 0).reshape(64, 256))


@pytest.mark.parametrize("N", [3, 64])
def test_conv_dgrad_layers(N):
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(N + 7)
    lib = _lib()
    w3 = _bf(torch.randn(64, 3, 3, 64, generator=g) * 0.04)
    w2 = _bf(torch.randn(64, 4, 4, 64, generator=g) * 0.03)
    # conv3 dgrad: dY3 (7x7) -> dX2 (9x9) masked by y2
    dy3 = _bf(torch.randn(N, 7, 7, 64, generator=g))
    y2 = _bf(torch.randn(N, 9, 9, 64, generator=g))
    out = torch.empty(N, 9, 9, 64, dtype=torch.bfloat16, device=DEV)
    C.conv3_dgrad(lib, dy3, w3, y2, out)
    ref = R.conv_dgrad(dy3.float(), w3.float(), (N, 9, 9, 64), 1, y2.float())
    assert _rel(out, ref) < 1e-2
    # conv2 dgrad: dY2 (9x9) -> dX1 (20x20), stride 2, masked by y1
    dy2 = _bf(torch.randn(N, 9, 9, 64, generator=g))
    y1 = _bf(torch.randn(N, 20, 20, 64, generator=g))
    out1 = torch.empty(N, 20, 20, 64, dtype=torch.bfloat16, device=DEV)
    C.conv2_dgrad(lib, dy2, w2, y1, out1)
    ref1 = R.conv_dgrad(dy2.float(), w2.float(), (N, 20, 20, 64), 2, y1.float())
    assert _rel(out1, ref1) < 1e-2


@pytest.mark.parametrize("N", [3, 64])
def test_conv_wgrad_layers(N):
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(N + 11)
    lib = _lib()
    ws = C.Workspace()
    for KH, stride, hin, hout in ((3, 1, 9, 7), (4, 2, 20, 9)):
        dy = _bf(torch.randn(N, hout, hout, 64, generator=g))
        x = _bf(torch.relu(torch.randn(N, hin, hin, 64, generator=g)))
        dw = torch.empty(64, KH, KH, 64, device=DEV)
        db = torch.empty(64, device=DEV)
        C.conv_wgrad(lib, ws, dy, x, KH, stride, dw, db, target_rows=256)
        rdw, rdb = R.conv_wgrad(dy.float(), x.float(), KH, stride)
        assert _rel(dw, rdw) < 5e-3, (KH, _rel(dw, rdw))
        assert _rel(db, rdb) < 1e-4


@pytest.mark.parametrize("N,grid", [(3, 0), (32, 0), (32, 5), (9, 16)])
def test_conv1_wgrad_from_ring(N, grid):
    """Image-resident conv1 wgrad (several images per workgroup, idle workgroups)
    and the tiled ring-mode wgrad, both against the fp32 autograd oracle."""
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(N + 5)
    from apex_dqn_amd.replay.gpu_replay import to_s2d
    raw = torch.randint(0, 256, (40, 84, 84), generator=g, dtype=torch.uint8).to(DEV)
    ring = to_s2d(raw)
    slots = torch.randint(0, 40, (N, 4), generator=g, dtype=torch.int32).to(DEV)
    dy = _bf(torch.randn(N, 20, 20, 64, generator=g))
    dw = torch.empty(64, 4, 8, 8, device=DEV)
    db = torch.empty(64, device=DEV)
    C.conv1_wgrad_ring(_lib(), C.Workspace(), dy, ring, slots, 1 / 255.0, dw, db, grid=grid)
    rdw, rdb = R.conv1_wgrad(dy.float(), raw[slots.long()], 1 / 255.0)
    assert _rel(dw, rdw) < 5e-3
    assert _rel(db, rdb) < 1e-4
    dw2, db2 = torch.empty_like(dw), torch.empty_like(db)
    C.conv1_wgrad_ring_tiled(_lib(), C.Workspace(), dy, ring, slots, 1 / 255.0, dw2, db2, target_rows=800)
    assert _rel(dw2, rdw) < 5e-3 and _rel(db2, rdb) < 1e-4


@pytest.mark.parametrize("M", [64, 512])
def test_dense_wgrad(M):
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(M + 1)
    dh = _bf(torch.randn(M, 1024, generator=g))
    x = _bf(torch.relu(torch.randn(M, 3136, generator=g)))
    dw = torch.empty(1024, 3136, device=DEV)
    db = torch.empty(1024, device=DEV)
    C.dense_wgrad(_lib(), dh, x, dw, db)
    assert _rel(dw, dh.float().t() @ x.float()) < 5e-3
    assert _rel(db, dh.float().sum(0)) < 1e-4


def test_fused_online_target_weight_switch():
    """One launch over [online rows | target rows] equals two separate launches."""
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(21)
    lib = _lib()
    N1, N2 = 128, 64  # 128*81 rows is a multiple of the 128-row tile
    x = _bf(torch.relu(torch.randn(N1 + N2, 20, 20, 64, generator=g)))
    wa = _bf(torch.randn(64, 4, 4, 64, generator=g) * 0.03)
    wb = _bf(torch.randn(64, 4, 4, 64, generator=g) * 0.03)
    ba = (torch.randn(64, generator=g) * 0.1).to(DEV)
    bb = (torch.randn(64, generator=g) * 0.1).to(DEV)
    out = torch.empty(N1 + N2, 9, 9, 64, dtype=torch.bfloat16, device=DEV)
    C.conv_fwd(lib, x, wa, ba, 2, out, wb, bb, N1)
    r1 = torch.empty(N1, 9, 9, 64, dtype=torch.bfloat16, device=DEV)
    r2 = torch.empty(N2, 9, 9, 64, dtype=torch.bfloat16, device=DEV)
    C.conv_fwd(lib, x[:N1], wa, ba, 2, r1)
    C.conv_fwd(lib, x[N1:], wb, bb, 2, r2)
    assert torch.equal(out[:N1], r1) and torch.equal(out[N1:], r2)
    # conv1 from the ring with the switch at a 400-row image boundary (N1*400 % 128 == 0)
    from apex_dqn_amd.replay.gpu_replay import to_s2d
    raw = torch.randint(0, 256, (30, 84, 84), generator=g, dtype=torch.uint8).to(DEV)
    ring = to_s2d(raw)
    slots = torch.randint(0, 30, (N1 + N2, 4), generator=g, dtype=torch.int32).to(DEV)
    w1a = _bf(torch.randn(64, 4, 8, 8, generator=g) * 0.05)
    w1b = _bf(torch.randn(64, 4, 8, 8, generator=g) * 0.05)
    o1 = torch.empty(N1 + N2, 20, 20, 64, dtype=torch.bfloat16, device=DEV)
    C.conv1_s2d_fwd(lib, C.Workspace(), ring, slots, w1a, ba, 1 / 255.0, o1, w1b, bb, N1)
    ref_a = R.conv1_fwd(raw[slots[:N1].long()], w1a.float(), ba, 1 / 255.0)
    ref_b = R.conv1_fwd(raw[slots[N1:].long()], w1b.float(), bb, 1 / 255.0)
    assert _rel(o1[:N1], ref_a) < 1e-2 and _rel(o1[N1:], ref_b) < 1e-2


@pytest.mark.parametrize("C", [1, 2, 4])
def test_conv1_s2d_frame_stacks_and_ring_layout(C):
    """Other frame-stack depths (reference parameters.json uses C=1) + the s2d ring
    written by the replay's append path."""
    from apex_dqn_amd.ops import conv as Cv
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    g = torch.Generator(device="cpu").manual_seed(C)
    rp = GpuReplayShard(64, 64, 80, C, device=DEV)
    raw = torch.randint(0, 256, (70, 84, 84), generator=g, dtype=torch.uint8)
    rp.append_frames(raw)
    N = 37
    slots = torch.randint(0, 70, (N, C), generator=g, dtype=torch.int32).to(DEV)
    assert torch.equal(rp.gather_frames(slots).cpu(), raw[slots.long().cpu()])
    w = _bf(torch.randn(64, C, 8, 8, generator=g) * 0.05)
    b = (torch.randn(64, generator=g) * 0.1).to(DEV)
    out = torch.empty(N, 20, 20, 64, dtype=torch.bfloat16, device=DEV)
    Cv.conv1_s2d_fwd(_lib(), Cv.Workspace(), rp.frames, slots, w, b, 1 / 255.0, out)
    ref = R.conv1_fwd(raw[slots.long().cpu()].to(DEV), w.float(), b, 1 / 255.0)
    assert _rel(out, ref) < 1e-2
    dy = _bf(torch.randn(N, 20, 20, 64, generator=g))
    dw = torch.empty(64, C, 8, 8, device=DEV)
    db = torch.empty(64, device=DEV)
    Cv.conv1_wgrad_ring(_lib(), Cv.Workspace(), dy, rp.frames, slots, 1 / 255.0, dw, db)
    rdw, _ = R.conv1_wgrad(dy.float(), raw[slots.long().cpu()].to(DEV), 1 / 255.0)
    assert _rel(dw, rdw) < 5e-3


@pytest.mark.parametrize("N,grid,switch", [(37, 3, 20), (300, 0, 200), (1, 0, 1)])
def test_conv2_image_resident_vs_torch(N, grid, switch):
    """csrc/conv2_img.hip: several images per workgroup (grid < N), the online /
    target weight switch inside a workgroup's image walk, vs the fp32 torch conv."""
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(N)
    x = _bf(torch.relu(torch.randn(N, 20, 20, 64, generator=g)))
    wa = _bf(torch.randn(64, 4, 4, 64, generator=g) * 0.03)
    wb = _bf(torch.randn(64, 4, 4, 64, generator=g) * 0.03)
    ba = (torch.randn(64, generator=g) * 0.1).to(DEV)
    bb = (torch.randn(64, generator=g) * 0.1).to(DEV)
    out = torch.empty(N, 9, 9, 64, dtype=torch.bfloat16, device=DEV)
    C.conv2_img_fwd(_lib(), x, wa, ba, out, wb, bb, switch, grid=grid)
    ref = torch.cat([R.conv_fwd(x[:switch].float(), wa.float(), ba, 2),
                     R.conv_fwd(x[switch:].float(), wb.float(), bb, 2)]) if switch < N else \
        R.conv_fwd(x.float(), wa.float(), ba, 2)
    assert _rel(out, ref) < 1e-2 and _maxrel(out, ref) < 2e-2


@pytest.mark.parametrize("N,grid", [(300, 0), (37, 5), (1, 0)])
def test_conv2_dgrad_image_resident_vs_torch(N, grid):
    """csrc/conv2_img.hip conv2_dgrad_img_kernel (several images per workgroup) vs the
    fp32 torch conv-transpose, ReLU-masked by y1."""
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(N + 7)
    dy2 = _bf(torch.randn(N, 9, 9, 64, generator=g))
    w2 = _bf(torch.randn(64, 4, 4, 64, generator=g) * 0.03)
    y1 = _bf(torch.randn(N, 20, 20, 64, generator=g))
    out = torch.full((N, 20, 20, 64), 7.0, dtype=torch.bfloat16, device=DEV)
    C.conv2_dgrad_img(_lib(), dy2, w2, y1, out, grid=grid)
    ref = R.conv_dgrad(dy2.float(), w2.float(), (N, 20, 20, 64), 2, y1.float())
    assert _rel(out, ref) < 1e-2 and _maxrel(out, ref) < 2e-2


@pytest.mark.parametrize("N,grid", [(300, 0), (37, 5), (1, 0)])
def test_conv3_dgrad_image_resident_vs_torch(N, grid):
    """csrc/conv2_img.hip conv3_dgrad_img_kernel vs the fp32 torch conv-transpose,
    ReLU-masked by y2."""
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(N + 11)
    dy3 = _bf(torch.randn(N, 7, 7, 64, generator=g))
    w3 = _bf(torch.randn(64, 3, 3, 64, generator=g) * 0.04)
    y2 = _bf(torch.randn(N, 9, 9, 64, generator=g))
    out = torch.full((N, 9, 9, 64), 7.0, dtype=torch.bfloat16, device=DEV)
    C.conv3_dgrad_img(_lib(), dy3, w3, y2, out, grid=grid)
    ref = R.conv_dgrad(dy3.float(), w3.float(), (N, 9, 9, 64), 1, y2.float())
    assert _rel(out, ref) < 1e-2 and _maxrel(out, ref) < 2e-2
