"""bk_conv3x3 (fp32 MFMA 3x3 conv with fused bias / residual / ReLU; NHWC activations, planar
observation input) against torch's fp32 convolution (the "plain PyTorch fp32 reference of the same op"), and LeafResNet against the
reference-layout ResNet. Tolerance: the MFMA kernel sums K = 9*cin products in a different order
than MIOpen, so agreement is to f32 rounding: |diff| <= 1e-5 * (sum_k |x_k w_k| + 1) per output."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(x, w, b, relu, res):
    y = F.conv2d(x.double(), w.double(), b.double(), padding=1)
    if res is not None:
        y = y + res.double()
    if relu:
        y = torch.relu(y)
    bound = F.conv2d(x.double().abs(), w.double().abs(), None, padding=1) + 1.0
    return y, bound


@pytest.mark.parametrize("B,N,cin", [(256, 20, 64), (3, 20, 64), (1, 20, 8), (256, 20, 8), (5, 7, 4), (7, 7, 64),
                                     (33, 20, 64), (1, 20, 64), (300, 20, 64), (9, 8, 64), (3, 2, 64), (2, 14, 64)])
@pytest.mark.parametrize("relu,use_res", [(True, False), (False, False), (True, True), (False, True)])
def test_conv3x3_matches_torch(B, N, cin, relu, use_res):
    from blokus_rl_amd.nets import conv3x3, pack_conv3x3

    g = torch.Generator(device="cuda").manual_seed(B * 1000 + N * 10 + cin)
    x = torch.randn((B, cin, N, N), device="cuda", generator=g)
    w = torch.randn((64, cin, 3, 3), device="cuda", generator=g) / (3 * cin ** 0.5)
    b = torch.randn(64, device="cuda", generator=g) * 0.1
    res = (torch.randn((B, 64, N, N), device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
           if use_res else None)
    # planar observation (cin 4, 8) / NHWC activation (cin 64)
    xin = x.contiguous(memory_format=torch.channels_last) if cin == 64 else x.contiguous()
    y = conv3x3(xin, pack_conv3x3(w), b, relu, res)
    torch.cuda.synchronize()
    assert y.is_contiguous(memory_format=torch.channels_last)
    ref, bound = _ref(x, w, b, relu, res)
    err = (y.double() - ref).abs()
    assert bool((err <= 1e-5 * bound).all()), float((err / bound).max())


@pytest.mark.parametrize("B,N,cin", [(256, 20, 64), (3, 20, 64), (33, 20, 64), (300, 20, 64), (9, 8, 64),
                                     (3, 2, 64), (2, 14, 64)])
@pytest.mark.parametrize("relu,use_res", [(True, False), (True, True), (False, True)])
def test_conv3x3_winograd_form1_matches_torch(B, N, cin, relu, use_res, monkeypatch):
    """BK_CONV_WINO=1: the Winograd form with U in LDS (k_conv3x3_wino) instead of form 2."""
    monkeypatch.setenv("BK_CONV_WINO", "1")
    test_conv3x3_matches_torch(B, N, cin, relu, use_res)


@pytest.mark.parametrize("B", [1, 37, 256])
def test_winograd_and_direct_forms_agree(B, monkeypatch):
    """Even N runs the Winograd F(2x2,3x3) form (2, or 1 with BK_CONV_WINO=1), BK_CONV_DIRECT=1
    the direct one: all f32, all within the f32 bound of the fp64 convolution, and close to each
    other (the two Winograd forms group the channel sum differently, so they agree to rounding)."""
    from blokus_rl_amd.nets import conv3x3, pack_conv3x3

    g = torch.Generator(device="cuda").manual_seed(B)
    x = torch.relu(torch.randn((B, 64, 20, 20), device="cuda", generator=g))
    w = torch.randn((64, 64, 3, 3), device="cuda", generator=g) / 24
    b = torch.randn(64, device="cuda", generator=g) * 0.1
    wp = pack_conv3x3(w)
    xin = x.contiguous(memory_format=torch.channels_last)
    y_w = conv3x3(xin, wp, b, True)
    monkeypatch.setenv("BK_CONV_WINO", "1")
    y_w1 = conv3x3(xin, wp, b, True)
    monkeypatch.setenv("BK_CONV_DIRECT", "1")
    y_d = conv3x3(xin, wp, b, True)
    torch.cuda.synchronize()
    ref, bound = _ref(x, w, b, True, None)
    assert bool(((y_w.double() - y_w1.double()).abs() <= 2e-5 * bound).all())
    for y in (y_w, y_w1, y_d):
        assert bool(((y.double() - ref).abs() <= 1e-5 * bound).all())
    assert bool(((y_w.double() - y_d.double()).abs() <= 2e-5 * bound).all())
    assert not torch.equal(y_w, y_d)  # two different kernels really ran


def test_leaf_resnet_matches_reference_forward():
    from blokus_rl_amd.nets import LeafResNet, ResNet

    torch.manual_seed(0)
    for N, P, A in ((20, 4, 30433), (7, 2, 2522)):
        net = ResNet(N, P, A, 3).cuda().eval()
        with torch.no_grad():
            for m in net.modules():
                if isinstance(m, torch.nn.BatchNorm2d):
                    m.running_mean.uniform_(-0.2, 0.2)
                    m.running_var.uniform_(0.5, 1.5)
        leaf = LeafResNet(net).eval()
        assert leaf.native
        x = (torch.rand(64, 2 * P, N, N, device="cuda") < 0.3).float()
        with torch.no_grad():
            lp_ref, v_ref = net(x)
            lp, v = leaf(x)
        assert (lp - lp_ref).abs().max().item() < 2e-4
        assert (lp.exp() - lp_ref.exp()).abs().max().item() < 1e-6
        assert (v - v_ref).abs().max().item() < 1e-5


def test_resnet_heads_kernel_matches_torch():
    from blokus_rl_amd.nets import FusedResNet, ResNet, resnet_heads

    torch.manual_seed(1)
    for N, P, A in ((20, 4, 30433), (7, 2, 2522)):
        f = FusedResNet(ResNet(N, P, A, 1).cuda().eval()).eval()
        x = torch.relu(torch.randn(37, 64, N, N, device="cuda")).contiguous(memory_format=torch.channels_last)
        pf, v = resnet_heads(x, f)
        with torch.no_grad():
            p_ref = torch.relu(f.policy_conv(x)).contiguous().flatten(1)
            v_ref = torch.tanh(f.value_fc2(torch.relu(f.value_fc1(torch.relu(f.value_conv(x)).contiguous().flatten(1)))))
        assert (pf - p_ref).abs().max().item() < 1e-5 * max(1.0, p_ref.abs().max().item())
        assert (v - v_ref).abs().max().item() < 1e-5


def test_leaf_resnet_raw_logits_give_same_masked_softmax():
    from blokus_rl_amd.nets import LeafResNet, ResNet

    torch.manual_seed(2)
    net = ResNet(20, 4, 30433, 2).cuda().eval()
    x = (torch.rand(8, 8, 20, 20, device="cuda") < 0.3).float()
    lp, v = LeafResNet(net).eval()(x)
    lg, v2 = LeafResNet(net, normalize=False).eval()(x)
    assert torch.equal(v, v2)
    ids = torch.randperm(30433, device="cuda")[:300]
    a = torch.softmax(lp[:, ids], 1)
    b = torch.softmax(lg[:, ids], 1)
    assert (a - b).abs().max().item() < 1e-6


@pytest.mark.parametrize("B,N,nblocks", [(256, 20, 5), (3, 20, 2), (300, 20, 1), (37, 14, 2), (5, 14, 3)])
def test_resnet_tower_matches_per_layer_convs(B, N, nblocks):
    """bk_resnet_tower (the whole tower in one launch, one workgroup per board) does the same
    arithmetic as the chain of per-layer Winograd form-2 bk_conv3x3 launches: bitwise equal; and
    within the f32 bound of an fp64 torch tower."""
    from blokus_rl_amd.engine import load_library
    from blokus_rl_amd.nets import conv3x3, pack_conv3x3, pack_tower, resnet_tower

    assert load_library().bk_tower_supported(N)
    g = torch.Generator(device="cuda").manual_seed(B + N + nblocks)
    x = torch.relu(torch.randn((B, 64, N, N), device="cuda", generator=g)).contiguous(memory_format=torch.channels_last)
    ws = [torch.randn((64, 64, 3, 3), device="cuda", generator=g) / 24 for _ in range(2 * nblocks)]
    bs = [torch.randn(64, device="cuda", generator=g) * 0.1 for _ in range(2 * nblocks)]
    out = resnet_tower(x, pack_tower(ws), torch.cat(bs).contiguous(), 2 * nblocks)
    h = x
    for i in range(2 * nblocks):
        last = i + 1 == 2 * nblocks
        h = conv3x3(h, pack_conv3x3(ws[i]), bs[i], last or i % 2 == 0, x if last else None)
    torch.cuda.synchronize()
    assert torch.equal(out, h)
    ref = x.double()
    for i in range(2 * nblocks):
        ref = F.conv2d(ref, ws[i].double(), bs[i].double(), padding=1)
        if i % 2 == 0:
            ref = torch.relu(ref)
    ref = torch.relu(ref + x.double())
    assert float((out.double() - ref).abs().max()) <= 1e-4 * (float(ref.abs().max()) + 1.0)


@pytest.mark.parametrize("B,N,nblocks", [(256, 20, 5), (3, 20, 2), (37, 14, 2)])
def test_resnet_tower_heads_matches_tower_then_heads(B, N, nblocks):
    """bk_resnet_tower_heads (heads fused into the tower launch): the tower output bitwise equal
    to bk_resnet_tower, policy features and values equal to bk_resnet_heads on it to f32
    rounding (the 1x1 convs sum the 64 channels in a different order)."""
    from blokus_rl_amd.nets import FusedResNet, ResNet, pack_tower, resnet_heads, resnet_tower, resnet_tower_heads

    torch.manual_seed(B + N)
    net = ResNet(N, 4, 100, nblocks).cuda().eval()
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
    f = FusedResNet(net).eval()
    convs = [c for blk in f.blocks for c in blk]
    ut = pack_tower([c.weight.detach() for c in convs])
    bt = torch.cat([c.bias.detach().float() for c in convs]).contiguous()
    x = torch.relu(torch.randn((B, 64, N, N), device="cuda")).contiguous(memory_format=torch.channels_last)
    h = resnet_tower(x, ut, bt, 2 * nblocks)
    pf_ref, v_ref = resnet_heads(h, f)
    pf, v, out = resnet_tower_heads(x, ut, bt, 2 * nblocks, f, want_out=True)
    pf2, v2 = resnet_tower_heads(x, ut, bt, 2 * nblocks, f)
    torch.cuda.synchronize()
    assert torch.equal(out, h)
    assert torch.equal(pf, pf2) and torch.equal(v, v2)
    assert torch.allclose(pf, pf_ref, rtol=1e-5, atol=1e-5)
    assert torch.allclose(v, v_ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,N,nblocks", [(256, 20, 5), (3, 20, 2), (37, 14, 1)])
def test_resnet_stem_tower_heads_matches_separate_launches(B, N, nblocks):
    """bk_resnet_stem_tower_heads (stem conv + tower + heads in one launch) against the separate
    stem bk_conv3x3 + bk_resnet_tower_heads: the stem output to f32 rounding (different K order),
    and the heads' outputs within the f32 bound of the fp64 torch reference of the whole net."""
    from blokus_rl_amd.nets import (FusedResNet, ResNet, pack_stem_tower, pack_tower, resnet_stem_tower_heads)

    torch.manual_seed(B * 7 + N)
    net = ResNet(N, 4, 100, nblocks).cuda().eval()
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
    f = FusedResNet(net).eval()
    convs = [c for blk in f.blocks for c in blk]
    ut = pack_tower([c.weight.detach() for c in convs])
    bt = torch.cat([c.bias.detach().float() for c in convs]).contiguous()
    obs = (torch.rand((B, 8, N, N), device="cuda") < 0.3).float()
    pf, v, x0 = resnet_stem_tower_heads(obs, pack_stem_tower(f.stem.weight.detach()), ut, bt, 2 * nblocks, f,
                                        want_x0=True)
    torch.cuda.synchronize()
    with torch.no_grad():
        ref_x0 = torch.relu(F.conv2d(obs.double(), f.stem.weight.double(), f.stem.bias.double(), padding=1))
    assert float((x0.double() - ref_x0).abs().max()) <= 1e-5 * (float(ref_x0.abs().max()) + 1.0)
    with torch.no_grad():
        fd = FusedResNet(net).double().eval()
        p_ref = torch.relu(fd.policy_conv(_tower_ref(fd, obs.double()))).flatten(1)
        xt = _tower_ref(fd, obs.double())
        v_ref = torch.tanh(fd.value_fc2(torch.relu(fd.value_fc1(torch.relu(fd.value_conv(xt)).flatten(1)))))
    assert float((pf.double() - p_ref).abs().max()) <= 1e-4 * (float(p_ref.abs().max()) + 1.0)
    assert float((v.double() - v_ref).abs().max()) <= 1e-4


def _tower_ref(fd, obs):
    x = torch.relu(fd.stem(obs))
    h = x
    for c1, c2 in fd.blocks:
        h = c2(torch.relu(c1(h)))
    return torch.relu(x + h)
