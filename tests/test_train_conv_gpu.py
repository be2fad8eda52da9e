"""The learner's device path (blokus_rl_amd/alphazero/train_conv.py, csrc/trainconv.hip): the
tower's 3x3 convolutions 64 -> 64 of a training step on split-f16 MFMA products (bk_conv_x3).

* bk_conv_x3_pack splits the weights on the device bit-for-bit as nets.pack_x3 does on the host
  (forward weights, and the flipped / transposed weights of the input gradient);
* the forward and both gradients are fp32-class against an fp64 torch reference: elementwise
  within 1e-5 of conv(|x|, |w|) + |b| (the scale of the sum; fp32's own rounding is ~1e-7 of it),
  on boards of very different magnitudes (the per-board power-of-two scaling) and an all-zero board;
* a Learner on the device path tracks the fp32 (MIOpen) learner step for step (the reference
  trains in fp32: neural_network.py:52-85)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _inputs(seed, B=5):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, 64, 20, 20, generator=g, dtype=torch.float64)
    scales = torch.tensor([1.0, 1e-6, 1e3, 0.0, 3.7][:B], dtype=torch.float64).view(B, 1, 1, 1)
    x = x * scales
    x[0, :, 3:7, :] = 0.0  # zero rows inside a board
    w = torch.randn(64, 64, 3, 3, generator=g, dtype=torch.float64) * (2.0 / 576) ** 0.5
    b = torch.randn(64, generator=g, dtype=torch.float64) * 0.1
    return x, w, b


def _bound(x, w, b=None):
    y = F.conv2d(x.abs(), w.abs(), padding=1)
    return y + (b.abs().view(1, -1, 1, 1) if b is not None else 0)


def test_pack_matches_host_pack():
    from blokus_rl_amd.alphazero.train_conv import pack_weight
    from blokus_rl_amd.nets import pack_x3

    _, w, _ = _inputs(1)
    w = w.float()
    w[3] *= 1e-5  # rows of different magnitudes
    w[7, 5] = 0.0
    for flip in (False, True):
        ref_w = w.transpose(0, 1).flip(2, 3).contiguous() if flip else w
        hp, hinv, _ = pack_x3(ref_w)
        dp, dinv = pack_weight(w.cuda(), flip)
        assert torch.equal(dp.cpu(), hp.cpu()), f"flip={flip}: split fragments differ"
        assert torch.equal(dinv.cpu(), hinv.cpu()), f"flip={flip}: inverse scales differ"


def test_conv_x3_forward_fp32_class():
    from blokus_rl_amd.alphazero.train_conv import conv_x3, pack_weight

    x, w, b = _inputs(2)
    ref = F.conv2d(x, w, b, padding=1)
    bound = _bound(x, w, b)
    xd = x.float().cuda().contiguous(memory_format=torch.channels_last)
    ws, inv = pack_weight(w.float().cuda(), False)
    y = conv_x3(xd, ws, inv, b.float().cuda())
    assert y.is_contiguous(memory_format=torch.channels_last)
    err = (y.double().cpu() - ref).abs()
    assert bool((err <= 1e-5 * bound + 1e-30).all()), f"max err/bound {(err / (bound + 1e-30)).max():.3e}"
    # the fp32 conv's own error on the same inputs, for scale (both far inside the bar)
    y32 = F.conv2d(x.float().cuda(), w.float().cuda(), b.float().cuda(), padding=1).double().cpu()
    r_x3 = float((err / (bound + 1e-30)).max())
    r_32 = float(((y32 - ref).abs() / (bound + 1e-30)).max())
    assert r_x3 <= max(20 * r_32, 1e-6), (r_x3, r_32)
    # the all-zero board gives the bias exactly
    assert torch.equal(y[3].cpu(), b.float().view(64, 1, 1).expand(64, 20, 20))


def test_conv_x3_gradients_fp32_class():
    from blokus_rl_amd.alphazero.train_conv import X3Conv2d

    x, w, b = _inputs(3)
    gy = torch.randn(x.shape, generator=torch.Generator().manual_seed(4), dtype=torch.float64)
    gy[1] *= 1e-4
    # fp64 reference gradients
    xr, wr, br = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    F.conv2d(xr, wr, br, padding=1).backward(gy)
    conv = torch.nn.Conv2d(64, 64, 3, padding=1).cuda()
    with torch.no_grad():
        conv.weight.copy_(w.float())
        conv.bias.copy_(b.float())
    conv.__class__ = X3Conv2d
    xd = x.float().cuda().contiguous(memory_format=torch.channels_last).requires_grad_()
    y = conv(xd)
    y.backward(gy.float().cuda().contiguous(memory_format=torch.channels_last))
    # input gradient: conv(dy, w flipped/transposed) on bk_conv_x3
    wt = w.transpose(0, 1).flip(2, 3)
    gx_bound = _bound(gy, wt)
    err = (xd.grad.double().cpu() - xr.grad).abs()
    assert bool((err <= 1e-5 * gx_bound + 1e-30).all()), f"dx max err/bound {(err / (gx_bound + 1e-30)).max():.3e}"
    # weight and bias gradients (fp32 PyTorch paths) against fp64
    gw_bound = torch.nn.grad.conv2d_weight(x.abs(), w.shape, gy.abs(), padding=1)
    assert bool(((conv.weight.grad.double().cpu() - wr.grad).abs() <= 1e-5 * gw_bound + 1e-30).all())
    gb_bound = gy.abs().sum(dim=(0, 2, 3))
    assert bool(((conv.bias.grad.double().cpu() - br.grad).abs() <= 1e-5 * gb_bound + 1e-30).all())


def test_conv_x3_rejects_bad_shapes():
    from blokus_rl_amd.alphazero.train_conv import conv_x3, pack_weight

    ws, inv = pack_weight(torch.zeros(64, 64, 3, 3, device="cuda"), False)
    with pytest.raises(ValueError):
        conv_x3(torch.zeros(2, 64, 14, 14, device="cuda"), ws, inv, None)
    with pytest.raises(ValueError):
        conv_x3(torch.zeros(2, 32, 20, 20, device="cuda"), ws, inv, None)


def test_learner_device_path_tracks_fp32():
    from blokus_rl_amd.alphazero.learner import DeviceReplay, Learner
    from blokus_rl_amd.alphazero.learner_bench import synthetic_replay
    from blokus_rl_amd.alphazero.train_conv import X3Conv2d
    from blokus_rl_amd.engine import Engine
    from blokus_rl_amd.nets import ResNet

    eng = Engine(20, 4, 5)
    buf, cap, *_ = synthetic_replay(eng, 512, seed=7)
    rb = DeviceReplay(eng, cap=cap)
    rb.add_packed(buf, cap)
    losses = {}
    for dp in (False, True):
        torch.manual_seed(0)
        model = ResNet(20, 4, eng.A, 2).cuda()
        L = Learner(model, lr=1e-3, weight_decay=1e-4, batch_size=256, seed=0, device_path=dp)
        assert L.device_path == dp
        n_x3 = sum(isinstance(m, X3Conv2d) for m in model.modules())
        assert n_x3 == (4 if dp else 0)
        gen = torch.Generator(device="cuda").manual_seed(1)
        out = []
        for _ in range(4):
            idx = torch.randint(0, 512, (256,), device="cuda", generator=gen)
            out.append(float(L.train_step(rb.batch(idx))))
        losses[dp] = out
    for a, b in zip(losses[False], losses[True]):
        assert abs(a - b) <= 2e-4 * abs(a), losses
    # "auto" picks the device path at large batches on the GPU only
    m2 = ResNet(20, 4, eng.A, 1).cuda()
    assert Learner(m2, batch_size=64).device_path is False
    assert Learner(ResNet(20, 4, eng.A, 1).cuda(), batch_size=1024).device_path is True
