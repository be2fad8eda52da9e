"""The learner's device path (blokus_rl_amd/alphazero/train_conv.py, csrc/trainconv.hip): the
tower's 3x3 convolutions 64 -> 64 of a training step on split-f16 MFMA products (bk_conv_x3).

* bk_conv_x3_pack splits the weights on the device bit-for-bit as nets.pack_x3 does on the host
  (forward weights, and the flipped / transposed weights of the input gradient);
* the forward and both gradients are fp32-class against an fp64 torch reference: elementwise
  within 1e-5 of conv(|x|, |w|) + |b| (the scale of the sum; fp32's own rounding is ~1e-7 of it),
  on boards of very different magnitudes (the per-board power-of-two scaling) and an all-zero board;
* a Learner on the device path tracks the fp32 (MIOpen) learner step for step (the reference
  trains in fp32: neural_network.py:52-85): one step's gradients parameter by parameter, and the
  losses over four SGD steps."""
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
    # weight gradient (bk_conv_x3_wgrad) and bias gradient (a PyTorch sum) against fp64
    gw_bound = torch.nn.grad.conv2d_weight(x.abs(), w.shape, gy.abs(), padding=1)
    assert bool(((conv.weight.grad.double().cpu() - wr.grad).abs() <= 1e-5 * gw_bound + 1e-30).all())
    gb_bound = gy.abs().sum(dim=(0, 2, 3))
    assert bool(((conv.bias.grad.double().cpu() - br.grad).abs() <= 1e-5 * gb_bound + 1e-30).all())


def test_conv_x3_wgrad_fp32_class():
    """bk_conv_x3_wgrad at 300 boards (256 workgroups, some with two boards) whose magnitudes
    differ by up to 1e8 (the workgroup's operand scales drop, and its sums are rescaled, when a
    later band holds larger values), with all-zero boards among them."""
    from blokus_rl_amd.alphazero.train_conv import conv_x3_wgrad

    B = 300
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(B, 64, 20, 20, device="cuda", dtype=torch.float64, generator=g)
    gy = torch.randn(B, 64, 20, 20, device="cuda", dtype=torch.float64, generator=g)
    sx = torch.logspace(-4, 4, B, device="cuda", dtype=torch.float64)[torch.randperm(B, device="cuda", generator=g)]
    sy = torch.logspace(-4, 4, B, device="cuda", dtype=torch.float64)[torch.randperm(B, device="cuda", generator=g)]
    x *= sx.view(B, 1, 1, 1)
    gy *= sy.view(B, 1, 1, 1)
    x[5] = 0.0
    gy[17] = 0.0
    gy[300 - 44, :, 10:, :] *= 1e6  # a large lower band after a small upper one (rescale inside a board)
    x32 = x.float().contiguous(memory_format=torch.channels_last)
    gy32 = gy.float().contiguous(memory_format=torch.channels_last)
    dw = conv_x3_wgrad(x32, gy32).double()
    xr, gyr = x32.double(), gy32.double()  # the fp64 reference on the same (f32-rounded) inputs
    ref = torch.nn.grad.conv2d_weight(xr, (64, 64, 3, 3), gyr, padding=1)
    bound = torch.nn.grad.conv2d_weight(xr.abs(), (64, 64, 3, 3), gyr.abs(), padding=1)
    err = (dw - ref).abs()
    ratio = float((err / (bound + 1e-30)).max())
    print(f"wgrad max err / bound = {ratio:.3e}")
    assert ratio <= 1e-5
    # deterministic: the partial sums are added in a fixed order
    assert torch.equal(conv_x3_wgrad(x32, gy32), conv_x3_wgrad(x32, gy32))
    # one board, and zero boards
    one = conv_x3_wgrad(x32[:1], gy32[:1]).double()
    ref1 = torch.nn.grad.conv2d_weight(xr[:1], (64, 64, 3, 3), gyr[:1], padding=1)
    b1 = torch.nn.grad.conv2d_weight(xr[:1].abs(), (64, 64, 3, 3), gyr[:1].abs(), padding=1)
    assert bool(((one - ref1).abs() <= 1e-5 * b1 + 1e-30).all())
    assert torch.equal(conv_x3_wgrad(x32[:0], gy32[:0]), torch.zeros(64, 64, 3, 3, device="cuda"))


def test_fused_batchnorm_matches_fp64():
    """FusedBatchNorm2d (bk_bn_forward / bk_bn_backward) against nn.BatchNorm2d in fp64: the
    output, the running statistics after two steps, and dx / dgamma / dbeta, to 2e-6 relative to
    each quantity's scale; eval mode is PyTorch's own path."""
    from blokus_rl_amd.alphazero.train_conv import FusedBatchNorm2d

    g = torch.Generator().manual_seed(5)
    ref = torch.nn.BatchNorm2d(64).double()
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5, generator=g)
        ref.bias.uniform_(-0.3, 0.3, generator=g)
    bn = torch.nn.BatchNorm2d(64).cuda()
    bn.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in ref.state_dict().items()})
    bn.__class__ = FusedBatchNorm2d
    for step in range(2):
        x = (torch.randn(37, 64, 20, 20, generator=g, dtype=torch.float64) * 3 + 5).float().double()
        gy = torch.randn(37, 64, 20, 20, generator=g, dtype=torch.float64).float().double()
        xr = x.clone().requires_grad_()
        ref.train()
        yr = ref(xr)
        yr.backward(gy)
        xd = x.float().cuda().contiguous(memory_format=torch.channels_last).requires_grad_()
        bn.train()
        y = bn(xd)
        y.backward(gy.float().cuda().contiguous(memory_format=torch.channels_last))
        assert float((y.detach().double().cpu() - yr.detach()).abs().max()) <= 2e-6 * float(yr.detach().abs().max())
        assert float((xd.grad.double().cpu() - xr.grad).abs().max()) <= 2e-6 * float(xr.grad.abs().max())
        for a, b in ((bn.weight.grad, ref.weight.grad), (bn.bias.grad, ref.bias.grad)):
            assert float((a.double().cpu() - b).abs().max()) <= 2e-6 * float(b.abs().max())
        bn.weight.grad = bn.bias.grad = None
        ref.zero_grad()
    for a, b in ((bn.running_mean, ref.running_mean), (bn.running_var, ref.running_var)):
        assert float((a.double().cpu() - b).abs().max()) <= 2e-6 * float(b.abs().max())
    assert int(bn.num_batches_tracked) == int(ref.num_batches_tracked) == 2
    bn.eval()
    ref.eval()
    x = torch.randn(3, 64, 20, 20, generator=g, dtype=torch.float64)
    assert torch.allclose(bn(x.float().cuda()).double().cpu(), ref(x), atol=1e-5, rtol=1e-5)


def test_conv_x3_rejects_bad_shapes():
    from blokus_rl_amd.alphazero.train_conv import conv_x3, pack_weight

    ws, inv = pack_weight(torch.zeros(64, 64, 3, 3, device="cuda"), False)
    with pytest.raises(ValueError):
        conv_x3(torch.zeros(2, 64, 14, 14, device="cuda"), ws, inv, None)
    with pytest.raises(ValueError):
        conv_x3(torch.zeros(2, 32, 20, 20, device="cuda"), ws, inv, None)


def _replay(n=512):
    from blokus_rl_amd.alphazero.learner import DeviceReplay
    from blokus_rl_amd.alphazero.learner_bench import synthetic_replay
    from blokus_rl_amd.engine import Engine

    eng = Engine(20, 4, 5)
    buf, cap, *_ = synthetic_replay(eng, n, seed=7)
    rb = DeviceReplay(eng, cap=cap)
    rb.add_packed(buf, cap)
    return eng, rb


def test_learner_device_path_gradients_match_fp32():
    """One training step's gradients (the reference's compute_loss through the whole ResNet) on the
    device path against the fp32 path, parameter by parameter: within 5e-4 of the gradient's norm
    (the fp32 path's own error: its batch-norm parameter gradients are f32 sums over 102k terms
    that largely cancel, ~1e-4 of their norm off the fp64 value; the device path sums in fp64 and
    is checked against fp64 directly in test_fused_batchnorm_matches_fp64).
    The biases of the convs that feed a batch norm are left out: under train-mode batch norm their
    gradient is zero in exact arithmetic (the channel mean is subtracted), so both paths return
    rounding noise."""
    from blokus_rl_amd.alphazero.learner import Learner, alphazero_loss
    from blokus_rl_amd.nets import ResNet

    eng, rb = _replay()
    idx = torch.randint(0, 512, (256,), device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
    batch = rb.batch(idx)
    grads = {}
    for dp in (False, True):
        torch.manual_seed(0)
        model = ResNet(20, 4, eng.A, 2).cuda()
        L = Learner(model, batch_size=256, device_path=dp)
        obs = batch["observation"].contiguous(memory_format=torch.channels_last) if dp else batch["observation"]
        model.train()
        p, v = model(obs)
        alphazero_loss(p, v, batch).backward()
        grads[dp] = {k: t.grad.detach().clone() for k, t in model.named_parameters()}
    for k, g32 in grads[False].items():
        if k in ("conv1.bias", "policy_conv.bias", "value_conv.bias") or (
                k.startswith("res_blocks") and k.endswith(".bias") and k.split(".")[2] in ("0", "3")):
            continue  # the bias of a conv that feeds a batch norm: zero in exact arithmetic
        d = (grads[True][k] - g32).norm()
        assert float(d) <= 5e-4 * float(g32.norm()) + 1e-12, (k, float(d), float(g32.norm()))


def test_learner_device_path_tracks_fp32():
    """Four SGD steps (an update proportional to the gradient, so rounding differences stay that
    size; Adam's first steps move every weight by +-lr whatever the gradient's size, which turns
    rounding-level gradients into O(lr) weight differences on both paths alike): the losses of the
    device path and the fp32 path agree to 1e-4."""
    from blokus_rl_amd.alphazero.learner import Learner
    from blokus_rl_amd.alphazero.train_conv import X3Conv2d
    from blokus_rl_amd.nets import ResNet

    eng, rb = _replay()
    losses = {}
    for dp in (False, True):
        torch.manual_seed(0)
        model = ResNet(20, 4, eng.A, 2).cuda()
        opt = torch.optim.SGD(model.parameters(), lr=1e-2)
        L = Learner(model, batch_size=256, seed=0, device_path=dp, optimizer=opt)
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
        assert abs(a - b) <= 1e-4 * abs(a), losses
    # "auto" picks the device path at large batches on the GPU only
    assert Learner(ResNet(20, 4, eng.A, 1).cuda(), batch_size=64).device_path is False
    assert Learner(ResNet(20, 4, eng.A, 1).cuda(), batch_size=1024).device_path is True


def test_fused_conv_bn_relu_matches_fp64():
    """ConvBNFunction (conv on bk_conv_x3 -> batch norm + ReLU on bk_bn_forward_ex; backward with the
    ReLU mask recomputed from the conv output and the conv's bias gradient as dx's column sums)
    against the fp64 conv -> BatchNorm2d -> ReLU: output, dx, dW, dgamma, dbeta at fp32-class
    tolerances; the conv bias gradient (zero in exact arithmetic under train-mode batch norm) to
    1e-6 of the summed |dz| scale; relu off as well."""
    from blokus_rl_amd.alphazero.train_conv import ConvBNFunction

    g = torch.Generator().manual_seed(9)
    for relu in (True, False):
        x = torch.randn(33, 64, 20, 20, generator=g, dtype=torch.float64)
        w = torch.randn(64, 64, 3, 3, generator=g, dtype=torch.float64) * 0.05
        b = torch.randn(64, generator=g, dtype=torch.float64) * 0.1
        gam = torch.rand(64, generator=g, dtype=torch.float64) + 0.5
        bet = torch.randn(64, generator=g, dtype=torch.float64) * 0.2
        gy = torch.randn(33, 64, 20, 20, generator=g, dtype=torch.float64)
        xr, wr, br, gr, btr = (t.clone().requires_grad_() for t in (x, w, b, gam, bet))
        z = F.conv2d(xr, wr, br, padding=1)
        yr = F.batch_norm(z, torch.zeros(64, dtype=torch.float64), torch.ones(64, dtype=torch.float64), gr, btr,
                          training=True, momentum=0.1, eps=1e-5)
        if relu:
            yr = F.relu(yr)
        yr.backward(gy)
        xd = x.float().cuda().contiguous(memory_format=torch.channels_last).requires_grad_()
        wd, bd, gd, btd = (t.float().cuda().requires_grad_() for t in (w, b, gam, bet))
        rm, rv = torch.zeros(64, device="cuda"), torch.ones(64, device="cuda")
        y = ConvBNFunction.apply(xd, wd, bd, gd, btd, rm, rv, 0.1, 1e-5, relu)
        y.backward(gy.float().cuda().contiguous(memory_format=torch.channels_last))
        scale = lambda t: float(t.abs().max())  # noqa: E731
        assert float((y.detach().double().cpu() - yr.detach()).abs().max()) <= 5e-6 * scale(yr.detach())
        for a, r in ((xd.grad, xr.grad), (wd.grad, wr.grad), (gd.grad, gr.grad), (btd.grad, btr.grad)):
            assert float((a.double().cpu() - r).abs().max()) <= 2e-5 * scale(r), (relu, scale(r))
        assert float(bd.grad.abs().max()) <= 1e-6 * float(gy.abs().sum(dim=(0, 2, 3)).max())
        assert float((rm.double().cpu() - 0.1 * z.detach().mean(dim=(0, 2, 3))).abs().max()) <= 1e-6 * float(z.detach().abs().max())


def test_train_resnet_matches_unfused_device_path():
    """TrainResNet (block-level fusion + raw policy logits) against the same model with the fusion
    off (the per-module device path), one step through the reference loss: the losses agree to
    1e-6 relative, the parameter gradients to 1e-4 of each gradient's norm (the conv biases that
    feed a batch norm aside: rounding noise on both paths)."""
    from blokus_rl_amd.alphazero.learner import alphazero_loss
    from blokus_rl_amd.alphazero.train_conv import TrainResNet, prepare_model
    from blokus_rl_amd.nets import ResNet

    eng, rb = _replay()
    idx = torch.randint(0, 512, (256,), device="cuda", generator=torch.Generator(device="cuda").manual_seed(5))
    batch = rb.batch(idx)
    out = {}
    for fused in (True, False):
        torch.manual_seed(0)
        model = prepare_model(ResNet(20, 4, eng.A, 2).cuda())
        assert isinstance(model, TrainResNet)
        if not fused:
            model.__class__ = ResNet
        model.train()
        p, v = model(batch["observation"].contiguous(memory_format=torch.channels_last))
        loss = alphazero_loss(p, v, batch)
        loss.backward()
        out[fused] = (float(loss.detach()), {k: t.grad.detach().clone() for k, t in model.named_parameters()})
    assert abs(out[True][0] - out[False][0]) <= 1e-6 * abs(out[False][0])
    for k, g0 in out[False][1].items():
        if k in ("conv1.bias", "policy_conv.bias", "value_conv.bias") or (
                k.startswith("res_blocks") and k.endswith(".bias") and k.split(".")[2] in ("0", "3")):
            continue  # the bias of a conv that feeds a batch norm: zero in exact arithmetic
        d = (out[True][1][k] - g0).norm()
        assert float(d) <= 1e-4 * float(g0.norm()) + 1e-12, (k, float(d), float(g0.norm()))


def test_sparse_policy_linear_matches_dense():
    """SparsePolicyLinear (trainfc.hip) against the dense Linear followed by the gather at the rows'
    legal ids, in fp64: the gathered logits, and the input / weight / bias gradients from an upstream
    gradient that lives on the legal ids only (what the masked loss produces). Rows of 0 and of
    `cap` ids, ids shared by many rows (the counting-sort index) and ids no row holds (zero rows of
    dW); deterministic (two runs bitwise equal)."""
    from blokus_rl_amd.alphazero.train_conv import SparsePolicyLinear

    g = torch.Generator().manual_seed(21)
    B, F, A, cap = 300, 800, 3000, 128
    pf = torch.relu(torch.randn(B, F, generator=g, dtype=torch.float64))
    W = torch.randn(A, F, generator=g, dtype=torch.float64) * 0.03
    bias = torch.randn(A, generator=g, dtype=torch.float64) * 0.1
    k = torch.randint(0, cap + 1, (B,), generator=g)
    k[0], k[1] = 0, cap
    ids = torch.full((B, cap), -1, dtype=torch.int16)
    for b in range(B):
        pool = 600 if b % 2 else A  # half the rows draw from a small pool: shared ids
        ids[b, : int(k[b])] = torch.randperm(pool, generator=g)[: int(k[b])].sort().values.to(torch.int16)
    valid = torch.arange(cap)[None, :] < k[:, None]
    gy = torch.randn(B, cap, generator=g, dtype=torch.float64) * valid
    # fp64 dense reference
    pr, Wr, br = (t.clone().requires_grad_() for t in (pf, W, bias))
    dense = torch.nn.functional.linear(pr, Wr, br)
    gat = torch.gather(dense, 1, ids.long().clamp(min=0)) * valid
    gat.backward(gy)
    outs = []
    for _ in range(2):
        pd, Wd, bd = (t.float().cuda().requires_grad_() for t in (pf, W, bias))
        xs = SparsePolicyLinear.apply(pd, Wd, bd, ids.cuda(), k.to(torch.int32).cuda())
        xs.backward(gy.float().cuda())
        outs.append((xs.detach().cpu(), pd.grad.cpu(), Wd.grad.cpu(), bd.grad.cpu()))
    assert all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))  # deterministic
    xs, dpf, dW, db = (t.double() for t in outs[0])
    assert float(((xs - gat.detach()) * valid).abs().max()) <= 1e-5 * float(gat.detach().abs().max())
    assert float((xs * ~valid).abs().max()) == 0.0
    for a, r in ((dpf, pr.grad), (dW, Wr.grad), (db, br.grad)):
        assert float((a - r).abs().max()) <= 1e-5 * float(r.abs().max()), float((a - r).abs().max())
    held = torch.zeros(A, dtype=torch.bool)
    held[ids[valid].long()] = True
    assert bool((dW[~held] == 0).all()) and bool((db[~held] == 0).all()) and int((~held).sum()) > 0

    # ids outside [0, A) inside k (-1 = 65535 unsigned, A itself): logit 0, no gradient, no access
    # past W; the rest of the row unchanged
    bad = ids.clone()
    rows = [b for b in range(2, B) if int(k[b]) >= 2][:20]
    for i, b in enumerate(rows):
        bad[b, i % 2] = -1 if i % 3 else A
    pd, Wd, bd = (t.float().cuda().requires_grad_() for t in (pf, W, bias))
    xb = SparsePolicyLinear.apply(pd, Wd, bd, bad.cuda(), k.to(torch.int32).cuda())
    gb = gy.clone()
    for i, b in enumerate(rows):
        gb[b, i % 2] = 0.0  # the reference: those pairs absent
    xb.backward(gb.float().cuda())
    xb = xb.detach().cpu().double()
    for i, b in enumerate(rows):
        assert float(xb[b, i % 2]) == 0.0
    keep = valid.clone()
    for i, b in enumerate(rows):
        keep[b, i % 2] = False
    assert float(((xb - gat.detach()) * keep).abs().max()) <= 1e-5 * float(gat.detach().abs().max())
    pr2, Wr2, br2 = (t.clone().requires_grad_() for t in (pf, W, bias))
    gat2 = torch.gather(torch.nn.functional.linear(pr2, Wr2, br2), 1, ids.long().clamp(min=0)) * keep
    gat2.backward(gb * keep)
    for a, r in ((pd.grad.cpu().double(), pr2.grad), (Wd.grad.cpu().double(), Wr2.grad), (bd.grad.cpu().double(), br2.grad)):
        assert float((a - r).abs().max()) <= 1e-5 * float(r.abs().max()), float((a - r).abs().max())


def test_learner_sparse_head_matches_dense_head():
    """The learner's step with the sparse policy head (Learner.sparse_head: logits at the legal ids
    only) against the same device path with the dense raw logits: loss to 1e-6 relative, every
    parameter gradient to 1e-4 of its norm (conv biases that feed a batch norm aside)."""
    from blokus_rl_amd.alphazero.learner import Learner, alphazero_loss, sparse_policy_loss
    from blokus_rl_amd.nets import ResNet

    eng, rb = _replay()
    idx = torch.randint(0, 512, (256,), device="cuda", generator=torch.Generator(device="cuda").manual_seed(8))
    batch = rb.batch(idx)
    out = {}
    for sparse in (True, False):
        torch.manual_seed(0)
        model = ResNet(20, 4, eng.A, 2).cuda()
        L = Learner(model, batch_size=256, device_path=True)
        assert L.sparse_head
        model.train()
        obs = batch["observation"].contiguous(memory_format=torch.channels_last)
        if sparse:
            xs, v = model(obs, ids=batch["ids"], k=batch["k"])
            loss = sparse_policy_loss(xs, batch["pi"], batch["k"]) + (v.squeeze() - batch["score"]).pow(2).mean()
        else:
            p, v = model(obs)
            loss = alphazero_loss(p, v, batch)
        loss.backward()
        out[sparse] = (float(loss.detach()), {n: t.grad.detach().clone() for n, t in model.named_parameters()})
    assert abs(out[True][0] - out[False][0]) <= 1e-6 * abs(out[False][0])
    for n, g0 in out[False][1].items():
        if n in ("conv1.bias", "policy_conv.bias", "value_conv.bias") or (
                n.startswith("res_blocks") and n.endswith(".bias") and n.split(".")[2] in ("0", "3")):
            continue
        d = (out[True][1][n] - g0).norm()
        assert float(d) <= 1e-4 * float(g0.norm()) + 1e-12, (n, float(d), float(g0.norm()))
