"""bk_leafnet_x3 (leafnet.hip: the whole leaf ResNet in one launch on split-f16 MFMA products)
against an fp64 torch forward of the same BN-folded net (FusedResNet, models/blokus_nnet.py:88-151).

Accuracy bar ("fp32-class"): on every output the x3 kernel's error against fp64 stays within a
small factor of the error of the round-1 fp32 kernel (f32 MFMA, bk_resnet_stem_tower_heads) on the
same inputs, and within 2e-6 of the output scale. Inputs include binary observations (what the
search feeds), and dense random planes scaled by 1e-3 and 1e3 (the per-board power-of-two
activation scaling must keep both ends exact)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _net(N, nblocks, seed, A=100):
    from blokus_rl_amd.nets import ResNet

    torch.manual_seed(seed)
    net = ResNet(N, 4, A, nblocks).cuda().eval()
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.1, 0.1)
    return net


def _ref64(net, obs):
    """fp64 forward of the BN-folded net: (policy features, values, tower output)."""
    from blokus_rl_amd.nets import FusedResNet

    with torch.no_grad():
        fd = FusedResNet(net).double().eval()
        x = torch.relu(fd.stem(obs.double()))
        h = x
        for c1, c2 in fd.blocks:
            h = c2(torch.relu(c1(h)))
        xt = torch.relu(x + h)
        pf = torch.relu(fd.policy_conv(xt)).flatten(1)
        v = torch.tanh(fd.value_fc2(torch.relu(fd.value_fc1(torch.relu(fd.value_conv(xt)).flatten(1)))))
    return pf, v, xt


def _rel(a, ref):
    return float((a.double() - ref).abs().max()) / (float(ref.abs().max()) + 1e-30)


@pytest.mark.parametrize("B,N,nblocks,kind", [(256, 20, 5, "binary"), (7, 20, 2, "dense"), (5, 20, 1, "tiny"),
                                             (6, 20, 2, "huge"), (37, 14, 2, "binary"), (3, 14, 1, "dense")])
def test_leafnet_x3_is_fp32_class(B, N, nblocks, kind):
    from blokus_rl_amd.nets import LeafResNet, leafnet_x3, resnet_stem_tower_heads

    net = _net(N, nblocks, seed=B + N + nblocks)
    g = torch.Generator(device="cuda").manual_seed(B * 3 + N)
    if kind == "binary":
        obs = (torch.rand((B, 8, N, N), device="cuda", generator=g) < 0.3).float()
    else:
        scale = {"dense": 1.0, "tiny": 1e-3, "huge": 1e3}[kind]
        obs = torch.randn((B, 8, N, N), device="cuda", generator=g) * scale
    leaf = LeafResNet(net, normalize=False, features=True).eval()
    assert leaf.x3
    pf, v, out = leafnet_x3(obs, leaf, want_out=True)
    pf32, v32 = resnet_stem_tower_heads(obs, leaf.w_stem_tower, leaf.u_tower, leaf.b_tower, 2 * nblocks, leaf.f)
    torch.cuda.synchronize()
    pf_ref, v_ref, xt_ref = _ref64(net, obs)
    assert torch.isfinite(pf).all() and torch.isfinite(v).all()
    e_x3, e_32 = _rel(pf, pf_ref), _rel(pf32, pf_ref)
    assert e_x3 <= max(4 * e_32, 2e-6), (e_x3, e_32)
    ev_x3, ev_32 = float((v.double() - v_ref).abs().max()), float((v32.double() - v_ref).abs().max())
    assert ev_x3 <= max(4 * ev_32, 2e-6), (ev_x3, ev_32)
    assert _rel(out, xt_ref) <= 2e-6


def test_leafnet_x3_outputs_do_not_depend_on_the_batch():
    """A board's outputs are a function of that board alone (one workgroup per board): the same
    boards in a batch of 256 and alone give bitwise equal outputs."""
    from blokus_rl_amd.nets import LeafResNet, leafnet_x3

    net = _net(20, 2, seed=11)
    leaf = LeafResNet(net, normalize=False, features=True).eval()
    obs = (torch.rand((256, 8, 20, 20), device="cuda") < 0.3).float()
    pf, v = leafnet_x3(obs, leaf)
    pf1, v1 = leafnet_x3(obs[17:18].contiguous(), leaf)
    assert torch.equal(pf[17:18], pf1) and torch.equal(v[17:18], v1)


def test_leaf_resnet_default_math_is_x3(monkeypatch):
    """LeafResNet runs bk_leafnet_x3 by default and the round-1 f32 kernels with BK_NET_MATH=f32;
    both are within fp32-class distance of each other."""
    from blokus_rl_amd.nets import LeafResNet, leafnet_x3

    net = _net(20, 5, seed=3, A=30433)
    leaf = LeafResNet(net, normalize=False, features=True).eval()
    obs = (torch.rand((64, 8, 20, 20), device="cuda") < 0.3).float()
    pf, v = leaf(obs)
    pfx, vx = leafnet_x3(obs, leaf)
    assert torch.equal(pf, pfx) and torch.equal(v, vx)
    monkeypatch.setenv("BK_NET_MATH", "f32")
    pf32, v32 = leaf(obs)
    assert not torch.equal(pf32, pf)
    assert torch.allclose(pf32, pf, rtol=1e-5, atol=1e-5) and torch.allclose(v32, v, rtol=1e-5, atol=1e-6)


def test_leaf_resnet_head_operands_are_buffers():
    """The x3 head operands are registered buffers: state_dict carries them and .to() moves them
    with the weight packs (a plain list kept device pointers of the old location)."""
    from blokus_rl_amd.nets import LeafResNet

    leaf = LeafResNet(_net(20, 1, seed=5), normalize=False, features=True).eval()
    sd = leaf.state_dict()
    assert all(f"x3_head{i}" in sd for i in range(9))
    cpu = leaf.to("cpu")
    assert all(t.device.type == "cpu" for t in cpu.x3_heads) and cpu.x3_wtower.device.type == "cpu"
    back = cpu.to("cuda")
    assert all(t.is_cuda for t in back.x3_heads)


@pytest.mark.parametrize("B,nblocks,kind", [(256, 5, "binary"), (7, 2, "dense"), (5, 1, "tiny"), (6, 2, "huge"),
                                           (3, 3, "binary")])
def test_leafnet_w3_is_fp32_class(B, nblocks, kind):
    """bk_leafnet_w3 (the tower as Winograd F(2x2,3x3) on split-f16 products) against the same fp64
    forward, at the same bar as x3: within 4x the round-1 f32 kernel's error (itself a Winograd
    tower on the f32 MFMA) or 2e-6 of the output scale, and the tower output within 2e-6."""
    from blokus_rl_amd.nets import LeafResNet, leafnet_w3, resnet_stem_tower_heads

    N = 20
    net = _net(N, nblocks, seed=B + 3 * nblocks)
    g = torch.Generator(device="cuda").manual_seed(B * 5 + nblocks)
    if kind == "binary":
        obs = (torch.rand((B, 8, N, N), device="cuda", generator=g) < 0.3).float()
    else:
        scale = {"dense": 1.0, "tiny": 1e-3, "huge": 1e3}[kind]
        obs = torch.randn((B, 8, N, N), device="cuda", generator=g) * scale
    leaf = LeafResNet(net, normalize=False, features=True).eval()
    pf, v, out = leafnet_w3(obs, leaf, want_out=True)
    pf32, v32 = resnet_stem_tower_heads(obs, leaf.w_stem_tower, leaf.u_tower, leaf.b_tower, 2 * nblocks, leaf.f)
    torch.cuda.synchronize()
    pf_ref, v_ref, xt_ref = _ref64(net, obs)
    assert torch.isfinite(pf).all() and torch.isfinite(v).all()
    e_w3, e_32 = _rel(pf, pf_ref), _rel(pf32, pf_ref)
    assert e_w3 <= max(4 * e_32, 2e-6), (e_w3, e_32)
    ev_w3, ev_32 = float((v.double() - v_ref).abs().max()), float((v32.double() - v_ref).abs().max())
    assert ev_w3 <= max(4 * ev_32, 2e-6), (ev_w3, ev_32)
    assert _rel(out, xt_ref) <= 2e-6


def test_leafnet_w3_outputs_do_not_depend_on_the_batch(monkeypatch):
    """One workgroup per board: a board's w3 outputs are the same alone and in a batch of 256, and
    BK_NET_MATH=w3 routes LeafResNet through bk_leafnet_w3."""
    from blokus_rl_amd.nets import LeafResNet, leafnet_w3

    net = _net(20, 2, seed=12)
    leaf = LeafResNet(net, normalize=False, features=True).eval()
    obs = (torch.rand((256, 8, 20, 20), device="cuda") < 0.3).float()
    pf, v = leafnet_w3(obs, leaf)
    pf1, v1 = leafnet_w3(obs[200:201].contiguous(), leaf)
    assert torch.equal(pf[200:201], pf1) and torch.equal(v[200:201], v1)
    monkeypatch.setenv("BK_NET_MATH", "w3")
    pfl, vl = leaf(obs)
    assert torch.equal(pfl, pf) and torch.equal(vl, v)
