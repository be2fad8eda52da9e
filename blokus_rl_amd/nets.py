"""Policy/value nets used as the MCTS leaf evaluator, kept on PyTorch-ROCm (MIOpen convs,
hipBLASLt GEMMs): the north star keeps the repo's existing net. Architectures, forward
semantics and `state_dict` keys follow the reference so its checkpoints load unchanged:

* `ResNet`  — blokus_rl/models/blokus_nnet.py:88-151: conv3x3(2P->64)+BN+ReLU, ONE residual
  around the whole stack of `num_res_blocks` (conv-BN-ReLU-conv-BN) blocks, policy head
  1x1 conv(2)+BN+ReLU+Linear(2*N*N -> A)+log_softmax, value head 1x1 conv(1)+BN+ReLU+
  Linear(N*N -> 64)+ReLU+Linear(64 -> P)+tanh.
* `DCNNet`  — blokus_nnet.py:9-85.
* `DumbNet` — models/dumbnet.py:6-21: logits 1, value 0 (the "uninformed MCTS" opponent).
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn.functional as F
from torch import nn


class NativeBatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d on PyTorch's own batch-norm kernels instead of MIOpen's (same parameters,
    buffers and state_dict keys; training-mode batch statistics and running-stat updates alike):
    nn.BatchNorm2d.forward's bookkeeping, then aten::native_batch_norm directly (F.batch_norm would
    pick MIOpen; switching the process-wide cudnn flag around it is not thread-safe)."""

    def forward(self, x):
        self._check_input_dim(x)
        factor = 0.0 if self.momentum is None else self.momentum
        if self.training and self.track_running_stats and self.num_batches_tracked is not None:
            self.num_batches_tracked.add_(1)
            factor = 1.0 / float(self.num_batches_tracked) if self.momentum is None else self.momentum
        use_batch = self.training or (self.running_mean is None and self.running_var is None)
        track = not self.training or self.track_running_stats
        rm = self.running_mean if track else None
        rv = self.running_var if track else None
        return torch.native_batch_norm(x, self.weight, self.bias, rm, rv, use_batch, factor, self.eps)[0]


def use_native_batchnorm(model: nn.Module) -> nn.Module:
    """Switch every BatchNorm2d of `model` to NativeBatchNorm2d in place."""
    for m in model.modules():
        if type(m) is nn.BatchNorm2d:
            m.__class__ = NativeBatchNorm2d
    return model


class ResNet(nn.Module):
    def __init__(self, board_size: int, num_players: int, action_size: int, num_res_blocks: int = 5,
                 channels: int = 64):
        super().__init__()
        self.board_x = self.board_y = board_size
        self.action_size = action_size
        self.num_players = num_players
        self.input_dim = [2 * num_players, board_size, board_size]
        c = channels
        self.conv1 = nn.Conv2d(2 * num_players, c, kernel_size=3, padding=1)
        self.bn1 = nn.BatchNorm2d(c)
        self.res_blocks = nn.Sequential(*[
            nn.Sequential(nn.Conv2d(c, c, 3, padding=1), nn.BatchNorm2d(c), nn.ReLU(),
                          nn.Conv2d(c, c, 3, padding=1), nn.BatchNorm2d(c))
            for _ in range(num_res_blocks)
        ])
        n2 = board_size * board_size
        self.policy_conv = nn.Conv2d(c, 2, kernel_size=1)
        self.policy_bn = nn.BatchNorm2d(2)
        self.policy_out = nn.Linear(2 * n2, action_size)
        self.value_conv = nn.Conv2d(c, 1, kernel_size=1)
        self.value_bn = nn.BatchNorm2d(1)
        self.value_fc1 = nn.Linear(n2, 64)
        self.value_fc2 = nn.Linear(64, num_players)

    def forward(self, x):
        x = F.relu(self.bn1(self.conv1(x)))
        x = F.relu(x + self.res_blocks(x))
        p = F.relu(self.policy_bn(self.policy_conv(x))).flatten(1)
        p = F.log_softmax(self.policy_out(p), dim=1)
        v = F.relu(self.value_bn(self.value_conv(x))).flatten(1)
        v = torch.tanh(self.value_fc2(F.relu(self.value_fc1(v))))
        return p, v


class DCNNet(nn.Module):
    def __init__(self, board_size: int, num_players: int, action_size: int, num_channels: int = 128,
                 linear_dim: int = 128, dropout: float = 0.3):
        super().__init__()
        n, c, d = board_size, num_channels, linear_dim
        self.num_channels, self.board_x, self.board_y, self.dropout = c, n, n, dropout
        self.conv1 = nn.Conv2d(2 * num_players, c, 3, stride=1, padding=1)
        self.conv2 = nn.Conv2d(c, c, 3, stride=1, padding=1)
        self.conv3 = nn.Conv2d(c, c, 3, stride=1)
        self.conv4 = nn.Conv2d(c, c, 3, stride=1)
        self.bn1, self.bn2, self.bn3, self.bn4 = (nn.BatchNorm2d(c) for _ in range(4))
        self.fc1 = nn.Linear(c * (n - 4) * (n - 4), d)
        self.fc_bn1 = nn.BatchNorm1d(d)
        self.fc2 = nn.Linear(d, d // 2)
        self.fc_bn2 = nn.BatchNorm1d(d // 2)
        self.fc3 = nn.Linear(d // 2, action_size)
        self.fc4 = nn.Linear(d // 2, num_players)

    def forward(self, x):
        x = F.relu(self.bn1(self.conv1(x)))
        x = F.relu(self.bn2(self.conv2(x)))
        x = F.relu(self.bn3(self.conv3(x)))
        x = F.relu(self.bn4(self.conv4(x)))
        x = x.reshape(-1, self.num_channels * (self.board_x - 4) * (self.board_y - 4))
        x = F.dropout(F.relu(self.fc_bn1(self.fc1(x))), p=self.dropout, training=self.training)
        x = F.dropout(F.relu(self.fc_bn2(self.fc2(x))), p=self.dropout, training=self.training)
        return F.log_softmax(self.fc3(x), dim=1), torch.tanh(self.fc4(x))


class DumbNet(nn.Module):
    """Uniform prior, zero value. Returns logits of 1 exactly like the reference (not a
    log-softmax); the masked log-softmax downstream makes the prior uniform either way."""

    def __init__(self, board_size: int, num_players: int, action_size: int):
        super().__init__()
        self.p_shape, self.v_shape = action_size, num_players

    def forward(self, x):
        b = x.shape[0]
        return (torch.ones((b, self.p_shape), device=x.device),
                torch.zeros((b, self.v_shape), device=x.device))


def get_model(model_type: str):
    """models/__init__.py:5-11 registry."""
    return {"dumbnet": DumbNet, "dcnnet": DCNNet, "resnet": ResNet}[model_type]


def build_model(model_type: str, board_size: int, num_players: int, action_size: int, **kw) -> nn.Module:
    cls = get_model(model_type)
    if cls is ResNet:
        return ResNet(board_size, num_players, action_size, num_res_blocks=kw.get("num_res_blocks", 5))
    if cls is DCNNet:
        return DCNNet(board_size, num_players, action_size, kw.get("num_channels", 128), kw.get("linear_dim", 128),
                      kw.get("dropout", 0.3))
    return DumbNet(board_size, num_players, action_size)


def _fold_bn(conv: nn.Conv2d, bn: nn.BatchNorm2d) -> nn.Conv2d:
    """conv followed by eval-mode BN -> one conv with scaled weights and shifted bias."""
    fused = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride, conv.padding,
                      bias=True).to(conv.weight.device)
    with torch.no_grad():
        scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
        fused.weight.copy_(conv.weight * scale.view(-1, 1, 1, 1))
        b = conv.bias if conv.bias is not None else torch.zeros_like(bn.running_mean)
        fused.bias.copy_((b - bn.running_mean) * scale + bn.bias)
    return fused


class FusedResNet(nn.Module):
    """Inference form of `ResNet` for the leaf batch: every eval-mode BatchNorm folded into its
    convolution (MIOpen's inference BN costs as much as the convs at batch 256). Same function
    as ResNet.eval() up to float32 rounding."""

    def __init__(self, net: ResNet):
        super().__init__()
        net = net.eval()
        self.stem = _fold_bn(net.conv1, net.bn1)
        self.blocks = nn.ModuleList()
        for blk in net.res_blocks:
            self.blocks.append(nn.ModuleList([_fold_bn(blk[0], blk[1]), _fold_bn(blk[3], blk[4])]))
        self.policy_conv = _fold_bn(net.policy_conv, net.policy_bn)
        self.policy_out = net.policy_out
        self.value_conv = _fold_bn(net.value_conv, net.value_bn)
        self.value_fc1 = net.value_fc1
        self.value_fc2 = net.value_fc2
        self._fc1_t = None

    def value_fc1_wt(self) -> torch.Tensor:
        """value_fc1.weight transposed to [N*N, 64] (bk_resnet_heads' layout), cached."""
        if self._fc1_t is None:
            self._fc1_t = self.value_fc1.weight.detach().float().t().contiguous()
        return self._fc1_t

    def forward(self, x):
        x = F.relu(self.stem(x))
        h = x
        for c1, c2 in self.blocks:
            h = c2(F.relu(c1(h)))
        x = F.relu(x + h)
        p = F.relu(self.policy_conv(x)).flatten(1)
        p = F.log_softmax(self.policy_out(p).float(), dim=1)
        v = F.relu(self.value_conv(x)).flatten(1)
        v = torch.tanh(self.value_fc2(F.relu(self.value_fc1(v)))).float()
        return p, v


def _bias_act(x: torch.Tensor, bias: torch.Tensor, relu: bool, residual: torch.Tensor | None = None):
    """In-place x = act(x + bias (+ residual)) on a channels_last activation (bk_bias_act)."""
    from .engine import _check, _ptr, _stream, load_library

    assert x.is_contiguous(memory_format=torch.channels_last) and x.dtype == torch.float32
    if residual is not None:
        assert residual.is_contiguous(memory_format=torch.channels_last) and residual.shape == x.shape
    _check(load_library().bk_bias_act(ctypes.c_void_p(x.data_ptr()), x.numel(), x.shape[1], _ptr(bias),
                                      None if residual is None else ctypes.c_void_p(residual.data_ptr()),
                                      int(relu), _stream(x.device)))
    return x


def pack_conv3x3(w: torch.Tensor) -> torch.Tensor:
    """[64, cin, 3, 3] weights -> bk_conv3x3's operand order: flat [9][cin/4][64 lanes][4 blocks]
    (cin 64: followed by pack_winograd(w) for the Winograd form used at even N),
    element (tap, s, l, j) = w[16j + (l & 15), cin(s, l >> 4), tap // 3, tap % 3] with
    cin(s, g) = 4*VEC*(s // VEC) + VEC*g + s % VEC, VEC = 4 (cin % 16 == 0), 2 (cin 8), 1 (cin 4)."""
    cout, cin = w.shape[0], w.shape[1]
    assert cout == 64 and w.shape[2:] == (3, 3) and cin in (4, 8, 64)
    vec = 4 if cin % 16 == 0 else (2 if cin == 8 else 1)
    dev = w.device
    tap = torch.arange(9, device=dev).view(9, 1, 1, 1)
    s = torch.arange(cin // 4, device=dev).view(1, -1, 1, 1)
    lane = torch.arange(64, device=dev).view(1, 1, 64, 1)
    j = torch.arange(4, device=dev).view(1, 1, 1, 4)
    ci = 4 * vec * (s // vec) + vec * (lane >> 4) + s % vec
    co = 16 * j + (lane & 15)
    out = w.float()[co, ci, tap // 3, tap % 3].contiguous().view(-1)
    if cin != 64:
        return out
    return torch.cat([out, pack_winograd(w)])


_WINO_G = ((1.0, 0.0, 0.0), (0.5, 0.5, 0.5), (0.5, -0.5, 0.5), (0.0, 0.0, 1.0))


def pack_winograd(w: torch.Tensor) -> torch.Tensor:
    """[64, 64, 3, 3] -> the Winograd F(2x2,3x3) form's U = G w G^T (computed in fp64, stored f32),
    twice: in k_conv3x3_wino's LDS order (form 1): flat [2 halves h][2 blocks k][16 positions p]
    [16 k-steps s][64 lanes], element = U[32h + 16k + (l & 15), 16 * (l >> 4) + s, p // 4, p % 4];
    then in k_conv3x3_wino2's register order (form 2, below)."""
    assert w.shape == (64, 64, 3, 3)
    G = torch.tensor(_WINO_G, dtype=torch.float64, device=w.device)
    U = torch.einsum("ik,ockl,jl->ocij", G, w.double(), G).reshape(64, 64, 16)  # [cout][cin][p]
    dev = w.device
    h = torch.arange(2, device=dev).view(2, 1, 1, 1, 1)
    k = torch.arange(2, device=dev).view(1, 2, 1, 1, 1)
    pos = torch.arange(16, device=dev).view(1, 1, 16, 1, 1)
    st = torch.arange(16, device=dev).view(1, 1, 1, 16, 1)
    lane = torch.arange(64, device=dev).view(1, 1, 1, 1, 64)
    out = U[32 * h + 16 * k + (lane & 15), 16 * (lane >> 4) + st, pos]
    # form 2 (k_conv3x3_wino2, U in registers): [4 blocks kb][64 q][64 lanes][4 e], i = 4q + e,
    # element = U[16kb + (l & 15), 4 * (i // 16) + (l >> 4), i % 16]
    kb = torch.arange(4, device=dev).view(4, 1, 1, 1)
    q = torch.arange(64, device=dev).view(1, 64, 1, 1)
    l2 = torch.arange(64, device=dev).view(1, 1, 64, 1)
    e = torch.arange(4, device=dev).view(1, 1, 1, 4)
    i = 4 * q + e
    out2 = U[16 * kb + (l2 & 15), 4 * (i // 16) + (l2 >> 4), i % 16]
    return torch.cat([out.float().contiguous().view(-1), out2.float().contiguous().view(-1)])


def conv3x3(x: torch.Tensor, wpacked: torch.Tensor, bias: torch.Tensor, relu: bool,
            residual: torch.Tensor | None = None) -> torch.Tensor:
    """bk_conv3x3: x = planar observation [B, cin, N, N] contiguous (cin 4 / 8) or a 64-channel
    activation in channels_last memory format (NHWC) -> [B, 64, N, N] channels_last."""
    from .engine import _check, _ptr, _stream, load_library

    B, cin, N, _ = x.shape
    assert x.dtype == torch.float32
    if cin == 64:
        assert x.is_contiguous(memory_format=torch.channels_last)
    else:
        assert x.is_contiguous()
    lib = load_library()
    assert wpacked.dtype == torch.float32 and wpacked.numel() == lib.bk_conv3x3_packed_floats(cin)
    y = torch.empty((B, 64, N, N), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
    if residual is not None:
        assert residual.is_contiguous(memory_format=torch.channels_last) and residual.shape == y.shape
    _check(lib.bk_conv3x3(ctypes.c_void_p(x.data_ptr()), B, N, cin, _ptr(wpacked), _ptr(bias),
                                     None if residual is None else ctypes.c_void_p(residual.data_ptr()), int(relu),
                                     ctypes.c_void_p(y.data_ptr()), _stream(x.device)))
    return y


def pack_tower(weights) -> torch.Tensor:
    """[64, 64, 3, 3] weights of the tower's convs, in order -> bk_resnet_tower's u2all: each
    layer's Winograd U in the form-2 register order (the tail of pack_winograd), concatenated."""
    return torch.cat([pack_winograd(w)[-(4 * 64 * 64 * 4):] for w in weights]).contiguous()


def pack_stem_tower(w: torch.Tensor) -> torch.Tensor:
    """[64, 8, 3, 3] stem weights -> bk_resnet_stem_tower_heads' MFMA order: flat [4 blocks kb]
    [18 k-steps s][64 lanes], element = w[16kb + (l & 15), 4 * (s % 2) + (l >> 4), t // 3, t % 3]
    with tap t = s // 2."""
    assert w.shape == (64, 8, 3, 3)
    dev = w.device
    kb = torch.arange(4, device=dev).view(4, 1, 1)
    st = torch.arange(18, device=dev).view(1, 18, 1)
    lane = torch.arange(64, device=dev).view(1, 1, 64)
    t = st // 2
    return w.float()[16 * kb + (lane & 15), 4 * (st % 2) + (lane >> 4), t // 3, t % 3].contiguous().view(-1)


def pack_x3(w: torch.Tensor, b: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """[64, cin, 3, 3] conv weights (cin 8: the stem, 64: a tower conv) and bias [64] ->
    bk_leafnet_x3's operands: (split weights as uint8 bytes, inverse scales f32 [64], output bound
    f32 [2] = (A, B) with |y| <= A max|x| + B for y = conv(x) + b: A the largest row L1 norm of
    the weights, B the largest |bias|, both rounded up).

    GEMM view: A[o][k] with k = tap * cin + c (tap = 3 ky + kx), K padded to 32-wide chunks (the
    stem's 72 -> 96 with zeros). Row o is scaled by 2^e_o so that its largest magnitude lies in
    [2^14, 2^15), then split hi = f16(x), lo = f16(x - hi); inverse scale 2^-e_o. Fragment order:
    [chunk][wave 4][part hi/lo][lane 64][8 f16], lane l of wave w holding row 16w + l%16, columns
    32 chunk + 8 (l/16) .. +7 (the A operand of v_mfma_f32_16x16x32_f16)."""
    cout, cin = w.shape[0], w.shape[1]
    assert cout == 64 and w.shape[2:] == (3, 3) and cin in (8, 64)
    a = w.detach().to("cpu", torch.float64).permute(0, 2, 3, 1).reshape(64, 9 * cin)  # k = tap * cin + c
    K = (a.shape[1] + 31) // 32 * 32
    a = torch.cat([a, a.new_zeros(64, K - a.shape[1])], dim=1)
    mx = a.abs().amax(dim=1)
    _, e = torch.frexp(mx)
    e = torch.where(mx > 0, 15 - e, torch.zeros_like(e)).to(torch.float64)
    scaled = a * torch.pow(2.0, e).view(64, 1)
    hi = scaled.to(torch.float16)
    lo = (scaled - hi.to(torch.float64)).to(torch.float16)
    parts = torch.stack([hi, lo])                                   # [2][64][K]
    parts = parts.view(2, 4, 16, K // 32, 4, 8)                     # [part][wave][row][chunk][k-group][8]
    packed = parts.permute(3, 1, 0, 4, 2, 5).contiguous()           # [chunk][wave][part][k-group][row][8]
    inv = torch.pow(2.0, -e).to(torch.float32)
    bmax = float(b.detach().abs().max()) if b is not None else 0.0
    bound = torch.tensor([float(a.abs().sum(dim=1).max()) * (1 + 2 ** -16), bmax * (1 + 2 ** -16)],
                         dtype=torch.float32)
    return packed.view(torch.uint8).view(-1).to(w.device), inv.to(w.device).contiguous(), bound.to(w.device)


def pack_w3(w: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """[64, 64, 3, 3] tower conv weights -> bk_leafnet_w3's operands: the Winograd F(2x2,3x3)
    transform U = G w G^T (fp64), each output channel's row scaled by 2^e_o so that its largest
    |U| lies in [2^14, 2^15), split hi = f16(x), lo = f16(x - hi); and the inverse scales 2^-e_o
    (f32 [64]). Fragment order [pos 16][chunk 2][wave 4][part hi/lo][lane 64][8 f16]: lane
    l = 16 g + r of wave w holds U[16 w + r][32 chunk + 8 g + i][pos], i = 0..7 (the A operand of
    v_mfma_f32_16x16x32_f16 for output channels 16 w.., input channels 32 chunk..)."""
    assert w.shape == (64, 64, 3, 3)
    G = torch.tensor(_WINO_G, dtype=torch.float64)
    U = torch.einsum("ik,ockl,jl->ocij", G, w.detach().to("cpu", torch.float64), G).reshape(64, 64, 16)
    mx = U.abs().amax(dim=(1, 2))
    _, e = torch.frexp(mx)
    e = torch.where(mx > 0, 15 - e, torch.zeros_like(e)).to(torch.float64)
    scaled = U * torch.pow(2.0, e).view(64, 1, 1)
    hi = scaled.to(torch.float16)
    lo = (scaled - hi.to(torch.float64)).to(torch.float16)
    parts = torch.stack([hi, lo]).view(2, 4, 16, 2, 4, 8, 16)      # [part][wave][row][chunk][g][i][pos]
    packed = parts.permute(6, 3, 1, 0, 4, 2, 5).contiguous()       # [pos][chunk][wave][part][g][row][i]
    inv = torch.pow(2.0, -e).to(torch.float32)
    return packed.view(torch.uint8).view(-1).to(w.device), inv.to(w.device).contiguous()


def net_math() -> str:
    """The leaf ResNet's arithmetic on the device: "x3" (default) = bk_leafnet_x3, split-f16 MFMA
    products with f32 accumulation (fp32-class accuracy, tests/test_leafnet_gpu.py); "w3" =
    bk_leafnet_w3, the same products with the residual tower as Winograd F(2x2,3x3) convolutions
    (2.25x fewer products per output); "f32" = the round-1 kernels on the f32 MFMA (BK_NET_MATH)."""
    import os

    m = os.environ.get("BK_NET_MATH", "x3")
    if m not in ("x3", "w3", "f32"):
        raise ValueError(f"BK_NET_MATH must be x3, w3 or f32, got {m!r}")
    return m


def leafnet_x3(obs: torch.Tensor, model: "LeafResNet", want_out: bool = False):
    """bk_leafnet_x3: the planar observation [B, 8, N, N] -> (policy features [B, 2*N*N], values
    [B, P][, tower output [B, 64, N, N] channels_last]) in one launch."""
    from .engine import _check, _ptr, _stream, load_library

    B, cin, N, _ = obs.shape
    assert cin == 8 and obs.dtype == torch.float32 and obs.is_contiguous()
    f = model.f
    lib = load_library()
    nl = 2 * len(f.blocks)
    assert model.x3_wtower.numel() == nl * lib.bk_leafnet_x3_weight_bytes(64)
    assert model.x3_wstem.numel() == lib.bk_leafnet_x3_weight_bytes(8)
    P = f.value_fc2.out_features
    pf = torch.empty((B, 2 * N * N), dtype=torch.float32, device=obs.device)
    v = torch.empty((B, P), dtype=torch.float32, device=obs.device)
    out = torch.empty((B, 64, N, N), dtype=torch.float32, device=obs.device,
                      memory_format=torch.channels_last) if want_out else None
    h = model.x3_heads
    _check(lib.bk_leafnet_x3(
        ctypes.c_void_p(obs.data_ptr()), B, N, cin, _ptr(model.x3_wstem), _ptr(model.x3_sstem), _ptr(h[0]), nl,
        _ptr(model.x3_wtower), _ptr(model.x3_stower), _ptr(model.b_tower), _ptr(model.x3_bounds),
        *[_ptr(t) for t in h[1:]], P, _ptr(pf),
        _ptr(v), None if out is None else ctypes.c_void_p(out.data_ptr()), _stream(obs.device)))
    return (pf, v, out) if want_out else (pf, v)


def leafnet_w3(obs: torch.Tensor, model: "LeafResNet", want_out: bool = False):
    """bk_leafnet_w3: leafnet_x3's network and outputs with the residual tower as Winograd
    F(2x2,3x3) convolutions on split-f16 products (20x20 boards)."""
    from .engine import _check, _ptr, _stream, load_library

    B, cin, N, _ = obs.shape
    assert cin == 8 and obs.dtype == torch.float32 and obs.is_contiguous()
    f = model.f
    lib = load_library()
    nl = 2 * len(f.blocks)
    assert model.w3_utower.numel() == nl * lib.bk_leafnet_w3_weight_bytes()
    P = f.value_fc2.out_features
    pf = torch.empty((B, 2 * N * N), dtype=torch.float32, device=obs.device)
    v = torch.empty((B, P), dtype=torch.float32, device=obs.device)
    out = torch.empty((B, 64, N, N), dtype=torch.float32, device=obs.device,
                      memory_format=torch.channels_last) if want_out else None
    # the stem output's workspace, kept per model instance, device, batch and stream (a captured graph
    # reuses the pointer; two evaluators or streams never share one)
    cache = model.__dict__.setdefault("_w3_ws", {})
    key = (obs.device, B, N, torch.cuda.current_stream(obs.device).cuda_stream)
    ws = cache.get(key)
    if ws is None:
        ws = cache[key] = torch.empty((B, N * N, 64), dtype=torch.float32, device=obs.device)
    h = model.x3_heads
    _check(lib.bk_leafnet_w3(
        ctypes.c_void_p(obs.data_ptr()), B, N, cin, _ptr(model.x3_wstem), _ptr(model.x3_sstem), _ptr(h[0]), nl,
        _ptr(model.w3_utower), _ptr(model.w3_stower), _ptr(model.b_tower), _ptr(model.x3_bounds),
        *[_ptr(t) for t in h[1:]], P, _ptr(pf), _ptr(v), _ptr(ws),
        None if out is None else ctypes.c_void_p(out.data_ptr()), _stream(obs.device)))
    return (pf, v, out) if want_out else (pf, v)


def tower_enabled() -> bool:
    """BK_TOWER=0 runs the residual tower as one bk_conv3x3 launch per layer instead of the fused
    bk_resnet_tower (same arithmetic; for comparisons)."""
    import os

    return os.environ.get("BK_TOWER", "1") != "0"


def resnet_tower(x: torch.Tensor, u2all: torch.Tensor, biasall: torch.Tensor, nlayers: int) -> torch.Tensor:
    """bk_resnet_tower: x = the stem output [B, 64, N, N] channels_last -> relu(x + tower(x))."""
    from .engine import _check, _ptr, _stream, load_library

    B, C, N, _ = x.shape
    assert C == 64 and x.dtype == torch.float32 and x.is_contiguous(memory_format=torch.channels_last)
    lib = load_library()
    assert u2all.numel() == nlayers * lib.bk_tower_u_floats() and biasall.numel() == nlayers * 64
    out = torch.empty_like(x, memory_format=torch.channels_last)
    ha = torch.empty_like(x, memory_format=torch.channels_last)
    hb = torch.empty_like(x, memory_format=torch.channels_last)
    _check(lib.bk_resnet_tower(ctypes.c_void_p(x.data_ptr()), B, N, nlayers, _ptr(u2all), _ptr(biasall),
                               ctypes.c_void_p(ha.data_ptr()), ctypes.c_void_p(hb.data_ptr()),
                               ctypes.c_void_p(out.data_ptr()), _stream(x.device)))
    return out


def resnet_tower_heads(x: torch.Tensor, u2all: torch.Tensor, biasall: torch.Tensor, nlayers: int, f: "FusedResNet",
                       want_out: bool = False):
    """bk_resnet_tower_heads: the tower and the heads in one launch, from the stem output x
    [B, 64, N, N] channels_last -> (policy features [B, 2*N*N], values [B, P][, tower output])."""
    from .engine import _check, _ptr, _stream, load_library

    B, C, N, _ = x.shape
    assert C == 64 and x.dtype == torch.float32 and x.is_contiguous(memory_format=torch.channels_last)
    lib = load_library()
    assert u2all.numel() == nlayers * lib.bk_tower_u_floats() and biasall.numel() == nlayers * 64
    P = f.value_fc2.out_features
    pf = torch.empty((B, 2 * N * N), dtype=torch.float32, device=x.device)
    v = torch.empty((B, P), dtype=torch.float32, device=x.device)
    out = torch.empty_like(x, memory_format=torch.channels_last) if want_out else None
    ha = torch.empty_like(x, memory_format=torch.channels_last)
    hb = torch.empty_like(x, memory_format=torch.channels_last)
    c = lambda t: t.detach().float().contiguous()  # noqa: E731
    wp, wv = c(f.policy_conv.weight.view(2, 64)), c(f.value_conv.weight.view(64))
    _check(lib.bk_resnet_tower_heads(ctypes.c_void_p(x.data_ptr()), B, N, nlayers, _ptr(u2all), _ptr(biasall),
                                     ctypes.c_void_p(ha.data_ptr()), ctypes.c_void_p(hb.data_ptr()),
                                     None if out is None else ctypes.c_void_p(out.data_ptr()), _ptr(wp),
                                     _ptr(c(f.policy_conv.bias)), _ptr(wv), _ptr(c(f.value_conv.bias)),
                                     _ptr(f.value_fc1_wt()), _ptr(c(f.value_fc1.bias)), _ptr(c(f.value_fc2.weight)),
                                     _ptr(c(f.value_fc2.bias)), P, _ptr(pf), _ptr(v), _stream(x.device)))
    return (pf, v, out) if want_out else (pf, v)


def resnet_stem_tower_heads(obs: torch.Tensor, wstem: torch.Tensor, u2all: torch.Tensor, biasall: torch.Tensor,
                            nlayers: int, f: "FusedResNet", want_x0: bool = False):
    """bk_resnet_stem_tower_heads: the planar observation [B, 8, N, N] -> (policy features
    [B, 2*N*N], values [B, P][, the stem output x0]) in one launch: stem conv, tower, heads."""
    from .engine import _check, _ptr, _stream, load_library

    B, cin, N, _ = obs.shape
    assert cin == 8 and obs.dtype == torch.float32 and obs.is_contiguous()
    lib = load_library()
    assert wstem.numel() == lib.bk_stem_tower_u_floats()
    assert u2all.numel() == nlayers * lib.bk_tower_u_floats() and biasall.numel() == nlayers * 64
    P = f.value_fc2.out_features
    pf = torch.empty((B, 2 * N * N), dtype=torch.float32, device=obs.device)
    v = torch.empty((B, P), dtype=torch.float32, device=obs.device)
    x0 = torch.empty((B, 64, N, N), dtype=torch.float32, device=obs.device, memory_format=torch.channels_last)
    ha, hb = torch.empty_like(x0), torch.empty_like(x0)
    c = lambda t: t.detach().float().contiguous()  # noqa: E731
    wp, wv = c(f.policy_conv.weight.view(2, 64)), c(f.value_conv.weight.view(64))
    _check(lib.bk_resnet_stem_tower_heads(
        ctypes.c_void_p(obs.data_ptr()), B, N, cin, _ptr(wstem), _ptr(c(f.stem.bias)), nlayers, _ptr(u2all),
        _ptr(biasall), ctypes.c_void_p(x0.data_ptr()), ctypes.c_void_p(ha.data_ptr()), ctypes.c_void_p(hb.data_ptr()),
        None, _ptr(wp), _ptr(c(f.policy_conv.bias)), _ptr(wv), _ptr(c(f.value_conv.bias)), _ptr(f.value_fc1_wt()),
        _ptr(c(f.value_fc1.bias)), _ptr(c(f.value_fc2.weight)), _ptr(c(f.value_fc2.bias)), P, _ptr(pf), _ptr(v),
        _stream(obs.device)))
    return (pf, v, x0) if want_x0 else (pf, v)


def resnet_heads(x: torch.Tensor, f: "FusedResNet"):
    """bk_resnet_heads: tower output [B, 64, N, N] channels_last -> (policy features [B, 2*N*N] in
    the NCHW flatten order, values [B, P])."""
    from .engine import _check, _ptr, _stream, load_library

    B, C, N, _ = x.shape
    assert C == 64 and x.dtype == torch.float32 and x.is_contiguous(memory_format=torch.channels_last)
    P = f.value_fc2.out_features
    pf = torch.empty((B, 2 * N * N), dtype=torch.float32, device=x.device)
    v = torch.empty((B, P), dtype=torch.float32, device=x.device)
    c = lambda t: t.detach().float().contiguous()  # noqa: E731
    wp, wv = c(f.policy_conv.weight.view(2, 64)), c(f.value_conv.weight.view(64))
    _check(load_library().bk_resnet_heads(ctypes.c_void_p(x.data_ptr()), B, N * N, _ptr(wp), _ptr(c(f.policy_conv.bias)),
                                          _ptr(wv), _ptr(c(f.value_conv.bias)), _ptr(f.value_fc1_wt()),
                                          _ptr(c(f.value_fc1.bias)), _ptr(c(f.value_fc2.weight)),
                                          _ptr(c(f.value_fc2.bias)), P, _ptr(pf), _ptr(v), _stream(x.device)))
    return pf, v


class LeafResNet(nn.Module):
    """The leaf evaluator's ResNet on the device (fp32): FusedResNet's function with the stem conv +
    bias + ReLU as one bk_conv3x3 launch, the whole residual tower (Winograd fp32 MFMA, NHWC
    activations; + the tower's residual and ReLU) as one bk_resnet_tower launch (board sizes it
    supports; one bk_conv3x3 launch per conv otherwise), both heads' 1x1 convs and the whole value MLP
    in one bk_resnet_heads launch, and the policy Linear in hipBLASLt (or, features=True, left to
    the search's sparse head). Input: the planar observation [B, 2P, N, N]. With normalize=False the policy
    comes back as raw logits (the leaf batch's consumer, k_expand_backup, takes a softmax over the
    legal ids, which a per-row shift does not change), skipping the full-row log-softmax."""

    def __init__(self, net: ResNet, normalize: bool = True, features: bool = False):
        super().__init__()
        self.f = FusedResNet(net).eval()
        self.normalize = normalize
        self.features = features  # return (policy features [B, 2*N*N], v): the search applies policy_out
        f = self.f
        self.native = f.stem.out_channels == 64 and f.stem.in_channels in (4, 8)
        self.x3 = False
        if self.native:
            self.register_buffer("w_stem", pack_conv3x3(f.stem.weight.detach()))
            for i, (c1, c2) in enumerate(f.blocks):
                self.register_buffer(f"w_{i}_1", pack_conv3x3(c1.weight.detach()))
                self.register_buffer(f"w_{i}_2", pack_conv3x3(c2.weight.detach()))
            if f.stem.in_channels == 8:  # the stem inside the tower launch (bk_resnet_stem_tower_heads)
                self.register_buffer("w_stem_tower", pack_stem_tower(f.stem.weight.detach()))
            if len(f.blocks):  # the fused tower's operands (bk_resnet_tower)
                convs = [c for blk in f.blocks for c in blk]
                self.register_buffer("u_tower", pack_tower([c.weight.detach() for c in convs]))
                self.register_buffer("b_tower", torch.cat([c.bias.detach().float() for c in convs]).contiguous())
            self.x3 = f.stem.in_channels == 8 and len(f.blocks) > 0
            if self.x3:  # bk_leafnet_x3's operands: split f16 weights + inverse scales
                ws, ss, bs = pack_x3(f.stem.weight, f.stem.bias)
                self.register_buffer("x3_wstem", ws)
                self.register_buffer("x3_sstem", ss)
                packs = [pack_x3(c.weight, c.bias) for c in convs]
                self.register_buffer("x3_wtower", torch.cat([p[0] for p in packs]).contiguous())
                self.register_buffer("x3_stower", torch.cat([p[1] for p in packs]).contiguous())
                self.register_buffer("x3_bounds", torch.cat([bs] + [p[2] for p in packs]).contiguous())
                # bk_leafnet_w3's tower operands: split Winograd U + inverse scales
                w3 = [pack_w3(c.weight) for c in convs]
                self.register_buffer("w3_utower", torch.cat([p[0] for p in w3]).contiguous())
                self.register_buffer("w3_stower", torch.cat([p[1] for p in w3]).contiguous())
                c = lambda t: t.detach().float().contiguous().clone()  # noqa: E731
                heads = [c(f.stem.bias), c(f.policy_conv.weight.view(2, 64)), c(f.policy_conv.bias),
                         c(f.value_conv.weight.view(64)), c(f.value_conv.bias), c(f.value_fc1_wt()),
                         c(f.value_fc1.bias), c(f.value_fc2.weight), c(f.value_fc2.bias)]
                # registered buffers, so .to(device) / state_dict see them like the weight packs
                for i, t in enumerate(heads):
                    self.register_buffer(f"x3_head{i}", t)

    @property
    def x3_heads(self) -> list[torch.Tensor]:
        """bk_leafnet_x3's head operands (stem bias, policy/value 1x1 convs, value MLP), on the
        module's current device."""
        return [getattr(self, f"x3_head{i}") for i in range(9)]

    @torch.no_grad()
    def forward(self, x):
        f = self.f
        n = len(f.blocks)
        if self.native:
            # planar observation in (as the search writes it), NHWC activations through the tower
            from .engine import load_library

            math = net_math() if self.x3 else "f32"
            if math == "w3" and load_library().bk_leafnet_w3_supported(x.shape[2]):
                # the tower as Winograd convolutions on split-f16 MFMA products (bk_leafnet_w3)
                pf, v = leafnet_w3(x.float().contiguous(), self)
                if self.features:
                    return pf, v
                logits = f.policy_out(pf)
                return (F.log_softmax(logits, dim=1) if self.normalize else logits), v
            if math in ("x3", "w3") and load_library().bk_leafnet_x3_supported(x.shape[2]):
                # the whole net in one launch on split-f16 MFMA products (bk_leafnet_x3)
                pf, v = leafnet_x3(x.float().contiguous(), self)
                if self.features:
                    return pf, v
                logits = f.policy_out(pf)
                return (F.log_softmax(logits, dim=1) if self.normalize else logits), v
            fused = n and tower_enabled() and load_library().bk_tower_supported(x.shape[2])
            if fused and f.stem.in_channels == 8:
                # stem conv, tower and heads in one launch (bk_resnet_stem_tower_heads)
                pf, v = resnet_stem_tower_heads(x.float().contiguous(), self.w_stem_tower, self.u_tower, self.b_tower,
                                                2 * n, f)
                if self.features:
                    return pf, v
                logits = f.policy_out(pf)
                return (F.log_softmax(logits, dim=1) if self.normalize else logits), v
            x = conv3x3(x.float().contiguous(), self.w_stem, f.stem.bias, True)
            h = x
            if fused:
                # the tower and the heads in one launch (bk_resnet_tower_heads)
                pf, v = resnet_tower_heads(x, self.u_tower, self.b_tower, 2 * n, f)
            else:
                for i, (c1, c2) in enumerate(f.blocks):
                    h = conv3x3(h, getattr(self, f"w_{i}_1"), c1.bias, True)
                    h = conv3x3(h, getattr(self, f"w_{i}_2"), c2.bias, i + 1 == n, x if i + 1 == n else None)
                if not n:
                    h = torch.relu(x + x)
                pf, v = resnet_heads(h, f)
            if self.features:
                return pf, v
            logits = f.policy_out(pf)
            return (F.log_softmax(logits, dim=1) if self.normalize else logits), v
        # other widths: MIOpen convolutions (channels_last) with the bk_bias_act epilogue
        x = x.float().contiguous(memory_format=torch.channels_last)
        conv = lambda t, c: F.conv2d(t, c.weight, None, c.stride, c.padding)  # noqa: E731
        x = _bias_act(conv(x, f.stem), f.stem.bias, True)
        h = x
        for i, (c1, c2) in enumerate(f.blocks):
            h = _bias_act(conv(h, c1), c1.bias, True)
            h = _bias_act(conv(h, c2), c2.bias, i + 1 == n, x if i + 1 == n else None)
        x = h if n else F.relu(x + x)
        conv1 = lambda t, c: F.conv2d(t, c.weight, None).contiguous(memory_format=torch.channels_last)  # noqa: E731
        p = _bias_act(conv1(x, f.policy_conv), f.policy_conv.bias, True)
        logits = f.policy_out(p.contiguous().flatten(1))
        v = _bias_act(conv1(x, f.value_conv), f.value_conv.bias, True)
        v = torch.tanh(f.value_fc2(F.relu(f.value_fc1(v.contiguous().flatten(1)))))
        if self.features:
            return p.contiguous().flatten(1), v
        return (F.log_softmax(logits, dim=1) if self.normalize else logits), v


def inference_model(model: nn.Module, normalize: bool = True, dtype: torch.dtype = torch.float32,
                    features: bool = False) -> nn.Module:
    """The leaf evaluator's form of a net: ResNet -> LeafResNet (fp32 HIP kernels) on a HIP
    device, FusedResNet for reduced-precision autocast runs or off the device; eval() otherwise.
    normalize=False lets LeafResNet return raw policy logits (see LeafResNet)."""
    if isinstance(model, ResNet):
        dev = next(model.parameters()).device
        if dev.type == "cuda" and dtype == torch.float32:
            return LeafResNet(model, normalize=normalize, features=features).eval()
        return FusedResNet(model).eval()
    return model.eval()
