"""The learner's device path for the ResNet: the residual tower's 3x3
convolutions 64 -> 64 on the f16 matrix cores (bk_conv_x3 / bk_conv_x3_wgrad: split-f16 products,
fp32-class), the activations in channels_last (NHWC), the 64-channel train-mode batch norms on
bk_bn_forward / bk_bn_backward (fp64 statistics) and the heads' small ones on PyTorch's kernels.

The reference trains models/blokus_nnet.py:88-151 in fp32 (neural_network.py:52-85); on MI355X
the fp32 convolutions (MIOpen igemm / Winograd on the f32 MFMA, 1/16 of the f16 rate on gfx950)
take most of a large-batch step. `ConvX3Function` runs a conv's forward and its input gradient
through bk_conv_x3 and its weight gradient through bk_conv_x3_wgrad; `prepare_model` switches a
ResNet to that path in place without touching its parameters or state_dict keys.
"""
from __future__ import annotations

import ctypes

import torch
from torch import nn

from ..engine import _check, _ptr, _stream, load_library
import torch.nn.functional as F

from ..nets import NativeBatchNorm2d, ResNet, use_native_batchnorm


def pack_weight(weight: torch.Tensor, flip: bool) -> tuple[torch.Tensor, torch.Tensor]:
    """[64, 64, 3, 3] f32 -> (split fragments, inverse row scales) of bk_conv_x3, on the device
    (bk_conv_x3_pack: nets.pack_x3's operands; flip = the input-gradient conv's weights)."""
    lib = load_library()
    w = weight.detach()
    if w.dtype != torch.float32 or not w.is_contiguous():
        w = w.float().contiguous()
    ws = torch.empty(lib.bk_conv_x3_weight_bytes(), dtype=torch.uint8, device=w.device)
    inv = torch.empty(64, dtype=torch.float32, device=w.device)
    _check(lib.bk_conv_x3_pack(_ptr(w), int(flip), _ptr(ws), _ptr(inv), _stream(w.device)))
    return ws, inv


def conv_x3(x: torch.Tensor, ws: torch.Tensor, inv: torch.Tensor, bias: torch.Tensor | None) -> torch.Tensor:
    """bk_conv_x3 on a channels_last [B, 64, 20, 20] f32 activation -> [B, 64, 20, 20] channels_last."""
    lib = load_library()
    B, C, N, N2 = x.shape
    if C != 64 or N != 20 or N2 != 20 or x.dtype != torch.float32 or not x.is_cuda:
        raise ValueError(f"conv_x3 takes a [B, 64, 20, 20] f32 device tensor, got {tuple(x.shape)} {x.dtype}")
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.empty((B, 64, N, N), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
    b = None
    if bias is not None:
        b = bias.detach()
        b = b if (b.dtype == torch.float32 and b.is_contiguous()) else b.float().contiguous()
    # NHWC: channels_last [B, 64, N, N] is the dense [B][N][N][64] buffer the kernel reads and writes
    _check(lib.bk_conv_x3(ctypes.c_void_p(x.data_ptr()), B, N, _ptr(ws), _ptr(inv), _ptr(b) if b is not None else None,
                          ctypes.c_void_p(y.data_ptr()), _stream(x.device)))
    return y


def conv_x3_wgrad(x: torch.Tensor, gy: torch.Tensor) -> torch.Tensor:
    """bk_conv_x3_wgrad: the weight gradient [64, 64, 3, 3] of the 20x20 64->64 conv from its
    input x and output gradient gy (channels_last [B, 64, 20, 20] f32)."""
    lib = load_library()
    B = x.shape[0]
    x = x.contiguous(memory_format=torch.channels_last)
    gy = gy.contiguous(memory_format=torch.channels_last)
    if tuple(x.shape[1:]) != (64, 20, 20) or x.shape != gy.shape or x.dtype != torch.float32 or gy.dtype != torch.float32:
        raise ValueError("conv_x3_wgrad takes two [B, 64, 20, 20] f32 tensors")
    ws = torch.empty(lib.bk_conv_x3_wgrad_workspace_floats(B), dtype=torch.float32, device=x.device)
    dw = torch.empty((64, 64, 3, 3), dtype=torch.float32, device=x.device)
    _check(lib.bk_conv_x3_wgrad(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(gy.data_ptr()), B, 20, _ptr(ws), _ptr(dw),
                                _stream(x.device)))
    return dw


class ConvX3Function(torch.autograd.Function):
    """y = conv2d(x, weight, bias, padding=1) with the forward, the input gradient and the weight
    gradient on bk_conv_x3 / bk_conv_x3_wgrad; the bias gradient the sum of dy over batch and
    pixels."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ws, inv = pack_weight(weight, flip=False)
        y = conv_x3(x, ws, inv, bias)
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            ws, inv = pack_weight(weight, flip=True)
            gx = conv_x3(gy, ws, inv, None)
        if ctx.needs_input_grad[1]:
            gw = conv_x3_wgrad(x, gy)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = gy.sum(dim=(0, 2, 3))
        return gx, gw, gb


def bn_forward(x: torch.Tensor, gamma, beta, rmean, rvar, momentum: float, eps: float, relu: bool):
    """bk_bn_forward_ex on a channels_last [B, 64, H, W] f32 activation -> (y, stats [256])."""
    lib = load_library()
    M = x.numel() // 64
    ws = torch.empty(lib.bk_bn_workspace_doubles(), dtype=torch.float64, device=x.device)
    stats = torch.empty(256, dtype=torch.float32, device=x.device)
    y = torch.empty_like(x, memory_format=torch.channels_last)
    _check(lib.bk_bn_forward_ex(ctypes.c_void_p(x.data_ptr()), M, _ptr(gamma), _ptr(beta), _ptr(rmean), _ptr(rvar),
                                float(momentum), float(eps), _ptr(ws), _ptr(stats), ctypes.c_void_p(y.data_ptr()),
                                int(relu), _stream(x.device)))
    return y, stats


def bn_backward(gy: torch.Tensor, x: torch.Tensor, gamma, stats, relu: bool, want_dsum: bool):
    """bk_bn_backward_ex -> (dx, dgamma, dbeta, dsum or None); dsum = the column sums of dx (the bias
    gradient of the conv that produced x)."""
    lib = load_library()
    M = x.numel() // 64
    ws = torch.empty(lib.bk_bn_workspace_doubles(), dtype=torch.float64, device=x.device)
    ws2 = torch.empty(lib.bk_bn_workspace2_doubles(), dtype=torch.float64, device=x.device) if want_dsum else None
    coef = torch.empty(256, dtype=torch.float32, device=x.device)
    dg = torch.empty(64, dtype=torch.float32, device=x.device)
    db = torch.empty(64, dtype=torch.float32, device=x.device)
    ds = torch.empty(64, dtype=torch.float32, device=x.device) if want_dsum else None
    dx = torch.empty_like(x, memory_format=torch.channels_last)
    _check(lib.bk_bn_backward_ex(ctypes.c_void_p(gy.data_ptr()), ctypes.c_void_p(x.data_ptr()), M, _ptr(gamma),
                                 _ptr(stats), _ptr(ws), _ptr(coef), _ptr(dg), _ptr(db), ctypes.c_void_p(dx.data_ptr()),
                                 int(relu), _ptr(ds), _ptr(ws2), _stream(x.device)))
    return dx, dg, db, ds


class BatchNormFunction(torch.autograd.Function):
    """Train-mode batch norm (+ the following ReLU when relu) of a channels_last [B, 64, H, W] f32
    activation on bk_bn_forward_ex / bk_bn_backward_ex (fp64 statistics, one streaming read per
    reduction; the ReLU's mask recomputed from x in the backward, no extra pass); updates the
    running statistics in place like nn.BatchNorm2d."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, relu):
        x = x.contiguous(memory_format=torch.channels_last)
        y, stats = bn_forward(x, weight, bias, running_mean, running_var, momentum, eps, relu)
        ctx.save_for_backward(x, weight, stats)
        ctx.relu = bool(relu)
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gy):
        x, weight, stats = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        dx, dg, db, _ = bn_backward(gy, x, weight, stats, ctx.relu, False)
        return dx, dg, db, None, None, None, None, None


class ConvBNFunction(torch.autograd.Function):
    """y = [relu](bn(conv(x))) in training (models/blokus_nnet.py:103-112's conv -> BatchNorm2d (->
    ReLU)): the conv on bk_conv_x3 (+ bias), the batch norm and ReLU on bk_bn_forward_ex; the
    backward on bk_bn_backward_ex — the ReLU's mask, dgamma, dbeta and the conv's bias gradient
    (dx's column sums, in the same pass) — then the conv's input gradient (bk_conv_x3, flipped
    weights) and weight gradient (bk_conv_x3_wgrad). Saves what the unfused pair saves (x, the conv
    output) and moves two fewer activation passes each way (the separate ReLU and bias sums)."""

    @staticmethod
    def forward(ctx, x, cw, cb, gamma, beta, running_mean, running_var, momentum, eps, relu):
        ws, inv = pack_weight(cw, flip=False)
        x = x.contiguous(memory_format=torch.channels_last)
        z = conv_x3(x, ws, inv, cb)
        y, stats = bn_forward(z, gamma, beta, running_mean, running_var, momentum, eps, relu)
        ctx.save_for_backward(x, cw, z, gamma, stats)
        ctx.relu, ctx.has_bias = bool(relu), cb is not None
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gy):
        x, cw, z, gamma, stats = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        need_cb = ctx.has_bias and ctx.needs_input_grad[2]
        dz, dg, db, dcb = bn_backward(gy, z, gamma, stats, ctx.relu, need_cb)
        gx = gw = None
        if ctx.needs_input_grad[0]:
            ws, inv = pack_weight(cw, flip=True)
            gx = conv_x3(dz, ws, inv, None)
        if ctx.needs_input_grad[1]:
            gw = conv_x3_wgrad(x, dz)
        return gx, gw, dcb, dg, db, None, None, None, None, None


class FusedBatchNorm2d(NativeBatchNorm2d):
    """nn.BatchNorm2d(64) (same parameters, buffers and state_dict keys) whose train-mode device
    calls on 64-channel f32 activations run BatchNormFunction; everything else (eval mode, CPU,
    other shapes, momentum=None) takes PyTorch's own batch norm."""

    def forward(self, x):
        if (self.training and x.is_cuda and x.dim() == 4 and x.shape[1] == 64 and x.dtype == torch.float32
                and self.affine and self.track_running_stats and self.momentum is not None
                and x.numel() > 64):
            self.num_batches_tracked.add_(1)
            return BatchNormFunction.apply(x, self.weight, self.bias, self.running_mean, self.running_var,
                                           self.momentum, self.eps, False)
        return super().forward(x)


def use_fused_batchnorm(model: nn.Module) -> int:
    """Switch every 64-channel BatchNorm2d of `model` to FusedBatchNorm2d in place."""
    k = 0
    for m in model.modules():
        if type(m) in (nn.BatchNorm2d, NativeBatchNorm2d) and m.num_features == 64:
            m.__class__ = FusedBatchNorm2d
            k += 1
    return k


def _eligible(m: nn.Module) -> bool:
    return (type(m) is nn.Conv2d and m.in_channels == 64 and m.out_channels == 64 and m.kernel_size == (3, 3)
            and m.stride == (1, 1) and m.padding == (1, 1) and m.dilation == (1, 1) and m.groups == 1
            and m.padding_mode == "zeros")


class X3Conv2d(nn.Conv2d):
    """nn.Conv2d (same parameters and state_dict keys) whose 20x20 64->64 device calls in training
    (train mode, gradients enabled) run ConvX3Function; anything else (eval mode, no_grad /
    inference, CPU, other shapes) takes nn.Conv2d's own fp32 path."""

    def forward(self, x):
        if (self.training and torch.is_grad_enabled() and x.is_cuda and x.dim() == 4
                and tuple(x.shape[1:]) == (64, 20, 20) and x.dtype == torch.float32):
            return ConvX3Function.apply(x, self.weight, self.bias)
        return super().forward(x)


def use_x3_convs(model: nn.Module) -> int:
    """Switch every eligible Conv2d (3x3, 64 -> 64, stride 1, padding 1) to X3Conv2d in place;
    returns how many were switched."""
    k = 0
    for m in model.modules():
        if _eligible(m):
            m.__class__ = X3Conv2d
            k += 1
    return k


class SparsePolicyLinear(torch.autograd.Function):
    """The policy Linear at each row's legal ids only (trainfc.hip): xs[b][j] = bias[ids[b][j]] +
    pf[b] . W[ids[b][j]] for j < k[b] — the logits compute_loss reads (neural_network.py:138-157);
    the backward's input gradient and dense weight / bias gradients (zero at ids no row holds) from
    the same pairs, in a fixed order."""

    @staticmethod
    def forward(ctx, pf, W, bias, ids, k):
        lib = load_library()
        pf = pf.float().contiguous()
        B, F = pf.shape
        cap = ids.shape[1]
        xs = torch.empty((B, cap), dtype=torch.float32, device=pf.device)
        _check(lib.bk_sparse_linear_fwd(_ptr(pf), B, F, _ptr(W.detach()), _ptr(bias.detach()), W.shape[0], _ptr(ids),
                                        _ptr(k), cap, _ptr(xs), _stream(pf.device)))
        ctx.save_for_backward(pf, W, ids, k)
        return xs

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        lib = load_library()
        pf, W, ids, k = ctx.saved_tensors
        g = g.float().contiguous()
        B, F = pf.shape
        A, cap = W.shape[0], ids.shape[1]
        dev, st = pf.device, _stream(pf.device)
        dpf = dW = db = None
        if ctx.needs_input_grad[0]:
            dpf = torch.empty_like(pf)
            _check(lib.bk_sparse_linear_dx(_ptr(g), B, F, _ptr(W.detach()), A, _ptr(ids), _ptr(k), cap, _ptr(dpf), st))
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            count = torch.zeros(A, dtype=torch.int32, device=dev)
            _check(lib.bk_sparse_linear_index(_ptr(ids), _ptr(k), cap, B, A, _ptr(count), None, None, None, st))
            start = torch.zeros(A + 1, dtype=torch.int32, device=dev)
            start[1:] = torch.cumsum(count, 0, dtype=torch.int32)
            cursor = torch.zeros(A, dtype=torch.int32, device=dev)
            pairs = torch.empty(B * cap, dtype=torch.int32, device=dev)
            _check(lib.bk_sparse_linear_index(_ptr(ids), _ptr(k), cap, B, A, _ptr(count), _ptr(start), _ptr(cursor),
                                              _ptr(pairs), st))
            dW = torch.empty((A, F), dtype=torch.float32, device=dev)
            db = torch.empty(A, dtype=torch.float32, device=dev)
            _check(lib.bk_sparse_linear_dw(_ptr(g), _ptr(pf), B, F, cap, A, _ptr(start), _ptr(pairs), _ptr(dW), _ptr(db),
                                           st))
        return dpf, dW, db, None, None


def _bn_ok(bn: nn.Module) -> bool:
    return (isinstance(bn, nn.BatchNorm2d) and bn.num_features == 64 and bn.affine and bn.track_running_stats
            and bn.momentum is not None)


def _bn_apply(bn: nn.Module, x: torch.Tensor, relu: bool) -> torch.Tensor:
    bn.num_batches_tracked.add_(1)
    return BatchNormFunction.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps, relu)


def _conv_bn(conv: nn.Module, bn: nn.Module, x: torch.Tensor, relu: bool) -> torch.Tensor:
    bn.num_batches_tracked.add_(1)
    return ConvBNFunction.apply(x, conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                bn.momentum, bn.eps, relu)


class TrainResNet(ResNet):
    """nets.ResNet (same modules, parameters and state_dict keys) whose training forward (train
    mode, gradients enabled, 20x20 f32 on the device) runs each residual block's conv -> BN -> ReLU
    and conv -> BN as one ConvBNFunction each and the stem's BN -> ReLU as one BatchNormFunction,
    and returns the policy head's raw logits instead of their log-softmax: the learner's loss is
    the masked log-softmax over the legal ids (bk_policy_loss, neural_network.py:138-157), which is
    invariant to the dense log-softmax's per-row shift, and its gradient sums to zero over a row,
    so the dense log-softmax (a [B, A] pass each way) changes neither the loss nor the gradients.
    Every other forward (eval, no_grad, CPU) is ResNet's own."""

    def _fused_ok(self, x: torch.Tensor) -> bool:
        return (self.training and torch.is_grad_enabled() and x.is_cuda and x.dtype == torch.float32
                and x.dim() == 4 and x.shape[2] == 20 and x.shape[3] == 20 and _bn_ok(self.bn1)
                and all(_eligible_x3(b[0]) and _eligible_x3(b[3]) and _bn_ok(b[1]) and _bn_ok(b[4])
                        and isinstance(b[2], nn.ReLU) and len(b) == 5 for b in self.res_blocks))

    def forward(self, x, ids: torch.Tensor | None = None, k: torch.Tensor | None = None):
        """ids / k (the batch's legal ids [B, cap] int16 and counts [B] int32): the policy head
        returns the logits at those ids only, [B, cap] (SparsePolicyLinear; the learner's loss reads
        nothing else), instead of the dense raw logits."""
        if not self._fused_ok(x):
            if ids is not None:
                raise ValueError("the sparse policy head is the device training path's (train mode, grad, cuda)")
            return super().forward(x)
        x = _bn_apply(self.bn1, self.conv1(x).contiguous(memory_format=torch.channels_last), True)
        h = x
        for b in self.res_blocks:
            h = _conv_bn(b[0], b[1], h, True)
            h = _conv_bn(b[3], b[4], h, False)
        x = F.relu(x + h)
        p = F.relu(self.policy_bn(self.policy_conv(x))).flatten(1)
        if ids is not None:
            p = SparsePolicyLinear.apply(p, self.policy_out.weight, self.policy_out.bias, ids, k)
        else:
            p = self.policy_out(p)  # raw logits (see the class docstring)
        v = F.relu(self.value_bn(self.value_conv(x))).flatten(1)
        v = torch.tanh(self.value_fc2(F.relu(self.value_fc1(v))))
        return p, v


def _eligible_x3(m: nn.Module) -> bool:
    return isinstance(m, nn.Conv2d) and m.in_channels == 64 and m.out_channels == 64 and m.kernel_size == (3, 3) \
        and m.stride == (1, 1) and m.padding == (1, 1) and m.dilation == (1, 1) and m.groups == 1 \
        and m.padding_mode == "zeros"


def prepare_model(model: nn.Module, x3_convs: bool = True, fused_bn: bool = True) -> nn.Module:
    """The device training path IN PLACE on the caller's model (Learner(device_path="auto") calls
    it): channels_last parameters, PyTorch batch norm (the 64-channel ones on bk_bn_forward /
    bk_bn_backward when fused_bn), and (x3_convs) the tower convs on bk_conv_x3. The swapped
    classes keep the parameters and state_dict keys; their eval-mode and no-grad forwards are
    PyTorch's fp32 ones, so a deepcopy of the model (e.g. the trainer's pnet) evaluates in fp32."""
    use_native_batchnorm(model)
    if fused_bn:
        use_fused_batchnorm(model)
    if x3_convs:
        use_x3_convs(model)
    if x3_convs and fused_bn and type(model) is ResNet:
        model.__class__ = TrainResNet  # the block-level fusion (conv + BN + ReLU per autograd node)
    return model.to(memory_format=torch.channels_last)
