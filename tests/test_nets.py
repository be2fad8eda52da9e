"""Leaf-eval nets and NNet-wrapper host logic against golden vectors produced by the
reference's own model and predict code (tests/golden/make_net_golden.py). CPU, float32."""
import importlib.util
import os
import types

import numpy as np
import pytest
import torch

from conftest import GOLDEN

_spec = importlib.util.spec_from_file_location("make_net_golden", os.path.join(GOLDEN, "make_net_golden.py"))
_mng = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(_mng)
det_state_dict = _mng.det_state_dict
G = np.load(os.path.join(GOLDEN, "net_golden.npz"))


def _load(model):
    sd = model.state_dict()
    model.load_state_dict(det_state_dict({k: v.shape for k, v in sd.items()}))  # strict: keys match the reference
    return model.eval()


def test_resnet_and_dcnnet_match_reference_7x7():
    from blokus_rl_amd.nets import DCNNet, FusedResNet, ResNet
    obs = torch.from_numpy(G["obs7"])
    r = _load(ResNet(7, 2, 2522, num_res_blocks=2))
    with torch.no_grad():
        lp, v = r(obs)
        torch.testing.assert_close(lp, torch.from_numpy(G["resnet7_logp"]), rtol=0, atol=2e-5)
        torch.testing.assert_close(v, torch.from_numpy(G["resnet7_v"]), rtol=0, atol=2e-6)
        flp, fv = FusedResNet(r)(obs)
        torch.testing.assert_close(flp, torch.from_numpy(G["resnet7_logp"]), rtol=0, atol=1e-4)
        torch.testing.assert_close(fv, torch.from_numpy(G["resnet7_v"]), rtol=0, atol=1e-5)
    d = _load(DCNNet(7, 2, 2522, num_channels=32, linear_dim=64))
    with torch.no_grad():
        lp, v = d(obs)
    torch.testing.assert_close(lp, torch.from_numpy(G["dcnnet7_logp"]), rtol=0, atol=2e-5)
    torch.testing.assert_close(v, torch.from_numpy(G["dcnnet7_v"]), rtol=0, atol=2e-6)


class _Game:
    board_size, number_of_players = 20, 4

    def get_action_size(self):
        return 30433


@pytest.mark.parametrize("blocks", [2, 5])
def test_predict_matches_reference_20x20(blocks):
    """The drop-in predict() on the CPU (the same module structure as the reference, fp32) against
    the reference predict() golden rows, 2-block and config-3 (5-block) nets, at fp32 rounding."""
    from blokus_rl_amd.neural_network import BlokusNNetWrapper
    hp = types.SimpleNamespace(model_type="resnet", num_res_blocks=blocks, lr=1e-3, weight_decay=1e-4)
    w = BlokusNNetWrapper(_Game(), hp, device="cpu")
    _load(w.model)
    sfx = "" if blocks == 2 else "b5"
    n20 = sum(1 for k in G.files if k.startswith("obs20_"))  # mid-game, empty and spread boards
    assert n20 >= 10
    for i in range(n20):
        mask = np.zeros(30433)
        mask[G[f"ids20_{i}"]] = 1
        p, v = w.predict(G[f"obs20_{i}"], mask)
        np.testing.assert_allclose(p, G[f"p20{sfx}_{i}"], rtol=1e-5, atol=1e-9)
        np.testing.assert_allclose(v, G[f"v20{sfx}_{i}"], rtol=0, atol=1e-6)


def test_vectorised_loss_equals_reference_loop():
    """compute_loss vs the reference's per-sample loop (neural_network.py:138-157)."""
    import torch.nn.functional as F
    from torch.nn.utils.rnn import pad_sequence
    from blokus_rl_amd.neural_network import BlokusNNetWrapper

    torch.manual_seed(0)
    B, A = 5, 300
    masks = torch.rand(B, A) < 0.2
    logits = torch.randn(B, A)
    pis = [torch.softmax(torch.randn(int(m.sum())), 0) for m in masks]
    p_gt = pad_sequence(pis, batch_first=True)
    v_pred, v_gt = torch.randn(B, 4), torch.randn(B, 4)
    ref_p = 0
    for mask, gt, lg in zip(masks, p_gt, logits):
        pred = F.log_softmax(torch.masked_select(lg, mask), dim=-1)
        pred = F.pad(pred, (0, gt.shape[0] - pred.shape[0]), value=0)
        ref_p += -torch.sum(gt * pred)
    ref = ref_p / B + (v_pred.squeeze() - v_gt).pow(2).mean()
    got = BlokusNNetWrapper.compute_loss(None, masks, (logits, v_pred), (p_gt, v_gt))
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)
