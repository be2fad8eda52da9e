"""Golden leaf-evaluation vectors from the reference's own model / predict code.

Run here (never on the GPU box): `python tests/golden/make_net_golden.py`.
Loads /root/reference/blokus_rl/models/blokus_nnet.py (ResNet, DCNNet) and
blokus_rl/neural_network.py (BlokusNNetWrapper.predict / get_valid_dist) by file path, with the
package modules they import but do not need for a forward pass (blokus_rl.colossumrl,
blokus_rl.utils) stubbed, fills every parameter/buffer deterministically by name
(`det_state_dict`, shared with the tests, so no weights are stored), and records on CPU:
  * 7x7 2-player (A=2522) ResNet(2 blocks) and DCNNet: full log-prob rows and values;
  * 20x20 4-player (A=30433) ResNet(2 and 5 blocks): predict(obs, mask) -> (p over legal ids, v)
    on 3 mid-game boards, the empty board and up to 8 boards spread over a game.
Observations/masks come from oracle random boards. Output: tests/golden/net_golden.npz.
"""
import importlib.util
import os
import sys
import types
import zlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

REF = "/root/reference/blokus_rl"


def det_state_dict(shapes: dict) -> dict:
    """Deterministic tensors for a state_dict layout {name: shape}, keyed by name."""
    out = {}
    for name, shape in shapes.items():
        rng = np.random.default_rng(zlib.crc32(name.encode()))
        shape = tuple(shape)
        if name.endswith("num_batches_tracked"):
            out[name] = torch.zeros(shape, dtype=torch.long)
            continue
        if name.endswith("running_mean"):
            a = rng.uniform(-0.2, 0.2, shape)
        elif name.endswith("running_var"):
            a = rng.uniform(0.5, 1.5, shape)
        elif ("bn" in name or name.split(".")[-2:-1] in (["1"], ["4"])) and name.endswith("weight") and len(shape) == 1:
            a = rng.uniform(0.8, 1.2, shape)
        elif name.endswith("bias"):
            a = rng.uniform(-0.1, 0.1, shape)
        else:
            fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 1
            a = rng.standard_normal(shape) / np.sqrt(fan_in)
        out[name] = torch.from_numpy(a.astype(np.float32))
    return out


def _load(modname, path, package):
    spec = importlib.util.spec_from_file_location(modname, path)
    mod = importlib.util.module_from_spec(spec)
    mod.__package__ = package
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    pkg = types.ModuleType("refbk")
    pkg.__path__ = []
    sys.modules["refbk"] = pkg
    col = types.ModuleType("refbk.colossumrl")
    col.ColosseumBlokusGameWrapper = object
    sys.modules["refbk.colossumrl"] = col
    utils = types.ModuleType("refbk.utils")

    class AverageMeter:
        def __init__(self):
            self.avg = 0

        def update(self, v, n=1):
            self.avg = v

    utils.AverageMeter = AverageMeter
    utils.log_info = utils.log_warning = lambda *a, **k: None
    utils.to_device = lambda x, d: x
    sys.modules["refbk.utils"] = utils
    _load("refbk.hparams", os.path.join(REF, "hparams.py"), "refbk")
    models = types.ModuleType("refbk.models")
    models.__path__ = []
    sys.modules["refbk.models"] = models
    dumb = _load("refbk.models.dumbnet", os.path.join(REF, "models", "dumbnet.py"), "refbk.models")
    nnet = _load("refbk.models.blokus_nnet", os.path.join(REF, "models", "blokus_nnet.py"), "refbk.models")
    models.DumbNet, models.DCNNet, models.ResNet = dumb.DumbNet, nnet.DCNNet, nnet.ResNet
    models.get_model = lambda t: {"dumbnet": dumb.DumbNet, "dcnnet": nnet.DCNNet, "resnet": nnet.ResNet}[t]
    nw = _load("refbk.neural_network", os.path.join(REF, "neural_network.py"), "refbk")
    return nnet, nw


class _Game:
    def __init__(self, n, p, a):
        self.n, self.number_of_players, self.a = n, p, a

    def get_board_size(self):
        return (self.n, self.n)

    def get_action_size(self):
        return self.a

    def get_number_of_players(self):
        return self.number_of_players

    def get_observation_size(self):
        return [2 * self.number_of_players, self.n, self.n]


class _HP(types.SimpleNamespace):
    pass


def main():
    from oracle.oracle import Oracle

    torch.set_num_threads(4)
    nnet, nw = load_reference()
    out = {}
    # 7x7: full outputs
    o7 = Oracle(7, 2, 5)
    boards7 = [o7.random_board(s, 12) for s in range(6)]
    obs7 = np.stack([o7.observe(b) for b in boards7])
    hp7 = _HP(num_res_blocks=2, num_channels=32, linear_dim=64, dropout=0.3, lr=1e-3, weight_decay=1e-4,
              model_type="resnet")
    g7 = _Game(7, 2, o7.A)
    for name, cls in (("resnet7", nnet.ResNet), ("dcnnet7", nnet.DCNNet)):
        m = cls(g7, hp7).eval()
        m.load_state_dict(det_state_dict({k: v.shape for k, v in m.state_dict().items()}))
        with torch.no_grad():
            lp, v = m(torch.from_numpy(obs7))
        out[f"{name}_logp"] = lp.numpy()
        out[f"{name}_v"] = v.numpy()
    out["obs7"] = obs7
    # 20x20: the reference predict() path
    o20 = Oracle(20, 4, 5)
    # three mid-game boards (the round-1 rows), the empty board (first move) and boards spread over
    # a whole game (seeds 4..11, up to 80 random plies; a mover without a legal move is skipped)
    boards20 = [o20.random_board(s, 40) for s in (1, 2, 3)] + [o20.init_state()]
    boards20 += [b for b in (o20.random_board(s, 80) for s in range(4, 12)) if len(o20.legal_ids(b)) > 0]
    hp20 = _HP(num_res_blocks=2, num_channels=128, linear_dim=128, dropout=0.3, lr=1e-3, weight_decay=1e-4,
               model_type="resnet")
    g20 = _Game(20, 4, o20.A)
    wrapper = nw.BlokusNNetWrapper(g20, hp20, device="cpu")
    wrapper.model.load_state_dict(det_state_dict({k: v.shape for k, v in wrapper.model.state_dict().items()}))
    for i, b in enumerate(boards20):
        obs = o20.observe(b)
        mask = np.zeros(o20.A)
        mask[o20.legal_ids(b)] = 1
        p, v = wrapper.predict(obs, mask)
        out[f"obs20_{i}"] = obs
        out[f"ids20_{i}"] = np.nonzero(mask)[0].astype(np.int32)
        out[f"p20_{i}"] = np.asarray(p, dtype=np.float32)
        out[f"v20_{i}"] = np.asarray(v, dtype=np.float32)
    # the config-3 net: 5 residual blocks, the same 30433-action predict() path
    hp20b5 = _HP(num_res_blocks=5, num_channels=128, linear_dim=128, dropout=0.3, lr=1e-3, weight_decay=1e-4,
                 model_type="resnet")
    wrapper5 = nw.BlokusNNetWrapper(g20, hp20b5, device="cpu")
    wrapper5.model.load_state_dict(det_state_dict({k: v.shape for k, v in wrapper5.model.state_dict().items()}))
    for i, b in enumerate(boards20):
        mask = np.zeros(o20.A)
        mask[o20.legal_ids(b)] = 1
        p, v = wrapper5.predict(o20.observe(b), mask)
        out[f"p20b5_{i}"] = np.asarray(p, dtype=np.float32)
        out[f"v20b5_{i}"] = np.asarray(v, dtype=np.float32)
    fp = os.path.join(HERE, "net_golden.npz")
    np.savez_compressed(fp, **out)
    print(fp, os.path.getsize(fp), "bytes;", sorted(out))


if __name__ == "__main__":
    main()
