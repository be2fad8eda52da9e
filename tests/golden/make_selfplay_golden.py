"""Golden self-play episodes from the reference trainer's own `_self_play` (trainer.py:92-137).

Run here (never on the GPU box): `python tests/golden/make_selfplay_golden.py`.
Loads /root/reference/blokus_rl/alphazero/{mcts,trainer}.py by file path. trainer.py's imports
that `_self_play` never calls are stubbed in sys.modules (imageio, pytablewriter, torchsummary,
torch.utils.tensorboard are absent in this image; the package-relative colossumrl / hparams /
neural_network / players / utils / arena / dataset modules are replaced by empty names); the
real reference MCTS class is bound as `.mcts.MCTS`. The trainer object is made with
object.__new__ (its __init__ builds tensorboard writers and a torch net) and given
  * game  = the reference Game interface over the C oracle (make_mcts_golden.OracleGame plus
            get_init_board, blokus_wrapper.py:64-70),
  * nnet  = make_mcts_golden.StubNet (priors/values from prior_value(hash, K, P)),
  * hparams with num_mcts_sims / cpuct.
np.random.seed(seed) precedes each episode, so the Dirichlet root noise (trainer.py:112) and
the per-ply np.random.choice (trainer.py:124) come from the legacy global generator exactly as in
a reference run. Recorded per episode: the action ids applied (the index of each
np.random.choice draw is recorded by a pass-through wrapper), each ply's pi (float32 bytes), K, and the final scores z.
Output: tests/golden/selfplay_golden.json (data only).
"""
import base64
import importlib.util
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from make_mcts_golden import OracleGame, StubNet  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

REF = "/root/reference/blokus_rl"


def _load(modname, path, package):
    spec = importlib.util.spec_from_file_location(modname, path)
    mod = importlib.util.module_from_spec(spec)
    mod.__package__ = package
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__path__ = []
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def load_reference_trainer():
    _stub("imageio")
    _stub("pytablewriter", MarkdownTableWriter=object)
    _stub("torchsummary", summary=lambda *a, **k: "")
    _stub("torch.utils.tensorboard", SummaryWriter=object)
    _stub("refaz")
    for sub, attrs in {
        "colossumrl": dict(ColosseumBlokusGameWrapper=object),
        "hparams": dict(AlphaZeroHparams=object),
        "neural_network": dict(BlokusNNetWrapper=object),
        "players": dict(MCTSPlayer=object),
        "utils": dict(calculate_n_parameters=lambda *a: 0, log_info=lambda *a, **k: None),
    }.items():
        _stub(f"refaz.{sub}", **attrs)
    _stub("refaz.alphazero")
    _stub("refaz.alphazero.arena", play_match=None)
    _stub("refaz.alphazero.dataset", AlphaZeroDataset=object, collate_dataset_fn=None)
    _load("refaz.alphazero.mcts", os.path.join(REF, "alphazero", "mcts.py"), "refaz.alphazero")
    tr = _load("refaz.alphazero.trainer", os.path.join(REF, "alphazero", "trainer.py"), "refaz.alphazero")
    return tr.AlphaZeroTrainer


class EpisodeGame(OracleGame):
    """OracleGame + get_init_board (blokus_wrapper.py:64-70)."""

    def get_init_board(self):
        return self.o.init_state(), 0


def run_episode(Trainer, preset, sims, cpuct, temperature, seed):
    o = Oracle(*preset)
    tr = object.__new__(Trainer)
    tr.game = EpisodeGame(o)
    tr.nnet = StubNet(tr.game)
    tr.hparams = types.SimpleNamespace(num_mcts_sims=sims, cpuct=cpuct)
    picks = []
    choice = np.random.choice

    def recording_choice(n, p=None):  # trainer.py:124 -- the same draw, index recorded
        i = choice(n, p=p)
        picks.append(int(i))
        return i

    np.random.seed(seed)
    np.random.choice = recording_choice
    try:
        data = tr._self_play(temperature)
    finally:
        np.random.choice = choice
    # dist rows are the legal ids in ascending order (mcts.py:67-70), so the applied action of
    # ply k is legal_ids(s_k)[pick k]
    s = o.init_state()
    applied = []
    assert len(picks) == len(data)
    for k, (obs, mask, pi, z) in enumerate(data):
        assert (o.observe(s) == obs).all()
        ids = o.legal_ids(s)
        assert (np.nonzero(mask)[0] == ids).all()
        applied.append(int(ids[picks[k]]))
        s, _ = o.next_state(s, applied[-1])
    z = data[0][3]
    assert (o.game_ended(s) == z).all()
    return {
        "preset": list(preset), "sims": sims, "cpuct": cpuct, "temperature": temperature, "seed": seed,
        "actions": applied,
        "K": [int(d[1].sum()) for d in data],
        "pi": [base64.b64encode(np.ascontiguousarray(d[2], dtype=np.float32).tobytes()).decode() for d in data],
        "z": [float(x) for x in z],
    }


def main():
    Trainer = load_reference_trainer()
    # (preset, sims, cpuct, temperature, seed)
    specs = [
        ((7, 2, 5), 16, 1, 1.0, 0),
        ((7, 2, 5), 24, 1, 1.0, 7),
        ((7, 2, 5), 12, 2, 0, 3),
        ((7, 2, 4), 16, 1, 1.0, 11),
        ((20, 4, 5), 4, 1, 1.0, 5),
    ]
    eps = []
    for spec in specs:
        e = run_episode(Trainer, *spec)
        print(f"preset {e['preset']} sims {e['sims']} T {e['temperature']} seed {e['seed']}: "
              f"{len(e['actions'])} plies z {e['z']}")
        eps.append(e)
    out = {"generator": "tests/golden/make_selfplay_golden.py driving /root/reference/blokus_rl/alphazero/trainer.py "
                        "_self_play + mcts.py", "prior": "make_mcts_golden.prior_value", "episodes": eps}
    fp = os.path.join(HERE, "selfplay_golden.json")
    with open(fp, "w", encoding="utf-8") as f:
        json.dump(out, f, separators=(",", ":"))
    print(fp, os.path.getsize(fp), "bytes")


if __name__ == "__main__":
    main()
