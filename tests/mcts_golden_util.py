"""Helpers shared by the MCTS golden tests (CPU oracle and GPU engine)."""
import base64
import json
import os

import numpy as np

from conftest import GOLDEN

import importlib.util

_spec = importlib.util.spec_from_file_location("make_mcts_golden", os.path.join(GOLDEN, "make_mcts_golden.py"))
_mod = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(_mod)
prior_value = _mod.prior_value


def load_cases():
    with open(os.path.join(GOLDEN, "mcts_golden.json"), encoding="utf-8") as f:
        return json.load(f)["cases"]


def state_of(b64: str) -> np.ndarray:
    return np.frombuffer(base64.b64decode(b64), dtype=np.uint8).copy()


def unhex(xs):
    return [float.fromhex(x) for x in xs]


def load_episodes():
    """tests/golden/selfplay_golden.json: reference trainer._self_play episodes
    (make_selfplay_golden.py)."""
    with open(os.path.join(GOLDEN, "selfplay_golden.json"), encoding="utf-8") as f:
        return json.load(f)["episodes"]


def pi_of(b64: str) -> np.ndarray:
    return np.frombuffer(base64.b64decode(b64), dtype=np.float32).copy()
