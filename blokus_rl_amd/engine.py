"""ctypes binding of libblokus_hip.so (include/blokus_engine.h) with torch as device plumbing.

torch provides device memory, streams and the policy/value net; every rules/search operation
runs in the HIP library. There is no CPU fallback: importing this module on a machine without
the built library raises, and every call needs a HIP device.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BK_LIB") or os.path.join(HERE, "_lib", "libblokus_hip.so")
STATE_BYTES = 384
STATE_WORDS = STATE_BYTES // 4

# Word offsets inside a state (include/blokus_engine.h)
W_PIECES, W_HASH, W_TO_MOVE, W_PLY, W_FLAGS = 80, 84, 86, 87, 88

_vp = ctypes.c_void_p
_i = ctypes.c_int
_SIGS = {
    "bk_last_error": (ctypes.c_char_p, []),
    "bk_version": (_i, []),
    "bk_state_bytes": (_i, []),
    "bk_ctx_create": (_i, [_i, _i, _i, _i, ctypes.POINTER(_vp)]),
    "bk_ctx_destroy": (_i, [_vp]),
    "bk_action_size": (_i, [_vp]),
    "bk_mask_words": (_i, [_vp]),
    "bk_num_pieces": (_i, [_vp]),
    "bk_action_table": (_i, [_vp, _vp]),
    "bk_action_cells": (_i, [_vp, _vp]),
    "bk_init_states": (_i, [_vp, _vp, _i, _vp]),
    "bk_legal_mask": (_i, [_vp, _vp, _vp, _i, _vp, _vp, _vp]),
    "bk_legal_ids": (_i, [_vp, _vp, _vp, _i, _vp, _i, _vp, _vp]),
    "bk_next_state": (_i, [_vp, _vp, _vp, _i, _vp, _vp, _vp, _vp]),
    "bk_game_ended": (_i, [_vp, _vp, _i, _vp, _vp, _vp]),
    "bk_observe": (_i, [_vp, _vp, _i, _vp, _vp]),
    "bk_square_counts": (_i, [_vp, _vp, _i, _vp, _vp]),
    "bk_mcts_create": (_i, [_vp, _i, _i, ctypes.c_int64, ctypes.POINTER(_vp)]),
    "bk_mcts_destroy": (_i, [_vp]),
    "bk_mcts_reset": (_i, [_vp, _vp, _vp]),
    "bk_mcts_select": (_i, [_vp, _vp, _vp, ctypes.c_double, _vp, _vp, _vp, _vp]),
    "bk_mcts_select_eps": (_i, [_vp, _vp, _vp, ctypes.c_double, ctypes.c_double, _vp, _vp, _vp, _vp]),
    "bk_mcts_expand_backup": (_i, [_vp, _vp, _vp, _i, _vp]),
    "bk_mcts_leaf_logits": (_i, [_vp, _vp, ctypes.c_int64, _i, _vp, _vp, _vp]),
    "bk_mcts_leaf_step": (_i, [_vp, _vp, ctypes.c_int64, _i, _vp, _vp, _vp, _i, _vp, _vp, ctypes.c_double, _vp,
                               _vp, _vp, _vp]),
    "bk_mcts_root_policy": (_i, [_vp, _vp, _vp, ctypes.c_double, _vp, _vp, _i, _vp, _vp]),
    "bk_mcts_root_stats": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp]),
    "bk_mcts_counters": (_i, [_vp, _vp, _vp]),
    "bk_mcts_leaf_info": (_i, [_vp, _vp, _vp, _vp]),
    "bk_ply_policy": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i, ctypes.c_double, ctypes.c_double, ctypes.c_uint64,
                           ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bk_ply_finish": (_i, [_i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                           ctypes.c_int64, _vp, _vp, _vp, _vp, _vp]),
    "bk_vec_reset": (_i, [_vp, _vp, _vp, _vp, _i, _vp, _vp, _vp]),
    "bk_vec_step": (_i, [_vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    "bk_vec_policy": (_i, [_vp, _vp, _vp, _vp, _i, _i, _vp, _vp, _vp]),
    "bk_vec_step_policy": (_i, [_vp, _vp, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bk_replay_stride": (ctypes.c_size_t, [_i]),
    "bk_replay_batch": (_i, [_vp, _vp, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bk_policy_loss": (_i, [_vp, ctypes.c_int64, _vp, _vp, _vp, _i, _i, _vp, _vp, _vp]),
    "bk_policy_loss_grad": (_i, [_vp, ctypes.c_int64, _vp, _vp, _vp, _i, _i, _vp, ctypes.c_float, _vp, _vp,
                                 ctypes.c_int64, _vp]),
    "bk_conv_x3_weight_bytes": (_i, []),
    "bk_conv_x3_pack": (_i, [_vp, _i, _vp, _vp, _vp]),
    "bk_conv_x3": (_i, [_vp, _i, _i, _vp, _vp, _vp, _vp, _vp]),
    "bk_conv_x3_wgrad_workspace_floats": (_i, [_i]),
    "bk_conv_x3_wgrad": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp]),
    "bk_bn_workspace_doubles": (_i, []),
    "bk_bn_forward": (_i, [_vp, ctypes.c_int64, _vp, _vp, _vp, _vp, ctypes.c_float, ctypes.c_float, _vp, _vp, _vp, _vp]),
    "bk_bn_backward": (_i, [_vp, _vp, ctypes.c_int64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bk_bn_workspace2_doubles": (_i, []),
    "bk_bn_forward_ex": (_i, [_vp, ctypes.c_int64, _vp, _vp, _vp, _vp, ctypes.c_float, ctypes.c_float, _vp, _vp, _vp,
                              _i, _vp]),
    "bk_bn_backward_ex": (_i, [_vp, _vp, ctypes.c_int64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp]),
    "bk_sparse_linear_fwd": (_i, [_vp, _i, _i, _vp, _vp, _i, _vp, _vp, _i, _vp, _vp]),
    "bk_sparse_linear_dx": (_i, [_vp, _i, _i, _vp, _i, _vp, _vp, _i, _vp, _vp]),
    "bk_sparse_linear_index": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp]),
    "bk_sparse_linear_dw": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp]),
    "bk_ppo_gae": (_i, [_i, _i, _vp, _vp, _vp, _vp, _vp, ctypes.c_float, ctypes.c_float, _vp, _vp, _vp]),
    "bk_filter_legal": (_i, [_vp, _i, _i, _vp, _i, _vp, _vp]),
    "bk_bias_act": (_i, [_vp, ctypes.c_int64, _i, _vp, _vp, _i, _vp]),
    "bk_conv3x3_packed_floats": (_i, [_i]),
    "bk_conv3x3_form": (_i, [_i, _i]),
    "bk_conv3x3": (_i, [_vp, _i, _i, _i, _vp, _vp, _vp, _i, _vp, _vp]),
    "bk_resnet_heads": (_i, [_vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp]),
    "bk_tower_u_floats": (_i, []),
    "bk_tower_supported": (_i, [_i]),
    "bk_resnet_tower": (_i, [_vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bk_resnet_tower_heads": (_i, [_vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _i, _vp, _vp, _vp]),
    "bk_stem_tower_u_floats": (_i, []),
    "bk_resnet_stem_tower_heads": (_i, [_vp, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                        _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp]),
    "bk_leafnet_x3_weight_bytes": (_i, [_i]),
    "bk_leafnet_x3_supported": (_i, [_i]),
    "bk_leafnet_x3": (_i, [_vp, _i, _i, _i, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp] + [_vp] * 8 + [_i, _vp, _vp, _vp, _vp]),
    "bk_leafnet_w3_weight_bytes": (_i, []),
    "bk_leafnet_w3_supported": (_i, [_i]),
    "bk_leafnet_w3": (_i, [_vp, _i, _i, _i, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp] + [_vp] * 8 + [_i, _vp, _vp, _vp, _vp, _vp]),
}

_LIB = None


class EngineError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load the HIP engine (torch first, so its libamdhip64.so.7 is the one in the process)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise EngineError(
            f"HIP engine library not built: {path}. Run `python -c 'import __graft_entry__ as g; g.build()'`."
        )
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def exported_symbols() -> list[str]:
    return list(_SIGS)


def _check(rc: int):
    if rc != 0:
        msg = _LIB.bk_last_error().decode() if _LIB else "?"
        raise EngineError(f"engine error {rc}: {msg}")


def _ptr(t: torch.Tensor | None):
    if t is None:
        return None
    assert t.is_contiguous()
    return ctypes.c_void_p(t.data_ptr())


def _stream(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


@dataclass(frozen=True)
class Preset:
    board_size: int = 20
    num_players: int = 4
    max_piece_cells: int = 5


class Engine:
    """One board preset on one HIP device. States are uint8 tensors [B, 384] on that device."""

    def __init__(self, board_size: int = 20, num_players: int = 4, max_piece_cells: int = 5,
                 device: int | str | torch.device | None = None):
        if not torch.cuda.is_available():
            raise EngineError("the Blokus engine needs a HIP device (torch.cuda.is_available() is False)")
        self.lib = load_library()
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.N, self.P, self.max_cells = board_size, num_players, max_piece_cells
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            _check(self.lib.bk_ctx_create(board_size, num_players, max_piece_cells, dev.index, ctypes.byref(h)))
        self.h = h
        self.A = self.lib.bk_action_size(h)
        self.W = self.lib.bk_mask_words(h)
        self.num_pieces = self.lib.bk_num_pieces(h)
        tab = np.zeros((self.A, 4), dtype=np.int32)
        _check(self.lib.bk_action_table(h, tab.ctypes.data_as(ctypes.c_void_p)))
        self.action_table = tab
        cells = np.zeros((self.A, 5), dtype=np.int16)
        _check(self.lib.bk_action_cells(h, cells.ctypes.data_as(ctypes.c_void_p)))
        self.action_cells = cells

    def __del__(self):
        try:
            if getattr(self, "h", None):
                self.lib.bk_ctx_destroy(self.h)
                self.h = None
        except Exception:  # pragma: no cover
            pass

    # ------------------------------------------------------------------ helpers
    @property
    def obs_shape(self):
        return (2 * self.P, self.N, self.N)

    def empty_states(self, B: int) -> torch.Tensor:
        return torch.empty((B, STATE_BYTES), dtype=torch.uint8, device=self.device)

    def _s(self):
        return _stream(self.device)

    # ------------------------------------------------------------------ batched env
    def init_states(self, B: int) -> torch.Tensor:
        st = self.empty_states(B)
        _check(self.lib.bk_init_states(self.h, _ptr(st), B, self._s()))
        return st

    def legal_mask(self, states: torch.Tensor, players: torch.Tensor | None = None):
        B = states.shape[0]
        masks = torch.empty((B, self.W), dtype=torch.int64, device=self.device)
        counts = torch.empty(B, dtype=torch.int32, device=self.device)
        _check(self.lib.bk_legal_mask(self.h, _ptr(states), _ptr(players), B, _ptr(masks), _ptr(counts),
                                      self._s()))
        return masks, counts

    def legal_mask_into(self, states, masks, counts, players=None):
        _check(self.lib.bk_legal_mask(self.h, _ptr(states), _ptr(players), states.shape[0], _ptr(masks),
                                      _ptr(counts), self._s()))

    def legal_ids(self, states: torch.Tensor, cap: int = 2048, players: torch.Tensor | None = None):
        B = states.shape[0]
        ids = torch.empty((B, cap), dtype=torch.int32, device=self.device)
        counts = torch.empty(B, dtype=torch.int32, device=self.device)
        _check(self.lib.bk_legal_ids(self.h, _ptr(states), _ptr(players), B, _ptr(ids), cap, _ptr(counts),
                                     self._s()))
        return ids, counts

    def next_state(self, states: torch.Tensor, actions: torch.Tensor):
        B = states.shape[0]
        out = self.empty_states(B)
        nxt = torch.empty(B, dtype=torch.int32, device=self.device)
        status = torch.empty(B, dtype=torch.int32, device=self.device)
        _check(self.lib.bk_next_state(self.h, _ptr(states), _ptr(actions), B, _ptr(out), _ptr(nxt),
                                      _ptr(status), self._s()))
        return out, nxt, status

    def game_ended(self, states: torch.Tensor):
        B = states.shape[0]
        ended = torch.empty(B, dtype=torch.int32, device=self.device)
        scores = torch.empty((B, self.P), dtype=torch.float64, device=self.device)
        _check(self.lib.bk_game_ended(self.h, _ptr(states), B, _ptr(ended), _ptr(scores), self._s()))
        return ended, scores

    def observe(self, states: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        B = states.shape[0]
        if out is None:
            out = torch.empty((B,) + self.obs_shape, dtype=torch.float32, device=self.device)
        _check(self.lib.bk_observe(self.h, _ptr(states), B, _ptr(out), self._s()))
        return out

    def replay_batch(self, rows: torch.Tensor, cap: int, index: torch.Tensor, with_states: bool = False):
        """Packed replay rows [E, stride] (uint8, device) + index [B] int64 -> the training batch
        {observation [B,2P,N,N] f32, ids [B,cap] int16, pi [B,cap] f32, k [B] int32,
        score [B,P] f32 (, states [B,384])} (bk_replay_batch)."""
        B = index.shape[0]
        dev = self.device
        assert rows.dtype == torch.uint8 and rows.shape[1] == self.lib.bk_replay_stride(cap)
        index = index.to(device=dev, dtype=torch.int64).contiguous()
        out = {
            "observation": torch.empty((B,) + self.obs_shape, dtype=torch.float32, device=dev),
            "ids": torch.empty((B, cap), dtype=torch.int16, device=dev),
            "pi": torch.empty((B, cap), dtype=torch.float32, device=dev),
            "k": torch.empty(B, dtype=torch.int32, device=dev),
            "score": torch.empty((B, self.P), dtype=torch.float32, device=dev),
        }
        st = self.empty_states(B) if with_states else None
        _check(self.lib.bk_replay_batch(self.h, _ptr(rows), cap, _ptr(index), B, _ptr(out["observation"]),
                                        _ptr(out["ids"]), _ptr(out["pi"]), _ptr(out["k"]), _ptr(out["score"]),
                                        _ptr(st), self._s()))
        if with_states:
            out["states"] = st
        return out

    def square_counts(self, states: torch.Tensor) -> torch.Tensor:
        B = states.shape[0]
        out = torch.empty((B, self.P), dtype=torch.int32, device=self.device)
        _check(self.lib.bk_square_counts(self.h, _ptr(states), B, _ptr(out), self._s()))
        return out

    # ------------------------------------------------------------------ state fields
    @staticmethod
    def words(states: torch.Tensor) -> torch.Tensor:
        return states.view(torch.int32)

    @staticmethod
    def to_move(states: torch.Tensor) -> torch.Tensor:
        return states.view(torch.int32)[:, W_TO_MOVE]

    @staticmethod
    def hashes(states: torch.Tensor) -> torch.Tensor:
        return states.view(torch.int64)[:, W_HASH // 2]

    def unpack_mask(self, masks: torch.Tensor) -> torch.Tensor:
        """[B, W] int64 bit words -> [B, A] bool (on device)."""
        bits = torch.arange(64, device=masks.device, dtype=torch.int64)
        m = (masks.unsqueeze(-1) >> bits) & 1
        return m.reshape(masks.shape[0], -1)[:, : self.A].bool()


def host_tables(board_size: int = 20, num_players: int = 4, max_piece_cells: int = 5):
    """Action table + cells from a host-only context (no device needed)."""
    lib = load_library()
    h = ctypes.c_void_p()
    _check(lib.bk_ctx_create(board_size, num_players, max_piece_cells, -1, ctypes.byref(h)))
    try:
        A = lib.bk_action_size(h)
        tab = np.zeros((A, 4), dtype=np.int32)
        cells = np.zeros((A, 5), dtype=np.int16)
        _check(lib.bk_action_table(h, tab.ctypes.data_as(ctypes.c_void_p)))
        _check(lib.bk_action_cells(h, cells.ctypes.data_as(ctypes.c_void_p)))
        return tab, cells
    finally:
        lib.bk_ctx_destroy(h)
