"""Batched Arena: `play_match` (blokus_rl/alphazero/arena.py:10-87) for
MCTSPlayer seats (players/mcts_player.py:8-28), every game of the match played at once on the
batched engine.

Reference semantics kept exactly:
  * game i seats the players in order matches[i % len(matches)] (all permutations of the
    player list when permute, else the identity); colour c is played by player order[c];
  * each player owns its own MCTS, fresh at the start of every game (player.reset()) and kept
    across that player's moves of the game;
  * a move = `simulations` MCTS.simulate calls from the current state, then the T=0
    distribution's argmax (first max N) — deterministic given the priors;
  * scores[order] += the game's -1 / 3 / 1 one-hot (get_game_ended).

Layout: one tree per (game, player) — T = games x P trees in one BatchedMCTS; at each ply only
the tree of the player to move is active in each game. The G leaves of a simulation step are
gathered into one [G, 2P, N, N] batch; each distinct net evaluates it once (the arena compare
has two: the new net and the previous one) and rows are picked per game by the seat's net.
DumbNet seats (the "uninformed MCTS" player) get the uniform log-prior and zero values.
"""
from __future__ import annotations

from itertools import permutations

import numpy as np
import torch

from ..engine import Engine
from .batched_mcts import BatchedMCTS
from .selfplay import LeafEvaluator


class ArenaSeat:
    """One arena player: a net (None / DumbNet = uninformed MCTS) and its simulation count."""

    def __init__(self, model: torch.nn.Module | None, simulations: int):
        self.model = model
        self.simulations = int(simulations)


def seat_of(player) -> ArenaSeat:
    """An MCTSPlayer of the drop-in API (players.MCTSPlayer) -> its seat."""
    nn = getattr(player, "nn", None)
    if nn is None or not hasattr(player, "simulations"):
        raise TypeError(f"the batched arena plays MCTSPlayer seats only, got {player}")
    model = getattr(nn, "model", nn)
    return ArenaSeat(model, player.simulations)


class BatchedArena:
    def __init__(self, eng: Engine, seats: list, cpuct: float = 1.0, node_cap: int | None = None,
                 child_cap_per_tree: int | None = None, nn_dtype: torch.dtype = torch.float32):
        self.eng = eng
        self.seats = [s if isinstance(s, ArenaSeat) else seat_of(s) for s in seats]
        if len(self.seats) != eng.P:
            raise ValueError(f"{eng.P} players expected, got {len(self.seats)}")
        self.cpuct = cpuct
        if node_cap is None:
            # a seat's tree lives for the whole game and grows by <= sims nodes on each of its
            # player's plies (at most num_pieces of them)
            node_cap = max(s.simulations for s in self.seats) * eng.num_pieces + 1
        self.node_cap = node_cap
        self.child_cap_per_tree = child_cap_per_tree or node_cap * (256 if eng.N >= 14 else 64)
        self.nn_dtype = nn_dtype
        # distinct nets (by identity) -> evaluator index; seat -> net index
        self._models: list = []
        self.seat_net = []
        for s in self.seats:
            m = s.model
            if m is not None and m.__class__.__name__ == "DumbNet":
                m = None
            for i, mm in enumerate(self._models):
                if mm is m:
                    self.seat_net.append(i)
                    break
            else:
                self._models.append(m)
                self.seat_net.append(len(self._models) - 1)

    def play(self, games_num: int, permute: bool = False, max_plies: int = 10_000):
        """-> (scores float64[P] accumulated per player, per-game score rows [G][P], final states)."""
        eng, P, G = self.eng, self.eng.P, games_num
        dev = eng.device
        matches = list(permutations(range(P))) if permute else [tuple(range(P))]
        orders = torch.tensor([matches[i % len(matches)] for i in range(G)], dtype=torch.int64, device=dev)  # [G,P]
        T = G * P
        mcts = BatchedMCTS(eng, T, node_cap=self.node_cap, child_cap=T * self.child_cap_per_tree)
        evals = [LeafEvaluator(m, eng, G, self.nn_dtype, use_graph=m is not None, sparse_policy=False)
                 for m in self._models]
        seat_net = torch.tensor(self.seat_net, dtype=torch.int64, device=dev)
        seat_sims = torch.tensor([s.simulations for s in self.seats], dtype=torch.int64, device=dev)
        max_sims = max(s.simulations for s in self.seats)
        states = eng.init_states(G)
        logp = torch.zeros((T, eng.A), dtype=torch.float32, device=dev)
        vals = torch.zeros((T, P), dtype=torch.float32, device=dev)
        garange = torch.arange(G, device=dev)
        over = torch.zeros(G, dtype=torch.bool, device=dev)
        final = torch.zeros((G, P), dtype=torch.float64, device=dev)
        for _ in range(max_plies):
            to_move = Engine.to_move(states).long()
            pidx = orders.gather(1, to_move.view(-1, 1)).view(-1)     # player index at each game's turn
            tree = garange * P + pidx                                    # its tree
            roots = states.repeat_interleave(P, dim=0)
            net_row = seat_net[pidx]
            sims_row = seat_sims[pidx]
            for s in range(max_sims):
                act_g = (~over) & (sims_row > s)
                active = torch.zeros(T, dtype=torch.int32, device=dev)
                active[tree] = act_g.to(torch.int32)
                _, obs, _ = mcts.select(roots, active, self.cpuct)
                obs_g = obs.index_select(0, tree)
                lp_g = None
                v_g = None
                for n, ev in enumerate(evals):
                    lp, v = ev(obs_g)
                    if len(evals) == 1:
                        lp_g, v_g = lp, v
                        break
                    pick = (net_row == n).view(-1, 1)
                    lp_g = lp if lp_g is None else torch.where(pick, lp, lp_g)
                    v_g = v if v_g is None else torch.where(pick, v, v_g)
                logp.index_copy_(0, tree, lp_g.expand(G, -1) if lp_g.shape[0] != G else lp_g)
                vals.index_copy_(0, tree, v_g.expand(G, -1) if v_g.shape[0] != G else v_g)
                mcts.expand_backup(logp, vals, prior_mode=0)
            act_t = torch.zeros(T, dtype=torch.int32, device=dev)
            act_t[tree] = (~over).to(torch.int32)
            ids, pi, counts = mcts.root_policy(roots, act_t, 0.0)
            ids_g, pi_g = ids.index_select(0, tree), pi.index_select(0, tree)
            k = counts.index_select(0, tree)
            if bool(((k < 0) & ~over).any()):
                raise RuntimeError("arena: a root had more children than the root_policy cap")
            k = k.clamp(min=0)
            col = torch.arange(pi_g.shape[1], device=dev).unsqueeze(0)
            pi_g = torch.where(col < k.unsqueeze(1), pi_g, torch.full_like(pi_g, -1.0))
            best = pi_g.argmax(dim=1)  # first max, as np.argmax over the one-hot distribution
            action = ids_g.gather(1, best.view(-1, 1)).view(-1)
            action = torch.where(over | (k == 0), torch.full_like(action, -1), action).to(torch.int32)
            states, _, status = eng.next_state(states, action.contiguous())
            if bool((status != 0).any()):
                raise RuntimeError("arena: an MCTS move was illegal")
            ended, scores = eng.game_ended(states)
            newly = ended.bool() & ~over
            final = torch.where(newly.view(-1, 1), scores.to(torch.float64), final)
            over |= ended.bool()
            if bool(over.all()):
                break
        mcts.check()
        per_game = final.cpu().numpy()
        ords = orders.cpu().numpy()
        total = np.zeros(P)
        for g in range(G):
            total[list(ords[g])] += per_game[g]
        return total, per_game, states


def play_match_batched(game, players: list, games_num: int, permute: bool = False, cpuct: float = 1.0,
                       node_cap: int | None = None):
    """play_match(game, players, games_num, permute) (arena.py:10-32) for MCTSPlayer seats,
    batched: -> (scores, items) with items[i] = {"scores": game i's one-hot, "frames": []}."""
    arena = BatchedArena(game.engine, players, cpuct=cpuct, node_cap=node_cap)
    scores, per_game, _ = arena.play(games_num, permute)
    return scores, [{"scores": per_game[i], "frames": []} for i in range(games_num)]
