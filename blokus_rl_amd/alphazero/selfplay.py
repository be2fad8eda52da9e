"""GPU self-play: G concurrent games, one batched search tree per game.

Restates `AlphaZeroTrainer._self_play` (blokus_rl/alphazero/trainer.py:92-137) for G games at
once, every step on the device:
  per ply: `num_sims` x { k_select -> net forward on the [G, 2P, N, N] leaf batch ->
           k_expand_backup }, then get_distribution(T) at the root (mcts.py:73-99), root-only
           Dirichlet(alpha=1) mixing 0.75/0.25 on a game's first ply (trainer.py:110-116),
           sampling from pi (trainer.py:124-125), recording (state, pi, player), next state.
  at game end: every example of the game gets z = the final one-hot scores (trainer.py:134-135).
The host only launches; random numbers come from torch's device generator (per-run seed), so
trajectories are statistically — not stream-for-stream — equivalent to np.random's.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field

import torch

from ..engine import Engine, _check, _ptr
from .batched_mcts import BatchedMCTS


@dataclass
class Examples:
    """Packed replay examples (the all-gathered (s, pi, z) of SURVEY.md §8e): fixed stride."""
    states: torch.Tensor  # [E, 384] u8 — the root state (observation and mask are recomputed)
    ids: torch.Tensor     # [E, cap] int16 — legal ids of pi (ascending), -1 padded
    pi: torch.Tensor      # [E, cap] f32 — MCTS policy over ids
    k: torch.Tensor       # [E] int32 — number of ids
    z: torch.Tensor       # [E, P] f32 — final scores of the game (-1 / 3 / 1)

    def __len__(self):
        return int(self.states.shape[0])


@dataclass
class SelfPlayStats:
    sims: int = 0
    plies: int = 0
    games_finished: int = 0
    seconds: float = 0.0
    nn_seconds: float = 0.0
    extra: dict = field(default_factory=dict)


class LeafEvaluator:
    """Wraps the policy/value net for the leaf batch: obs [G, 2P, N, N] -> (logp [G, A] f32,
    v [G, P] f32). DumbNet needs no forward: a constant uniform log-prior and zero values."""

    def __init__(self, model: torch.nn.Module | None, eng: Engine, G: int, dtype: torch.dtype = torch.float32,
                 use_graph: bool = True, sparse_policy: bool = True):
        self.model = model
        self.eng = eng
        self.G = G
        self.sparse = False
        self.planar = False
        self.dtype = dtype
        dev = eng.device
        self.const_logp = None
        if model is None or model.__class__.__name__ == "DumbNet":
            self.const_logp = torch.full((G, eng.A), -float(torch.log(torch.tensor(float(eng.A)))),
                                         dtype=torch.float32, device=dev)
            self.const_v = torch.zeros((G, eng.P), dtype=torch.float32, device=dev)
            self.model = None
            return
        from ..nets import LeafResNet, inference_model
        # raw policy logits are enough: k_expand_backup takes the softmax over the legal ids; with
        # the HIP ResNet, even the policy Linear is left to the search (bk_mcts_leaf_logits computes
        # only the leaf's legal ids' logits), so the net returns (policy features, v)
        self.model = inference_model(model, normalize=False, dtype=dtype, features=sparse_policy).to(
            memory_format=torch.channels_last)
        self.sparse = isinstance(self.model, LeafResNet) and self.model.native and sparse_policy
        if isinstance(self.model, LeafResNet) and not self.sparse:
            self.model.features = False
        if self.sparse:
            po = self.model.f.policy_out
            self.policy_w = po.weight.detach().float().contiguous()
            self.policy_b = po.bias.detach().float().contiguous()
            # the sparse head leaves out W float4s whose four features are zero (exact: 0 * w adds
            # +-0 for finite w); a non-finite weight there would have made the reference's logit
            # NaN, so a diverged policy layer is refused here instead of silently giving finite priors
            if not (bool(torch.isfinite(self.policy_w).all()) and bool(torch.isfinite(self.policy_b).all())):
                from ..engine import EngineError

                raise EngineError("the policy layer holds non-finite weights (diverged net): refusing the sparse "
                                  "policy head, whose zero-feature skip would hide the NaN logits")
        # the HIP ResNet reads the planar observation k_select writes (the search can write straight
        # into static_obs: no copy); the MIOpen paths want channels_last
        self.planar = isinstance(self.model, LeafResNet) and self.model.native
        self.static_obs = torch.zeros((G,) + eng.obs_shape, dtype=torch.float32, device=dev)
        if not self.planar:
            self.static_obs = self.static_obs.contiguous(memory_format=torch.channels_last)
        self.graph = None
        if use_graph:
            self._capture()

    def _forward(self, obs):
        obs = obs.contiguous() if self.planar else obs.contiguous(memory_format=torch.channels_last)
        with torch.inference_mode():
            if self.dtype != torch.float32:
                with torch.autocast("cuda", dtype=self.dtype):
                    lp, v = self.model(obs)
            else:
                lp, v = self.model(obs)
            return lp.float().contiguous(), v.float().contiguous()

    def _capture(self):
        s = torch.cuda.Stream(self.eng.device)
        s.wait_stream(torch.cuda.current_stream(self.eng.device))
        with torch.cuda.stream(s):
            for _ in range(2):
                self._forward(self.static_obs)
        torch.cuda.current_stream(self.eng.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.static_lp, self.static_v = self._forward(self.static_obs)
        self.graph = g

    def __call__(self, obs: torch.Tensor):
        if self.model is None:
            return self.const_logp, self.const_v
        if self.graph is not None:
            if obs.data_ptr() != self.static_obs.data_ptr():
                self.static_obs.copy_(obs)
            self.graph.replay()
            return self.static_lp, self.static_v
        return self._forward(obs)


class SelfPlay:
    def __init__(self, eng: Engine, model: torch.nn.Module | None, games: int, num_sims: int = 100,
                 cpuct: float = 1.0, temperature: float = 1.0, dirichlet_alpha: float = 1.0,
                 dirichlet_weight: float = 0.25, node_cap: int | None = None, child_cap: int | None = None,
                 cap: int = 2048, seed: int = 0, nn_dtype: torch.dtype = torch.float32, use_graph: bool = True,
                 continuous: bool = False, sim_graph_sims: int | None = None, record_plies: int | None = None):
        self.eng = eng
        self.G = games
        self.num_sims = num_sims
        # BK_SIM_GRAPH_SIMS is read here (not at import) like the other BK_* knobs
        self.sim_graph_sims = (sim_graph_sims or int(os.environ.get("BK_SIM_GRAPH_SIMS", "0"))
                               or self.graph_sims_for(num_sims))
        self.cpuct = cpuct
        self.temperature = temperature
        self.alpha = dirichlet_alpha
        self.weight = dirichlet_weight
        self.cap = cap
        self.continuous = continuous
        # records kept on the device (~3 MB per ply at 256 games): all of them in finite mode (a run
        # ends with every game), the last `record_plies` plies in continuous mode, where games never
        # stop (examples(drain=True) / window_packed() take them out; older plies are dropped)
        self.record_plies = record_plies if record_plies is not None else (
            4 * self.max_game_plies(eng) if continuous else 0)
        if node_cap is None:
            node_cap = self.node_cap_for(eng, num_sims)
        self.mcts = BatchedMCTS(eng, games, node_cap=node_cap, child_cap=child_cap)
        self.evaluator = LeafEvaluator(model, eng, games, nn_dtype, use_graph)
        self._use_graph = use_graph
        if getattr(self.evaluator, "planar", False) and self.evaluator.graph is not None:
            self.mcts.obs = self.evaluator.static_obs  # k_select writes the net's input buffer directly
        dev = eng.device
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed)
        self._seed = int(seed) & 0xFFFFFFFFFFFFFFFF  # bk_ply_policy's counter-based draws
        self._init_state = eng.init_states(1)  # bk_ply_finish restarts finished games from it
        self.roots = eng.init_states(games)
        self.active = torch.ones(games, dtype=torch.int32, device=dev)
        self.first_ply = torch.ones(games, dtype=torch.bool, device=dev)
        self.game_id = torch.arange(games, dtype=torch.int64, device=dev)
        self._stats = SelfPlayStats()
        # device-side bookkeeping: no host sync anywhere in play_ply
        self._next_gid = torch.full((), games, dtype=torch.int64, device=dev)
        self._sims_dev = torch.zeros((), dtype=torch.int64, device=dev)
        self._fin_dev = torch.zeros((), dtype=torch.int64, device=dev)
        self._zcap = 0
        self.z_table = torch.zeros((0, eng.P), dtype=torch.float32, device=dev)  # z of game id g
        self.z_known = torch.zeros(0, dtype=torch.bool, device=dev)
        self._ensure_zcap()
        self._records: list[tuple[torch.Tensor, ...]] = []  # per-ply records (z resolved lazily)
        self.timers = None
        self._graph = None  # the captured simulations (_sim_graph)
        self._window: list[tuple[torch.Tensor, ...]] = []  # records since mark_window()
        self._dropped_plies = 0  # continuous mode: plies that fell out of the record ring
        # an active game whose root had more children than `cap` (k_root returns counts = -K):
        # latched on the device, raised by check() at the next host sync
        self._cap_overflow = torch.zeros((), dtype=torch.int32, device=dev)
        self.last_action = torch.full((games,), -1, dtype=torch.int32, device=dev)

    @staticmethod
    def max_game_plies(eng: Engine) -> int:
        """Upper bound on the plies of one game: every ply places one of a player's pieces."""
        return eng.num_pieces * eng.P

    @classmethod
    def node_cap_for(cls, eng: Engine, num_sims: int) -> int:
        """Nodes one tree can need over a whole game. A tree lives for one game (trainer.py:95)
        and a simulation adds at most one node, so num_sims x plies + 1 (the first root) bounds it."""
        return int(num_sims) * cls.max_game_plies(eng) + 1

    def check(self) -> dict:
        """Raise EngineError if any tree ran out of nodes/children (the search would otherwise
        keep re-selecting an unexpanded leaf and distort pi) or a root had more than `cap`
        children (the ply would be dropped). Synchronises the stream; returns the MCTS counters."""
        from ..engine import EngineError

        c = self.mcts.check()
        if int(self._cap_overflow.item()):
            raise EngineError(f"a root had more than cap={self.cap} children: raise SelfPlay(cap=...)")
        return c

    @property
    def stats(self) -> SelfPlayStats:
        """Host copy of the counters (synchronises the stream once)."""
        self._stats.sims = int(self._sims_dev.item())
        self._stats.games_finished = int(self._fin_dev.item())
        return self._stats

    def _ensure_zcap(self):
        """z_table rows for every game id that can exist after the next ply (ids < G*(plies+2))."""
        need = self.G * (self._stats.plies + 2)
        if need > self._zcap:
            cap = max(need, 2 * self._zcap)
            dev = self.eng.device
            self.z_table = torch.cat([self.z_table, torch.zeros((cap - self._zcap, self.eng.P), dtype=torch.float32,
                                                                device=dev)])
            self.z_known = torch.cat([self.z_known, torch.zeros(cap - self._zcap, dtype=torch.bool, device=dev)])
            self._zcap = cap

    # ------------------------------------------------------------------ one simulation
    def _evaluate(self, obs):
        """Net on the leaf batch, leaving the priors' inputs in the search state: dense logits,
        or (HIP ResNet) policy features + the sparse policy head over the legal ids."""
        out, v = self.evaluator(obs)
        if self.evaluator.sparse:
            self.mcts.leaf_logits(out, self.evaluator.policy_w, self.evaluator.policy_b)
            return None, v, 2
        return out, v, 0

    def simulate(self):
        """One simulation in every active tree (= num active trees simulate() calls)."""
        if self.timers is not None:
            return self._simulate_timed()
        _, obs, _ = self.mcts.select(self.roots, self.active, self.cpuct)
        logp, v, mode = self._evaluate(obs)
        self.mcts.expand_backup(logp, v, prior_mode=mode)

    # simulations per captured graph (the constructor's sim_graph_sims or BK_SIM_GRAPH_SIMS; a ply's
    # n simulations = n // k replays + eager rest). Default: the whole ply in one graph (one k_select
    # per ply instead of one per replay: +0.5% sims/s at 100 sims vs k = 10), see graph_sims_for

    @staticmethod
    def graph_sims_for(num_sims: int) -> int:
        """num_sims itself up to 100, else its largest divisor <= 100 (10 if that is below 10)."""
        if num_sims <= 100:
            return max(num_sims, 1)
        d = max(k for k in range(1, 101) if num_sims % k == 0)
        return d if d >= 10 else 10

    def _simulations(self, n: int):
        """n simulations of every active tree: replays of a graph of sim_graph_sims captured
        simulations (no per-launch host work) and eager ones."""
        k = self.sim_graph_sims
        if n >= k and self._graph_usable():
            g = self._sim_graph()
            self._g_roots.copy_(self.roots)
            self._g_active.copy_(self.active)
            for _ in range(n // k):
                g.replay()
            n -= (n // k) * k
        for _ in range(n):
            self.simulate()

    def _graph_usable(self) -> bool:
        ev = self.evaluator
        return (self.timers is None and self._use_graph and (ev.model is None or ev.graph is not None)
                and os.environ.get("BK_SIM_GRAPH", "1") != "0")

    def _sim_body(self):
        """One simulation on the captured buffers (_g_roots, _g_active)."""
        _, obs, _ = self.mcts.select(self._g_roots, self._g_active, self.cpuct)
        ev = self.evaluator
        if ev.model is None:
            self.mcts.expand_backup(ev.const_logp, ev.const_v, prior_mode=0)
            return
        out, v = ev._forward(obs)
        if ev.sparse:
            self.mcts.leaf_logits(out, ev.policy_w, ev.policy_b)
            self.mcts.expand_backup(None, v, prior_mode=2)
        else:
            self.mcts.expand_backup(out, v, prior_mode=0)

    def _sim_graph(self):
        """sim_graph_sims simulations captured once. With the sparse policy head the search half of
        a simulation and the next one's descent are one launch (bk_mcts_leaf_step): select, then
        sim_graph_sims x {net, leaf_step (+ select, except the last)} — the trees of the per-stage
        launches, bitwise (tests/test_sims_gpu.py)."""
        if self._graph is None:
            self._g_roots = self.roots.clone()
            self._g_active = self.active.clone()
            ev = self.evaluator
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                if ev.model is not None and ev.sparse:
                    _, obs, _ = self.mcts.select(self._g_roots, self._g_active, self.cpuct)
                    for i in range(self.sim_graph_sims):
                        out, v = ev._forward(obs)
                        last = i == self.sim_graph_sims - 1
                        self.mcts.leaf_step(out, ev.policy_w, ev.policy_b, v, None if last else self._g_roots,
                                            self._g_active, self.cpuct, want_mask=False)
                else:
                    for _ in range(self.sim_graph_sims):
                        self._sim_body()
            self._graph = g
        return self._graph

    def enable_timers(self, on: bool = True):
        """HIP events around each stage on the launch stream (bench.py roofline inputs)."""
        self.timers = {"select": [], "net": [], "expand": []} if on else None

    def _simulate_timed(self):
        st = torch.cuda.current_stream(self.eng.device)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record(st)
        _, obs, _ = self.mcts.select(self.roots, self.active, self.cpuct)
        ev[1].record(st)
        logp, v, mode = self._evaluate(obs)
        ev[2].record(st)
        self.mcts.expand_backup(logp, v, prior_mode=mode)
        ev[3].record(st)
        self.timers["select"].append((ev[0], ev[1]))
        self.timers["net"].append((ev[1], ev[2]))
        self.timers["expand"].append((ev[2], ev[3]))

    def timer_ms(self) -> dict:
        torch.cuda.synchronize(self.eng.device)
        return {k: (sum(a.elapsed_time(b) for a, b in v) / len(v) if v else 0.0) for k, v in self.timers.items()}

    # ------------------------------------------------------------------ one ply
    def play_ply(self, record: bool = True):
        self._simulations(self.num_sims)
        if os.environ.get("BK_PLY_FUSED", "1") != "0":
            return self._ply_tail_fused(record)
        ids, pi, counts = self.mcts.root_policy(self.roots, self.active, self.temperature, self.cap)
        G, cap = self.G, self.cap
        col = torch.arange(cap, device=self.eng.device).unsqueeze(0)
        valid = col < counts.clamp(min=0).unsqueeze(1)
        pi = torch.where(valid, pi, torch.zeros_like(pi))
        self._cap_overflow |= ((counts < 0) & self.active.bool()).any().to(torch.int32)
        # root-only Dirichlet noise on each game's first ply (trainer.py:110-116); drawn every
        # ply and applied where first_ply, so no host round trip decides it
        gam = torch._standard_gamma(torch.full((G, cap), self.alpha, dtype=torch.float64,
                                               device=self.eng.device), generator=self.gen)
        gam = torch.where(valid, gam, torch.zeros_like(gam))
        noise = gam / gam.sum(dim=1, keepdim=True).clamp(min=1e-300)
        mixed = pi * (1 - self.weight) + noise * self.weight
        pi = torch.where(self.first_ply.unsqueeze(1), mixed, pi)
        pi32 = pi.to(torch.float32)
        act_mask = self.active.bool() & (counts > 0)
        probs = torch.where(act_mask.unsqueeze(1), pi32, (col == 0).to(torch.float32))
        idx = torch.multinomial(probs, 1, generator=self.gen).view(-1)
        action = ids.gather(1, idx.view(-1, 1)).view(-1)
        action = torch.where(act_mask, action, torch.full_like(action, -1)).to(torch.int32).contiguous()
        if record:
            player = Engine.to_move(self.roots).clone()
            rec = (self.roots.clone(), ids.to(torch.int16), pi32, counts.clone(), player, self.game_id.clone(),
                   act_mask.clone())
            self._records.append(rec)
            self._window.append(rec)
            if self.record_plies and len(self._records) > self.record_plies:
                self._dropped_plies += len(self._records) - self.record_plies
                del self._records[:-self.record_plies]
                del self._window[:-self.record_plies]
        self.last_action = action
        self.roots, _, status = self.eng.next_state(self.roots, action)
        self.first_ply &= ~act_mask
        self._stats.plies += 1
        self._sims_dev += int(self.num_sims) * act_mask.sum()
        ended, scores = self.eng.game_ended(self.roots)
        done = ended.bool() & self.active.bool()
        self._finish(done, scores)
        return status

    def _ply_tail_fused(self, record: bool):
        """The ply's tail (the tensor code of play_ply/_finish below, which BK_PLY_FUSED=0 keeps)
        in six engine launches: k_root, bk_ply_policy (noise on first plies, float32 pi, the
        sampled action, the record fields), k_next_state, k_game_ended, bk_ply_finish (z, counters,
        restarts, next game ids), then the tree resets (k_reset). The noise and the action come from
        counter-based random numbers of (seed, ply, game) instead of self.gen: the same law
        (tests/test_selfplay_gpu.py::test_play_ply_sampling_statistics), ~0.45 ms less per ply."""
        eng, G, cap, dev = self.eng, self.G, self.cap, self.eng.device
        lib = self.mcts.lib
        ids, pi, counts = self.mcts.root_policy(self.roots, self.active, self.temperature, cap, zero=False)
        action = torch.empty(G, dtype=torch.int32, device=dev)
        ids16 = torch.empty((G, cap), dtype=torch.int16, device=dev)
        pi32 = torch.empty((G, cap), dtype=torch.float32, device=dev)
        act = torch.empty(G, dtype=torch.bool, device=dev)
        player = torch.empty(G, dtype=torch.int32, device=dev)
        st = self.mcts._s()
        _check(lib.bk_ply_policy(_ptr(ids), _ptr(pi), _ptr(counts), _ptr(self.active), _ptr(self.first_ply), G, cap,
                                 float(self.weight), float(self.alpha), self._seed, self._stats.plies,
                                 _ptr(self.roots), _ptr(action), _ptr(ids16), _ptr(pi32), _ptr(act), _ptr(player),
                                 st))
        if record:
            # nothing here is written in place later (the next roots and game ids are new tensors)
            rec = (self.roots, ids16, pi32, counts, player, self.game_id, act)
            self._records.append(rec)
            self._window.append(rec)
            if self.record_plies and len(self._records) > self.record_plies:
                self._dropped_plies += len(self._records) - self.record_plies
                del self._records[:-self.record_plies]
                del self._window[:-self.record_plies]
        self.last_action = action  # the ply's sampled action per game (-1: none), for checkers
        nxt, _, status = eng.next_state(self.roots, action)
        ended, scores = eng.game_ended(nxt)
        self._stats.plies += 1
        self._ensure_zcap()
        roots_out = eng.empty_states(G)
        gid_out = torch.empty_like(self.game_id)
        flags = torch.empty(G, dtype=torch.int32, device=dev)
        _check(lib.bk_ply_finish(G, eng.P, _ptr(ended), _ptr(scores), _ptr(counts), _ptr(act), _ptr(self.game_id),
                                 _ptr(nxt), _ptr(self._init_state), int(self.continuous), int(self.num_sims),
                                 _ptr(self.active), _ptr(self.first_ply), _ptr(flags), _ptr(gid_out), _ptr(roots_out),
                                 _ptr(self.z_table), _ptr(self.z_known), self._zcap, _ptr(self._next_gid),
                                 _ptr(self._fin_dev), _ptr(self._sims_dev), _ptr(self._cap_overflow), st))
        self.mcts.reset(flags)  # a new MCTS per episode (trainer.py:95); no-op for unflagged trees
        self.roots, self.game_id = roots_out, gid_out
        return status

    def _finish(self, done: torch.Tensor, scores: torch.Tensor):
        """Record z of the games that ended this ply (z_table[game id]); reset their trees and,
        in continuous mode, start new games in their slots. Masked device ops only."""
        self._ensure_zcap()
        gid = self.game_id
        self.z_table[gid] = torch.where(done.unsqueeze(1), scores.float(), self.z_table[gid])
        self.z_known[gid] = self.z_known[gid] | done
        self._fin_dev += done.sum()
        flags = done.to(torch.int32)
        self.mcts.reset(flags)  # a new MCTS per episode (trainer.py:95); no-op for unflagged trees
        if self.continuous:
            fresh = self.eng.init_states(self.G)
            self.roots = torch.where(done.unsqueeze(1), fresh, self.roots)
            self.first_ply |= done
            d = done.to(torch.int64)
            self.game_id = torch.where(done, self._next_gid + torch.cumsum(d, 0) - 1, self.game_id)
            self._next_gid += d.sum()
        else:
            self.active = self.active & ~flags

    def mark_window(self):
        self._window = []

    def window_packed(self):
        """Packed replay rows (blokus_rl_amd.replay layout) of every ply recorded since
        mark_window(). z is the final one-hot score of the row's game (trainer.py:131-135) for
        games that have ended, zero for games still running (their outcome is not known yet)."""
        from ..replay import pack

        if not self._window:
            return None, 0
        m = torch.cat([r[6] for r in self._window])
        states = torch.cat([r[0] for r in self._window])[m]
        k = torch.cat([r[3] for r in self._window])[m]
        kmax = int(k.max().item())
        cap = max(64, (kmax + 63) // 64 * 64)
        ids = torch.cat([r[1][:, :cap] for r in self._window])[m]
        pi = torch.cat([r[2][:, :cap] for r in self._window])[m]
        player = torch.cat([r[4] for r in self._window])[m]
        gids = torch.cat([r[5] for r in self._window])[m]
        z = torch.where(self.z_known[gids].unsqueeze(1), self.z_table[gids], torch.zeros_like(self.z_table[gids]))
        return pack(states, ids, pi, k, z, player, cap=cap)

    def run(self, plies: int, check_every: int = 8):
        """Up to `plies` plies; in finite mode stops once every game is over (checked every
        `check_every` plies — extra plies of finished games are no-ops)."""
        t0 = time.perf_counter()
        for i in range(plies):
            if not self.continuous and i % check_every == 0 and not bool(self.active.any()):
                break
            self.play_ply()
        torch.cuda.synchronize(self.eng.device)
        self._stats.seconds += time.perf_counter() - t0
        self.check()
        return self.stats

    def examples(self, drain: bool = False) -> Examples | None:
        """Every recorded example of a finished game (z known), in ply order. drain=True drops
        them from the record list (records of running games stay)."""
        if not self._records:
            return None
        m = torch.cat([r[6] for r in self._records])
        gids = torch.cat([r[5] for r in self._records])
        sel = m & self.z_known[gids]
        if not bool(sel.any()):
            return None
        ex = Examples(torch.cat([r[0] for r in self._records])[sel], torch.cat([r[1] for r in self._records])[sel],
                      torch.cat([r[2] for r in self._records])[sel], torch.cat([r[3] for r in self._records])[sel],
                      self.z_table[gids[sel]])
        if drain:
            keep = []
            for r in self._records:
                mr = r[6] & ~self.z_known[r[5]]
                if bool(mr.any()):
                    keep.append(r[:6] + (mr,))
            self._records = keep
        return ex
