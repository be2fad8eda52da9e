"""Config-5 vector env on the GPU against its CPU restatement (oracle/vecenv_oracle.py):
states, observations, masks, rewards, dones and the per-env random streams bit-exact over many
steps and episodes — agent actions given (random legal ids chosen on the host, plus out-of-range
and illegal ids, which end the episode as a loss) and drawn in-kernel; a partial last workgroup
(E not a multiple of the envs per workgroup), both lane widths of k_vec_step7 and the
one-wave-per-env kernel; and the benchmark size (8192 envs, and 8190) driven through a captured
HIP graph of back-to-back step_raw launches as bench.py replays it (ppo/trainer.py:128-175)."""
import numpy as np
import pytest
import torch

from oracle.vecenv_oracle import VecEnvOracle

pytestmark = pytest.mark.gpu


def _obs_of(states: np.ndarray, N: int = 7) -> np.ndarray:
    """VecEnvOracle.obs for every env at once: 1 where colour 0 sits, 2 for colour 1, else 0."""
    occ = np.ascontiguousarray(states[:, :320]).view(np.uint32).reshape(-1, 4, 20)[:, :2, :N]
    bits = (occ[..., None] >> np.arange(N, dtype=np.uint32)) & 1
    return np.where(bits[:, 0] == 1, 1, np.where(bits[:, 1] == 1, 2, 0)).astype(np.uint8)


def _assert_env_equal(env, ref, tag):
    E = env.num_envs
    st = env.states.cpu().numpy()
    want = np.stack(ref.states)
    bad = np.nonzero((st != want).any(axis=1))[0]
    assert bad.size == 0, (tag, "state", bad[:8])
    assert (env.obs.cpu().numpy() == _obs_of(want)).all(), (tag, "obs")
    m = env.mask_words.cpu().numpy().view(np.uint64)
    for e in range(E):
        assert (m[e] == ref.mask(e)).all(), (tag, "mask", e)
    assert (env.rng.cpu().numpy().view(np.uint64) == np.array(ref.rng, dtype=np.uint64)).all(), (tag, "rng")


@pytest.mark.parametrize("max_cells,E,kernel", [(4, 32, "16"), (5, 32, "16"), (4, 37, "16"), (5, 37, "8"),
                                                (4, 32, "8"), (4, 37, "wave")])
def test_vector_env_matches_oracle(max_cells, E, kernel, monkeypatch):
    """E = 37: the last workgroup holds 5 (16 lanes) or 5 of 32 (8 lanes) envs — spare lane groups
    and the byte-wise obs copy. kernel: lanes per env of k_vec_step7 (BK_VEC_LANES), or the
    one-wave-per-env k_vec_step (BK_VEC_WAVE=1). Every 7th step gives each env an out-of-range id
    (>= A) or an id that is in range but not legal: reward -1, done, auto-reset, rng untouched."""
    from blokus_rl_amd.vector_env import BlokusVectorEnv

    if kernel == "wave":
        monkeypatch.setenv("BK_VEC_WAVE", "1")
    else:
        monkeypatch.setenv("BK_VEC_LANES", kernel)
    env = BlokusVectorEnv(E, 7, max_cells)
    ref = VecEnvOracle(E, 7, max_cells)
    A = env.eng.A
    env.reset(seed=5)
    ref.reset(seed=5)
    rng = np.random.default_rng(0)
    episodes = losses = 0
    for t in range(60):
        _assert_env_equal(env, ref, t)
        m = env.mask_words.cpu().numpy().view(np.uint64)
        legal = [np.nonzero(np.unpackbits(m[e].view(np.uint8), bitorder="little")[:A])[0] for e in range(E)]
        if t % 7 == 6:
            acts = np.empty(E, dtype=np.int32)
            for e in range(E):
                if e % 3 == 0:
                    acts[e] = A + int(rng.integers(0, 4096))  # out of range
                else:
                    illegal = np.setdiff1d(np.arange(A), legal[e])
                    acts[e] = int(rng.choice(illegal)) if e % 3 == 1 else int(rng.choice(legal[e]))
        elif t % 3 == 2:
            acts = np.full(E, -1, dtype=np.int32)  # in-kernel random agent
        else:
            acts = np.array([int(rng.choice(legal[e])) for e in range(E)], dtype=np.int32)
        _, rew, term, _, _ = env.step(torch.from_numpy(acts))
        rew, term = rew.cpu().numpy(), term.cpu().numpy()
        for e in range(E):
            r, d = ref.step(e, int(acts[e]))
            assert rew[e] == r and bool(term[e]) == bool(d), (t, e)
            episodes += d
            if t % 7 == 6 and e % 3 != 2:
                assert r == -1.0 and d == 1, (t, e)
                losses += 1
    _assert_env_equal(env, ref, "end")
    assert episodes > E and losses > 0  # several episodes per env ended and auto-reset


def _graph_rollout(E, steps_per_graph, replays, seed):
    """The bench's config-5 loop: a HIP graph of `steps_per_graph` in-kernel-agent step_raw
    launches, replayed; the env checked against the oracle after every replay."""
    from blokus_rl_amd.vector_env import BlokusVectorEnv

    env = BlokusVectorEnv(E, 7, 4)
    ref = VecEnvOracle(E, 7, 4)
    env.reset(seed=seed)
    ref.reset(seed=seed)
    g = torch.cuda.CUDAGraph()
    # capture on a side stream, as torch.cuda.graph does; nothing runs until the first replay
    with torch.cuda.graph(g):
        for _ in range(steps_per_graph):
            env.step_raw(None)
    torch.cuda.synchronize()
    _assert_env_equal(env, ref, "reset")
    ended = 0
    for r in range(replays):
        g.replay()
        torch.cuda.synchronize()
        for _ in range(steps_per_graph):
            last = [ref.step(e, -1) for e in range(E)]
            ended += sum(d for _, d in last)
        _assert_env_equal(env, ref, r)
        rew, done = env.reward.cpu().numpy(), env.done.cpu().numpy()
        assert rew.tolist() == [x for x, _ in last] and done.tolist() == [d for _, d in last], r
    return ended


def test_vector_env_benchmark_size_graph_matches_oracle():
    """8192 envs (config 5), the bench's 25-step graph replayed once: 25 back-to-back launches,
    thousands of episodes ending and auto-resetting inside the graph."""
    assert _graph_rollout(8192, 25, 1, seed=3) > 8192


def test_vector_env_ragged_size_graph_matches_oracle():
    """8190 envs: not a multiple of the 16 envs of a k_vec_step7 workgroup (the last one holds
    14); a 5-step graph replayed 4 times, checked after each replay."""
    assert _graph_rollout(8190, 5, 4, seed=9) > 8190


def test_step_raw_rejects_bad_action_tensors():
    from blokus_rl_amd.vector_env import BlokusVectorEnv

    env = BlokusVectorEnv(8, 7, 4)
    env.reset(seed=0)
    for bad in (torch.zeros(8, dtype=torch.int32), torch.zeros(8, dtype=torch.int64, device=env.device),
                torch.zeros(7, dtype=torch.int32, device=env.device),
                torch.zeros(16, dtype=torch.int32, device=env.device)[::2]):
        with pytest.raises(ValueError):
            env.step_raw(bad)
    env.step_raw(torch.full((8,), -1, dtype=torch.int32, device=env.device))


def test_ai_possible_indexes_and_masked_logits():
    from blokus_rl_amd.vector_env import BlokusVectorEnv

    env = BlokusVectorEnv(4, 7, 4)
    env.reset(seed=1)
    assert env.single_action_space_n == 919
    lists = env.get_attr("ai_possible_indexes")
    mask = env.valid_mask()
    for e in range(4):
        assert lists[e] == torch.nonzero(mask[e]).view(-1).tolist()
    logits = torch.randn(4, 919, device=env.device)
    ml = env.masked_logits(logits)
    assert bool((ml[~mask] == -1e9).all()) and torch.equal(ml[mask], logits[mask])


# ------------------------------------------------------------------ the masked-policy draw
def _policy_logits(E, A, t, rng):
    """Seeded logits with the edge cases of FilterLegalMoves (ppo/agent.py:27-42): exact zeros
    (+0 and -0) on ~1/8 of the ids, an all-zero row every 5th env (under zero_masked: no
    candidate -> the reference's all -1e9 row, uniform over every id), and a large spread."""
    x = (rng.standard_normal((E, A)) * (0.5 + 4.0 * (t % 3))).astype(np.float32)
    x[rng.random((E, A)) < 0.125] = 0.0
    x[rng.random((E, A)) < 0.02] = -0.0
    x[::5] = 0.0
    return x


@pytest.mark.parametrize("max_cells,E", [(4, 37), (5, 32), (4, 8)])
def test_policy_sample_matches_oracle(max_cells, E):
    """bk_vec_policy vs oracle.vecenv_oracle.policy_sample every step of a rollout: actions,
    log-probs and the env's random stream bitwise; zero_masked on and off; then the env steps
    with the drawn actions (states, masks, rewards bitwise, as test_vector_env_matches_oracle)."""
    from blokus_rl_amd.vector_env import BlokusVectorEnv

    env = BlokusVectorEnv(E, 7, max_cells)
    ref = VecEnvOracle(E, 7, max_cells)
    A = env.eng.A
    env.reset(seed=2)
    ref.reset(seed=2)
    rng = np.random.default_rng(11)
    uniform_rows = 0
    for t in range(40):
        zm = t % 4 != 3
        x = _policy_logits(E, A, t, rng)
        a, lp = env.sample_policy(torch.from_numpy(x).to(env.device), zero_masked=zm)
        ra, rlp = ref.sample_policy(x, zero_masked=zm)
        assert (a.cpu().numpy() == ra).all(), (t, np.nonzero(a.cpu().numpy() != ra)[0][:8])
        assert (lp.cpu().numpy().view(np.uint32) == rlp.view(np.uint32)).all(), t
        assert (env.rng.cpu().numpy().view(np.uint64) == np.array(ref.rng, dtype=np.uint64)).all(), t
        if zm:
            uniform_rows += int((rlp[::5] == 0.0).sum())
        env.step_raw(a)
        for e in range(E):
            r, d = ref.step(e, int(ra[e]))
            assert float(env.reward[e]) == r and int(env.done[e]) == d, (t, e)
        _assert_env_equal(env, ref, t)
    assert uniform_rows > 0  # the all -1e9 rows were drawn (log-prob 0, as torch gives them)


def _policy_graph_rollout(E, steps_per_graph, replays, seed):
    from blokus_rl_amd.vector_env import BlokusVectorEnv

    env = BlokusVectorEnv(E, 7, 4)
    ref = VecEnvOracle(E, 7, 4)
    env.reset(seed=seed)
    ref.reset(seed=seed)
    x = np.random.default_rng(seed).standard_normal((E, env.eng.A)).astype(np.float32) * 3.0
    logits = torch.from_numpy(x).to(env.device)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(steps_per_graph):
            env.step_policy(logits)
    torch.cuda.synchronize()
    ended = 0
    for r in range(replays):
        g.replay()
        torch.cuda.synchronize()
        for _ in range(steps_per_graph):
            ra, rlp = ref.sample_policy(x)
            last = [ref.step(e, int(ra[e])) for e in range(E)]
            ended += sum(d for _, d in last)
        assert (env.actions.cpu().numpy() == ra).all(), r
        assert (env.logp.cpu().numpy().view(np.uint32) == rlp.view(np.uint32)).all(), r
        _assert_env_equal(env, ref, r)
        assert env.reward.cpu().numpy().tolist() == [x_ for x_, _ in last], r
    return ended


def test_policy_rollout_benchmark_size_graph_matches_oracle():
    """8192 envs (config 5) through the bench's path: a HIP graph of 5 x (bk_vec_policy +
    k_vec_step7) replayed twice, checked against the oracle after each replay."""
    assert _policy_graph_rollout(8192, 5, 2, seed=4) > 0


def test_policy_rollout_ragged_size_graph_matches_oracle():
    assert _policy_graph_rollout(8190, 3, 2, seed=6) > 0


def test_policy_sample_law_and_logprob_vs_torch():
    """The draw's law and log-probs against the reference's own ops: 8192 envs on the empty board
    (the same legal set), one logits row: the action histogram vs softmax over the legal ids
    (chi-square), log-probs vs Categorical(logits=FilterLegalMoves(x)).log_prob (the reference's
    get_action_and_value, ppo/agent.py:148-156) at rtol 2e-6; with zero_masked, legal ids whose
    logit is exactly 0 are never drawn, without it they are."""
    from scipy import stats

    from blokus_rl_amd.ppo.agent import FilterLegalMoves
    from blokus_rl_amd.vector_env import BlokusVectorEnv

    E = 8192
    env = BlokusVectorEnv(E, 7, 4)
    env.reset(seed=0)
    A = env.eng.A
    g = torch.Generator().manual_seed(0)
    row = torch.randn(A, generator=g) * 1.5
    legal = env.valid_mask()[0].cpu()
    lid = torch.nonzero(legal).view(-1)
    row[lid[::4]] = 0.0  # every 4th legal id at exactly 0
    x = row.repeat(E, 1).contiguous().to(env.device)
    filt = FilterLegalMoves()(x, env.mask_words)
    dist = torch.distributions.Categorical(logits=filt)
    counts = torch.zeros(A, dtype=torch.int64)
    for _ in range(8):  # 8 draws per env from the same state (the stream advances)
        a, lp = env.sample_policy(x, zero_masked=True)
        want = dist.log_prob(a.long())
        torch.testing.assert_close(lp, want, rtol=2e-6, atol=2e-6)
        counts += torch.bincount(a.long().cpu(), minlength=A)
    probs = dist.probs[0].double().cpu()
    assert int(counts[probs == 0].sum()) == 0  # illegal ids and the zero-logit legal ids
    keep = probs > 0
    exp = probs[keep] * counts.sum()
    big = exp >= 5
    chi = float((((counts[keep][big] - exp[big]) ** 2) / exp[big]).sum())
    dof = int(big.sum()) - 1
    assert stats.chi2.sf(chi, dof) > 1e-4, (chi, dof)
    a, _ = env.sample_policy(x, zero_masked=False)
    zero_ids = set(lid[::4].tolist())
    hits = sum(1 for v in a.cpu().tolist() if v in zero_ids)
    assert hits > 0


@pytest.mark.parametrize("max_cells,E", [(4, 37), (5, 21)])
def test_fused_policy_step_matches_two_launches(max_cells, E):
    """bk_vec_step_policy (the draw inside k_vec_step7) against bk_vec_policy + bk_vec_step on a
    twin env: actions, log-probs, states, observations, masks, rewards, dones and random streams
    bit for bit every step, zero_masked on and off, with all-zero (no-candidate) rows."""
    from blokus_rl_amd.vector_env import BlokusVectorEnv

    env1, env2 = BlokusVectorEnv(E, 7, max_cells), BlokusVectorEnv(E, 7, max_cells)
    A = env1.eng.A
    env1.reset(seed=7)
    env2.reset(seed=7)
    rng = np.random.default_rng(3)
    for t in range(30):
        zm = t % 5 != 4
        x = torch.from_numpy(_policy_logits(E, A, t, rng)).to(env1.device)
        a1, l1 = env1.step_policy(x, zero_masked=zm)
        a2, l2 = env2.step_policy(x, zero_masked=zm, fused=False)
        assert torch.equal(a1, a2) and torch.equal(l1.view(torch.int32), l2.view(torch.int32)), t
        for n in ("states", "obs", "mask_words", "rng", "reward", "done"):
            assert torch.equal(getattr(env1, n), getattr(env2, n)), (t, n)
