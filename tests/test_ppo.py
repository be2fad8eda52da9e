"""PPO remainder against the reference's own outputs
(tests/golden/ppo_golden.npz from tests/golden/make_ppo_golden.py): GAE, FilterLegalMoves, the
agent's log-prob/entropy/value, and whole _optimize_agent passes; plus the device kernels at the
config-5 scale against the CPU restatement (oracle/ppo_oracle.py)."""
import os
import sys
import types

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from make_net_golden import det_state_dict  # noqa: E402
from make_ppo_golden import AGENT_HP, PPO_DEFAULTS  # noqa: E402

from oracle.ppo_oracle import filter_legal, gae_f32  # noqa: E402

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "ppo_golden.npz"))
N, A = 7, 919


def _hp(**kw):
    from blokus_rl_amd.ppo.trainer import PPOHparams

    d = dict(PPO_DEFAULTS, **AGENT_HP, num_steps=7, num_envs=6, agent_type="cnn", board_size=7, max_piece_cells=4)
    d.update(kw)
    return PPOHparams(**d)


def _agent(device="cpu"):
    from blokus_rl_amd.ppo.agent import CnnAgent

    agent = CnnAgent((N, N), A, types.SimpleNamespace(**AGENT_HP))
    agent.load_state_dict(det_state_dict({k: t.shape for k, t in agent.state_dict().items()}))
    return agent.to(device)


def _batch(device="cpu"):
    return {
        "obs": torch.from_numpy(G["agent_obs"]).to(device),
        "actions": torch.from_numpy(G["agent_actions"].astype(np.float32)).to(device),
        "logprobs": torch.from_numpy(G["update_in_logprobs"]).to(device),
        "advantages": torch.from_numpy(G["update_in_advantages"]).to(device),
        "returns": torch.from_numpy(G["update_in_returns"]).to(device),
        "values": torch.from_numpy(G["update_in_values"]).to(device),
    }


# ---------------------------------------------------------------- CPU: oracle + torch parts
def test_oracle_gae_matches_reference_bit_exact():
    adv, ret = gae_f32(G["gae_r"], G["gae_v"], G["gae_d"], G["gae_nv"], G["gae_nd"], 0.99, 0.95)
    assert np.array_equal(adv, G["gae_adv"])
    assert np.array_equal(ret, G["gae_adv"] + G["gae_v"])


def test_oracle_filter_matches_reference():
    assert np.array_equal(filter_legal(G["filter_x"], G["filter_mask"]), G["filter_out"])


def test_agent_layout_and_unmasked_outputs_match_reference():
    agent = _agent()
    ref_keys = sorted(k[len("update_param_"):] for k in G.files if k.startswith("update_param_"))
    assert sorted(agent.state_dict()) == ref_keys
    for k, t in agent.state_dict().items():
        assert tuple(t.shape) == G[f"update_param_{k}"].shape
    with torch.no_grad():
        _, lp, ent, _ = agent.get_action_and_value(torch.from_numpy(G["agent_obs"]),
                                                   torch.from_numpy(G["agent_actions"]))
    np.testing.assert_allclose(lp.numpy(), G["agent_logprob_unmasked"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ent.numpy(), G["agent_entropy_unmasked"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("case,seed,kl", [("update", 123, 0.01), ("update2", 321, None)])
def test_optimize_agent_matches_reference_cpu(case, seed, kl):
    from blokus_rl_amd.ppo.trainer import optimize_agent

    hp = _hp(target_kl=kl)
    agent = _agent()
    opt = torch.optim.Adam(agent.parameters(), lr=hp.learning_rate, eps=hp.eps)
    batch = _batch()
    if case == "update2":
        batch["logprobs"] = torch.from_numpy(G["agent_logprob_unmasked"])
    np.random.seed(seed)
    log = optimize_agent(agent, opt, batch, hp)
    for k, t in agent.state_dict().items():
        np.testing.assert_allclose(t.numpy(), G[f"{case}_param_{k}"], rtol=1e-4, atol=1e-6, err_msg=k)
    for k in ("loss", "value_loss", "policy_loss", "entropy", "approx_kl", "clipfrac"):
        np.testing.assert_allclose(log[k], G[f"{case}_log_{k}"][0], rtol=1e-4, atol=1e-6, err_msg=k)


def test_mask_words_from_id_lists():
    from blokus_rl_amd.ppo.agent import ids_to_mask_words

    m = G["filter_mask"]
    words = ids_to_mask_words([np.flatnonzero(r) for r in m], A, "cpu").numpy().view(np.uint64)
    bits = ((words[:, :, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).reshape(m.shape[0], -1)[:, :A]
    assert np.array_equal(bits.astype(np.uint8), m)


# ---------------------------------------------------------------- GPU kernels
@pytest.mark.gpu
def test_gae_kernel_matches_reference_and_oracle():
    from blokus_rl_amd.ppo.trainer import compute_gae

    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    adv, ret = compute_gae(t(G["gae_r"]), t(G["gae_v"]), t(G["gae_d"]), t(G["gae_nv"]), t(G["gae_nd"]), 0.99, 0.95)
    assert np.array_equal(adv.cpu().numpy(), G["gae_adv"])
    assert np.array_equal(ret.cpu().numpy(), G["gae_adv"] + G["gae_v"])
    # config-5 scale: 32 steps x 8192 envs
    rng = np.random.default_rng(0)
    T, E = 32, 8192
    r = (rng.integers(-1, 2, (T, E)) * (rng.random((T, E)) < 0.1)).astype(np.float32)
    v = rng.standard_normal((T, E)).astype(np.float32)
    d = (rng.random((T, E)) < 0.1).astype(np.float32)
    nv = rng.standard_normal(E).astype(np.float32)
    nd = (rng.random(E) < 0.1).astype(np.float32)
    adv, ret = compute_gae(t(r), t(v), t(d), t(nv), t(nd), 0.99, 0.95)
    ra, rr = gae_f32(r, v, d, nv, nd, 0.99, 0.95)
    assert np.array_equal(adv.cpu().numpy(), ra) and np.array_equal(ret.cpu().numpy(), rr)


@pytest.mark.gpu
def test_filter_kernel_matches_reference():
    from blokus_rl_amd.ppo.agent import FilterLegalMoves, ids_to_mask_words

    m = G["filter_mask"]
    x = torch.from_numpy(G["filter_x"]).cuda()
    out = FilterLegalMoves()(x, [np.flatnonzero(r) for r in m])
    assert np.array_equal(out.cpu().numpy(), G["filter_out"])
    out2 = FilterLegalMoves()(x, ids_to_mask_words([np.flatnonzero(r) for r in m], A, "cuda"))
    assert torch.equal(out, out2)


@pytest.mark.gpu
def test_agent_masked_outputs_match_reference_gpu():
    agent = _agent("cuda")
    with torch.no_grad():
        _, lp, ent, val = agent.get_action_and_value(torch.from_numpy(G["agent_obs"]).cuda(),
                                                     torch.from_numpy(G["agent_actions"]).cuda(),
                                                     possible_moves=[np.flatnonzero(r) for r in G["agent_mask"]])
    np.testing.assert_allclose(lp.cpu().numpy(), G["agent_logprob"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(ent.cpu().numpy(), G["agent_entropy"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(val.cpu().numpy(), G["agent_value"], rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_optimize_agent_matches_reference_gpu():
    from blokus_rl_amd.ppo.trainer import optimize_agent

    hp = _hp(target_kl=None)
    agent = _agent("cuda")
    opt = torch.optim.Adam(agent.parameters(), lr=hp.learning_rate, eps=hp.eps)
    batch = _batch("cuda")
    batch["logprobs"] = torch.from_numpy(G["agent_logprob_unmasked"]).cuda()
    np.random.seed(321)
    optimize_agent(agent, opt, batch, hp)
    for k, t in agent.state_dict().items():
        np.testing.assert_allclose(t.cpu().numpy(), G[f"update2_param_{k}"], rtol=1e-3, atol=1e-5, err_msg=k)


@pytest.mark.gpu
def test_ppo_trainer_updates_on_device_env(tmp_path):
    from blokus_rl_amd.ppo.trainer import PPOTrainer

    hp = _hp(num_envs=64, num_steps=16, total_timesteps=64 * 16 * 3, agent_type="cnn", save_interval=2,
             checkpoint_dir=tmp_path)
    tr = PPOTrainer(hp)
    logs = tr.train()
    assert len(logs) == 3 and all(np.isfinite(l["loss"]) for l in logs)
    assert tr.global_step == 64 * 16 * 3 and tr.total_episodes > 0
    assert (tmp_path / "checkpoint_2.pt").exists()
    tr2 = PPOTrainer(hp)
    tr2._load_checkpoint(2)
    assert tr2.update == 3


@pytest.mark.gpu
@pytest.mark.parametrize("device_sampling", [True, False])
def test_ppo_rollout_draws(device_sampling):
    """The rollout's draw on the device (bk_vec_policy over the actor's raw logits) or through torch's
    Categorical over FilterLegalMoves: the stored actions are the drawn ones and their log-probs are
    finite and <= 0; a device draw is a legal id unless every legal logit of its row is exactly 0 —
    the reference filter's all -1e9 row (ppo/agent.py:40-41), uniform over every id, which the
    freshly initialised agent produces for a few envs whose last hidden layer is all zero."""
    from blokus_rl_amd.ppo.trainer import PPOTrainer

    hp = _hp(num_envs=64, num_steps=16, total_timesteps=64 * 16, agent_type="cnn", save_interval=10**6)
    tr = PPOTrainer(hp, device_sampling=device_sampling)
    obs, _ = tr.envs.reset(seed=0)
    masks, acts, rows = [], [], []
    orig_step, orig_sample = tr.envs.step, tr.envs.sample_policy

    def rec_step(action):
        masks.append(tr.envs.valid_mask().clone())
        acts.append(action.long().clone())
        return orig_step(action)

    def rec_sample(logits, zero_masked=True):
        rows.append(logits.clone())
        return orig_sample(logits, zero_masked)

    orig_sp = tr.envs.step_policy

    def rec_step_policy(logits, zero_masked=True):
        masks.append(tr.envs.valid_mask().clone())
        rows.append(logits.clone())
        a, lp = orig_sp(logits, zero_masked)
        acts.append(a.long().clone())
        return a, lp

    tr.envs.step, tr.envs.sample_policy, tr.envs.step_policy = rec_step, rec_sample, rec_step_policy
    tr._play_env(obs.float(), torch.zeros(64, device=tr.device))
    assert len(acts) == hp.num_steps
    illegal = 0
    for t, (m, a) in enumerate(zip(masks, acts)):
        assert torch.equal(tr.memory.actions[t].long(), a)
        bad = ~m.gather(1, a.view(-1, 1)).view(-1)
        if device_sampling:
            no_candidate = ~(m & (rows[t] != 0)).any(dim=1)
            assert bool((no_candidate | ~bad).all()), (t, torch.nonzero(bad & ~no_candidate).view(-1).tolist())
        illegal += int(bad.sum())
    lp = tr.memory.logprobs
    assert bool(torch.isfinite(lp).all()) and bool((lp <= 0).all())
    assert device_sampling or illegal <= 64  # torch's draw over the same filter (same quirk)
