"""Golden vectors for the PPO remainder from the reference's own code.

Run here (never on the GPU box): `python tests/golden/make_ppo_golden.py`.
Loads /root/reference/blokus_rl/ppo/{agent,memory,trainer}.py by file path. The modules they
import but the recorded functions never call are stubbed in sys.modules: gymnasium (absent in
this image), torchsummary (absent), torch.utils.tensorboard (absent), blokus_rl.utils (logging /
env factory). Hyper-parameters come in a SimpleNamespace with PPOHparams' field names and
defaults (hparams.py:97-185), so nothing is written to disk. Recorded, on CPU:
  * gae_*    — PPOTrainer._compute_gae (trainer.py:177-211) on a seeded rollout (T=7, E=6);
  * filter_* — FilterLegalMoves (agent.py:27-42) on logits with exact zeros;
  * agent_*  — CnnAgent.get_action_and_value (agent.py:152-160) with given actions, masked;
  * update_* — PPOTrainer._optimize_agent (trainer.py:213-311) from deterministic weights
               (dropout 0), np.random.seed(123) for its minibatch shuffles: final parameters and
               the last minibatch's losses (this batch trips the target_kl early stop);
  * update2_* — the same with target_kl None and ratio ~ 1 (all update_epochs run), seed 321.
Weights come from make_net_golden.det_state_dict (regenerated in the tests). Output:
tests/golden/ppo_golden.npz.
"""
import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

REF = "/root/reference/blokus_rl"

PPO_DEFAULTS = dict(update_epochs=4, learning_rate=2.5e-4, num_minibatches=4, eps=1e-5, anneal_lr=True,
                    gae=True, gamma=0.99, gae_lambda=0.95, clip_coef=0.2, norm_adv=True, clip_vloss=True,
                    ent_coef=0.01, vf_coef=0.5, max_grad_norm=0.5, target_kl=0.01)
AGENT_HP = dict(d_model=8, cnn_layers=2, cnn_kernel_size=3, cnn_stride=1, cnn_padding=1, cnn_dropout=0.0,
                dropout=0.0)
N, A = 7, 919


class FakeEnvs:
    class _Obs:
        shape = (N, N)

    class _Act:
        n = A
        shape = ()

    single_observation_space = _Obs()
    single_action_space = _Act()


def _load(modname, path, package):
    spec = importlib.util.spec_from_file_location(modname, path)
    mod = importlib.util.module_from_spec(spec)
    mod.__package__ = package
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference_ppo():
    sys.modules["gymnasium"] = types.ModuleType("gymnasium")
    ts = types.ModuleType("torchsummary")
    ts.summary = lambda *a, **k: ""
    sys.modules["torchsummary"] = ts
    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = object
    sys.modules["torch.utils.tensorboard"] = tb
    pkg = types.ModuleType("refppo")
    pkg.__path__ = []
    sys.modules["refppo"] = pkg
    utils = types.ModuleType("refppo.utils")
    utils.log_info = utils.log_warning = lambda *a, **k: None
    utils.make_envs = None
    sys.modules["refppo.utils"] = utils
    _load("refppo.hparams", os.path.join(REF, "hparams.py"), "refppo")
    sub = types.ModuleType("refppo.ppo")
    sub.__path__ = []
    sys.modules["refppo.ppo"] = sub
    agent = _load("refppo.ppo.agent", os.path.join(REF, "ppo", "agent.py"), "refppo.ppo")
    memory = _load("refppo.ppo.memory", os.path.join(REF, "ppo", "memory.py"), "refppo.ppo")
    trainer = _load("refppo.ppo.trainer", os.path.join(REF, "ppo", "trainer.py"), "refppo.ppo")
    return agent, memory, trainer


def rollout(T, E, seed):
    rng = np.random.default_rng(seed)
    r = (rng.integers(-1, 2, (T, E)) * (rng.random((T, E)) < 0.3)).astype(np.float32)
    v = rng.standard_normal((T, E)).astype(np.float32)
    d = (rng.random((T, E)) < 0.25).astype(np.float32)
    nv = rng.standard_normal(E).astype(np.float32)
    nd = (rng.random(E) < 0.25).astype(np.float32)
    return r, v, d, nv, nd


def obs_batch(B, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 3, (B, N, N)).astype(np.float32)


def main():
    from make_net_golden import det_state_dict

    torch.set_num_threads(4)
    agent_m, memory_m, trainer_m = load_reference_ppo()
    hp = types.SimpleNamespace(**PPO_DEFAULTS, **AGENT_HP, num_steps=7, num_envs=6)
    hp.batch_size = hp.num_envs * hp.num_steps
    hp.minibatch_size = hp.batch_size // hp.num_minibatches
    out = {}

    # GAE
    tr = trainer_m.PPOTrainer.__new__(trainer_m.PPOTrainer)
    tr.hparams, tr.device = hp, "cpu"
    tr.memory = memory_m.Memory(hp, FakeEnvs(), "cpu")
    r, v, d, nv, nd = rollout(hp.num_steps, hp.num_envs, 5)
    tr.memory.rewards[:] = torch.from_numpy(r)
    tr.memory.values[:] = torch.from_numpy(v)
    tr.memory.dones[:] = torch.from_numpy(d)
    adv = tr._compute_gae(torch.from_numpy(nv).reshape(1, -1), torch.from_numpy(nd))
    out.update(gae_r=r, gae_v=v, gae_d=d, gae_nv=nv, gae_nd=nd, gae_adv=adv.numpy())

    # FilterLegalMoves (exact zeros on a legal and an illegal id)
    rng = np.random.default_rng(9)
    x = rng.standard_normal((3, A)).astype(np.float32)
    x[0, 5] = 0.0
    x[1, 7] = 0.0
    moves = [sorted(rng.choice(A, 40, replace=False).tolist()) + [5] for _ in range(3)]
    moves[1] = [m for m in moves[1] if m != 7]
    f = agent_m.FilterLegalMoves()(torch.from_numpy(x), moves)
    mask = np.zeros((3, A), np.uint8)
    for i, m in enumerate(moves):
        mask[i, m] = 1
    out.update(filter_x=x, filter_mask=mask, filter_out=f.numpy())

    # CnnAgent outputs and one _optimize_agent pass
    agent = agent_m.CnnAgent(FakeEnvs(), hp)
    agent.load_state_dict(det_state_dict({k: t.shape for k, t in agent.state_dict().items()}))
    B = hp.batch_size
    obs = obs_batch(B, 11)
    acts = np.random.default_rng(12).integers(0, A, B)
    amask = np.zeros((B, A), np.uint8)
    rng = np.random.default_rng(13)
    for i in range(B):
        amask[i, rng.choice(A, 30, replace=False)] = 1
        amask[i, acts[i]] = 1
    with torch.no_grad():
        _, lp, ent, val = agent.get_action_and_value(torch.from_numpy(obs), torch.from_numpy(acts),
                                                     possible_moves=[np.flatnonzero(m) for m in amask])
        _, lp_u, ent_u, _ = agent.get_action_and_value(torch.from_numpy(obs), torch.from_numpy(acts))
    out.update(agent_obs=obs, agent_actions=acts, agent_mask=amask, agent_logprob=lp.numpy(),
               agent_entropy=ent.numpy(), agent_value=val.numpy(), agent_logprob_unmasked=lp_u.numpy(),
               agent_entropy_unmasked=ent_u.numpy())
    rb = rollout(hp.num_steps, hp.num_envs, 21)
    batch = {
        "obs": torch.from_numpy(obs),
        "actions": torch.from_numpy(acts.astype(np.float32)),
        "logprobs": lp.clone() + torch.from_numpy(np.random.default_rng(14).normal(0, 0.05, B).astype(np.float32)),
        "advantages": torch.from_numpy(rb[0].reshape(-1) + rb[1].reshape(-1)),
        "returns": torch.from_numpy(rb[1].reshape(-1) * 0.5),
        "values": val.view(-1).clone(),
    }
    tr.agent = agent
    tr.optimizer = torch.optim.Adam(agent.parameters(), lr=hp.learning_rate, eps=hp.eps)
    from collections import defaultdict
    tr.running_vals = defaultdict(list)
    np.random.seed(123)
    tr._optimize_agent(batch)
    for k in ("logprobs", "advantages", "returns", "values"):
        out[f"update_in_{k}"] = batch[k].numpy()
    for k, t in agent.state_dict().items():
        out[f"update_param_{k}"] = t.numpy()
    for k, vals in tr.running_vals.items():
        out[f"update_log_{k.split('/')[-1]}"] = np.asarray(vals, dtype=np.float64)
    # second pass: old log-probs from the unmasked policy (ratio ~ 1), no KL early stop -> all epochs
    agent2 = agent_m.CnnAgent(FakeEnvs(), hp)
    agent2.load_state_dict(det_state_dict({k: t.shape for k, t in agent2.state_dict().items()}))
    hp2 = types.SimpleNamespace(**vars(hp))
    hp2.target_kl = None
    tr.hparams = hp2
    tr.agent = agent2
    tr.optimizer = torch.optim.Adam(agent2.parameters(), lr=hp.learning_rate, eps=hp.eps)
    tr.running_vals = defaultdict(list)
    batch2 = dict(batch)
    batch2["logprobs"] = lp_u.clone()
    np.random.seed(321)
    tr._optimize_agent(batch2)
    for k, t in agent2.state_dict().items():
        out[f"update2_param_{k}"] = t.numpy()
    for k, vals in tr.running_vals.items():
        out[f"update2_log_{k.split('/')[-1]}"] = np.asarray(vals, dtype=np.float64)
    fp = os.path.join(HERE, "ppo_golden.npz")
    np.savez_compressed(fp, **out)
    print(fp, os.path.getsize(fp), "bytes;", len(out), "arrays")
    print({k: out[k] for k in out if "_log_" in k})


if __name__ == "__main__":
    main()
