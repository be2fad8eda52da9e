"""Config-5 vector env on the GPU against its CPU restatement (oracle/vecenv_oracle.py):
states, observations, masks, rewards and dones bit-exact over many steps and episodes, with
agent actions both given (random legal, chosen on the host) and drawn in-kernel."""
import numpy as np
import pytest
import torch

from oracle.vecenv_oracle import VecEnvOracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("max_cells", [4, 5])
def test_vector_env_matches_oracle(max_cells):
    from blokus_rl_amd.vector_env import BlokusVectorEnv

    E = 32
    env = BlokusVectorEnv(E, 7, max_cells)
    ref = VecEnvOracle(E, 7, max_cells)
    env.reset(seed=5)
    ref.reset(seed=5)
    rng = np.random.default_rng(0)
    episodes = 0
    for t in range(60):
        m = env.mask_words.cpu().numpy().view(np.uint64)
        obs = env.obs.cpu().numpy()
        for e in range(E):
            assert (m[e] == ref.mask(e)).all(), (t, e)
            assert (obs[e] == ref.obs(e)).all(), (t, e)
            assert (env.states[e].cpu().numpy() == ref.states[e]).all(), (t, e)
        if t % 3 == 2:
            acts = np.full(E, -1, dtype=np.int32)  # in-kernel random agent
        else:
            acts = np.array([int(rng.choice(np.nonzero(np.unpackbits(m[e].view(np.uint8), bitorder="little")[:env.eng.A])[0]))
                             for e in range(E)], dtype=np.int32)
        _, rew, term, _, _ = env.step(torch.from_numpy(acts))
        rew, term = rew.cpu().numpy(), term.cpu().numpy()
        for e in range(E):
            r, d = ref.step(e, int(acts[e]))
            assert rew[e] == r and bool(term[e]) == bool(d), (t, e)
            episodes += d
        assert (env.rng.cpu().numpy().view(np.uint64) == np.array(ref.rng, dtype=np.uint64)).all()
    assert episodes > E  # several episodes per env ended and auto-reset


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
