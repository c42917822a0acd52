"""muz_detmadn_random_round (the env-only micro-benchmark's kernel and a random-play actor) against the
oracle (GPU): every round, every game's state, next legal mask and int8 observation equal the NumPy
restatement of valid_action -> k-th legal action (engine counter RNG) -> env_step / no_step -> env_reset of
finished games -> encode_board."""
import numpy as np
import pytest
import torch

from oracle import detmadn as dm
from oracle.dog import _game_key, _mix64, _u24
from tests._detmadn_util import RULE_SETS, legal_bits_oracle

pytestmark = pytest.mark.gpu
STREAM = 0xD37A11D0


def oracle_round(envs, seed, turn, kw):
    out = []
    for g, e in enumerate(envs):
        va = dm.valid_action(e).flatten()
        legal = np.flatnonzero(va)
        if legal.size == 0:
            e2 = dm.no_step(e)[0]
        else:
            u = _u24(_mix64(_game_key(seed ^ STREAM, g, turn)))
            k = min(int(np.float32(u) * np.float32(legal.size)), legal.size - 1)
            e2 = dm.env_step(e, dm.map_action(int(legal[k])))[0]
        fin = bool(e2.done)
        if fin:
            e2 = dm.env_reset(**kw)
        out.append((e2, fin))
    return out


@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("rule_set", ["selfplay_2p", "selfplay_4p_teams", "exotic_4p"])
def test_random_round_matches_oracle(cuda, rule_set, variant):
    """variant 1: one game per lane (k_det_round), 2 / 3 / 4 / 5: one game per 32 / 8 / 4 / 16 lanes
    (k_det_round_g)."""
    from exploring_muzero_on_dog_amd import detmadn as E
    kw = RULE_SETS[rule_set]
    B, seed, rounds = 48, 9, 400
    env = E.env_reset(B, **kw)
    legal = E.legal_bits(env)
    P = kw["num_players"]
    C = dm.num_channels(P)
    obs = torch.empty((B, C, 56), dtype=torch.int8, device="cuda")
    done = torch.empty(B, dtype=torch.uint8, device="cuda")
    envs = [dm.env_reset(**kw) for _ in range(B)]
    finished = 0
    for t in range(rounds):
        E.random_round(env, legal, seed, t, obs=obs, done=done, variant=variant)
        res = oracle_round(envs, seed, t, kw)
        envs = [e for e, _ in res]
        fin = np.array([f for _, f in res])
        finished += int(fin.sum())
        assert np.array_equal(done.cpu().numpy().astype(bool), fin), t
        pins = env.pins_bp().cpu().numpy()
        assert np.array_equal(pins, np.stack([e.pins for e in envs])), t
        assert np.array_equal(env.current_player.cpu().numpy(), [e.current_player for e in envs]), t
        assert np.array_equal(env.action_set_bp().cpu().numpy(), np.stack([e.action_set for e in envs])), t
        assert np.array_equal(env.board.T.cpu().numpy(), np.stack([e.board for e in envs])), t
        assert np.array_equal(legal.cpu().numpy(), [legal_bits_oracle(e) for e in envs]), t
        assert np.array_equal(obs.cpu().numpy(), np.stack([dm.encode_board(e) for e in envs]).astype(np.int8)), t
    assert finished > 0, "games must finish and restart within the rounds"


@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5])
def test_random_round_large_batch_properties(cuda, variant):
    """B = 2^20 games (the micro-benchmark's HBM-sized batch): the observation written by the fused kernel
    equals encode_board of the stored state, and the returned mask equals valid_action of it."""
    from exploring_muzero_on_dog_amd import detmadn as E
    kw = RULE_SETS["selfplay_2p"]
    B = 1 << 20
    env = E.env_reset(B, **kw)
    legal = E.legal_bits(env)
    obs = torch.empty((B, 18, 56), dtype=torch.int8, device="cuda")
    for t in range(40):
        E.random_round(env, legal, 3, t, obs=obs, variant=variant)
    assert torch.equal(obs, E.encode_board(env, dtype=torch.int8))
    assert torch.equal(legal, E.legal_bits(env))


def test_random_round_variants_identical_ragged(cuda):
    """Every kernel variant (one game per 1 / 32 / 8 / 4 / 16 lanes) leaves the same state, mask, observation,
    rewards and done flags at a batch that fills no workgroup evenly (5001 games, 4p teams rules)."""
    from exploring_muzero_on_dog_amd import detmadn as E
    kw = RULE_SETS["selfplay_4p_teams"]
    B = 5001
    outs = []
    for variant in (1, 2, 3, 4, 5):
        env = E.env_reset(B, **kw)
        legal = E.legal_bits(env)
        C = E.num_channels(kw["num_players"])
        obs = torch.empty((B, C, 56), dtype=torch.int8, device="cuda")
        reward = torch.empty(B, dtype=torch.int8, device="cuda")
        done = torch.empty(B, dtype=torch.uint8, device="cuda")
        acc = torch.zeros(B, dtype=torch.int64, device="cuda")
        for t in range(60):
            E.random_round(env, legal, 11, t, obs=obs, reward=reward, done=done, variant=variant)
            acc += reward.long() * (t + 1) + done.long() * 1000
        outs.append((env.board.clone(), env.pins.clone(), env.action_set.clone(), env.current_player.clone(),
                     legal.clone(), obs.clone(), acc))
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert torch.equal(x, y)
