"""Classic-MADN HIP env kernels vs the CPU oracle (GPU).

* the reference's 64 golden step vectors (MADN/test.py:7-475), through the C ABI;
* seeded random play in lockstep for four rule sets: die from the same uniform numbers on both sides
  (throw_die), legal masks, dice distributions, soft-lock flags, observations, step / no_step, all
  compared bit-exactly after every ply.
"""
import numpy as np
import pytest
import torch

from oracle import classic_madn as cm
from tests.test_oracle_golden import CLASSIC_CASES, DICE_CASES, classic_env_from_case, dice_env_from_case

pytestmark = pytest.mark.gpu

RULE_SETS = {
    # config (c): game_agent_stochastic.py:13-24, 4 players in teams, dice rethrow
    "selfplay_4p_teams": dict(num_players=4, **cm.SELFPLAY_RULES),
    "selfplay_2p": dict(num_players=2, **cm.SELFPLAY_RULES),
    "exotic_4p": dict(num_players=4, enable_teams=False, enable_initial_free_pin=True, enable_circular_board=True,
                      enable_start_blocking=True, enable_jump_in_goal_area=False, enable_friendly_fire=True,
                      enable_start_on_1=False, enable_bonus_turn_on_6=True, enable_dice_rethrow=True,
                      must_traverse_start=True),
    "exotic_3p": dict(num_players=3, enable_teams=False, enable_initial_free_pin=False, enable_circular_board=False,
                      enable_start_blocking=True, enable_jump_in_goal_area=False, enable_friendly_fire=False,
                      enable_start_on_1=True, enable_bonus_turn_on_6=False, enable_dice_rethrow=False,
                      must_traverse_start=True),
}


def _C():
    from exploring_muzero_on_dog_amd import classic as C
    return C


def rules_of(env):
    return _C().make_rules(num_players=env.num_players, starting_player=0, **env.rules)


def to_gpu(envs, rules):
    return _C().state_from_host(
        pins=np.stack([e.pins for e in envs]), current_player=np.array([e.current_player for e in envs]),
        rules=rules, die=np.array([e.die for e in envs], np.int8), done=np.array([e.done for e in envs], np.uint8),
        reward=np.array([e.reward for e in envs], np.int8), board=np.stack([e.board for e in envs]))


def assert_same(gpu, envs, what):
    B, P = len(envs), envs[0].num_players
    torch.cuda.synchronize()
    pins = gpu.pins.cpu().numpy().T.reshape(B, P, 4)
    board = gpu.board.cpu().numpy().T
    cp = gpu.current_player.cpu().numpy()
    done = gpu.done.cpu().numpy()
    die = gpu.die.cpu().numpy()
    for b, e in enumerate(envs):
        ok = (np.array_equal(pins[b], e.pins) and np.array_equal(board[b], e.board) and cp[b] == e.current_player
              and bool(done[b]) == e.done and die[b] == e.die)
        assert ok, (what, b, pins[b].tolist(), e.pins.tolist(), int(cp[b]), e.current_player, int(die[b]), e.die)


def test_classic_dice_probs_notebook_outputs(cuda):
    """muz_classic_dice_probs on the 8 positions of MADN/jupyter_code/test_functions.ipynb cells 3-4 against the
    reference's recorded is_soft_locked / dice_probabilities outputs (classic_madn.py:180-228)."""
    C = _C()
    for case in DICE_CASES:
        env = dice_env_from_case(case)
        gpu = to_gpu([env], rules_of(env))
        probs, soft = C.dice_probabilities(gpu, with_soft_lock=True)
        torch.cuda.synchronize()
        assert bool(soft.cpu()[0]) == case["soft_locked"], case
        assert np.allclose(probs.cpu().numpy()[0], case["dice_probabilities"], rtol=0, atol=5e-9), case


def test_classic_golden_step_vectors(cuda):
    C = _C()
    for case in CLASSIC_CASES:
        env = classic_env_from_case(case)
        gpu = to_gpu([env], rules_of(env))
        valid = C.valid_action(gpu)[0].cpu().numpy()
        assert np.array_equal(valid, cm.valid_action(env)), case["source"]
        _, reward, done = C.env_step(gpu, torch.tensor([case["pin"]]))
        torch.cuda.synchronize()
        pins = gpu.pins_bp()[0].cpu().numpy()
        assert np.array_equal(pins, np.array(case["expected_valid"])), case["source"]
        assert valid[case["pin"]] or int(reward[0]) == -1, case["source"]      # MADN/test.py:474


@pytest.mark.parametrize("rule_set", sorted(RULE_SETS))
def test_classic_random_play_lockstep(cuda, rule_set):
    """Every ply: the GPU batch is rebuilt from the oracle states, then dice distribution, soft lock, die,
    observation, legal mask and the transition (step on games with a legal pin -- 10 % of them an
    arbitrary, possibly illegal pin -- no_step elsewhere) must match the oracle bit for bit."""
    C = _C()
    kw = RULE_SETS[rule_set]
    n, plies = 192, 400
    rng = np.random.default_rng(7)
    envs = [cm.env_reset(**kw) for _ in range(n)]
    gpu = C.env_reset(n, **kw)
    assert_same(gpu, envs, "reset")
    rules = gpu.rules
    steps = 0
    for ply in range(plies):
        gpu = to_gpu(envs, rules)
        probs, soft = C.dice_probabilities(gpu, with_soft_lock=True)
        probs, soft = probs.cpu().numpy(), soft.cpu().numpy()
        for i, e in enumerate(envs):
            assert bool(soft[i]) == cm.is_soft_locked(e), (ply, i)
            assert np.array_equal(probs[i], cm.dice_probabilities(e)), (ply, i)
        u = rng.random(n, dtype=np.float32)
        C.throw_die(gpu, torch.from_numpy(u))
        envs = [cm.throw_die(e, float(u[i])) for i, e in enumerate(envs)]
        assert_same(gpu, envs, f"die ply {ply}")
        obs = C.encode_board(gpu, torch.int8).cpu().numpy()
        legal = C.valid_action(gpu).cpu().numpy()
        pins = np.zeros(n, np.int64)
        step_idx, nost_idx = [], []
        for i, e in enumerate(envs):
            assert np.array_equal(obs[i], cm.encode_board(e)), (ply, i)
            va = cm.valid_action(e)
            assert np.array_equal(legal[i], va), (ply, i, legal[i], va)
            if e.done:
                continue
            if va.any():
                pins[i] = int(rng.choice(np.flatnonzero(va))) if rng.random() > 0.1 else int(rng.integers(0, 4))
                step_idx.append(i)
            else:
                nost_idx.append(i)
        if not step_idx and not nost_idx:
            break
        if step_idx:
            sub = to_gpu([envs[i] for i in step_idx], rules)
            _, reward, done = C.env_step(sub, torch.from_numpy(pins[step_idx]))
            reward = reward.cpu().numpy()
            for j, i in enumerate(step_idx):
                envs[i], r, _ = cm.env_step(envs[i], int(pins[i]))
                assert int(reward[j]) == r, (ply, i)
            assert_same(sub, [envs[i] for i in step_idx], f"step ply {ply}")
            steps += len(step_idx)
        if nost_idx:
            sub = to_gpu([envs[i] for i in nost_idx], rules)
            C.no_step(sub)
            for i in nost_idx:
                envs[i] = cm.no_step(envs[i])[0]
            assert_same(sub, [envs[i] for i in nost_idx], f"nostep ply {ply}")
    assert steps > 1000
