"""The C++ classic Stochastic-MuZero restatement behind bench.py --workload classic's cpu_baseline
(oracle/cpu_classic.cpp) against the NumPy oracle (CPU only): the reference's 64 golden step vectors and its
notebook dice outputs, lockstep random play of four rule sets (die draw from the same uniforms, legal masks,
dice distributions, observations, transitions), the networks (Repr2 / StochasticDynamicsNetwork4 / Pred4) at
1e-5, and a short self-play trace against oracle/selfplay.py's loop + oracle/mctx_stochastic.py under the
strict parity bar of tests/_parity.py (same network outputs on both sides)."""
import numpy as np
import pytest

from oracle import classic_madn as cm
from oracle import classic_nets as CN
from oracle import cpu_selfplay as CS
from oracle import selfplay as OS
from tests._parity import selfplay_parity
from tests.test_oracle_golden import CLASSIC_CASES, DICE_CASES, classic_env_from_case, dice_env_from_case

RULE_SETS = {
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


@pytest.fixture(scope="module", autouse=True)
def _built():
    CS._classic_lib()


def test_golden_step_vectors():
    for case in CLASSIC_CASES:
        env = classic_env_from_case(case)
        d = CS.classic_from_oracle(env)
        assert np.array_equal(CS.classic_valid_action(d), cm.valid_action(env)), case["source"]
        CS.classic_step(d, case["pin"])
        assert np.array_equal(np.array(d.pins[:8], np.int8).reshape(2, 4), np.array(case["expected_valid"])), case["source"]


def test_notebook_dice_outputs():
    for case in DICE_CASES:
        soft, p = CS.classic_dice(CS.classic_from_oracle(dice_env_from_case(case)))
        assert soft == case["soft_locked"]
        assert np.allclose(p, case["dice_probabilities"], rtol=0, atol=5e-9)


@pytest.mark.parametrize("rule_set", sorted(RULE_SETS))
def test_lockstep_random_play(rule_set):
    rules = dict(RULE_SETS[rule_set])
    P = rules.pop("num_players")
    rng = np.random.default_rng(11)
    n = 0
    for game in range(5):
        env = cm.env_reset(num_players=P, **rules)
        d = CS.classic_from_oracle(env)
        for ply in range(250):
            if env.done:
                break
            u = float(rng.random(dtype=np.float32))
            env = cm.throw_die(env, u)
            CS.classic_throw_die(d, u)
            assert d.die == env.die
            soft, p = CS.classic_dice(d)
            assert soft == cm.is_soft_locked(env) and np.array_equal(p, cm.dice_probabilities(env))
            va = cm.valid_action(env)
            assert np.array_equal(CS.classic_valid_action(d), va)
            assert np.array_equal(CS.classic_encode(d), cm.encode_board(env).astype(np.float32))
            if va.any():
                pin = int(rng.choice(np.flatnonzero(va))) if rng.random() > 0.1 else int(rng.integers(0, 4))
                env, r2, dn2 = cm.env_step(env, pin)
                r, dn = CS.classic_step(d, pin)
                assert (r, dn) == (r2, bool(dn2))
            else:
                env, _, _ = cm.no_step(env)
                CS.classic_no_step(d)
            assert np.array_equal(np.array(d.pins[:P * 4], np.int8).reshape(P, 4), env.pins)
            assert np.array_equal(np.array(d.board[:], np.int8), env.board)
            assert d.current_player == env.current_player and bool(d.done) == env.done
            n += 1
    assert n > 300


def test_networks_match_numpy_oracle():
    C = cm.num_channels(4)
    params = CN.init_params(C, seed=31, randomize_affine=True)
    net = CS.CpuClassicNet(params, C)
    rng = np.random.default_rng(4)
    obs = rng.integers(0, 4, (10, C, 56)).astype(np.float32)
    lg, v, e = net.root(obs)
    olg, ov, oe = CN.root_inference(params, obs)
    assert np.abs(lg - olg).max() < 1e-5 and np.abs(v - ov).max() < 1e-5 and np.abs(e - oe).max() < 1e-5
    act = rng.integers(0, 4, len(obs)).astype(np.int32)
    out = net.decision(act, oe)
    ref = CN.decision_recurrent(params, act, oe)
    for a, b in zip(out, ref):
        assert np.abs(a - b).max() < 1e-5
    ch = rng.integers(0, 6, len(obs)).astype(np.int32)
    out = net.chance(ch, ref[2])
    ref = CN.chance_recurrent(params, ch, ref[2])
    for a, b in zip(out, ref):
        assert np.abs(a - b).max() < 1e-5


def test_selfplay_trace_matches_oracle_loop():
    P, n, S, D, T, temp, seed = 4, 6, 8, 6, 70, 1.0, 91
    C = cm.num_channels(P)
    params = CN.init_params(C, seed=7, randomize_affine=True)
    net = CS.CpuClassicNet(params, C)
    buf, turns = net.selfplay(P, cm.SELFPLAY_RULES, n, S, D, T, temp, seed)
    envs = [cm.env_reset(num_players=P, **cm.SELFPLAY_RULES) for _ in range(n)]
    ref, steps = OS.play_batch_of_games_stochastic(
        params, lambda _, o: net.root(o), lambda _, a, e: net.decision(a, e), lambda _, c, a: net.chance(c, a),
        envs, S, D, T, temp, seed)
    diverged = selfplay_parity("C++ classic CPU restatement vs oracle loop", buf, ref, ("act", "mask", "dice"))
    if not diverged:
        assert turns == steps


def test_bench_counts_work():
    C = cm.num_channels(4)
    net = CS.CpuClassicNet(CN.init_params(C, seed=1), C)
    r = net.bench(4, cm.SELFPLAY_RULES, 4, 4, 4, 500, 1.0, 3, 2, 0.5)
    assert r["env_steps"] > 0 and r["searches"] > 0 and r["elapsed"] >= 0.5
