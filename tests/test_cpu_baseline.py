"""The C++ CPU restatement behind bench.py's cpu_baseline (oracle/cpu_selfplay.cpp) against the NumPy oracle
(CPU only): the reference's 64 golden step vectors, lockstep random play of four rule sets (legal masks,
transitions, no-move turns, observations), the three networks at 1e-5, and a short self-play trace under
the strict parity bar of tests/_parity.py (same network outputs on both sides)."""
import numpy as np
import pytest

from oracle import cpu_selfplay as CS
from oracle import detmadn as dm
from oracle import nets as ON
from oracle import selfplay as OS
from tests._detmadn_util import RULE_SETS, random_play_transitions
from tests._parity import selfplay_parity
from tests.test_oracle_golden import DET_CASES, det_env_from_case


@pytest.fixture(scope="module", autouse=True)
def _built():
    CS.load()


def test_golden_step_vectors():
    for case in DET_CASES:
        d = CS.env_from_oracle(det_env_from_case(case))
        CS.env_step(d, case["pin"], case["move"])
        assert np.array_equal(CS.pins(d), np.array(case["expected_valid"])), case["source"]


@pytest.mark.parametrize("rule_set", sorted(RULE_SETS))
def test_lockstep_random_play(rule_set):
    n = 0
    for _, batch in random_play_transitions(rule_set, 6, 11, max_plies=300, p_illegal=0.1):
        for _, env, kind, a in batch:
            d = CS.env_from_oracle(env)
            assert np.array_equal(CS.valid_action(d), dm.valid_action(env))
            assert np.array_equal(CS.encode(d), dm.encode_board(env).astype(np.float32))
            if kind == "step":
                r, done = CS.env_step(d, *dm.map_action(a))
                e2, r2, done2 = dm.env_step(env, dm.map_action(a))
            else:
                CS.no_step(d)
                e2, r2, done2 = dm.no_step(env)
                r = r2
                done = bool(d.done)
            assert (r, bool(done)) == (r2, bool(done2))
            assert np.array_equal(CS.pins(d), e2.pins)
            assert np.array_equal(np.array(d.board[:], np.int8), e2.board)
            assert np.array_equal(np.array(d.action_set[:e2.num_players * 6], np.int8).reshape(-1, 6), e2.action_set)
            assert d.current_player == e2.current_player
            n += 1
    assert n > 500


@pytest.mark.parametrize("P", [2, 4])
def test_networks_match_numpy_oracle(P):
    from tests.test_gpu_nets import random_obs
    C = dm.num_channels(P)
    params = ON.init_params(C, seed=21, randomize_affine=True)
    net = CS.CpuNet(params, C)
    obs, _ = random_obs("selfplay_2p" if P == 2 else "selfplay_4p_teams", 12, 4)
    lg, v, e = net.root(obs)
    olg, ov, oe = ON.root_inference(params, obs)
    assert np.abs(lg - olg).max() < 1e-5 and np.abs(v - ov).max() < 1e-5 and np.abs(e - oe).max() < 1e-5
    act = np.random.default_rng(0).integers(0, 24, len(obs)).astype(np.int32)
    out = net.recurrent(act, oe)
    ref = ON.recurrent_inference(params, act, oe)
    for a, b in zip(out, ref):
        assert np.abs(a - b).max() < 1e-5


def test_selfplay_trace_matches_oracle_loop():
    P, n, S, D, T, temp, seed = 2, 6, 8, 8, 80, 1.0, 77
    C = dm.num_channels(P)
    params = ON.init_params(C, seed=5, randomize_affine=True)
    net = CS.CpuNet(params, C)
    buf, turns = net.selfplay(P, dm.SELFPLAY_RULES, n, S, D, T, temp, seed)
    envs = [dm.env_reset(num_players=P, **dm.SELFPLAY_RULES) for _ in range(n)]
    ref, steps = OS.play_batch_of_games(params, lambda _, o: net.root(o), lambda _, a, e: net.recurrent(a, e), envs,
                                        S, D, T, temp, seed)
    diverged = selfplay_parity("C++ CPU restatement vs oracle loop", buf, ref, ("act", "mask"))
    if not diverged:
        assert turns == steps


def test_bench_counts_work():
    C = dm.num_channels(2)
    net = CS.CpuNet(ON.init_params(C, seed=1), C)
    r = net.bench(2, dm.SELFPLAY_RULES, 4, 4, 4, 500, 1.0, 3, 2, 0.5)
    assert r["env_steps"] > 0 and r["searches"] > 0 and r["elapsed"] >= 0.5
