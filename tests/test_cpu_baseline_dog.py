"""The C++ DOG restatement behind bench.py --workload dog's cpu_baseline (oracle/cpu_dog.cpp) against the NumPy
oracle (CPU only): the reference's golden step vectors (DOG/test.py, incl. the code-vs-test case the oracle
follows the code on), the 806-action mask and every transition of lockstep random play through swap phases,
deals and game restarts with the engine's counter-RNG deal keys / action choice, and the bench loop's action
sequence against the oracle's."""
import numpy as np
import pytest

from oracle import cpu_selfplay as CS
from oracle import dog as dg
from tests.test_oracle_golden import DOG_CASES, dog_env_from_case, dog_step_case


@pytest.fixture(scope="module", autouse=True)
def _built():
    CS._dog_lib()


def test_golden_step_vectors_follow_the_oracle():
    n = 0
    for kind, cases in DOG_CASES.items():
        for c in cases:
            env = dog_env_from_case(c)
            pins, reward, done = CS.dog_step_kind(CS.dog_from_oracle(env), kind, c)
            _, opins, oreward, odone = dog_step_case(kind, c)
            assert np.array_equal(pins, opins) and (reward, done) == (oreward, odone), (kind, c["source"])
            n += 1
    assert n == 112


def _same(d, e):
    P = e.num_players
    assert np.array_equal(np.array(d.board[:], np.int8), e.board)
    assert np.array_equal(np.array(d.pins[:P * 4], np.int32).reshape(P, 4), e.pins)
    assert np.array_equal(np.array(d.hands[:P * 14], np.int8).reshape(P, 14), e.hands)
    assert np.array_equal(np.array(d.deck[:], np.int8), e.deck)
    assert np.array_equal(np.array(d.swap_choices[:], np.int8), e.swap_choices)
    assert (d.current_player, d.phase, d.round_starter, d.hand_size, d.deal, bool(d.done)) == \
        (e.current_player, e.phase, e.round_starter, e.hand_size, e.deal, e.done)


@pytest.mark.parametrize("P,rules", [(4, dg.SELFPLAY_RULES), (4, dict(dg.DEFAULT_RULES)),
                                     (2, dict(dg.SELFPLAY_RULES, enable_circular_board=False,
                                              enable_jump_in_goal_area=True))])
def test_lockstep_random_play(P, rules):
    seed, games, turns = 13, 3, 260
    rng = np.random.default_rng(P)
    n = 0
    for g in range(games):
        keys = dg.engine_shuffle_keys(seed, g)
        e = dg.env_reset(num_players=P, shuffle_keys=keys, **rules)
        d = CS.dog_from_oracle(e, seed, g)
        for t in range(turns):
            if e.done:
                break
            mask = dg.valid_actions(e)
            assert np.array_equal(CS.dog_valid_actions(d), mask), (g, t)
            legal = np.flatnonzero(mask)
            if legal.size == 0:
                e = dg.no_step(e, keys)[0]
                CS.dog_no_step(d)
            else:   # mostly legal actions, sometimes an arbitrary one (invalid moves keep the reference's -1 path)
                a = int(rng.choice(legal)) if rng.random() > 0.05 else int(rng.integers(0, 806))
                e, r2, dn2 = dg.env_step(e, a, keys)
                r, dn = CS.dog_step(d, a)
                assert (r, dn) == (r2, bool(dn2)), (g, t, a)
            _same(d, e)
            n += 1
    assert n > 300


def test_bench_loop_follows_the_oracle_loop():
    """muzcpu_dog_play = bench.py's former NumPy loop (8 games, engine action choice, in-place restarts)."""
    seed, n, turns = 5, 2, 1300            # random DOG games last ~840 turns: restarts happen
    acts, steps = CS.dog_play(4, dg.SELFPLAY_RULES, n, turns, seed)
    gids = list(range(n))
    envs = [dg.env_reset(num_players=4, shuffle_keys=dg.engine_shuffle_keys(seed, g), **dg.SELFPLAY_RULES) for g in gids]
    nxt = n
    for t in range(turns):
        for i in range(n):
            if envs[i].done:
                gids[i], nxt = nxt, nxt + 1
                envs[i] = dg.env_reset(num_players=4, shuffle_keys=dg.engine_shuffle_keys(seed, gids[i]),
                                       **dg.SELFPLAY_RULES)
            keys = dg.engine_shuffle_keys(seed, gids[i])
            a = dg.engine_random_action(dg.valid_actions(envs[i]), seed, gids[i], t)
            assert acts[t, i] == a, (t, i)
            envs[i] = (dg.no_step(envs[i], keys) if a < 0 else dg.env_step(envs[i], a, keys))[0]
    assert steps == n * turns and nxt > n


def test_bench_counts_work():
    r = CS.dog_bench(4, dg.SELFPLAY_RULES, 8, 3, 2, 0.3)
    assert r["env_steps"] > 0 and r["elapsed"] >= 0.3
