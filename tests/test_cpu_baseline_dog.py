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


# ---- the DOG MuZero slice (bench.py --workload dog --policy muzero's cpu_baseline) --------------------------------
def _slice_states(n=24, seed=13):
    """(oracle state, C++ state) pairs from lockstep random play of 4p DOG, spread over a few hundred turns."""
    rng = np.random.default_rng(seed)
    out = []
    for g in range(3):
        keys = dg.engine_shuffle_keys(seed, g)
        e = dg.env_reset(num_players=4, shuffle_keys=keys, **dg.SELFPLAY_RULES)
        for t in range(300):
            if e.done:
                break
            if t % 37 == 5:
                out.append((e, CS.dog_from_oracle(e, seed, g)))
            legal = np.flatnonzero(dg.valid_actions(e))
            e = dg.no_step(e, keys)[0] if legal.size == 0 else dg.env_step(e, int(rng.choice(legal)), keys)[0]
    return out[:n]


def test_dog_encode_matches_oracle():
    from oracle import dog_muzero as DM
    states = _slice_states()
    assert len(states) >= 12
    for e, d in states:
        assert np.array_equal(CS.dog_encode(d), DM.encode_board(e).astype(np.float32))


def _dog_net(seed=13):
    from oracle import dog_muzero as DM
    params = DM.init_params(seed=seed, randomize_affine=True)
    return params, CS.CpuNet(params, DM.NUM_CHANNELS)


def test_dog_networks_match_numpy_oracle():
    """RepresentationNetwork (LayerNorm head) + Pred4 / Dyn4 at A = 806 against oracle/dog_muzero.py, 1e-5."""
    from oracle import dog_muzero as DM
    params, net = _dog_net()
    obs = np.stack([DM.encode_board(e) for e, _ in _slice_states(12)]).astype(np.float32)
    lg, v, e = net.root(obs)
    olg, ov, oe = DM.root_inference(params, obs)
    assert lg.shape == (12, 806)
    assert np.abs(lg - olg).max() < 1e-5 and np.abs(v - ov).max() < 1e-5 and np.abs(e - oe).max() < 1e-5
    act = np.random.default_rng(0).integers(-1, 806, len(obs)).astype(np.int32)   # -1: the all-zero one-hot
    for a, b in zip(net.recurrent(act, oe), DM.recurrent_inference(params, act, oe)):
        assert np.abs(a - b).max() < 1e-5


def _numpy_search(params, net, lg, v, e, valid, gum, S, D):
    from oracle import mctx_gumbel as G
    return G.gumbel_muzero_policy(params, lg, v, e, lambda _, a, x: net.recurrent(a, x), S, ~valid, gum, max_depth=D)


def test_dog_search_matches_numpy_search_bit_for_bit():
    """The C++ Gumbel search at A = 806 (oracle/cpu_search.hpp, lane-order sums) against oracle/mctx_gumbel.py driven
    by the same C++ recurrent inference: actions, action weights and root values identical."""
    from oracle import dog_muzero as DM
    from oracle import selfplay as OS
    params, net = _dog_net(7)
    states = _slice_states(6, seed=3)
    obs = np.stack([DM.encode_board(e) for e, _ in states]).astype(np.float32)
    valid = np.stack([dg.valid_actions(e) for e, _ in states]).astype(bool)
    keep = valid.any(1)
    obs, valid = obs[keep], valid[keep]
    lg, v, e = net.root(obs)
    gum = np.stack([OS.gumbel_noise(9, g, 2, A=806, scale=1.0) for g in range(len(obs))]).astype(np.float32)
    for S, D in ((8, 4), (12, 12)):
        a, w, rv = net.dog_search(lg, v, e, ~valid, gum, S, D)
        oa, ow, orv, _ = _numpy_search(params, net, lg, v, e, valid, gum, S, D)
        assert np.array_equal(a, oa) and np.array_equal(w, ow) and np.array_equal(rv, orv), (S, D)
        assert valid[np.arange(len(a)), a].all()


def test_dog_selfplay_follows_the_numpy_loop():
    """muzcpu_dog_mz_play (the cpu_baseline's turn) against the NumPy loop: oracle/dog.py transitions with the engine's
    deal keys, oracle/dog_muzero.py encoding, the engine's Gumbel stream of (seed, game, turn) and mctx_gumbel.py
    driven by the C++ networks -- every action identical."""
    from oracle import dog_muzero as DM
    from oracle import selfplay as OS
    params, net = _dog_net(11)
    n, turns, S, D, temp, seed = 3, 10, 4, 3, 1.0, 7
    acts, searches = net.dog_play(dg.SELFPLAY_RULES, n, turns, S, D, temp, seed)
    keys = [dg.engine_shuffle_keys(seed, g) for g in range(n)]
    envs = [dg.env_reset(num_players=4, shuffle_keys=keys[g], **dg.SELFPLAY_RULES) for g in range(n)]
    want_searches = 0
    for t in range(turns):
        valid = np.stack([dg.valid_actions(x) for x in envs]).astype(bool)
        has = np.flatnonzero(valid.any(1))
        want = np.full(n, -1)
        if has.size:
            obs = np.stack([DM.encode_board(envs[g]) for g in has]).astype(np.float32)
            lg, v, e = net.root(obs)
            gum = np.stack([OS.gumbel_noise(seed, int(g), t, A=806, scale=temp) for g in has]).astype(np.float32)
            want[has] = _numpy_search(params, net, lg, v, e, valid[has], gum, S, D)[0]
            want_searches += has.size
        assert np.array_equal(acts[t], want), (t, acts[t].tolist(), want.tolist())
        envs = [(dg.no_step(x, keys[g]) if want[g] < 0 else dg.env_step(x, int(want[g]), keys[g]))[0]
                for g, x in enumerate(envs)]
    assert searches == want_searches > 0


def test_dog_mz_bench_counts_work():
    _, net = _dog_net(1)
    r = net.dog_bench(dg.SELFPLAY_RULES, 2, 2, 2, 1.0, 3, 2, 0.3)
    assert r["env_steps"] > 0 and r["searches"] > 0 and r["elapsed"] >= 0.3
