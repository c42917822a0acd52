"""DOG HIP env kernels vs the CPU oracle (GPU), all through the C ABI (include/muz.h DOG section).

* reset: the device deal (counter-RNG keys, wave-parallel stable ranking) equals oracle env_reset with
  oracle/dog.py:engine_shuffle_keys, for four rule sets;
* the reference's golden step vectors (DOG/test.py) replayed as full env_step calls (card gating, hand
  consumption, next player) on both sides, and their expected pins;
* lockstep fuzzing from random mid-game states: legal masks (806 bits), the random-action kernel, and
  env_step / no_step (85 % legal actions, 15 % arbitrary ones, so refused moves are covered) must match
  the oracle bit for bit on every field;
* the engine's own loop (``dog.RandomPlay``, device RNG only) followed by the oracle on a subset of games.
"""
import numpy as np
import pytest
import torch

from oracle import dog as dg
from tests.dog_states import RULE_SETS, diff, fields_of, random_state, reset
from tests.test_oracle_golden import DOG_CASES, DOG_CODE_VS_TEST, dog_env_from_case

pytestmark = pytest.mark.gpu


def _D():
    from exploring_muzero_on_dog_amd import dog as D
    return D


def rules_of(kw_or_env):
    D = _D()
    if isinstance(kw_or_env, dict):
        kw = dict(kw_or_env)
        return D.make_rules(**kw)
    e = kw_or_env
    return D.make_rules(num_players=e.num_players, starting_player=0, **e.rules)


def to_gpu(envs, rules, seed):
    return _D().state_from_host(fields_of(envs), rules, seed=seed)


@pytest.mark.parametrize("rule_set", sorted(RULE_SETS))
def test_dog_reset_matches_oracle(cuda, rule_set):
    D = _D()
    kw = RULE_SETS[rule_set]
    n, seed = 96, 12345
    gpu = D.env_reset(n, seed=seed, **kw)
    envs = [reset(kw, seed, g) for g in range(n)]
    assert diff(D.to_host(gpu), envs) is None


def test_dog_golden_through_abi(cuda):
    D = _D()
    seed, ran = 77, 0
    for kind, cases in DOG_CASES.items():
        for i, c in enumerate(cases):
            if kind == "normal_move" and c["move"] == 7:
                continue          # step_normal_move(7) has no action index (7 is the hot-7 card)
            if kind == "hot7_move" and not np.all(dg.DISTS_7_4 == np.array(c["dist"])[None, :], axis=1).any():
                continue          # a distribution that does not sum to 7 has no action index either
            env = dog_env_from_case(c)
            env = env.replace(hands=np.ones((env.num_players, 14), np.int8), phase=0)
            joker = bool(i % 2)
            if kind == "normal_move":
                a = D.map_move_to_action("normal", c["pin"], c["move"], joker)
            elif kind == "neg_move":
                a = D.map_move_to_action("neg", c["pin"], -4, joker)
            elif kind == "swap_move":
                a = D.map_move_to_action("swap", c["pin"], c["pos"], joker)
            else:
                row = int(np.flatnonzero(np.all(dg.DISTS_7_4 == np.array(c["dist"])[None, :], axis=1))[0])
                a = D.map_move_to_action("hot7", -1, row, joker)
            gpu = to_gpu([env], rules_of(env), seed)
            _, reward, done = D.env_step(gpu, torch.tensor([a]))
            env2, r, d = dg.env_step(env, a, dg.engine_shuffle_keys(seed, 0))
            host = D.to_host(gpu)
            assert diff(host, [env2]) is None, (c["source"], diff(host, [env2]))
            assert int(reward[0]) == r and bool(done[0]) == d, c["source"]
            if c["source"] not in DOG_CODE_VS_TEST:
                assert np.array_equal(host["pins"][0], np.array(c["expected_valid"])), c["source"]
            ran += 1
    assert ran == 112 - 5 - 24       # all but the 5 move-7 and 24 non-7-sum cases


def test_dog_golden_step_functions(cuda):
    """All 112 reference cases through muz_dog_step_move, batched per (players, rules): the step function
    the reference test calls, with its own arguments (including hot-7 splits that do not sum to 7)."""
    D = _D()
    groups = {}
    for kind, cases in DOG_CASES.items():
        for c in cases:
            env = dog_env_from_case(c)
            key = (env.num_players, tuple(sorted(env.rules.items())))
            groups.setdefault(key, []).append((kind, c, env))
    ran = 0
    for (P, _), items in groups.items():
        envs = [e for _, _, e in items]
        kinds, args = [], []
        for kind, c, _ in items:
            if kind == "swap_move":
                kinds.append("swap"), args.append([c["pin"], c["pos"], 0, 0])
            elif kind == "hot7_move":
                kinds.append("hot7"), args.append(list(c["dist"]))
            else:
                kinds.append("normal" if kind == "normal_move" else "neg"), args.append([c["pin"], c["move"], 0, 0])
        gpu = to_gpu(envs, rules_of(envs[0]), 0)
        _, reward, done = D.step_move(gpu, kinds, args)
        host = D.to_host(gpu)
        reward, done = reward.cpu().numpy(), done.cpu().numpy()
        for b, (kind, c, env) in enumerate(items):
            from tests.test_oracle_golden import dog_step_case
            board, pins, r, d = dog_step_case(kind, c)
            assert np.array_equal(host["pins"][b], pins) and np.array_equal(host["board"][b], board), c["source"]
            assert int(reward[b]) == r and bool(done[b]) == d, c["source"]
            if c["source"] not in DOG_CODE_VS_TEST:
                assert np.array_equal(host["pins"][b], np.array(c["expected_valid"])), c["source"]
            ran += 1
    assert ran == 112


def test_dog_random_action_kernel(cuda):
    D = _D()
    rng = np.random.default_rng(0)
    B = 2000
    bits = (rng.random((B, 806)) < rng.random((B, 1)) * 0.05)
    bits[::17] = False
    words = np.zeros((B, 26), np.uint32)
    for a in range(806):
        words[:, a // 32] |= bits[:, a].astype(np.uint32) << np.uint32(a % 32)
    mask = torch.from_numpy(words.view(np.int32)).cuda()
    u = rng.random(B, dtype=np.float32)
    got = D.random_action(mask, torch.from_numpy(u)).cpu().numpy()
    for b in range(B):
        legal = np.flatnonzero(bits[b])
        want = -1 if legal.size == 0 else int(legal[min(int(u[b] * np.float32(legal.size)), legal.size - 1)])
        assert got[b] == want, b
    got = D.random_action(mask, None, seed=31, turn=4).cpu().numpy()
    for b in range(0, B, 7):
        assert got[b] == dg.engine_random_action(bits[b], 31, b, 4), b


@pytest.mark.parametrize("rule_set", sorted(RULE_SETS))
def test_dog_lockstep_fuzz(cuda, rule_set):
    D = _D()
    kw = RULE_SETS[rule_set]
    seed = 4242
    rng = np.random.default_rng(sorted(RULE_SETS).index(rule_set))
    n_rand, n_fresh, plies = 48, 16, 40
    envs = [random_state(rng, kw, seed, g) for g in range(n_rand)] + \
           [reset(kw, seed, n_rand + g) for g in range(n_fresh)]
    n = len(envs)
    keys = [dg.engine_shuffle_keys(seed, g) for g in range(n)]
    rules = rules_of(kw)
    steps = refused = nosteps = deals = dones = 0
    for ply in range(plies):
        gpu = to_gpu(envs, rules, seed)
        mask_words = D.legal_mask(gpu)
        legal = D.unpack_mask(mask_words).cpu().numpy()
        ract = D.random_action(mask_words, None, seed=seed, turn=ply).cpu().numpy()
        acts = np.zeros(n, np.int64)
        for g, e in enumerate(envs):
            va = dg.valid_actions(e)
            assert np.array_equal(legal[g], va), (rule_set, ply, g, np.flatnonzero(legal[g] != va)[:8])
            ra = dg.engine_random_action(va, seed, g, ply)
            assert ract[g] == ra, (ply, g)
            acts[g] = ra if (ra < 0 or rng.random() > 0.15) else int(rng.integers(0, 806))
        _, reward, done = D.env_step(gpu, torch.from_numpy(acts))
        reward, done = reward.cpu().numpy(), done.cpu().numpy()
        for g in range(n):
            d0 = envs[g].deal
            if acts[g] < 0:
                envs[g], r, d = dg.no_step(envs[g], keys[g])
                nosteps += 1
            else:
                envs[g], r, d = dg.env_step(envs[g], int(acts[g]), keys[g])
                steps += 1
                refused += r == -1
            deals += envs[g].deal != d0
            dones += bool(d)
            assert int(reward[g]) == r and bool(done[g]) == bool(d), (ply, g, int(reward[g]), r)
        bad = diff(D.to_host(gpu), envs)
        assert bad is None, (rule_set, ply, bad)
    assert steps > 1500 and refused > 50 and deals > 20, (steps, refused, nosteps, deals, dones)


@pytest.mark.parametrize("fused", [False, True])
def test_dog_engine_loop_followed_by_oracle(cuda, fused):
    """dog.RandomPlay (legal -> random action -> step, device RNG only; three launches or the fused
    muz_dog_random_turn) for 150 turns; the oracle replays every 16th game with the same counter streams
    and must land on the same state every turn."""
    D = _D()
    B, seed, T = 256, 99, 150
    rp = D.RandomPlay(B, seed=seed, fused=fused)
    kw = RULE_SETS["selfplay_4p_teams"]
    follow = list(range(0, B, 16))
    envs = {g: reset(kw, seed, g) for g in follow}
    keys = {g: dg.engine_shuffle_keys(seed, g) for g in follow}
    for t in range(T):
        rp.turn()
        for g in follow:
            if fused and envs[g].done:
                continue          # the fused turn leaves finished games alone
            a = dg.engine_random_action(dg.valid_actions(envs[g]), seed, g, t)
            envs[g] = (dg.no_step(envs[g], keys[g]) if a < 0 else dg.env_step(envs[g], a, keys[g]))[0]
        if t % 10 == 9 or t == T - 1:
            host = D.to_host(rp.env)
            sub = {k: v[follow] for k, v in host.items()}
            bad = diff(sub, [envs[g] for g in follow])
            assert bad is None, (t, bad)


def test_dog_multi_turn_kernel_equals_single_turns(cuda):
    """muz_dog_random_play(20 turns, one launch) == 20 x muz_dog_random_turn, state and step counts."""
    D = _D()
    B, seed = 300, 7
    a, b = D.RandomPlay(B, seed=seed), D.RandomPlay(B, seed=seed)
    steps = torch.zeros(B, dtype=torch.int32, device="cuda")
    for chunk in (1, 7, 12):
        for _ in range(chunk):
            a.turn()
        b.play(chunk, steps)
        ha, hb = D.to_host(a.env), D.to_host(b.env)
        for k in ha:
            assert np.array_equal(ha[k], hb[k]), k
    assert int(steps.sum()) == B * 20 - 0 or int(steps.min()) >= 1
    want = 20 - 0
    done = D.to_host(b.env)["done"]
    assert (steps.cpu().numpy()[done == 0] == want).all()


def test_dog_auto_reset_followed_by_oracle(cuda):
    """muz_dog_random_play with auto_reset over 1500 turns (longer than a random game): finished games
    restart in place with the deal counter continued; the oracle follows 8 games through their restarts."""
    D = _D()
    B, seed, T, chunk = 128, 3, 1500, 100
    rp = D.RandomPlay(B, seed=seed)
    kw = RULE_SETS["selfplay_4p_teams"]
    follow = list(range(0, B, 16))
    envs = {g: reset(kw, seed, g) for g in follow}
    keys = {g: dg.engine_shuffle_keys(seed, g) for g in follow}
    steps = torch.zeros(B, dtype=torch.int32, device="cuda")
    eps = torch.zeros(B, dtype=torch.int32, device="cuda")
    n_eps = {g: 0 for g in follow}
    for t0 in range(0, T, chunk):
        rp.play(chunk, steps, auto_reset=True, episodes=eps)
        for t in range(t0, t0 + chunk):
            for g in follow:
                e = envs[g]
                if e.done:      # dog_reset_lds: env_reset, deal counter continued
                    base = e.deal
                    e = dg.env_reset(num_players=4, shuffle_keys=lambda x, b=base, k=keys[g]: k(x.replace(deal=x.deal + b)),
                                     **dg.SELFPLAY_RULES)
                    e = e.replace(deal=e.deal + base)
                a = dg.engine_random_action(dg.valid_actions(e), seed, g, t)
                e = (dg.no_step(e, keys[g]) if a < 0 else dg.env_step(e, a, keys[g]))[0]
                n_eps[g] += int(e.done)
                envs[g] = e
        host = D.to_host(rp.env)
        bad = diff({k: v[follow] for k, v in host.items()}, [envs[g] for g in follow])
        assert bad is None, (t0, bad)
    assert (steps.cpu().numpy() == T).all()
    e_dev = eps.cpu().numpy()
    assert all(e_dev[g] == n_eps[g] for g in follow)
    assert e_dev.sum() > B // 2, "random DOG games end within ~1000 turns; restarts must have happened"


def test_dog_play_deterministic_and_launch_split_invariant(cuda):
    """Config (d)'s workload (1024 games, 16-turn launches with in-place restarts): two runs agree exactly,
    and so does the same schedule cut into single-turn launches (the state carried in LDS across turns
    of one launch must equal the state round-tripped through HBM every turn)."""
    D = _D()
    # 100 launches = 1600 turns: most games end and restart at least once inside a launch, which is where
    # round 1's unordered s.done read (fixed in k_dog_play) made runs differ
    B, seed, launches = 1024, 4, 100

    def run(turns_per_launch):
        rp = D.RandomPlay(B, seed=seed)
        steps = torch.zeros(B, dtype=torch.int32, device="cuda")
        eps = torch.zeros(B, dtype=torch.int32, device="cuda")
        for _ in range(launches * 16 // turns_per_launch):
            rp.play(turns_per_launch, steps, auto_reset=True, episodes=eps)
        return D.to_host(rp.env), steps.cpu().numpy(), eps.cpu().numpy()

    a, b, b2, c = run(16), run(16), run(16), run(1)
    for other in (b, b2, c):
        for k in a[0]:
            assert np.array_equal(a[0][k], other[0][k]), k
        assert np.array_equal(a[1], other[1]) and np.array_equal(a[2], other[2])
    assert a[2].sum() > B // 2      # most games finished and restarted inside a launch


def test_dog_records_follow_the_oracle(cuda):
    """muz_dog_random_play_record: every recorded row (action, mover, reward, legal count, finished flag)
    of the followed games equals the oracle's turn, across launches and in-place restarts; the packed
    records locate each game's rows."""
    D = _D()
    B, seed, T, chunk, launches = 64, 6, 900, 100, 9
    rp = D.RandomPlay(B, seed=seed)
    rec = D.DogTrajectory(B, T)
    follow = list(range(0, B, 8))
    envs = {g: reset(RULE_SETS["selfplay_4p_teams"], seed, g) for g in follow}
    keys = {g: dg.engine_shuffle_keys(seed, g) for g in follow}
    rows = {g: [] for g in follow}
    for li in range(launches):
        rp.play(chunk, auto_reset=True, record=rec)
        for t in range(li * chunk, (li + 1) * chunk):
            for g in follow:
                e = envs[g]
                if e.done:
                    base = e.deal
                    e = dg.env_reset(num_players=4, shuffle_keys=lambda x, b=base, k=keys[g]: k(x.replace(deal=x.deal + b)),
                                     **dg.SELFPLAY_RULES)
                    e = e.replace(deal=e.deal + base)
                mask = dg.valid_actions(e)
                a = dg.engine_random_action(mask, seed, g, t)
                mover = e.current_player
                if a < 0:
                    e2, r, d = dg.no_step(e, keys[g])
                else:
                    e2, r, d = dg.env_step(e, a, keys[g])
                rows[g].append((a, mover, int(r), int(np.asarray(mask).sum()), int(bool(d))))
                envs[g] = e2
    buf = {k: v.cpu().numpy() for k, v in rec.buf.items()}
    n = launches * chunk
    assert (buf["idx"] == n).all()
    for g in follow:
        got = list(zip(buf["act"][g, :n], buf["player"][g, :n], buf["reward"][g, :n], buf["legal"][g, :n],
                       buf["done"][g, :n]))
        assert [tuple(int(x) for x in r) for r in got] == rows[g], g
    assert sum(sum(r[4] for r in rows[g]) for g in follow) > 0, "games must finish within the records"
    packed = rec.pack()
    off, idx = packed["row_offset"].cpu().numpy(), packed["idx"].cpu().numpy()
    for g in follow:
        assert np.array_equal(packed["act"].cpu().numpy()[off[g]:off[g] + idx[g]], buf["act"][g, :idx[g]])
