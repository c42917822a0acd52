"""DOG MuZero slice on the GPU (csrc/dog_muzero.hip, csrc/dog_search.hip) against oracle/dog_muzero.py.

The reference defines only the DOG RepresentationNetwork (MuZero_DOG/muzero_dog.py:25-83); the observation, the
Dyn / Pred networks at A = 806 and the search there are builder-defined (parity unpinned beyond the env, whose
transitions the other DOG tests pin).  Bars: the encoding bit-exact; network outputs within atol 1e-5 (fp32, MFMA
k-order vs BLAS order, as tests/test_gpu_nets.py)."""
import numpy as np
import pytest
import torch

from oracle import dog as dg
from oracle import dog_muzero as DM
from tests.dog_states import RULE_SETS, random_state, reset
from tests.test_gpu_dog import rules_of, to_gpu

pytestmark = pytest.mark.gpu

ATOL = 1e-5


def _MD():
    from exploring_muzero_on_dog_amd import muzero_dog as MD
    return MD


def finished_mover(e):
    """e with the current player's four pins in its goal (a finished player: with teams it plays the partner's hand,
    dog.py sub_player) and the board rebuilt."""
    pins = np.asarray(e.pins).copy()
    cp = e.current_player
    board = np.asarray(e.board).copy()
    for k in range(4):
        cell = int(e.goal[cp][k])
        for p in range(pins.shape[0]):        # a pin of another player on that cell goes home
            pins[p][pins[p] == cell] = -1
        pins[cp][k] = cell
    board = dg.set_pins_on_board(-np.ones(56, np.int8), pins)
    return e.replace(pins=pins, board=board)


def dog_states(rule_set, n_rand, n_fresh, seed):
    kw = RULE_SETS[rule_set]
    rng = np.random.default_rng(seed)
    envs = [random_state(rng, kw, seed, g) for g in range(n_rand)] + \
           [reset(kw, seed, n_rand + g) for g in range(n_fresh)]
    for g in range(0, n_rand, 8):           # every 8th random state: the mover has finished
        envs[g] = finished_mover(envs[g])
    return kw, envs


@pytest.mark.parametrize("rule_set", ["selfplay_4p_teams", "exotic_4p"])
def test_dog_encode_matches_oracle(cuda, rule_set):
    MD = _MD()
    kw, envs = dog_states(rule_set, 80, 16, 7)
    gpu = to_gpu(envs, rules_of(kw), 7)
    obs = MD.encode_board(gpu).cpu().numpy()
    subs = 0
    for b, e in enumerate(envs):
        want = DM.encode_board(e)
        assert np.array_equal(obs[b], want), (rule_set, b, np.argwhere(obs[b] != want)[:6].tolist())
        subs += int(want[30, 0])
    if RULE_SETS[rule_set].get("enable_teams"):
        assert subs > 0   # the substituted hand (a finished player plays the partner's cards) was exercised


def test_dog_encode_rejects_non_4p(cuda):
    MD = _MD()
    from exploring_muzero_on_dog_amd import dog as D
    from exploring_muzero_on_dog_amd import lib as L
    gpu = D.env_reset(8, num_players=2)
    with pytest.raises(L.MuzError):
        MD.encode_board(gpu)


def _obs(n, seed):
    kw, envs = dog_states("selfplay_4p_teams", n, 0, seed)
    return np.stack([DM.encode_board(e) for e in envs]).astype(np.float32)


def test_dog_root_inference(cuda):
    MD = _MD()
    params = DM.init_params(seed=11, randomize_affine=True)
    net = MD.DeviceDogNet(params)
    obs = _obs(61, 3)                                 # 61: a partial 16-row tile
    lg, v, e = MD.root_inference_fn(net, torch.from_numpy(obs).cuda())
    rl, rv, re = DM.root_inference(params, obs)
    d_l = np.abs(lg.cpu().numpy() - rl).max()
    d_v = np.abs(v.cpu().numpy() - rv).max()
    d_e = np.abs(e.cpu().numpy() - re).max()
    print(f"dog root: |dlogits| {d_l:.2e} |dvalue| {d_v:.2e} |dlatent| {d_e:.2e} (latent std {re.std():.2f})")
    assert d_e < ATOL and d_l < ATOL and d_v < ATOL


@pytest.mark.parametrize("seed", [0, 1])
def test_dog_recurrent_inference(cuda, seed):
    MD = _MD()
    params = DM.init_params(seed=20 + seed, randomize_affine=True)
    net = MD.DeviceDogNet(params)
    rng = np.random.default_rng(seed)
    B = 77
    emb = rng.standard_normal((B, 256)).astype(np.float32)
    act = rng.integers(0, 806, B).astype(np.int32)
    act[:3] = [-1, 806, 805]                          # out of range -> zero one-hot row (jax.nn.one_hot)
    out = MD.recurrent_inference_fn(net, torch.from_numpy(act).cuda(), torch.from_numpy(emb).cuda())
    want = DM.recurrent_inference(params, act, emb)
    names = ("reward", "discount", "logits", "value", "next_latent")
    ds = {k: float(np.abs(o.cpu().numpy() - w).max()) for k, o, w in zip(names, out, want)}
    print("dog recurrent:", {k: f"{v:.2e}" for k, v in ds.items()})
    assert all(v < ATOL for v in ds.values()), ds


def _search_setup(B, seed):
    MD = _MD()
    params = DM.init_params(seed=seed, randomize_affine=True)
    net = MD.DeviceDogNet(params)
    kw, envs = dog_states("selfplay_4p_teams", B, 8, seed + 5)
    valid = np.stack([dg.valid_actions(e) for e in envs]).astype(bool)
    keep = valid.any(1)
    envs = [e for e, k in zip(envs, keep) if k]
    valid = valid[keep]
    obs = np.stack([DM.encode_board(e) for e in envs]).astype(np.float32)
    words = MD.invalid_to_words(torch.from_numpy(~valid))
    return MD, params, net, obs, valid, words


def _gpu_recurrent_fn(MD, net):
    def fn(params, action, emb):
        out = MD.recurrent_inference_fn(net, torch.from_numpy(np.asarray(action, np.int32)).cuda(),
                                        torch.from_numpy(np.ascontiguousarray(emb)).cuda())
        return tuple(t.cpu().numpy() for t in out)
    return fn


def test_dog_invalid_to_words_matches_legal_mask(cuda):
    MD = _MD()
    from exploring_muzero_on_dog_amd import dog as D
    gpu = D.env_reset(40, seed=3, **RULE_SETS["selfplay_4p_teams"])
    words = D.legal_mask(gpu)
    valid = D.unpack_mask(words).bool()
    assert torch.equal(MD.invalid_to_words(~valid.cpu()).cuda(), words)


@pytest.mark.parametrize("S,D,exact,rows", [(50, 25, False, None), (16, 4, False, None), (8, 50, False, "16"),
                                            (50, 25, True, "16"), (100, 50, False, None), (100, 50, False, "16")])
def test_dog_search_logic_matches_mctx_restatement(cuda, S, D, exact, rows, monkeypatch):
    """The oracle search driven by the GPU's own recurrent kernel: both sides see identical network outputs, so the
    tree arithmetic (lane-order sums at A = 806, oracle/mctx_gumbel.py lane_tree_sum) must agree bit for bit.
    exact: every interior selection on the 806-exponential path (MUZ_DOG_EXACT_SELECT=1) instead of the certified
    argmax (dog_search.hip wselect_certified) -- both must give the restatement's actions.  rows: 16 games per
    workgroup (MUZ_DOG_TILE_ROWS=16) instead of the one game per wave this batch size gets by default."""
    if exact:
        monkeypatch.setenv("MUZ_DOG_EXACT_SELECT", "1")
    if rows:
        monkeypatch.setenv("MUZ_DOG_TILE_ROWS", rows)
    from tests._parity import search_parity
    from oracle import mctx_gumbel as G
    MD, params, net, obs, valid, words = _search_setup(40, 7)
    B = obs.shape[0]
    lg, v, e = MD.root_inference_fn(net, torch.from_numpy(obs).cuda())
    gum = np.random.default_rng(3).gumbel(size=(B, 806)).astype(np.float32)
    pol, rv = MD.gumbel_muzero_policy(net, lg, v, e, words, S, D, 1.0, gumbel=torch.from_numpy(gum))
    trace = {}
    a, w, orv, _ = G.gumbel_muzero_policy(params, lg.cpu().numpy(), v.cpu().numpy(), e.cpu().numpy(),
                                          _gpu_recurrent_fn(MD, net), S, ~valid, gum, max_depth=D, trace=trace)
    torch.cuda.synchronize()
    ga, gw, grv = pol.action.cpu().numpy(), pol.action_weights.cpu().numpy(), rv.cpu().numpy()
    search_parity(f"dog search logic A806 S{S} D{D}", ga, gw, grv, a, w, orv, trace["margin"], trace["gain"])
    assert valid[np.arange(B), ga].all(), "search picked an invalid root action"
    assert np.array_equal(ga, a) and np.array_equal(gw, w) and np.array_equal(grv, orv), \
        "identical network outputs: the tree arithmetic must agree bit for bit"


def test_dog_run_muzero_mcts_reference_signature(cuda):
    """muzero_dog.py:101-137's signature on the flat params: same result as the device-native calls."""
    MD, params, net, obs, valid, words = _search_setup(24, 9)
    pol, rv = MD.run_muzero_mcts(params, 5, obs, ~valid, 8, 4, 1.0)
    lg, v, e = MD.root_inference_fn(net, torch.from_numpy(obs).cuda())
    pol2, rv2 = MD.gumbel_muzero_policy(net, lg, v, e, words, 8, 4, 1.0, seed=5)
    assert torch.equal(pol.action, pol2.action) and torch.equal(pol.action_weights, pol2.action_weights)
    assert torch.equal(rv, rv2)
    assert valid[np.arange(len(valid)), pol.action.cpu().numpy()].all()


@pytest.mark.parametrize("rows", [None, "16"])
def test_dog_muzero_selfplay_followed_by_oracle(cuda, rows, monkeypatch):
    """game_agent_dog.DogSelfPlay (legal -> encode -> root -> search at A = 806 -> step, finished games restarting in
    place) followed turn by turn by the oracle: oracle/dog.py transitions with the engine's deal keys, the oracle's
    own encoding fed to the GPU root kernel, and oracle/mctx_gumbel.py driven by the GPU recurrent kernel with the
    engine's Gumbel stream -- every action, weight, root value and state bit-identical.  rows: as above."""
    if rows:
        monkeypatch.setenv("MUZ_DOG_TILE_ROWS", rows)
    from oracle import mctx_gumbel as G
    from oracle import selfplay as OS
    from exploring_muzero_on_dog_amd import dog as D
    from exploring_muzero_on_dog_amd import game_agent_dog as GA
    MD = _MD()
    params = DM.init_params(seed=13, randomize_affine=True)
    net = MD.DeviceDogNet(params)
    B, S, Dd, T, seed, temp = 10, 4, 3, 24, 21, 1.0
    sp = GA.DogSelfPlay(net, B, S, Dd, temp, seed=seed)
    kw = RULE_SETS["selfplay_4p_teams"]
    envs = [reset(kw, seed, g) for g in range(B)]
    keys = [dg.engine_shuffle_keys(seed, g) for g in range(B)]
    rec = _gpu_recurrent_fn(MD, net)
    searched = 0
    for t in range(T):
        act, w, rv = sp.turn()
        act, w, rv = act.cpu().numpy(), w.cpu().numpy(), rv.cpu().numpy()
        valid = np.stack([dg.valid_actions(e) for e in envs]).astype(bool)
        has = np.flatnonzero(valid.any(1))
        want = np.full(B, -1)
        if has.size:
            obs = np.stack([DM.encode_board(envs[g]) for g in has]).astype(np.float32)
            lg, v, e = (x.cpu().numpy() for x in MD.root_inference_fn(net, torch.from_numpy(obs).cuda()))
            gum = np.stack([OS.gumbel_noise(seed, int(g), t, A=806, scale=temp) for g in has]).astype(np.float32)
            a, ow, orv, _ = G.gumbel_muzero_policy(params, lg, v, e, rec, S, ~valid[has], gum, max_depth=Dd)
            want[has] = a
            assert np.array_equal(w[has], ow) and np.array_equal(rv[has], orv), t
            searched += has.size
        assert np.array_equal(act, want), (t, act.tolist(), want.tolist())
        for g in range(B):
            e0 = envs[g]
            e1 = (dg.no_step(e0, keys[g]) if want[g] < 0 else dg.env_step(e0, int(want[g]), keys[g]))[0]
            if e1.done:      # muz_dog_step_restart: env_reset in place, deal counter continued
                base = e1.deal
                e1 = dg.env_reset(num_players=4, shuffle_keys=lambda x, b=base, k=keys[g]: k(x.replace(deal=x.deal + b)),
                                  **dg.SELFPLAY_RULES)
                e1 = e1.replace(deal=e1.deal + base)
            envs[g] = e1
        from tests.dog_states import diff
        bad = diff(D.to_host(sp.env), envs)
        assert bad is None, (t, bad)
    assert searched > B * T // 2


def test_dog_certified_select_equals_exact_at_bench_shape(cuda, monkeypatch):
    """the certified interior argmax (wselect_certified) at the benched shape -- 1500 games, S = 100, D = 50,
    seeded random weights, roots from 8 self-play turns -- against the exact 806-exponential selection
    (MUZ_DOG_EXACT_SELECT=1) on the same roots: actions, weights and root values bit-identical (about 10^6 interior
    selections, no oracle involved)."""
    from exploring_muzero_on_dog_amd import dog as D
    from exploring_muzero_on_dog_amd import game_agent_dog as GA
    MD = _MD()
    net = MD.DeviceDogNet(MD.init_muzero_params(2))
    B, S, Dd = 1500, 100, 50
    sp = GA.DogSelfPlay(net, B, S, Dd, 1.0, seed=4)
    sp.play(8)
    words = D.legal_mask(sp.env)
    obs = MD.encode_board(sp.env)
    lg, v, e = MD.root_inference_fn(net, obs)
    out = {}
    for exact in ("0", "1"):
        monkeypatch.setenv("MUZ_DOG_EXACT_SELECT", exact)
        pol, rv = MD.gumbel_muzero_policy(net, lg, v, e, words, S, Dd, 1.0, seed=4, turn=8)
        torch.cuda.synchronize()
        out[exact] = (pol.action.clone(), pol.action_weights.clone(), rv.clone())
    (a0, w0, v0), (a1, w1, v1) = out["0"], out["1"]
    assert int((a0 >= 0).sum()) > B // 2
    assert torch.equal(a0, a1) and torch.equal(w0, w1) and torch.equal(v0, v1)
