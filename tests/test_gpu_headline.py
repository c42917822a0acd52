"""Config (b) at its real shape (BASELINE.json headline): det-MADN 2p, B = 4096, S = 50, D = 25 (GPU).

* One full-batch muz_gumbel_search launch (256 workgroups of 16 games) on 4096 mid-game positions, checked
  against the mctx restatement on one lane of EVERY tile (the lane's position inside its tile varies), with
  the strict margin-aware bar of tests/_parity.py.  Rows of a tile are computed independently, so the
  oracle can run on the sampled lanes alone.
* The benchmark's own call, muz_detmadn_selfplay_stream over 4096 lanes: two runs are identical, and every
  recorded game replays through the (bit-exact) env kernels: each MCTS action legal, each no-move turn
  without a legal action, the recorded observation equal to encode_board, and the game done exactly at
  its recorded length (or truncated at max_steps)."""
import numpy as np
import pytest
import torch

from oracle import detmadn as dm
from oracle import mctx_gumbel as G
from oracle import nets as ON
from tests._parity import log, search_parity

pytestmark = pytest.mark.gpu

B, S, D, P = 4096, 50, 25, 2
FIELDS = ("board", "pins", "current_player", "reward", "done", "action_set")


def _mods():
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import mcts as M
    from exploring_muzero_on_dog_amd import nets as N
    return E, GA, M, N


def _merge(dst, src, sel):
    for f in FIELDS:
        getattr(dst, f)[..., sel] = getattr(src, f)[..., sel]


def _random_action(bits, rng):
    """A uniformly random legal action index per lane (-1 when nothing is legal), on the host."""
    m = ((bits[:, None] >> np.arange(24)[None, :]) & 1).astype(bool)
    u = rng.random(m.shape)
    score = np.where(m, u, -1.0)
    a = score.argmax(1).astype(np.int32)
    return np.where(m.any(1), a, -1).astype(np.int32)


def _step_mixed(E, env, act):
    """env_step where act >= 0, no_step where act < 0, games already done left untouched (in place)."""
    dev = env.board.device
    a = torch.from_numpy(act).to(dev)
    done_before = env.done.clone().bool()
    nos = env.clone()
    E.no_step(nos)
    E.env_step(env, torch.clamp(a, min=0))
    _merge(env, nos, a < 0)
    frozen = env.clone()
    return env, done_before, frozen


def mid_game_positions(E, rules, rng, max_plies=300):
    """4096 positions after 0..max_plies plies of seeded random legal play (a snapshot per lane at its
    drawn ply), each with at least one legal action."""
    env = E.env_reset(B, num_players=P, **rules)
    snap = env.clone()
    fresh = env.clone()
    target = rng.integers(0, max_plies + 1, B)
    for ply in range(max_plies + 1):
        sel = torch.from_numpy(target == ply).cuda()
        _merge(snap, env, sel)
        if ply == max_plies:
            break
        prev = env.clone()
        bits = E.legal_bits(env).cpu().numpy()
        act = _random_action(bits, rng)
        _step_mixed(E, env, act)
        _merge(env, prev, prev.done.bool())   # finished games stay finished
    bits = E.legal_bits(snap)
    bad = (bits == 0) | snap.done.bool()
    _merge(snap, fresh, bad)
    return snap


def test_full_batch_search_matches_oracle_on_every_tile(cuda):
    E, GA, M, N = _mods()
    C = dm.num_channels(P)
    params = ON.init_params(C, seed=17, randomize_affine=True)
    net = N.DeviceNet(params, C)
    rng = np.random.default_rng(0)
    env = mid_game_positions(E, dm.SELFPLAY_RULES, rng)
    bits = E.legal_bits(env)
    assert int((bits == 0).sum()) == 0
    obs = E.encode_board(env)
    gum = torch.from_numpy(np.random.default_rng(1).gumbel(size=(B, 24)).astype(np.float32)).cuda()
    lg, v, e = N.root_inference_fn(net, obs)
    pol, rv = M.gumbel_muzero_policy(net, lg, v, e, bits, S, D, 1.0, gumbel=gum)
    torch.cuda.synchronize()
    lanes = np.array([t * 16 + (t * 7) % 16 for t in range(B // 16)])      # one lane per tile
    sel = torch.from_numpy(lanes).cuda()
    b = bits.cpu().numpy()[lanes]
    invalid = ((b[:, None] >> np.arange(24)[None, :]) & 1) == 0

    def rec(params_, action, emb):
        out = N.recurrent_inference_fn(net, torch.from_numpy(np.asarray(action, np.int32)).cuda(),
                                       torch.from_numpy(np.ascontiguousarray(emb)).cuda())
        return tuple(t.cpu().numpy() for t in out)

    trace = {}
    a, w, orv, _ = G.gumbel_muzero_policy(params, lg[sel].cpu().numpy(), v[sel].cpu().numpy(), e[sel].cpu().numpy(),
                                          rec, S, invalid, gum[sel].cpu().numpy(), max_depth=D, trace=trace)
    ga = pol.action.cpu().numpy()
    search_parity("headline B=4096 S=50 D=25, one lane per tile (256 lanes)", ga[lanes],
                  pol.action_weights.cpu().numpy()[lanes], rv.cpu().numpy()[lanes], a, w, orv, trace["margin"], trace["gain"])
    allb = bits.cpu().numpy()
    assert ((allb >> ga) & 1).all(), "an action outside the legal mask"
    wts = pol.action_weights.cpu().numpy()
    assert np.allclose(wts.sum(1), 1.0, atol=1e-5)


def test_headline_stream_deterministic_and_replays_legally(cuda):
    E, GA, M, N = _mods()
    C = dm.num_channels(P)
    net = N.DeviceNet(N.init_muzero_params(0, C), C)
    T, games = 500, 2 * B
    eng = GA.SelfPlayEngine(net, B, num_players=P, max_steps=T, num_simulations=S, max_depth=D)
    one = {k: v.clone() for k, v in eng.play_stream(games, seed=1001, temperature=1.0).items()}
    st = dict(eng.last_stats)
    two = eng.play_stream(games, seed=1001, temperature=1.0)
    for k in one:
        assert torch.equal(one[k], two[k]), k
    del two
    idx = one["idx"]
    act = one["act"]
    env = E.env_reset(games, num_players=P, **dm.SELFPLAY_RULES)
    t_ar = torch.arange(T, device="cuda")
    live = t_ar[None, :] < idx[:, None]
    assert torch.equal((act >= 0) & live, (one["mask"] > 0) & live), "mask must mark exactly the MCTS turns"
    for t in range(int(idx.max().item())):
        active = (t < idx)
        assert not env.done.bool()[active].any(), f"turn {t}: a game continues after it was done"
        bits = E.legal_bits(env)
        a = act[:, t]
        mcts = active & (a >= 0)
        assert (((bits >> a.clamp(min=0)) & 1).bool() | ~mcts).all(), f"turn {t}: illegal recorded action"
        assert ((bits == 0) | ~(active & (a < 0))).all(), f"turn {t}: no-move turn with a legal action"
        obs = E.encode_board(env, dtype=torch.int8)
        assert torch.equal(obs[mcts], one["obs"][mcts, t]), f"turn {t}: recorded observation != encode_board"
        prev = env.clone()
        _step_mixed(E, env, a.cpu().numpy())
        _merge(env, prev, ~active)
    done = env.done.bool()
    assert torch.equal(done | (idx == T), torch.ones_like(done)), "a game stopped before done / max_steps"
    steps = int(idx.sum().item())
    log(f"headline stream B={B} S={S} D={D}: {games} games, {steps} env-steps, {st['searches']} searches, "
        f"deterministic, every game replays legally through the env kernels")
