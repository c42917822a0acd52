"""Config (c) at its real shape (BASELINE.json): classic MADN 4p teams, B = 4096, S = 50, D = 25 (GPU).

One full-batch muz_stochastic_search launch (256 workgroups of 16 games) over 4096 mid-game positions with
the die thrown, checked against the mctx restatement (oracle/mctx_stochastic.py, driven by the GPU's own
decision / chance recurrent kernels) on one lane of EVERY tile, with the strict bar of tests/_parity.py.
Rows of a tile are independent (a tile only skips a trunk no row needs), so the oracle runs on the sampled
lanes alone, with their game ids for the counter-RNG tie-break uniforms."""
import dataclasses

import numpy as np
import pytest
import torch

from oracle import classic_madn as cm
from oracle import classic_nets as CN
from oracle import mctx_stochastic as MS
from tests._parity import search_parity

pytestmark = pytest.mark.gpu

B, S, D, P = 4096, 50, 25, 4
FIELDS = ("board", "pins", "current_player", "reward", "done", "die")


def _mods():
    from exploring_muzero_on_dog_amd import classic as CL
    from exploring_muzero_on_dog_amd import stochastic as ST
    return CL, ST


def _copy(env):
    return dataclasses.replace(env, **{f: getattr(env, f).clone() for f in FIELDS})


def _merge(dst, src, sel):
    for f in FIELDS:
        getattr(dst, f)[..., sel] = getattr(src, f)[..., sel]


def _random_action(bits, rng):
    """A uniformly random legal pin per lane (-1 when nothing is legal), on the host."""
    m = ((bits[:, None] >> np.arange(4)[None, :]) & 1).astype(bool)
    score = np.where(m, rng.random(m.shape), -1.0)
    return np.where(m.any(1), score.argmax(1), -1).astype(np.int32)


def mid_game_positions(CL, rng, max_plies=240):
    """4096 positions after 0..max_plies plies of seeded random legal play through the (bit-exact) env
    kernels, die thrown; lanes without a legal pin (or finished) become a fresh game with a 6."""
    env = CL.env_reset(B, num_players=P, **cm.SELFPLAY_RULES)
    fresh = _copy(env)
    snap = _copy(env)
    target = rng.integers(0, max_plies + 1, B)
    for ply in range(max_plies + 1):
        CL.throw_die(env, torch.from_numpy(rng.random(B).astype(np.float32)).cuda())
        _merge(snap, env, torch.from_numpy(target == ply).cuda())
        if ply == max_plies:
            break
        prev = _copy(env)
        act = _random_action(CL.legal_bits(env).cpu().numpy(), rng)
        nos = _copy(env)
        CL.no_step(nos)
        CL.env_step(env, torch.from_numpy(np.maximum(act, 0)).cuda())
        _merge(env, nos, torch.from_numpy(act < 0).cuda())
        _merge(env, prev, prev.done.bool())   # finished games stay finished
    bad = (CL.legal_bits(snap) == 0) | snap.done.bool()
    _merge(snap, fresh, bad)
    CL.set_die(snap, torch.where(bad, torch.full_like(snap.die, 6), snap.die).int())
    return snap


def test_full_batch_stochastic_search_matches_oracle_on_every_tile(cuda):
    CL, ST = _mods()
    C = cm.num_channels(P)
    params = CN.init_params(C, seed=21, randomize_affine=True)
    net = ST.DeviceClassicNet(params, C)
    rng = np.random.default_rng(5)
    env = mid_game_positions(CL, rng)
    bits = CL.legal_bits(env)
    assert int((bits == 0).sum()) == 0
    obs = CL.encode_board(env)
    lg, v, e = ST.root_inference_fn(net, obs)
    r2 = np.random.default_rng(6)
    dirichlet = r2.dirichlet(np.full(4, 0.3), B).astype(np.float32)
    gumbel = r2.gumbel(size=(B, 4)).astype(np.float32)
    seed, turn = 4242, 13
    act, w, rv = ST.stochastic_muzero_policy(net, lg, v, e, bits, S, D, 1.0, seed=seed, turn=turn,
                                             dirichlet=torch.from_numpy(dirichlet), gumbel=torch.from_numpy(gumbel))
    torch.cuda.synchronize()
    lanes = np.array([t * 16 + (t * 5) % 16 for t in range(B // 16)])      # one lane per tile
    sel = torch.from_numpy(lanes).cuda()
    b = bits.cpu().numpy()[lanes]
    valid = ((b[:, None] >> np.arange(4)[None, :]) & 1).astype(bool)

    def dec(params_, action, emb):
        return tuple(t.cpu().numpy() for t in ST.decision_recurrent_fn(
            net, torch.from_numpy(np.asarray(action, np.int32)).cuda(), torch.from_numpy(np.ascontiguousarray(emb)).cuda()))

    def cha(params_, chance, after):
        return tuple(t.cpu().numpy() for t in ST.chance_recurrent_fn(
            net, torch.from_numpy(np.asarray(chance, np.int32)).cuda(), torch.from_numpy(np.ascontiguousarray(after)).cuda()))

    trace = {}
    oa, ow, orv, _ = MS.stochastic_muzero_policy(params, lg[sel].cpu().numpy(), v[sel].cpu().numpy(),
                                                 e[sel].cpu().numpy(), dec, cha, S, ~valid, dirichlet[lanes],
                                                 gumbel[lanes], max_depth=D, temperature=1.0, seed=seed, turn=turn,
                                                 gids=lanes, trace=trace)
    ga = act.cpu().numpy()
    search_parity("classic headline B=4096 S=50 D=25, one lane per tile (256 lanes)", ga[lanes],
                  w.cpu().numpy()[lanes], rv.cpu().numpy()[lanes], oa, ow, orv, trace["margin"])
    allb = bits.cpu().numpy()
    assert ((allb >> ga) & 1).all(), "a pin outside the legal mask"
    assert np.allclose(w.cpu().numpy().sum(1), 1.0, atol=1e-5)
