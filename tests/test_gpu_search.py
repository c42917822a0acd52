"""Persistent Gumbel-search kernel vs the NumPy restatement of mctx 0.0.6 (GPU).

Two levels:
  * search logic: the oracle search is driven by the GPU's own recurrent_inference kernel, so both
    sides see identical network outputs and only the tree arithmetic is compared;
  * end to end: the oracle uses its own NumPy networks (fp32, different summation order).
Parity vs mctx itself is unpinned (mctx is not vendored in the reference)."""
import numpy as np
import pytest
import torch

from oracle import detmadn as dm
from oracle import mctx_gumbel as G
from oracle import nets as ON
from tests._parity import search_parity
from tests.test_gpu_nets import random_obs

pytestmark = pytest.mark.gpu


def _mods():
    from exploring_muzero_on_dog_amd import mcts as M
    from exploring_muzero_on_dog_amd import nets as N
    return N, M


def setup(P, B, seed, rule_set):
    N, M = _mods()
    C = dm.num_channels(P)
    params = ON.init_params(C, seed=seed, randomize_affine=True)
    net = N.DeviceNet(params, C)
    obs, envs = random_obs(rule_set, B, seed + 5)
    valid = np.stack([dm.valid_action(e).flatten() for e in envs])
    keep = valid.any(1)
    obs, valid = obs[keep], valid[keep]
    bits = (valid.astype(np.int64) << np.arange(24)).sum(1).astype(np.int32)
    return N, M, params, net, obs, valid, bits


def gpu_recurrent_fn(N, net):
    def fn(params, action, emb):
        r, d, lg, v, ne = N.recurrent_inference_fn(net, torch.from_numpy(np.asarray(action, np.int32)).cuda(),
                                                   torch.from_numpy(np.ascontiguousarray(emb)).cuda())
        return r.cpu().numpy(), d.cpu().numpy(), lg.cpu().numpy(), v.cpu().numpy(), ne.cpu().numpy()
    return fn


@pytest.mark.parametrize("P,S,D,rule_set", [(2, 50, 25, "selfplay_2p"), (4, 16, 4, "selfplay_4p_teams"),
                                            (2, 8, 50, "selfplay_2p"),
                                            (4, 100, 50, "selfplay_4p_teams")])   # config (e)'s search shape
def test_search_logic_matches_mctx_restatement(cuda, P, S, D, rule_set):
    N, M, params, net, obs, valid, bits = setup(P, 48, 7, rule_set)
    B = obs.shape[0]
    lg, v, e = N.root_inference_fn(net, torch.from_numpy(obs).cuda())
    gum = np.random.default_rng(3).gumbel(size=(B, 24)).astype(np.float32)
    pol, rv = M.gumbel_muzero_policy(net, lg, v, e, torch.from_numpy(bits), S, D, 1.0,
                                     gumbel=torch.from_numpy(gum))
    trace = {}
    a, w, orv, tree = G.gumbel_muzero_policy(params, lg.cpu().numpy(), v.cpu().numpy(), e.cpu().numpy(),
                                             gpu_recurrent_fn(N, net), S, ~valid, gum, max_depth=D, trace=trace)
    torch.cuda.synchronize()
    ga, gw, grv = pol.action.cpu().numpy(), pol.action_weights.cpu().numpy(), rv.cpu().numpy()
    search_parity(f"search logic P{P} S{S} D{D}", ga, gw, grv, a, w, orv, trace["margin"], trace["gain"])
    assert valid[np.arange(B), ga].all(), "search picked an invalid root action"


def test_search_end_to_end_vs_numpy_networks(cuda):
    N, M, params, net, obs, valid, bits = setup(2, 32, 9, "selfplay_2p")
    B = obs.shape[0]
    gum = np.random.default_rng(4).gumbel(size=(B, 24)).astype(np.float32)
    pol, rv = M.muzero_mcts(net, torch.from_numpy(obs).cuda(), torch.from_numpy(bits), 50, 25, 1.0,
                                gumbel=torch.from_numpy(gum))
    lg, v, e = ON.root_inference(params, obs)
    trace = {}
    a, w, orv, _ = G.gumbel_muzero_policy(params, lg, v, e, ON.recurrent_inference, 50, ~valid, gum, max_depth=25,
                                          trace=trace)
    torch.cuda.synchronize()
    # the NumPy networks sum in another order (|d logits|, |d values| ~3e-6 = ~6 DQ, tests/test_gpu_nets.py):
    # decisions count as near-ties within 50x the tree-arithmetic bound, weights get 10x its gain term; the
    # root value and the weights' base tolerance are the north star's 1e-5 (measured: max|dv| 1.2e-7)
    search_parity("search end-to-end (NumPy nets)", pol.action.cpu().numpy(), pol.action_weights.cpu().numpy(),
                  rv.cpu().numpy(), a, w, orv, trace["margin"], 10 * trace["gain"], tie=50.0)


def test_device_noise_is_deterministic_and_valid(cuda):
    N, M, params, net, obs, valid, bits = setup(2, 40, 5, "selfplay_2p")
    t = torch.from_numpy(obs).cuda()
    p1, v1 = M.muzero_mcts(net, t, torch.from_numpy(bits), 16, 8, 1.0, seed=123, turn=7)
    p2, v2 = M.muzero_mcts(net, t, torch.from_numpy(bits), 16, 8, 1.0, seed=123, turn=7)
    assert torch.equal(p1.action, p2.action) and torch.equal(v1, v2)
    ga = p1.action.cpu().numpy()
    assert valid[np.arange(len(ga)), ga].all()
    w = p1.action_weights.cpu().numpy()
    assert np.allclose(w.sum(1), 1.0, atol=1e-5) and (w[~valid] < 1e-30).all()
