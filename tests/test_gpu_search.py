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
from tests._parity import DQ, log, search_parity
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
    # The NumPy networks sum in another order, so every value / reward / discount entering the two trees differs
    # by up to eps (measured here on the root batch and one recurrent step of it, ~1e-6..3e-6); those differences
    # reach the weights through the same Q-rescale gain as the tree arithmetic's ulps.  The allowance is scaled
    # by the MEASURED eps / DQ (logged) instead of a fixed factor; the root value keeps the literal 1e-5.
    glg, gv, ge = N.root_inference_fn(net, torch.from_numpy(obs).cuda())
    acts = np.asarray(a, np.int32)
    gr, gd, _, grv_, _ = N.recurrent_inference_fn(net, torch.from_numpy(acts).cuda(), ge)
    r_, d_, _, v_, _ = ON.recurrent_inference(params, acts, e)
    eps = max(np.abs(gv.cpu().numpy() - v).max(), np.abs(gr.cpu().numpy() - r_).max(),
              np.abs(gd.cpu().numpy() - d_).max(), np.abs(grv_.cpu().numpy() - v_).max())
    factor = max(1.0, float(eps) / DQ)
    log(f"search end-to-end (NumPy nets): measured network deviation eps {eps:.2e} -> allowance factor "
        f"eps / DQ = {factor:.2f} on the gain term and the near-tie bound")
    search_parity("search end-to-end (NumPy nets)", pol.action.cpu().numpy(), pol.action_weights.cpu().numpy(),
                  rv.cpu().numpy(), a, w, orv, trace["margin"] / factor, factor * trace["gain"])


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
