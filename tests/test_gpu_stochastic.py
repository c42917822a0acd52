"""Stochastic MuZero (classic MADN) on the GPU vs the NumPy restatements (GPU).

* networks: root_inference_fn / decision_recurrent_fn / chance_recurrent_fn vs oracle/classic_nets.py
  (atol 1e-5 on logits / values / rewards / discounts, 2e-5 on the min-max normalised 256-d states,
  the tolerances of tests/test_gpu_nets.py);
* search logic: the oracle search (oracle/mctx_stochastic.py) is driven by the GPU's own recurrent
  kernels, so both trees see identical network outputs; root noise and the final Gumbel draws are
  explicit inputs on both sides, the tie-break uniforms come from the same counter RNG.
Parity vs mctx itself is unpinned (mctx is not vendored in the reference)."""
import numpy as np
import pytest
import torch

from oracle import classic_madn as cm
from oracle import classic_nets as CN
from oracle import mctx_stochastic as MS

from tests._parity import search_parity  # noqa: E402

pytestmark = pytest.mark.gpu

ATOL_OUT = 1e-5
ATOL_LATENT = 2e-5


def _S():
    from exploring_muzero_on_dog_amd import stochastic as S
    return S


def random_classic_states(n, seed, P=4):
    """Observations + envs from seeded random classic self-play (rules of game_agent_stochastic.py)."""
    rng = np.random.default_rng(seed)
    envs = [cm.env_reset(num_players=P, **cm.SELFPLAY_RULES) for _ in range(n)]
    out = []
    for ply in range(int(rng.integers(20, 160))):
        nxt = []
        for e in envs:
            if e.done:
                nxt.append(e)
                continue
            e = cm.throw_die(e, float(rng.random()))
            out.append(e)
            va = cm.valid_action(e)
            e = cm.env_step(e, int(rng.choice(np.flatnonzero(va))))[0] if va.any() else cm.no_step(e)[0]
            nxt.append(e)
        envs = nxt
    pick = rng.choice(len(out), size=min(n, len(out)), replace=False)
    sel = [out[i] for i in pick]
    return np.stack([cm.encode_board(e) for e in sel]).astype(np.float32), sel


def test_classic_networks(cuda):
    S = _S()
    C = cm.num_channels(4)
    params = CN.init_params(C, seed=5, randomize_affine=True)
    net = S.DeviceClassicNet(params, C)
    obs, _ = random_classic_states(61, 1)
    lg, v, e = S.root_inference_fn(net, torch.from_numpy(obs).cuda())
    rl, rv, re = CN.root_inference(params, obs)
    assert np.abs(lg.cpu().numpy() - rl).max() < ATOL_OUT
    assert np.abs(v.cpu().numpy() - rv).max() < ATOL_OUT
    assert np.abs(e.cpu().numpy() - re).max() < ATOL_LATENT
    B = re.shape[0]
    rng = np.random.default_rng(2)
    act = rng.integers(-1, 5, B).astype(np.int32)          # includes out-of-range actions (zero one-hot)
    cl, av, after, r, d = S.decision_recurrent_fn(net, torch.from_numpy(act).cuda(), torch.from_numpy(re).cuda())
    ocl, oav, oafter, orr, od = CN.decision_recurrent(params, act, re)
    diffs = {"chance_logits": np.abs(cl.cpu().numpy() - ocl).max(), "afterstate_value": np.abs(av.cpu().numpy() - oav).max(),
             "reward": np.abs(r.cpu().numpy() - orr).max(), "discount": np.abs(d.cpu().numpy() - od).max(),
             "afterstate": np.abs(after.cpu().numpy() - oafter).max()}
    print("decision", {k: f"{v:.2e}" for k, v in diffs.items()})
    assert max(diffs[k] for k in diffs if k != "afterstate") < ATOL_OUT and diffs["afterstate"] < ATOL_LATENT
    ch = rng.integers(-1, 7, B).astype(np.int32)
    lg2, v2, nx = S.chance_recurrent_fn(net, torch.from_numpy(ch).cuda(), torch.from_numpy(oafter).cuda())
    olg2, ov2, onx = CN.chance_recurrent(params, ch, oafter)
    print(f"chance |dlogits| {np.abs(lg2.cpu().numpy() - olg2).max():.2e} |dnext| {np.abs(nx.cpu().numpy() - onx).max():.2e}")
    assert np.abs(lg2.cpu().numpy() - olg2).max() < ATOL_OUT
    assert np.abs(v2.cpu().numpy() - ov2).max() < ATOL_OUT
    assert np.abs(nx.cpu().numpy() - onx).max() < ATOL_LATENT


def gpu_fns(S, net):
    def dec(params, action, emb):
        out = S.decision_recurrent_fn(net, torch.from_numpy(np.asarray(action, np.int32)).cuda(),
                                      torch.from_numpy(np.ascontiguousarray(emb)).cuda())
        return tuple(t.cpu().numpy() for t in out)

    def cha(params, chance, after):
        out = S.chance_recurrent_fn(net, torch.from_numpy(np.asarray(chance, np.int32)).cuda(),
                                    torch.from_numpy(np.ascontiguousarray(after)).cuda())
        return tuple(t.cpu().numpy() for t in out)
    return dec, cha


@pytest.mark.parametrize("Ssim,D,temp", [(16, 8, 1.0), (50, 25, 0.6), (8, 3, 2.0)])
def test_stochastic_search_logic(cuda, Ssim, D, temp):
    S = _S()
    C = cm.num_channels(4)
    params = CN.init_params(C, seed=9, randomize_affine=True)
    net = S.DeviceClassicNet(params, C)
    obs, envs = random_classic_states(48, 4)
    valid = np.stack([cm.valid_action(e) for e in envs])
    keep = valid.any(1)
    obs, valid = obs[keep], valid[keep]
    B = obs.shape[0]
    bits = (valid.astype(np.int64) << np.arange(4)).sum(1).astype(np.int32)
    lg, v, e = S.root_inference_fn(net, torch.from_numpy(obs).cuda())
    rng = np.random.default_rng(3)
    dirichlet = rng.dirichlet(np.full(4, 0.3), B).astype(np.float32)
    gumbel = rng.gumbel(size=(B, 4)).astype(np.float32)
    seed, turn = 1234, 7
    act, w, rv = S.stochastic_muzero_policy(net, lg, v, e, torch.from_numpy(bits), Ssim, D, temp, seed=seed, turn=turn,
                                            dirichlet=torch.from_numpy(dirichlet), gumbel=torch.from_numpy(gumbel))
    dec, cha = gpu_fns(S, net)
    trace = {}
    oa, ow, orv, _ = MS.stochastic_muzero_policy(params, lg.cpu().numpy(), v.cpu().numpy(), e.cpu().numpy(), dec, cha,
                                                 Ssim, ~valid, dirichlet, gumbel, max_depth=D, temperature=temp,
                                                 seed=seed, turn=turn, trace=trace)
    torch.cuda.synchronize()
    ga, gw, grv = act.cpu().numpy(), w.cpu().numpy(), rv.cpu().numpy()
    search_parity(f"stochastic search S{Ssim} D{D} T{temp}", ga, gw, grv, oa, ow, orv, trace["margin"])
    assert valid[np.arange(B), ga].all(), "search picked an illegal pin"
    assert np.allclose(gw.sum(1), 1.0, atol=1e-6)


def test_stochastic_search_device_rng(cuda):
    """Device Dirichlet (Gamma sampler) and Gumbel streams: legal actions, proper visit distributions,
    deterministic for a fixed seed, different for another."""
    S = _S()
    C = cm.num_channels(4)
    net = S.DeviceClassicNet(CN.init_params(C, seed=1), C)
    obs, envs = random_classic_states(64, 8)
    valid = np.stack([cm.valid_action(e) for e in envs])
    keep = valid.any(1)
    obs, valid = obs[keep], valid[keep]
    bits = torch.from_numpy((valid.astype(np.int64) << np.arange(4)).sum(1).astype(np.int32))
    o = torch.from_numpy(obs).cuda()
    a1, w1, _ = S.stochastic_muzero_mcts(net, o, bits, 32, 10, 1.0, seed=5)
    a2, w2, _ = S.stochastic_muzero_mcts(net, o, bits, 32, 10, 1.0, seed=5)
    a3, w3, _ = S.stochastic_muzero_mcts(net, o, bits, 32, 10, 1.0, seed=6)
    torch.cuda.synchronize()
    assert torch.equal(a1, a2) and torch.equal(w1, w2)
    assert not torch.equal(w1, w3)
    ga = a1.cpu().numpy()
    assert valid[np.arange(len(ga)), ga].all()
    assert np.allclose(w1.cpu().numpy().sum(1), 1.0, atol=1e-6)
