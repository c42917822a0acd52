"""HIP MFMA network kernels vs the NumPy fp32 restatement of the Flax modules (GPU).

Tolerance: the north star asks for 1e-5 fp32 agreement of policy/value outputs.  The GPU sums
in MFMA k-order, the oracle in BLAS order, so per-layer rounding differs (~1e-7 relative);
outputs (values, logits, rewards, and the 256-d latent, measured |d| <= 8e-7 after its min-max
normalisation) are compared at atol 1e-5."""
import numpy as np
import pytest
import torch

from oracle import detmadn as dm
from oracle import nets as ON
from tests._detmadn_util import random_play_transitions

pytestmark = pytest.mark.gpu

ATOL_OUT = 1e-5
ATOL_LATENT = 1e-5


def _N():
    from exploring_muzero_on_dog_amd import nets as N
    return N


def random_obs(rule_set, n, seed):
    envs = []
    for _, batch in random_play_transitions(rule_set, n, seed, max_plies=400, p_illegal=0.0):
        envs.extend(e for _, e, _, _ in batch)
    rng = np.random.default_rng(seed)
    pick = rng.choice(len(envs), size=min(n, len(envs)), replace=False)
    return np.stack([dm.encode_board(envs[i]) for i in pick]).astype(np.float32), [envs[i] for i in pick]


@pytest.mark.parametrize("rule_set,P", [("selfplay_2p", 2), ("selfplay_4p_teams", 4)])
def test_root_inference(cuda, rule_set, P):
    N = _N()
    C = dm.num_channels(P)
    params = ON.init_params(C, seed=11, randomize_affine=True)
    net = N.DeviceNet(params, C)
    obs, _ = random_obs(rule_set, 61, 3)          # 61: exercises a partial 16-row tile
    lg, v, e = N.root_inference_fn(net, torch.from_numpy(obs).cuda())
    rl, rv, re = ON.root_inference(params, obs)
    torch.cuda.synchronize()
    d_l = np.abs(lg.cpu().numpy() - rl).max()
    d_v = np.abs(v.cpu().numpy() - rv).max()
    d_e = np.abs(e.cpu().numpy() - re).max()
    print(f"root {rule_set}: |dlogits| {d_l:.2e} |dvalue| {d_v:.2e} |dlatent| {d_e:.2e}")
    assert d_e < ATOL_LATENT and d_l < ATOL_OUT and d_v < ATOL_OUT


@pytest.mark.parametrize("seed", [0, 1])
def test_recurrent_inference(cuda, seed):
    N = _N()
    C = dm.num_channels(2)
    params = ON.init_params(C, seed=20 + seed, randomize_affine=True)
    net = N.DeviceNet(params, C)
    rng = np.random.default_rng(seed)
    B = 77
    emb = rng.random((B, 256), dtype=np.float32)
    emb = ((emb - emb.min(1, keepdims=True)) / (emb.max(1, keepdims=True) - emb.min(1, keepdims=True))).astype(np.float32)
    act = rng.integers(-1, 24, B).astype(np.int32)   # -1: jax.nn.one_hot gives a zero row (learner path)
    r, d, lg, v, ne = N.recurrent_inference_fn(net, torch.from_numpy(act).cuda(), torch.from_numpy(emb).cuda())
    rr, rd, rlg, rv, rne = ON.recurrent_inference(params, act, emb)
    torch.cuda.synchronize()
    diffs = {k: float(np.abs(a.cpu().numpy() - b).max()) for k, a, b in
             [("reward", r, rr), ("discount", d, rd), ("logits", lg, rlg), ("value", v, rv), ("latent", ne, rne)]}
    print("recurrent", diffs)
    assert diffs["latent"] < ATOL_LATENT
    for k in ("reward", "discount", "logits", "value"):
        assert diffs[k] < ATOL_OUT, (k, diffs[k])
