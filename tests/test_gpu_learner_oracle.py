"""The device learner against the oracle at config (e)'s shape.

One graph-captured ``Learner.train_step`` -- fused bias / LayerNorm epilogues (_DenseLN), the K-step
latent chain as one node (_TrunkChain), im2col convolutions, clip + AdamW in muz_adamw_step -- on a
batch drawn from the device ring (4 players in teams, batch 128, unroll 10, td 50:
train_with_reward.py:327-352) against:
  * oracle/learner.py ``loss_fn`` (the fp32 NumPy restatement of train_with_reward.py:24-146): total and
    every part within 1e-5 relative;
  * oracle/learner_grad.py (float64 restatement of value_and_grad in the reference's step order): every
    parameter gradient;
  * oracle/learner.py ``AdamW`` (optax clip_by_global_norm(5) -> adamw restated): applied to the oracle's
    gradients, the updated parameters; applied to the device's own gradients, the device's update.
The same for ``StochasticLearner`` against train_stochastic.py:34-199 (classic ring, td 25)."""
import numpy as np
import pytest
import torch

from oracle import learner as OL
from oracle import learner_grad as OG
from tests._parity import log

pytestmark = pytest.mark.gpu

GRAD_TOL = 1e-4      # max |g_dev - g_f64| / max |g_f64| per tensor (fp32 through an 11-step unroll)
LOSS_TOL = 1e-5


def _np_batch(batch):
    return {k: v.detach().cpu().numpy() for k, v in batch.items()}


def _check(name, learner, params, batch, classic):
    K = learner.unroll_steps
    b = _np_batch(batch)
    out = learner.train_step(batch)
    torch.cuda.synchronize()
    # losses vs the fp32 NumPy restatement
    if classic:
        wt, wparts = OL.loss_fn_stochastic(params, b, unroll_steps=K)
        keys = ("v_loss", "p_loss", "c_loss", "d_loss", "r_loss")
    else:
        wt, wparts = OL.loss_fn(params, b, unroll_steps=K)
        keys = ("v_loss", "p_loss", "d_loss", "r_loss")
    lerr = abs(float(out["total_loss"]) - wt) / abs(wt)
    perr = max(abs(float(out[k]) - y) / max(abs(y), 1e-3) for k, y in zip(keys, wparts))
    # gradients vs the float64 restatement
    _, _, ref = OG.loss_and_grads(params, b, unroll_steps=K, classic=classic)
    dev = {k: p.grad.detach().double().cpu().numpy() for k, p in learner.nets.p.items()}
    gerr = {k: float(np.abs(dev[k] - ref[k]).max()) / max(float(np.abs(ref[k]).max()), 1e-12) for k in ref}
    worst = max(gerr, key=gerr.get)
    # one clipped AdamW step: the oracle's update of the oracle's gradients, and of the device's gradients
    ora = OL.AdamW(params).update(params, {k: v.astype(np.float32) for k, v in ref.items()})
    own = OL.AdamW(params).update(params, {k: v.astype(np.float32) for k, v in dev.items()})
    newp = {k: p.detach().cpu().numpy() for k, p in learner.nets.p.items()}
    d_ora = {k: float(np.abs(newp[k] - ora[k]).max()) for k in ora}
    d_own = max(float(np.abs(newp[k] - own[k]).max()) for k in own)
    gnorm = float(np.sqrt(sum(float((v.astype(np.float64) ** 2).sum()) for v in ref.values())))
    n_par = sum(v.size for v in ora.values())
    n_off = sum(int((np.abs(newp[k] - ora[k]) > 1e-6).sum()) for k in ora)
    log(f"{name}: loss rel err {lerr:.2e}, parts {perr:.2e}; grads max rel err {gerr[worst]:.2e} ({worst}), "
        f"global norm {gnorm:.3f}; params after one AdamW step vs oracle step: max |d| {max(d_ora.values()):.2e} "
        f"({n_off} of {n_par} entries > 1e-6); vs oracle AdamW of the device grads: {d_own:.2e}")
    assert lerr <= LOSS_TOL and perr <= LOSS_TOL, (lerr, perr)
    assert gerr[worst] <= GRAD_TOL, (worst, gerr[worst])
    assert d_own <= 1e-6, d_own
    return d_ora, n_off


def test_det_learner_step_matches_oracle_config_e(cuda):
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import learner as L
    from exploring_muzero_on_dog_amd import nets as N
    from exploring_muzero_on_dog_amd import replay as R
    from oracle import nets as ON
    P, T = 4, 550
    C = E.num_channels(P)
    params = ON.init_params(C, seed=31, randomize_affine=True)
    net = N.DeviceNet(params, C)
    eng = GA.SelfPlayEngine(net, 64, num_players=P, max_steps=T, num_simulations=4, max_depth=4)
    ring = R.VectorizedReplayBuffer(20000, 128, 10, 50, obs_shape=(C, 56), max_episode_length=T,
                                    rng=np.random.RandomState(5))
    ring.save_games_from_buffers(eng.play_stream(96, seed=2, temperature=1.0))
    learner = L.Learner(params, C, unroll_steps=10, graph=True)
    d_ora, n_off = _check("det learner (config e: 4p, batch 128, unroll 10, td 50)", learner, params,
                          ring.sample_batch(), classic=False)
    assert max(d_ora.values()) <= 1e-5 and n_off <= 1e-4 * sum(p.numel() for p in learner.nets.p.values())


def test_classic_learner_step_matches_oracle(cuda):
    from exploring_muzero_on_dog_amd import classic as CL
    from exploring_muzero_on_dog_amd import game_agent_stochastic as GS
    from exploring_muzero_on_dog_amd import learner as L
    from exploring_muzero_on_dog_amd import replay as R
    from exploring_muzero_on_dog_amd import stochastic as S
    from oracle import classic_nets as CN
    C, T = CL.num_channels(4), 800
    params = CN.init_params(C, seed=32, randomize_affine=True)
    net = S.DeviceClassicNet(params, C)
    eng = GS.StochasticSelfPlayEngine(net, 64, max_steps=T, num_simulations=4, max_depth=4)
    ring = R.VectorizedReplayBufferStochastic(20000, 128, 10, 25, obs_shape=(C, 56), max_episode_length=T,
                                              rng=np.random.RandomState(6))
    ring.save_games_from_buffers(eng.play_stream(96, seed=3))
    learner = L.StochasticLearner(params, C, unroll_steps=10, graph=True)
    d_ora, n_off = _check("classic learner (4p, batch 128, unroll 10, td 25)", learner, params,
                          ring.sample_batch(), classic=True)
    assert max(d_ora.values()) <= 1e-5 and n_off <= 1e-4 * sum(p.numel() for p in learner.nets.p.values())
