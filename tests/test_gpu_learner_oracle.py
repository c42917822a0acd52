"""The device learner against the oracle at config (e)'s shape.

One graph-captured ``Learner.train_step`` -- fused bias / LayerNorm epilogues (_DenseLN), the K-step
latent chain as one node (_TrunkChain), im2col convolutions, clip + AdamW in muz_adamw_step -- on a
batch drawn from the device ring (4 players in teams, batch 128, unroll 10, td 50:
train_with_reward.py:327-352) against:
  * oracle/learner.py ``loss_fn`` (the fp32 NumPy restatement of train_with_reward.py:24-146): total and
    every part within 1e-5 relative;
  * oracle/learner_grad.py (float64 restatement of value_and_grad in the reference's step order): every
    parameter gradient, Frobenius-relative error per tensor <= max(1e-3, 3x the deviation of the same
    restatement run in fp32, the reference's own precision; the ADVICE round-2 head-scaling bug was 0.2);
  * oracle/learner.py ``AdamW`` (optax clip_by_global_norm(5) -> adamw restated): applied to the device's own
    gradients, the device's update within 1e-6; applied to the float64 oracle's gradients, the updated
    parameters -- entries off by > 1e-6 may only be where the exact gradient is below 1e-3 of its tensor's
    largest (Adam's first step is lr * sign(g), so fp32 noise flips it on near-zero gradients).
The same for ``StochasticLearner`` against train_stochastic.py:34-199 (classic ring, td 25)."""
import numpy as np
import pytest
import torch

from oracle import learner as OL
from oracle import learner_grad as OG
from tests._parity import log

pytestmark = pytest.mark.gpu

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
    # gradients vs the float64 restatement, with the same restatement in fp32 (the reference's own precision)
    # as the yardstick: the device may deviate from exact arithmetic by no more than the fp32 reference does
    _, _, ref = OG.loss_and_grads(params, b, unroll_steps=K, classic=classic)
    _, _, r32 = OG.loss_and_grads(params, b, unroll_steps=K, classic=classic, dtype=torch.float32)
    dev = {k: p.grad.detach().double().cpu().numpy() for k, p in learner.nets.p.items()}

    def rel(g):     # per tensor: (max-abs error / max |g|, Frobenius error / Frobenius norm)
        return {k: (float(np.abs(g[k] - ref[k]).max()) / max(float(np.abs(ref[k]).max()), 1e-12),
                    float(np.linalg.norm(g[k] - ref[k])) / max(float(np.linalg.norm(ref[k])), 1e-12)) for k in ref}
    gerr, gerr32 = rel(dev), rel({k: v.astype(np.float64) for k, v in r32.items()})
    worst = max(gerr, key=lambda k: gerr[k][0])
    worst_f = max(gerr, key=lambda k: gerr[k][1])
    worst32 = max(gerr32, key=lambda k: gerr32[k][1])
    # one clipped AdamW step: the oracle's update of the float64 / fp32 oracle gradients and of the device's
    f32 = lambda g: {k: v.astype(np.float32) for k, v in g.items()}      # noqa: E731
    ora = OL.AdamW(params).update(params, f32(ref))
    ora32 = OL.AdamW(params).update(params, f32(r32))
    own = OL.AdamW(params).update(params, f32(dev))
    newp = {k: p.detach().cpu().numpy() for k, p in learner.nets.p.items()}
    d_ora = {k: float(np.abs(newp[k] - ora[k]).max()) for k in ora}
    d_own = max(float(np.abs(newp[k] - own[k]).max()) for k in own)
    gnorm = float(np.sqrt(sum(float((v.astype(np.float64) ** 2).sum()) for v in ref.values())))
    n_par = sum(v.size for v in ora.values())
    off = {k: np.abs(newp[k] - ora[k]) > 1e-6 for k in ora}
    n_off = sum(int(m.sum()) for m in off.values())
    n_off32 = sum(int((np.abs(ora32[k] - ora[k]) > 1e-6).sum()) for k in ora)
    # where the updated parameters differ, the exact gradient is small against its tensor (Adam's
    # m / (sqrt(v) + eps) = sign(g) for any |g| >> eps, so fp32 noise on a near-zero g flips the update)
    g_at_off = max([float(np.abs(ref[k][m]).max()) / max(float(np.abs(ref[k]).max()), 1e-30)
                    for k, m in off.items() if m.any()] or [0.0])
    log(f"{name}: loss rel err {lerr:.2e}, parts {perr:.2e}; grads vs float64 (max-abs / Frobenius relative): "
        f"device worst {gerr[worst][0]:.2e} ({worst}) / {gerr[worst_f][1]:.2e} ({worst_f}); fp32 restatement "
        f"Frobenius worst {gerr32[worst32][1]:.2e} ({worst32}); global norm {gnorm:.3f}; one AdamW step vs the "
        f"float64 oracle step: {n_off} of {n_par} entries differ > 1e-6 (fp32 restatement: {n_off32}), max |d| "
        f"{max(d_ora.values()):.2e}, all at |g| <= {g_at_off:.1e} x max|g| of their tensor; optimizer vs oracle "
        f"AdamW of the device grads: {d_own:.2e}")
    assert lerr <= LOSS_TOL and perr <= LOSS_TOL, (lerr, perr)
    for k in ref:     # per tensor, Frobenius: within 1e-3 or 3x the fp32 reference's own deviation
        assert gerr[k][1] <= max(1e-3, 3.0 * gerr32[k][1]), (k, gerr[k], gerr32[k])
    assert d_own <= 1e-6, d_own
    assert g_at_off <= 1e-3, g_at_off


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
    _check("det learner (config e: 4p, batch 128, unroll 10, td 50)", learner, params, ring.sample_batch(),
           classic=False)


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
    _check("classic learner (4p, batch 128, unroll 10, td 25)", learner, params, ring.sample_batch(), classic=True)
