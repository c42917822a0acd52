"""Learner gradients (CPU, float64) against oracle/learner_grad.py, the reference's loss_fn /
loss_fn_stochastic restated step by step (train_with_reward.py:24-146, train_stochastic.py:34-181).

Every weight is nonzero (the dynamics heads included), so the check covers where the 0.5 gradient scaling of
the carried latent applies: the det reward / discount heads read the UNSCALED next latent inside
dynamics_net (muzero_deterministic_madn.py:437-455), only the latent carried to the next step is scaled."""
import numpy as np
import torch

from oracle import learner_grad as OG
from oracle import nets as ON


def _L():
    import muzpkg
    muzpkg.load()
    from exploring_muzero_on_dog_amd import learner as L
    return L


def _batch(B, K, C, A=24, seed=0):
    rng = np.random.default_rng(seed)
    pol = rng.random((B, K + 1, A)).astype(np.float32)
    pol /= pol.sum(-1, keepdims=True)
    return {"observations": rng.integers(0, 3, (B, C, 56)).astype(np.float32),
            "actions": rng.integers(-1, A, (B, K)).astype(np.int32),
            "rewards": rng.choice([0, 1, 1, 1, 2], (B, K)).astype(np.int32),
            "policies": pol, "masks": (rng.random((B, K + 1)) < 0.85).astype(np.float32),
            "target_values": rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
            "discount_targets": rng.choice([0, 1, 2, 2, 0], (B, K)).astype(np.int32)}


def _torch_batch(b):
    return {k: (torch.from_numpy(v).double() if v.dtype == np.float32 else torch.from_numpy(v)) for k, v in b.items()}


def _compare(grads, ref, what, tol=1e-9):
    worst = ("", 0.0)
    for k, g in grads.items():
        r = ref[k]
        err = float(np.abs(g - r).max()) / max(float(np.abs(r).max()), 1e-12)
        if err > worst[1]:
            worst = (k, err)
    assert worst[1] <= tol, f"{what}: {worst[0]} relative gradient error {worst[1]:.2e}"


def test_det_gradients_match_reference_step_order():
    L = _L()
    C, K = 18, 4
    params = ON.init_params(C, seed=21, randomize_affine=True)
    b = _batch(10, K, C, seed=4)
    tot, parts, ref = OG.loss_and_grads(params, b, unroll_steps=K)
    nets = L.MuZeroNets(params, C, device="cpu", dtype=torch.float64)
    loss, lparts = L.loss_fn(nets, _torch_batch(b), unroll_steps=K)
    loss.backward()
    assert abs(float(loss) - tot) <= 1e-12 * abs(tot)
    for x, y in zip(lparts, parts):
        assert abs(float(x) - y) <= 1e-12 * max(abs(y), 1.0)
    _compare({k: p.grad.numpy() for k, p in nets.p.items()}, ref, "det")


def test_det_oracle_forward_matches_numpy_oracle():
    """The float64 autograd restatement and the fp32 NumPy restatement (oracle/learner.py) compute the same
    losses (1e-5 relative: fp32 vs float64 forward)."""
    from oracle import learner as OL
    C, K = 18, 3
    params = ON.init_params(C, seed=22, randomize_affine=True)
    b = _batch(8, K, C, seed=5)
    tot, parts, _ = OG.loss_and_grads(params, b, unroll_steps=K)
    wt, wparts = OL.loss_fn(params, b, unroll_steps=K)
    assert abs(tot - wt) <= 1e-5 * abs(wt)
    for x, y in zip(parts, wparts):
        assert abs(x - y) <= 1e-5 * max(abs(y), 1e-3)


def test_classic_gradients_match_reference_step_order():
    L = _L()
    from oracle import classic_nets as CN
    C, K, B = 11, 4, 10
    params = CN.init_params(C, seed=23, randomize_affine=True)
    rng = np.random.default_rng(6)
    b = _batch(B, K, C, A=4, seed=6)
    b["dice_outcomes"] = rng.integers(0, 6, (B, K)).astype(np.int32)
    pr = rng.random((B, K, 6)).astype(np.float32)
    pr[::2] = 1.0
    b["dice_probs"] = (pr / pr.sum(-1, keepdims=True)).astype(np.float32)
    tot, parts, ref = OG.loss_and_grads(params, b, unroll_steps=K, classic=True)
    nets = L.ClassicMuZeroNets(params, C, device="cpu", dtype=torch.float64)
    loss, lparts = L.loss_fn_stochastic(nets, _torch_batch(b), unroll_steps=K)
    loss.backward()
    assert abs(float(loss) - tot) <= 1e-12 * abs(tot)
    _compare({k: p.grad.numpy() for k, p in nets.p.items()}, ref, "classic")


def test_minmax_gradient_splits_ties():
    """jnp.min / jnp.max split the gradient evenly over tied entries (JAX's reduce-chooser JVP); the learner's
    min-max scaling must too."""
    L = _L()
    x = torch.tensor([[0.5, -1.0, 2.0, -1.0, 2.0, 0.25]], dtype=torch.float64, requires_grad=True)
    w = torch.tensor([[0.3, -0.7, 1.1, 0.2, -0.4, 0.9]], dtype=torch.float64)
    (g1,) = torch.autograd.grad((L.MuZeroNets._minmax(x) * w).sum(), x)
    xo = x.detach().clone().requires_grad_(True)
    (g2,) = torch.autograd.grad((OG._Net.minmax(xo) * w).sum(), xo)
    assert torch.allclose(g1, g2, rtol=1e-12, atol=1e-15)
    den = float(x[0, 2] - x[0, 1]) + 1e-8
    # both tied minima (columns 1, 3) carry the same share of the min's gradient on top of their own w / den
    assert abs(float(g2[0, 1] - w[0, 1] / den) - float(g2[0, 3] - w[0, 3] / den)) < 1e-12
    assert abs(float(g2[0, 2] - w[0, 2] / den) - float(g2[0, 4] - w[0, 4] / den)) < 1e-12
