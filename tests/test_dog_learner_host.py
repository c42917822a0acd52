"""The DOG learner (MuZero_DOG/train.py:24-164, whose loss is train_with_reward.py's, on the DOG slice's nets:
RepresentationNetwork with its LayerNorm head, Dyn4 / Pred4 at A = 806) on the CPU host path: the loss against the
fp32 NumPy restatement (oracle/learner.py, generic in the head and the action width) and the gradients against the
float64 restatement (oracle/learner_grad.py).  The device path is tests/test_gpu_dog_learner.py."""
import numpy as np
import torch

from oracle import dog_muzero as DM
from oracle import learner as OL
from oracle import learner_grad as OG


def dog_batch(B=6, K=3, seed=0):
    """A synthetic sample_batch at the DOG shapes: int8-valued observations, actions in [-1, 806), policies on the
    806 actions, reward / discount classes, masks with a no-move step."""
    rng = np.random.default_rng(seed)
    pol = rng.random((B, K + 1, 806)).astype(np.float32)
    pol /= pol.sum(-1, keepdims=True)
    b = {"observations": rng.integers(0, 5, (B, 34, 56)).astype(np.float32),
         "actions": rng.integers(-1, 806, (B, K)).astype(np.int32),
         "rewards": rng.integers(0, 3, (B, K)).astype(np.int32),
         "policies": pol, "values": rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
         "masks": (rng.random((B, K + 1)) > 0.2).astype(np.float32),
         "target_values": rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
         "discount_targets": rng.integers(0, 3, (B, K)).astype(np.int32)}
    return b


def test_dog_learner_loss_and_grads_host():
    import muzpkg
    muzpkg.load()
    from exploring_muzero_on_dog_amd import learner as L
    params = DM.init_params(seed=4, randomize_affine=True)
    b = dog_batch()
    K = b["actions"].shape[1]
    nets = L.DogMuZeroNets(params, device="cpu")
    tb = {k: torch.from_numpy(v) for k, v in b.items()}
    total, parts = L.loss_fn(nets, tb, unroll_steps=K)
    total.backward()
    want, wparts = OL.loss_fn(params, b, unroll_steps=K)
    assert abs(float(total) - want) <= 1e-5 * abs(want), (float(total), want)
    for x, y in zip(parts, wparts):
        assert abs(float(x) - y) <= 1e-5 * max(abs(y), 1e-3), (float(x), y)
    t64, _, ref = OG.loss_and_grads(params, b, unroll_steps=K)
    assert abs(t64 - want) <= 1e-5 * abs(want)
    # gradients on the rows without a decision within 1e-6 of its threshold (tests/test_gpu_learner_oracle.py: a
    # ReLU input at its kink sends a whole gradient element one way or the other; here batch row 3's is 6.6e-7 off)
    dist, _ = OG.decision_margins(params, b, unroll_steps=K)
    keep = np.flatnonzero(dist >= 1e-6)
    assert 0 < len(keep) < len(dist)
    b = {k: v[keep] for k, v in b.items()}
    nets = L.DogMuZeroNets(params, device="cpu")
    total, _ = L.loss_fn(nets, {k: torch.from_numpy(v) for k, v in b.items()}, unroll_steps=K)
    total.backward()
    _, _, ref = OG.loss_and_grads(params, b, unroll_steps=K)
    for k, p in nets.p.items():
        g = p.grad.double().numpy()
        err = np.linalg.norm(g - ref[k]) / max(np.linalg.norm(ref[k]), 1e-12)
        assert err < 1e-4, (k, err)
    assert "representation/LayerNorm_7/scale" in nets.p and nets.p["dynamics/Dense_0/kernel"].shape[0] == 806
