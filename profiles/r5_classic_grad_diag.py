"""Round-5 diagnosis of the classic learner's gradient error.

Builds test_gpu_learner_oracle.py::test_classic_learner_step_matches_oracle's batch once, computes the float64
restatement's gradients once, then runs one eager StochasticLearner step per switch setting of learner.py
(CHAIN_KERNEL, RESBLOCK_STACK, RESBLOCK_NODE, FUSED_HEADS, FUSED_LOSS, GROUPED_GRADS) and logs, per setting, the
worst per-tensor max-abs / Frobenius relative error and the 5 worst tensors.  Test infrastructure (imports oracle/).

usage: python profiles/r5_classic_grad_diag.py [det]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import muzpkg  # noqa: E402

muzpkg.load()
from exploring_muzero_on_dog_amd import learner as L  # noqa: E402
from oracle import learner_grad as OG  # noqa: E402

SWITCHES = ("CHAIN_KERNEL", "RESBLOCK_STACK", "RESBLOCK_NODE", "FUSED_HEADS", "FUSED_LOSS", "GROUPED_GRADS",
            "FUSED_BWD", "FUSED_BOUNDARY", "FUSED_FILM")
ROUND4 = ("CHAIN_KERNEL", "RESBLOCK_STACK", "RESBLOCK_NODE", "FUSED_HEADS")


def classic_setup():
    from exploring_muzero_on_dog_amd import classic as CL
    from exploring_muzero_on_dog_amd import game_agent_stochastic as GS
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
    return params, C, ring.sample_batch(), (lambda: L.StochasticLearner(params, C, unroll_steps=10, graph=False))


def det_setup():
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import game_agent as GA
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
    return params, C, ring.sample_batch(), (lambda: L.Learner(params, C, unroll_steps=10, graph=False))


def main():
    det = len(sys.argv) > 1 and sys.argv[1] == "det"
    params, C, batch, make = det_setup() if det else classic_setup()
    b = {k: v.detach().cpu().numpy() for k, v in batch.items()}
    _, _, ref = OG.loss_and_grads(params, b, unroll_steps=10, classic=not det)
    _, _, r32 = OG.loss_and_grads(params, b, unroll_steps=10, classic=not det, dtype=torch.float32)

    def rel(g):
        return {k: (float(np.abs(g[k] - ref[k]).max()) / max(float(np.abs(ref[k]).max()), 1e-12),
                    float(np.linalg.norm(g[k] - ref[k])) / max(float(np.linalg.norm(ref[k])), 1e-12)) for k in ref}

    e32 = rel({k: v.astype(np.float64) for k, v in r32.items()})
    w32 = max(e32, key=lambda k: e32[k][1])
    print(f"{'det' if det else 'classic'}: fp32 restatement Frobenius worst {e32[w32][1]:.2e} ({w32})", flush=True)
    default = {s: getattr(L, s) for s in SWITCHES}
    off = lambda *names: (" + ".join(names) + " off", {n: False for n in names})   # noqa: E731
    settings = [("default", {})] + [off(s) for s in SWITCHES] + \
        [off("RESBLOCK_STACK", "RESBLOCK_NODE"), off("CHAIN_KERNEL", "RESBLOCK_STACK", "RESBLOCK_NODE"),
         off(*ROUND4), off(*SWITCHES)]
    for label, over in settings:
        for s in SWITCHES:
            setattr(L, s, over.get(s, default[s]))
        torch.manual_seed(0)
        learner = make()
        learner.train_step(batch)
        torch.cuda.synchronize()
        dev = {k: p.grad.detach().double().cpu().numpy() for k, p in learner.nets.p.items()}
        e = rel(dev)
        worst = sorted(e, key=lambda k: -e[k][1])[:5]
        wm = max(e, key=lambda k: e[k][0])
        ratio = max(e[k][1] / max(3.0 * e32[k][1], 1e-30) for k in e)
        print(f"[{label}] worst max-abs {e[wm][0]:.2e} ({wm}); Frobenius top5: " +
              ", ".join(f"{k} {e[k][1]:.2e} (fp32 {e32[k][1]:.1e})" for k in worst) +
              f"; max Frobenius / (3 x fp32) {ratio:.2f}", flush=True)
        del learner
    for s in SWITCHES:
        setattr(L, s, default[s])


if __name__ == "__main__":
    main()
