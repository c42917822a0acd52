"""Diagnostic: where do eager and graph-captured learner steps differ?  Runs two eager learners and one
graph learner from identical parameters on the same batches and reports bitwise equality of the loss,
the gradients (after the first backward) and the parameters, per step; then repeats eager with
torch.use_deterministic_algorithms(True)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
from exploring_muzero_on_dog_amd import detmadn as E  # noqa: E402
from exploring_muzero_on_dog_amd import game_agent as GA  # noqa: E402
from exploring_muzero_on_dog_amd import learner as L  # noqa: E402
from exploring_muzero_on_dog_amd import nets as N  # noqa: E402
from exploring_muzero_on_dog_amd import replay as R  # noqa: E402
from oracle import nets as ON  # noqa: E402

C = E.num_channels(2)
params = ON.init_params(C, seed=10)
net = N.DeviceNet(params, C)
eng = GA.SelfPlayEngine(net, 32, num_players=2, max_steps=80, num_simulations=4, max_depth=4)
ring = R.VectorizedReplayBuffer(64, 32, 5, 10, obs_shape=(C, 56), max_episode_length=80, rng=np.random.RandomState(3))
ring.save_games_from_buffers(eng.play(seed=2))
batches = [ring.sample_batch() for _ in range(6)]


def grads_after_backward(lr, b):
    for p in lr.nets.parameters():
        p.grad = None
    loss, _ = L.loss_fn(lr.nets, b, lr.unroll_steps)
    loss.backward()
    return loss.detach().clone(), {k: v.grad.detach().clone() for k, v in lr.nets.p.items()}


def report(tag, a, b):
    la, ga = a
    lb, gb = b
    diff = [k for k in ga if not torch.equal(ga[k], gb[k])]
    print(f"{tag}: loss equal {torch.equal(la, lb)} ({la.item():.9g} vs {lb.item():.9g}); gradients differing in "
          f"{len(diff)} of {len(ga)} tensors: {diff[:8]}")


for det in (False, True):
    torch.use_deterministic_algorithms(det, warn_only=True)
    e1, e2 = L.Learner(params, C, unroll_steps=5), L.Learner(params, C, unroll_steps=5)
    report(f"eager vs eager (deterministic={det})", grads_after_backward(e1, batches[0]),
           grads_after_backward(e2, batches[0]))
torch.use_deterministic_algorithms(False)
for cdet in (False,):
    torch.backends.cudnn.deterministic = cdet
    e1, e2 = L.Learner(params, C, unroll_steps=5), L.Learner(params, C, unroll_steps=5)
    report(f"eager vs eager (cudnn.deterministic={cdet})", grads_after_backward(e1, batches[0]),
           grads_after_backward(e2, batches[0]))
    e1, g1 = L.Learner(params, C, unroll_steps=5), L.Learner(params, C, unroll_steps=5, graph=True)
    for i, b in enumerate(batches):
        le, lg = e1.train_step(b), g1.train_step(b)
        pd = max((e1.nets.p[k] - g1.nets.p[k]).abs().max().item() for k in e1.nets.p)
        dk = [k for k in e1.nets.p if not torch.equal(e1.nets.p[k], g1.nets.p[k])]
        mu = [k for k, a, b in zip(e1.nets.p, e1.opt.mu, g1.opt.mu) if not torch.equal(a, b)]
        print(f"  step {i}: eager loss {float(le['total_loss']):.9g} graph {float(lg['total_loss']):.9g}; "
              f"max |param diff| {pd:.3e} in {dk[:4]}; mu differs in {mu[:4]}; count {e1.opt.count.item()} "
              f"{g1.opt.count.item()}")
    # timing of the graph step at the config (e) batch
    ring2 = R.VectorizedReplayBuffer(64, 128, 10, 50, obs_shape=(C, 56), max_episode_length=80,
                                     rng=np.random.RandomState(5))
    ring2.save_games_from_buffers(eng.play(seed=4))
    g = L.Learner(params, C, unroll_steps=10, graph=True)
    bb = ring2.sample_batch()
    for _ in range(3):
        g.train_step(bb)
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(20):
        g.train_step(bb)
    t1.record()
    t1.synchronize()
    print(f"  graph train step at batch 128 / unroll 10: {t0.elapsed_time(t1) / 20:.2f} ms")
