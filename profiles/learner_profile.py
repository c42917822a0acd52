"""Config (e) learner step, split: ring.sample_batch alone, train_step alone on a fixed batch (HIP graph
replay), and both together, at batch 128 / unroll 10 / td 50 (train_with_reward.py).  The ring is filled
by a short self-play run (content does not change the step's cost).

    python profiles/learner_profile.py [steps]
    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_learner -- python3 profiles/learner_profile.py 20
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import detmadn as E, game_agent as GA, learner as L, nets as N, replay as R  # noqa

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
C = E.num_channels(4)
params = N.init_muzero_params(0, C)
net = N.DeviceNet(params, C)
eng = GA.SelfPlayEngine(net, 256, num_players=4, max_steps=550, num_simulations=8, max_depth=8)
ring = R.VectorizedReplayBuffer(20000, 128, 10, 50, obs_shape=(C, 56), max_episode_length=550,
                                rng=np.random.RandomState(0))
buf = eng.play_stream(512, seed=1)
ring.save_games_from_buffers(buf)
torch.cuda.synchronize()


def timed(label, fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    ms = (time.time() - t) / steps * 1000
    print(f"{label}: {ms:.3f} ms", flush=True)
    return ms


batch = ring.sample_batch()
# the dynamics chain as the per-layer launch train (round 3) instead of csrc/learner_chain.hip's two launches
L.CHAIN_KERNEL = False
lr0 = L.Learner(params, C, unroll_steps=10, graph=True)
timed("train_step (graph replay, fixed batch, chain kernel off)", lambda: lr0.train_step(batch))
L.CHAIN_KERNEL = True
del lr0
L.RESBLOCK_STACK = False
lr0 = L.Learner(params, C, unroll_steps=10, graph=True)
timed("train_step (graph replay, fixed batch, ResBlock stack kernel off)", lambda: lr0.train_step(batch))
L.RESBLOCK_NODE = False
lr0 = L.Learner(params, C, unroll_steps=10, graph=True)
timed("train_step (graph replay, fixed batch, ResBlock stack kernel and node off)", lambda: lr0.train_step(batch))
L.RESBLOCK_NODE = L.RESBLOCK_STACK = True
del lr0
L.FUSED_HEADS = False
lr0 = L.Learner(params, C, unroll_steps=10, graph=True)
timed("train_step (graph replay, fixed batch, fused output heads off)", lambda: lr0.train_step(batch))
L.FUSED_HEADS = True
del lr0
lr = L.Learner(params, C, unroll_steps=10, graph=True)
timed("sample_batch", ring.sample_batch)
timed("train_step (graph replay, fixed batch)", lambda: lr.train_step(batch))
timed("sample_batch + train_step", lambda: lr.train_step(ring.sample_batch()))

if os.environ.get("MUZ_PROFILE_DET_ONLY"):      # (for a kernel trace of the det step alone)
    sys.exit(0)

# classic (train_stochastic.py) step at the same batch / unroll / td, chain node on and off
from exploring_muzero_on_dog_amd import classic as CL, game_agent_stochastic as GS, stochastic as S  # noqa: E402
Cc = CL.num_channels(4)
cparams = S.init_classic_params(Cc, 0)
ceng = GS.StochasticSelfPlayEngine(S.DeviceClassicNet(cparams, Cc), 256, max_steps=550, num_simulations=8, max_depth=8)
cring = R.VectorizedReplayBufferStochastic(20000, 128, 10, 50, obs_shape=(Cc, 56), max_episode_length=550,
                                           rng=np.random.RandomState(0))
cring.save_games_from_buffers(ceng.play_stream(512, seed=1))
cbatch = cring.sample_batch()
for chain in (True,):   # (CHAIN = False, the per-step graph, records shared weights twice into a GradSink)
    L.CHAIN = chain
    for graph in (True, False):
        clr = L.StochasticLearner(cparams, Cc, unroll_steps=10, graph=graph)
        timed(f"classic train_step ({'graph replay' if graph else 'eager'}, chain node {'on' if chain else 'off'})",
              lambda: clr.train_step(cbatch))
    lr_d = L.Learner(params, C, unroll_steps=10, graph=True)
    timed(f"det train_step (graph replay, chain node {'on' if chain else 'off'})", lambda: lr_d.train_step(batch))
L.CHAIN = True
L.CHAIN_KERNEL = False
clr = L.StochasticLearner(cparams, Cc, unroll_steps=10, graph=True)
timed("classic train_step (graph replay, chain node on, chain kernel off)", lambda: clr.train_step(cbatch))
L.CHAIN_KERNEL = True

if len(sys.argv) > 2:   # also time with the other BLAS backend (rocBLAS vs hipBLASLt)
    torch.backends.cuda.preferred_blas_library(sys.argv[2])
    lr2 = L.Learner(params, C, unroll_steps=10, graph=True)
    timed(f"train_step (graph replay, fixed batch, blas={sys.argv[2]})", lambda: lr2.train_step(batch))
    lr3 = L.Learner(params, C, unroll_steps=10, graph=False)
    timed(f"train_step (eager, fixed batch, blas={sys.argv[2]})", lambda: lr3.train_step(batch))
