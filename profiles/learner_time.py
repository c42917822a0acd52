"""Config (e) component timings on one MI355X: streamed self-play of 1500 4p games (S=100, D=50,
max_len 550) and the learner step at batch 128, unroll 10 (eager vs HIP-graph replay)."""
import sys
import time

sys.path.insert(0, ".")
import muzpkg  # noqa: E402

muzpkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import detmadn as E, game_agent as GA, learner as L, nets as N, replay as R  # noqa

C = E.num_channels(4)
params = N.init_muzero_params(0, C)
net = N.DeviceNet(params, C)
eng = GA.SelfPlayEngine(net, 1500, num_players=4, max_steps=550, num_simulations=100, max_depth=50)
ring = R.VectorizedReplayBuffer(20000, 128, 10, 50, obs_shape=(C, 56), max_episode_length=550,
                                rng=np.random.RandomState(0))
t = time.time()
buf = eng.play_stream(1500, seed=1)
torch.cuda.synchronize()
print("selfplay 1500 games S=100 D=50: %.2f s, %d env-steps" % (time.time() - t, int(buf["idx"].sum())))
ring.save_games_from_buffers(buf)
for graph in (False, True):
    lr = L.Learner(params, C, unroll_steps=10, graph=graph)
    for _ in range(3):
        lr.train_step(ring.sample_batch())
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(50):
        lr.train_step(ring.sample_batch())
    torch.cuda.synchronize()
    print("train_step (graph=%s): %.2f ms" % (graph, (time.time() - t) / 50 * 1000))
