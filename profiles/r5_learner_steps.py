"""The config (e) learner step as the train loop runs it (Learner.train_step_from: the ring writes the batch into the
captured graph's inputs, then one HIP-graph replay of forward + backward + AdamW), det or DOG, batch 128 / unroll 10 /
td 50.  Prints the mean step time over `steps` replays (HIP events); under rocprofv3 --kernel-trace the last step's
dispatches follow the last k_ring_sample (profiles/r5_learner_trace.sh).

    python profiles/r5_learner_steps.py [steps] [det|dog]

MUZ_DUMP=path.npz: also save the trained parameters (bit-for-bit comparisons of library builds).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import learner as L, replay as R  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
game = sys.argv[2] if len(sys.argv) > 2 else "det"
if game == "dog":
    from exploring_muzero_on_dog_amd import game_agent_dog as GAD, muzero_dog as MD
    params = MD.init_muzero_params(0)
    sp = GAD.DogSelfPlay(MD.DeviceDogNet(params), 256, 8, 8, 1.0, seed=1)
    ring = R.VectorizedReplayBuffer(2000, 128, 10, 50, obs_shape=(MD.NUM_CHANNELS, 56), action_dim=MD.NUM_ACTIONS,
                                    max_episode_length=550, rng=np.random.RandomState(0))
    ring.save_games_from_buffers(sp.play_stream(256, 550, seed=3))
    lr = L.DogLearner(params, unroll_steps=10, graph=True)
else:
    from exploring_muzero_on_dog_amd import detmadn as E, game_agent as GA, nets as N
    C = E.num_channels(4)
    params = N.init_muzero_params(0, C)
    eng = GA.SelfPlayEngine(N.DeviceNet(params, C), 256, num_players=4, max_steps=550, num_simulations=8, max_depth=8)
    ring = R.VectorizedReplayBuffer(20000, 128, 10, 50, obs_shape=(C, 56), max_episode_length=550,
                                    rng=np.random.RandomState(0))
    ring.save_games_from_buffers(eng.play_stream(512, seed=1))
    lr = L.Learner(params, C, unroll_steps=10, graph=True)
for _ in range(3):
    lr.train_step_from(ring)
torch.cuda.synchronize()
for losses in (True, False):   # with the per-step copy of the loss row (a logging loop) / without (the bench's loop)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        out = lr.train_step_from(ring, losses=losses)
    e1.record()
    torch.cuda.synchronize()
    tag = "" if losses else ", no loss handout"
    last = f"; loss {float(out['total_loss']):.4f}" if losses else ""
    print(f"{game} train_step_from (sample into the graph inputs + graph replay{tag}): "
          f"{e0.elapsed_time(e1) / steps:.3f} ms per step over {steps} steps{last}", flush=True)
if os.environ.get("MUZ_DUMP"):
    np.savez(os.environ["MUZ_DUMP"], **{k: np.asarray(v) for k, v in lr.nets.numpy().items()})
