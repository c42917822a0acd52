"""Config (e) 7-actor + 1-learner prediction from measured parts.

One MI355X, the train workload's classes and shapes (bench.py run_train: 4p, S = 100, D = 50, max_len 550):
  * self-play of one iteration's games by ONE actor: 1500 games (the 1-GPU loop) and ceil(1500 / 7) = 215 games
    (one actor of seven) -- wall time of play_stream, env steps, longest game (records);
  * the learner's graph-captured train_step_from(ring) at batch 128 / unroll 10 (mean over 300 steps);
  * transfer.pack of an actor's records: wall time and the bytes one actor sends (the packed rows).
Prints one JSON object per (game, part) and a summary.  Usage: python profiles/config_e_parts.py [det|dog ...]
"""
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import muzpkg  # noqa: E402

muzpkg.load()
from exploring_muzero_on_dog_amd import detmadn as E  # noqa: E402
from exploring_muzero_on_dog_amd import game_agent as GA  # noqa: E402
from exploring_muzero_on_dog_amd import learner as LR  # noqa: E402
from exploring_muzero_on_dog_amd import nets as N  # noqa: E402
from exploring_muzero_on_dog_amd import replay as R  # noqa: E402
from exploring_muzero_on_dog_amd import transfer as TR  # noqa: E402

P, GAMES, T, S, D, ACTORS = 4, 1500, 550, 100, 50, 7


def emit(**kw):
    print(json.dumps(kw), flush=True)


def actor(game, n, dev):
    if game == "dog":
        from exploring_muzero_on_dog_amd import game_agent_dog as GAD
        from exploring_muzero_on_dog_amd import muzero_dog as MD
        params = MD.init_muzero_params(0)
        net = MD.DeviceDogNet(params, device=dev)
        sp = GAD.DogSelfPlay(net, n, S, D, 1.0, seed=0, device=dev)
        return params, (lambda seed: sp.play_stream(n, T, temperature=1.0, seed=seed)), MD.NUM_CHANNELS, MD.NUM_ACTIONS
    C = E.num_channels(P)
    params = N.init_muzero_params(42, C)
    net = N.DeviceNet(params, C, device=dev)
    eng = GA.SelfPlayEngine(net, n, num_players=P, max_steps=T, num_simulations=S, max_depth=D, device=dev)
    return params, (lambda seed: eng.play_stream(n, seed=seed, temperature=1.0)), C, 24


def main(games):
    dev = torch.device("cuda", 0)
    summary = {}
    for game in games:
        parts = {}
        ring = learner = None
        for n in (GAMES, math.ceil(GAMES / ACTORS)):
            params, play, C, A = actor(game, n, dev)
            if ring is None:
                ring = R.VectorizedReplayBuffer(20000, 128, 10, 50, obs_shape=(C, 56), action_dim=A,
                                                max_episode_length=T, device=dev, rng=np.random.RandomState(0))
            walls = []
            for rep in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                buf = play(1000 + rep)
                torch.cuda.synchronize()
                walls.append(time.perf_counter() - t0)
                idx = buf["idx"].cpu().numpy()
                emit(game=game, part="self-play", games=n, rep=rep, wall_s=round(walls[-1], 3),
                     env_steps=int(idx.sum()), longest_game=int(idx.max()), mean_game=round(float(idx.mean()), 1))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            packed = TR.pack(buf)
            torch.cuda.synchronize()
            pack_s = time.perf_counter() - t0
            nbytes = sum(v.numel() * v.element_size() for v in packed.values())
            emit(game=game, part="pack", games=n, wall_ms=round(1e3 * pack_s, 3), bytes=int(nbytes),
                 rows=int(packed["act"].shape[0]), bytes_per_row=round(nbytes / max(1, packed["act"].shape[0]), 1))
            ring.save_packed(packed)
            parts[n] = dict(play_s=min(walls), pack_ms=1e3 * pack_s, bytes=int(nbytes))
            if learner is None:
                learner = (LR.DogLearner(params, unroll_steps=10, device=dev, graph=True) if game == "dog" else
                           LR.Learner(params, C, unroll_steps=10, device=dev, graph=True))
            del buf, packed, play
            torch.cuda.empty_cache()
        for _ in range(20):
            learner.train_step_from(ring, losses=False)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(300):
            learner.train_step_from(ring, losses=False)
        e1.record()
        e1.synchronize()
        step_ms = e0.elapsed_time(e1) / 300
        emit(game=game, part="learner", step_ms=round(step_ms, 4), iteration_s=round(2.5 * step_ms, 3))
        small = parts[math.ceil(GAMES / ACTORS)]
        learn_s = 2.5 * step_ms
        summary[game] = {
            "one_gpu_selfplay_s": round(parts[GAMES]["play_s"], 3), "actor_of_7_selfplay_s": round(small["play_s"], 3),
            "learner_2500_steps_s": round(learn_s, 3), "actor_bytes_per_iteration": small["bytes"],
            "predicted_7p1_sequential_s": round(small["play_s"] + learn_s, 3),
            "predicted_7p1_overlapped_s": round(max(small["play_s"], learn_s), 3),
        }
    emit(part="summary", **summary)


if __name__ == "__main__":
    main(sys.argv[1:] or ["det", "dog"])
