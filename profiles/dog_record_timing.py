import os, sys, time
sys.path.insert(0, os.getcwd())
import muzpkg; muzpkg.load()
import torch
from exploring_muzero_on_dog_amd import dog as DG
B, T = 1024, 16
rp = DG.RandomPlay(B, seed=4, fused=True)
es = torch.zeros(B, dtype=torch.int32, device="cuda"); ep = torch.zeros_like(es)
traj = DG.DogTrajectory(B, T)
for rec in (None, traj):
    for _ in range(3): rp.play(T, es, auto_reset=True, episodes=ep, record=rec)
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(20):
        if rec is not None: rec.reset()
        rp.play(T, es, auto_reset=True, episodes=ep, record=rec)
    torch.cuda.synchronize()
    print("record" if rec is not None else "plain", (time.time() - t) / 20 * 1000, "ms per play")
t = time.time()
for _ in range(20): p = traj.pack()
torch.cuda.synchronize(); print("pack", (time.time() - t) / 20 * 1000, "ms")
import cProfile, pstats
pr = cProfile.Profile(); pr.enable()
for _ in range(20): p = traj.pack()
torch.cuda.synchronize(); pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(8)
