"""Dump the DOG bench workload's state (config d: 1024 games, 16-turn launches with in-place restarts) after
each launch, to compare two builds game by game:  MUZ_LIB=<lib> python profiles/dog_state_dump.py <out.npz> [launches]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import dog as DG  # noqa: E402


def main():
    out = sys.argv[1]
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 205
    rp = DG.RandomPlay(1024, seed=4, fused=True)
    steps = torch.zeros(1024, dtype=torch.int32, device="cuda")
    eps = torch.zeros(1024, dtype=torch.int32, device="cuda")
    hist = []
    for _ in range(launches):
        rp.play(16, steps, auto_reset=True, episodes=eps)
        h = DG.to_host(rp.env)
        hist.append(np.concatenate([np.asarray(h[k]).reshape(1024, -1).astype(np.int64) for k in sorted(h)], axis=1))
    np.savez(out, hist=np.stack(hist).astype(np.int16), steps=steps.cpu().numpy(), eps=eps.cpu().numpy())
    print(out, int(eps.sum()))


if __name__ == "__main__":
    main()
