"""Compare two dog_state_dump.py outputs: first launch / games where the builds diverge, and the state of
the first diverging game in both builds at the launch before and at the divergence (small npz for a replay
with the oracle).  python profiles/dog_state_compare.py a.npz b.npz out.npz"""
import sys

import numpy as np


def main():
    a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
    ha, hb = a["hist"], b["hist"]
    diff = (ha != hb).any(axis=2)
    if not diff.any():
        print("identical over", ha.shape[0], "launches")
        return
    first = int(np.argmax(diff.any(axis=1)))
    games = np.flatnonzero(diff[first])
    g = int(games[0])
    print("first diverging launch", first, "games", games[:16].tolist(), "games differing at the end", int(diff[-1].sum()))
    lo = max(first - 1, 0)
    np.savez(sys.argv[3], game=g, launch=first, a=ha[lo:first + 1, g], b=hb[lo:first + 1, g])


if __name__ == "__main__":
    main()
