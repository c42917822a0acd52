"""Extract the reference's trained TicTacToeV2 policy (TicTacToe/Checkpoints/
TicTacToeV2_imp_net_3000ep_00001lr.params, flax msgpack: data only, nothing executed) into
tests/golden/ttt_imp_net_3000ep.npz, plus the evaluation it is pinned by (TicTacToe/results.md:
"ImpNet | 3k | 0.0001 | 82,20% | 17.60% | 0.20% | 444/378").  Run from the repo root:
    python tests/golden/make_ttt_checkpoint_fixture.py /root/reference"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import muzpkg  # noqa: E402

muzpkg.load()
from exploring_muzero_on_dog_amd import checkpoint as CK  # noqa: E402

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
src = os.path.join(ref, "TicTacToe", "Checkpoints", "TicTacToeV2_imp_net_3000ep_00001lr.params")
flat = CK.flatten(CK.load_flax_msgpack(src))
out = os.path.join(ROOT, "tests", "golden")
np.savez(os.path.join(out, "ttt_imp_net_3000ep.npz"), **{k.replace("/", "__"): v for k, v in flat.items()})
json.dump({"source": "TicTacToe/results.md (TicTacToeV2 results, 1000 games against random Bot)",
           "network": "ImprovedTicTacToeNet (TicTacToe/train.py), 3000 episodes, lr 0.0001",
           "win": 0.822, "loss": 0.176, "draw": 0.002, "wins_as_first": 444, "wins_as_second": 378,
           "games_per_seat": 500}, open(os.path.join(out, "ttt_imp_net_3000ep_results.json"), "w"), indent=1)
print("wrote", sorted(flat))
