"""Cycle shares inside k_dog_search (diagnostic build with -DMUZ_STAMPS2; thread 0 of each workgroup stamps).

    make -C exploring-muzero-on-dog_amd/csrc BUILD=build_st2 EXTRA=-DMUZ_STAMPS2 OUT=../variants/libmuz_st2.so
    MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_st2.so python profiles/diag_dog_stamps.py [B] [S] [D]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import lib as L  # noqa: E402
from exploring_muzero_on_dog_amd import muzero_dog as MD  # noqa: E402

CATS = {0: "mfma-loops", 1: "dense-epilogue", 2: "barrier-wait", 3: "row-ops", 4: "select scores", 5: "Q transform",
        6: "tree / backup", 7: "node loads + passes", 8: "dense-entry", 11: "first-walk es + top"}


def report(buf, wg_sims, header):
    tot = sum(buf[i] for i in CATS)
    print(f"{header}: {tot / wg_sims:.0f} cycles per workgroup-simulation")
    for i, c in CATS.items():
        print(f"{c:>20}: {100.0 * buf[i] / tot:6.2f} %   {buf[i] / wg_sims:9.0f} cycles/sim")
    print(f"interior selections of thread 0's game: {buf[9]}, on the exact path: {buf[10]}, first walks: {buf[12]}, full loads: {buf[13]}")


def games_per_wg(B):
    """k_dog_search's games per workgroup as the library launches it (muz_dog_search_games_per_workgroup; round 5's
    logs divided by ceil(B / 8) workgroups while 1500 games ran on 250 of 6: their cycles per workgroup-simulation
    are 250 / 188 = 1.33x too high, the shares unaffected)."""
    return int(L.load().muz_dog_search_games_per_workgroup(B))


def main():
    lib = L.load()
    fn = lib.muz_diag_dog_stamps2
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    D = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    net = MD.DeviceDogNet(MD.init_muzero_params(0))
    rng = np.random.default_rng(0)
    obs = torch.from_numpy(rng.integers(0, 3, (B, 34, 56)).astype(np.float32)).cuda()
    lg, v, e = MD.root_inference_fn(net, obs)
    valid = torch.from_numpy(rng.random((B, 806)) < 0.1)
    words = MD.invalid_to_words(~valid).cuda()
    ws = MD.SearchWorkspace(B, S)
    MD.gumbel_muzero_policy(net, lg, v, e, words, S, D, 1.0, seed=1, workspace=ws)
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * 14)()
    fn(buf, 1)
    reps = 2
    for r in range(reps):
        MD.gumbel_muzero_policy(net, lg, v, e, words, S, D, 1.0, seed=r, workspace=ws)
    torch.cuda.synchronize()
    fn(buf, 0)
    wg_sims = reps * ((B + games_per_wg(B) - 1) // games_per_wg(B)) * S
    report(buf, wg_sims, f"B={B} S={S} D={D}")


def selfplay(turns=6):
    """The same shares over DogSelfPlay turns (real states and legal masks, the bench's setting)."""
    from exploring_muzero_on_dog_amd import game_agent_dog as GA
    lib = L.load()
    fn = lib.muz_diag_dog_stamps2
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    B, S, D = int(os.environ.get("DIAG_B", "1500")), 100, 50
    net = MD.DeviceDogNet(MD.init_muzero_params(2))
    sp = GA.DogSelfPlay(net, B, S, D, 1.0, seed=4)
    sp.play(2)
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * 14)()
    fn(buf, 1)
    depth = []
    sp.play(turns)
    torch.cuda.synchronize()
    fn(buf, 0)
    wg_sims = turns * ((B + games_per_wg(B) - 1) // games_per_wg(B)) * S
    report(buf, wg_sims, f"DogSelfPlay B={B} S={S} D={D}, {turns} turns")
    words = sp.words.cpu().numpy().view(np.uint32)
    nleg = np.array([sum(bin(int(w)).count("1") for w in row) for row in words])
    print(f"legal actions per game: mean {nleg.mean():.1f}, max {nleg.max()}, phase-1 games {int(sp.env.phase.sum())}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "selfplay":
        selfplay()
    else:
        main()
