"""Executed / algorithmic MAC of k_stochastic_search's expansions, measured, and the same ratio
for a branch-sorted schedule of 4-row blocks (v_mfma_f32_4x4x1_16b: each block of a sorted tile picks its own
trunk).  Diagnostic build with -DMUZ_BRANCH_STATS (thread 0 of every workgroup histograms, per expansion, the tile's
decision-parent rows n_d and chance-parent rows n_c):

    make -C exploring-muzero-on-dog_amd/csrc BUILD=/tmp/build_br EXTRA=-DMUZ_BRANCH_STATS OUT=../variants/libmuz_br.so
    MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_br.so python profiles/diag_classic_branches.py

MAC per row (bench.py CLASSIC_FLOP_PER_SIM): action dynamics 518,432, chance dynamics 491,904, Pred4 (A = 4) 401,984
(every expansion runs Pred4: on the afterstate or on the next state).
  algorithmic  = n_d (518,432 + 401,984) + n_c (491,904 + 401,984)
  executed now = 16 (518,432 [n_d > 0] + 491,904 [n_c > 0] + 401,984)       (16-row MFMA passes)
  sorted 4-row = 4 ceil(n_d / 4) 518,432 + 4 ceil(n_c / 4) 491,904 + 4 ceil((n_d + n_c) / 4) 401,984"""
import ctypes
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import lib as L  # noqa: E402

M_ACT, M_CHA, M_PRED = 518_432, 491_904, 401_984


def main():
    from exploring_muzero_on_dog_amd import classic as CL
    from exploring_muzero_on_dog_amd import game_agent_stochastic as GS
    from exploring_muzero_on_dog_amd import stochastic as ST
    lib = L.load()
    fn = lib.muz_diag_branch_hist
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    B = int(os.environ.get("DIAG_B", "4096"))
    C = CL.num_channels(4)
    net = ST.DeviceClassicNet(ST.init_classic_params(C, seed=0), C)
    eng = GS.StochasticSelfPlayEngine(net, B, num_players=4, max_steps=500, num_simulations=50, max_depth=25)
    eng.play(seed=1, temperature=1.0)      # warm-up
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * 289)()
    fn(buf, 1)
    eng.play(seed=2, temperature=1.0)
    torch.cuda.synchronize()
    fn(buf, 0)
    h = np.array(buf[:], np.float64).reshape(17, 17)
    n = h.sum()
    alg = now = srt = 0.0
    both = single = 0.0
    for nd in range(17):
        for nc in range(17):
            c = h[nd, nc]
            if not c:
                continue
            alg += c * (nd * (M_ACT + M_PRED) + nc * (M_CHA + M_PRED))
            now += c * 16 * ((M_ACT if nd else 0) + (M_CHA if nc else 0) + M_PRED)
            srt += c * (4 * math.ceil(nd / 4) * M_ACT + 4 * math.ceil(nc / 4) * M_CHA + 4 * math.ceil((nd + nc) / 4) * M_PRED)
            both += c if (nd and nc) else 0
            single += c if (bool(nd) != bool(nc)) else 0
    nd_mean = (h.sum(1) * np.arange(17)).sum() / n
    nc_mean = (h.sum(0) * np.arange(17)).sum() / n
    print(f"B={B} S=50 D=25, one play() batch: {int(n)} tile expansions; mean decision-parent rows {nd_mean:.2f}, "
          f"chance-parent rows {nc_mean:.2f} of 16")
    print(f"tiles running both trunks {100 * both / n:.1f} %, one trunk {100 * single / n:.1f} %")
    print(f"executed / algorithmic MAC: current 16-row passes {now / alg:.3f}, branch-sorted 4-row blocks {srt / alg:.3f}")
    print("histogram rows n_d, columns n_c (share of expansions, %):")
    for nd in range(17):
        if h[nd].sum():
            print(f"  n_d={nd:2d}: " + " ".join(f"{100 * h[nd, nc] / n:5.2f}" for nc in range(17)))


if __name__ == "__main__":
    main()
