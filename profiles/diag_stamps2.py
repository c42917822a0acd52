"""Fine-grained cycle shares inside the Gumbel-search kernel (diagnostic build with -DMUZ_STAMPS2).

    make -C exploring-muzero-on-dog_amd/csrc BUILD=build_st2 EXTRA=-DMUZ_STAMPS2 OUT=../variants/libmuz_st2.so
    MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_st2.so python profiles/diag_stamps2.py

Wave 0 of each workgroup stamps: MFMA loops, dense epilogues, barrier waits, row ops (LayerNorm...),
tree selection, other, expansion + backup, elementwise passes + heads.  Shares only (stamps perturb the schedule)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import lib as L  # noqa: E402
from exploring_muzero_on_dog_amd import mcts as M  # noqa: E402
from exploring_muzero_on_dog_amd import nets as N  # noqa: E402

CATS = ["mfma-loops", "dense-epilogue", "barrier-wait", "row-ops", "select", "other", "expand+backup", "passes+heads", "dense-entry"]


def main():
    lib = L.load()
    fn = lib.muz_diag_stamps2
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    C = 18
    net = N.DeviceNet(N.init_muzero_params(0, C), C)
    rng = np.random.default_rng(0)
    obs = torch.from_numpy(rng.integers(0, 2, (B, C, 56)).astype(np.float32)).cuda()
    lg, v, e = N.root_inference_fn(net, obs)
    bits = torch.full((B,), (1 << 24) - 1, dtype=torch.int32, device="cuda")
    ws = M.SearchWorkspace(B, 50)
    M.gumbel_muzero_policy(net, lg, v, e, bits, 50, 25, 1.0, seed=1, workspace=ws)
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * 12)()
    fn(buf, 1)
    for r in range(3):
        M.gumbel_muzero_policy(net, lg, v, e, bits, 50, 25, 1.0, seed=r, workspace=ws)
    torch.cuda.synchronize()
    fn(buf, 0)
    tot = sum(buf[i] for i in range(12))
    wg_sims = 3 * ((B + 15) // 16) * 50
    print(f"B={B}: {tot / wg_sims:.0f} cycles per workgroup-simulation")
    for i, c in enumerate(CATS):
        print(f"{c:>15}: {100.0 * buf[i] / tot:6.2f} %   {buf[i] / wg_sims:9.0f} cycles/sim")


if __name__ == "__main__":
    main()
