"""Microbenchmark of one batched Gumbel search (k_gumbel_search) at B games, S sims.

    MUZ_LIB=<variant .so> python profiles/search_microbench.py [B] [S]

Reports device ms per search (HIP events on the launch stream) and algorithmic TFLOP/s."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import mcts as M  # noqa: E402
from exploring_muzero_on_dog_amd import nets as N  # noqa: E402

FLOP_PER_SIM = 2 * (529_280 + 404_544)        # algorithmic
EXEC_FLOP_PER_SIM = 2 * (491_904 + 404_544)   # executed (FiLM tabulated, one-hot rows gathered)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    C = 18
    net = N.DeviceNet(N.init_muzero_params(0, C), C)
    rng = np.random.default_rng(0)
    obs = torch.from_numpy(rng.integers(0, 2, (B, C, 56)).astype(np.float32)).cuda()
    lg, v, e = N.root_inference_fn(net, obs)
    bits = torch.full((B,), (1 << 24) - 1, dtype=torch.int32, device="cuda")
    ws = M.SearchWorkspace(B, S)
    for _ in range(2):
        M.gumbel_muzero_policy(net, lg, v, e, bits, S, 25, 1.0, seed=1, workspace=ws)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    st.record()
    for r in range(reps):
        M.gumbel_muzero_policy(net, lg, v, e, bits, S, 25, 1.0, seed=r, workspace=ws)
    en.record()
    torch.cuda.synchronize()
    ms = st.elapsed_time(en) / reps
    tf = B * S * FLOP_PER_SIM / (ms * 1e-3) / 1e12
    print(f"{os.path.basename(os.environ.get('MUZ_LIB', 'libmuz.so'))}: B={B} S={S}: {ms:.3f} ms/search, "
          f"{tf:.1f} TFLOP/s ({100 * tf / 157.3:.1f}% of fp32 MFMA peak), {1e3 * ms / S:.1f} us/sim")


if __name__ == "__main__":
    main()
