"""k_chain_fwd / k_chain_bwd alone at the learner's shape (batch 128, 10 applications of the det trunk; classic:
20 alternating), timed with HIP events on the launching stream.  MUZ_LIB selects a build variant.

    python profiles/chain_bench.py [B] [K] [reps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import learner as L  # noqa: E402
from oracle import nets as ON  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
g = torch.Generator().manual_seed(1)
nets = L.MuZeroNets(ON.init_params(18, seed=4, randomize_affine=True), 18, 24, "cuda")
P = [nets.p[n].detach() for n in L.DYN_TRUNK_PARAMS]
apps, scaled = (0,) * K, (True,) * K
lat0 = torch.rand(B, 256, generator=g).cuda()
scale1 = 1.0 + (0.3 * torch.randn(K, B, 256, generator=g)).cuda()
shift = (0.3 * torch.randn(K, B, 256, generator=g)).cuda()
G, H = (torch.randn(K, B, 256, generator=g).cuda() for _ in range(2))
slot, seen = L._slots(apps, 1)
X = {(0, n): torch.empty((K, B, 256), device="cuda") for n in L._GEMM_LAYERS}
outs, qs = torch.empty(K, B, 256, device="cuda"), torch.empty(K, B, 256, device="cuda")
lohi, idx = torch.empty(K, B, 2, device="cuda"), torch.empty(K, B, 2, dtype=torch.int32, device="cuda")
st = torch.cuda.Stream()
with torch.cuda.stream(st), torch.no_grad():
    def fwd():
        return L._chain_forward(lat0, scale1, shift, apps, slot, scaled, P, X, outs, qs, lohi, idx)
    chain = fwd()

    def bwd():
        chain.keep = chain.keep0
        return L._chain_backward(chain, G, H, 0.5, apps, P, B, 256)
    chain.keep0 = chain.keep
    for label, fn in (("forward (pack + k_chain_fwd)", fwd), ("backward (k_chain_bwd)", bwd)):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"B={B} K={K} {label}: {ms * 1000:.1f} us ({ms * 1000 / (7 * K):.2f} us per weight layer)", flush=True)
