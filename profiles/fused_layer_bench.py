"""Micro-benchmark of one learner layer at the step's shapes (M = 128 chain rows, 1408 prediction rows;
K = N = 256): muz_dense_ln_fwd / muz_dense_ln_bwd (csrc/learner_fused.hip, with and without the transposed
weight copy) against the library GEMM + muz_ln_fwd / muz_ln_bwd_rows pair they replace.  Per-call times from
100 calls captured in a HIP graph (as the learner step runs), replayed.
Usage: python profiles/fused_layer_bench.py [libmuz.so path]"""
import os
import sys

sys.path.insert(0, ".")
if len(sys.argv) > 1:
    os.environ["MUZ_LIB"] = sys.argv[1]
import muzpkg  # noqa: E402

muzpkg.load()
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import learner as L  # noqa: E402

L.prefer_rocblas()


def timed(fn, n=100):
    """Device time per call: n calls captured in one HIP graph, replayed (no host launch overhead)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(n):
            fn()
    gr.replay()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(5):
        gr.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (5 * n)


g = torch.Generator(device="cuda").manual_seed(0)
for M in (128, 1408):
    K = N = 256
    x = torch.randn((M, K), generator=g, device="cuda")
    W = torch.randn((K, N), generator=g, device="cuda") / 16
    b, gam, bet = (torch.randn((N,), generator=g, device="cuda") for _ in range(3))
    wt = L.WeightTranspose({"l/kernel": W})
    wt.refresh()
    f = L._dense_ln_fwd(x, W, b, gam, bet, None, 1)
    dout = torch.randn((M, N), generator=g, device="cuda")
    scr = torch.empty((L._ln_scratch_floats(M, N, K),), device="cuda")
    scr0 = torch.empty((L._L.load().muz_ln_bwd_scratch_floats(M, N),), device="cuda")
    L.FUSED_DENSE = L.FUSED_FWD = True
    t_f = timed(lambda: L._dense_ln_fwd(x, W, b, gam, bet, None, 1))
    with wt:
        t_ft = timed(lambda: L._dense_ln_fwd(x, W, b, gam, bet, None, 1))
    t_b = timed(lambda: L._dense_ln_bwd(dout, f, gam, 1, W, scr))
    t_bz = timed(lambda: L._dense_ln_bwd(dout, f, gam, 1, W, scr, need_dx=False))
    t_gemm = timed(lambda: x @ W)
    t_ln = timed(lambda: L._ln_fwd(x @ W, b, gam, bet, None, 1))
    t_lnb = timed(lambda: L._ln_bwd_rows(dout, f, gam, 1, scr0)[0] @ W.t())
    print(f"M={M}: fused fwd {t_f:.2f} us, fused fwd (W^T) {t_ft:.2f} us, fused bwd {t_b:.2f} us "
          f"(no dx {t_bz:.2f}); library GEMM {t_gemm:.2f} us, GEMM + ln_fwd {t_ln:.2f} us, "
          f"ln_bwd_rows + GEMM {t_lnb:.2f} us", flush=True)
