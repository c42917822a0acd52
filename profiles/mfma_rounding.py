"""How does v_mfma_f32_16x16x4_f32 round?  (profiles/mfma_rounding.hip)

D = C + sum_{k<4} A[.,k] B[k,.] for one wave per trial.  Operands are crafted so that the candidate rounding orders
give different results: C in [1, 2) and products straddling C's half-ulp (ties and near-ties), products with large
mutual cancellation, and plain random operands.  Candidates, computed exactly with fractions on the host:
  chain     fmaf chain k = 0, 1, 2, 3 (one rounding per product-add, each product exact)
  chain_rev fmaf chain k = 3, 2, 1, 0
  once      the exact C + sum of the 4 products, rounded once
  pairwise  RN(RN(RN(p0 + p1) + RN(p2 + p3)) + C)
The device's own fmaf chain (k_fma_chain) checks the host emulation.  Prints match counts per candidate and per case.
Usage: python profiles/mfma_rounding.py [trials]   (needs profiles/_bin/libmfma_round.so: hipcc -shared; see below)
"""
import ctypes
import os
import subprocess
import sys
from fractions import Fraction

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_bin", "libmfma_round.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-shared", "-ffp-contract=off",
                    os.path.join(HERE, "mfma_rounding.hip"), "-o", SO], check=True)


def rn32(x: Fraction) -> float:
    """Round a rational to the nearest float32, ties to even (normal range only)."""
    if x == 0:
        return 0.0
    s = -1 if x < 0 else 1
    x = abs(x)
    e = x.numerator.bit_length() - x.denominator.bit_length()
    if Fraction(2) ** e > x:
        e -= 1
    while Fraction(2) ** (e + 1) <= x:
        e += 1
    m = x / Fraction(2) ** (e - 23)          # in [2^23, 2^24)
    q, r = divmod(m.numerator, m.denominator)
    twice = 2 * r
    if twice > m.denominator or (twice == m.denominator and q % 2 == 1):
        q += 1
    return float(np.float32(s * q * 2.0 ** (e - 23)))


def cases(trials, rng):
    """a, b [trials][64] lane operands, c [trials][64][4]."""
    a = np.zeros((trials, 64), np.float32)
    b = np.zeros((trials, 64), np.float32)
    c = np.zeros((trials, 64, 4), np.float32)
    kind = np.arange(trials) % 3
    for t in range(trials):
        if kind[t] == 0:       # products around half an ulp of C (C in [1, 2): ulp 2^-23)
            a[t] = rng.choice([1.0, 1.5, 0.75, -1.0, -0.5, 1.25], 64) * 2.0 ** -12
            b[t] = rng.choice([1.0, 0.5, 1.5, 0.75, -1.0], 64) * 2.0 ** -12
            c[t] = 1.0 + rng.integers(0, 2 ** 23, (64, 4)) * 2.0 ** -23
        elif kind[t] == 1:     # large cancelling products plus small ones
            a[t] = rng.choice([1.0, -1.0], 64) * (1.0 + rng.integers(0, 2 ** 12, 64) * 2.0 ** -12)
            b[t] = rng.choice([1.0, -1.0], 64) * (1.0 + rng.integers(0, 2 ** 12, 64) * 2.0 ** -12)
            c[t] = rng.standard_normal((64, 4)) * 2.0 ** -10
        else:                  # plain random
            a[t] = rng.standard_normal(64)
            b[t] = rng.standard_normal(64)
            c[t] = rng.standard_normal((64, 4))
    return a, b, c, kind


def exact_mats(a, b, c, t):
    """the lane -> element maps of 16x16x4 f32: A[row][k] = a[row + 16k], B[k][col] = b[col + 16k],
    D lane l register j = D[4 (l // 16) + j][l % 16]"""
    A = a[t].reshape(4, 16).T.astype(np.float64)            # [row][k]
    B = b[t].reshape(4, 16).astype(np.float64)              # [k][col]
    C = np.zeros((16, 16))
    for l in range(64):
        for j in range(4):
            C[4 * (l // 16) + j, l % 16] = c[t, l, j]
    return A, B, C


def main(trials):
    if not os.path.exists(SO):
        build()
    lib = ctypes.CDLL(SO)
    rng = np.random.default_rng(6)
    a, b, c, kind = cases(trials, rng)
    ta, tb, tc = (torch.from_numpy(x).cuda() for x in (a, b, c))
    d = torch.empty((trials, 64, 4), dtype=torch.float32, device="cuda")
    ch = torch.empty_like(d)
    chr_ = torch.empty_like(d)
    s = torch.cuda.current_stream().cuda_stream
    ptr = lambda x: ctypes.c_void_p(x.data_ptr())   # noqa: E731
    assert lib.mfma_probe(ptr(ta), ptr(tb), ptr(tc), ptr(d), trials, ctypes.c_void_p(s)) == 0
    assert lib.fma_chain(ptr(ta), ptr(tb), ptr(tc), ptr(ch), trials, 0, ctypes.c_void_p(s)) == 0
    assert lib.fma_chain(ptr(ta), ptr(tb), ptr(tc), ptr(chr_), trials, 1, ctypes.c_void_p(s)) == 0
    torch.cuda.synchronize()
    d, ch, chr_ = d.cpu().numpy(), ch.cpu().numpy(), chr_.cpu().numpy()
    names = ("chain", "chain_rev", "once", "pairwise", "device_fma_chain", "device_fma_chain_rev")
    hits = {k: np.zeros(3, np.int64) for k in names}
    tot = np.zeros(3, np.int64)
    emul_ok = True
    for t in range(trials):
        A, B, C = exact_mats(a, b, c, t)
        for l in range(64):
            for j in range(4):
                row, col = 4 * (l // 16) + j, l % 16
                p = [Fraction(float(A[row, k])) * Fraction(float(B[k, col])) for k in range(4)]
                c0 = Fraction(float(C[row, col]))
                sc = c0
                for k in range(4):
                    sc = Fraction(rn32(sc + p[k]))
                sr = c0
                for k in (3, 2, 1, 0):
                    sr = Fraction(rn32(sr + p[k]))
                cand = {"chain": float(sc), "chain_rev": float(sr), "once": rn32(c0 + sum(p)),
                        "pairwise": rn32(Fraction(rn32(Fraction(rn32(p[0] + p[1])) + Fraction(rn32(p[2] + p[3]))))
                                         + c0)}
                got = float(d[t, l, j])
                for k, v in cand.items():
                    hits[k][kind[t]] += got == v
                hits["device_fma_chain"][kind[t]] += got == float(ch[t, l, j])
                hits["device_fma_chain_rev"][kind[t]] += got == float(chr_[t, l, j])
                emul_ok &= float(ch[t, l, j]) == cand["chain"] and float(chr_[t, l, j]) == cand["chain_rev"]
                tot[kind[t]] += 1
    labels = ("half-ulp products", "cancelling products", "random")
    print(f"v_mfma_f32_16x16x4_f32 on gfx950, {trials} waves, {int(tot.sum())} outputs "
          f"(per case: {', '.join(f'{labels[i]} {tot[i]}' for i in range(3))})")
    print(f"host emulation of the fmaf chains equals the device's fmaf chains: {emul_ok}")
    for k in names:
        print(f"  D == {k:22s}: " + ", ".join(f"{labels[i]} {hits[k][i]}/{tot[i]}" for i in range(3)))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        main(int(sys.argv[1]) if len(sys.argv) > 1 else 300)
