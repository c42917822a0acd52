"""Per-wave timeline of one simulation of one Gumbel-search workgroup (diagnostic build with -DMUZ_TIMELINE).

    make -C exploring-muzero-on-dog_amd/csrc BUILD=/tmp/build_tl EXTRA=-DMUZ_TIMELINE OUT=../variants/libmuz_tl.so
    MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_tl.so python profiles/diag_timeline.py

Lane 0 of each of the 8 waves stamps the end of every segment (MFMA loop, dense entry / epilogue, barrier
wait, row op, select, tree, other) of simulation MUZ_TL_SIM in workgroup MUZ_TL_WG.  For every SIMD (waves s
and s+4) the script reports how much of the simulation at least one of its two waves was inside an MFMA loop
("pipe fed"), and charges the rest (the pipe-idle time) to what the two waves were doing meanwhile."""
import ctypes
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import lib as L  # noqa: E402
from exploring_muzero_on_dog_amd import mcts as M  # noqa: E402
from exploring_muzero_on_dog_amd import nets as N  # noqa: E402

CATS = ["mfma", "epi", "bar", "row", "sel", "other", "tree", "pass", "entry", "c9", "c10", "sim"]
W, TMAX = 8, 1024


def segments(rec, n):
    """[(start, end, cat)] of one wave from its (time << 8 | cat) records.  The first record and the last
    one are 100 MHz real-time stamps (category 10) around the simulation."""
    out = []
    rec = rec[1:min(n, TMAX) - 1]
    for i in range(1, len(rec)):
        t0, t1 = rec[i - 1] >> 8, rec[i] >> 8
        out.append((t0, t1, CATS[rec[i] & 0xFF]))
    return out


def clock_ghz(rec, n):
    """Shader clock of the recorded simulation: shader cycles / 100 MHz ticks between its first and last stamp."""
    n = min(n, TMAX)
    return ((rec[n - 2] >> 8) - (rec[1] >> 8)) / ((rec[n - 1] >> 8) - (rec[0] >> 8)) * 0.1


def main():
    lib = L.load()
    fn = lib.muz_diag_timeline
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    C = 18
    net = N.DeviceNet(N.init_muzero_params(0, C), C)
    rng = np.random.default_rng(0)
    obs = torch.from_numpy(rng.integers(0, 2, (B, C, 56)).astype(np.float32)).cuda()
    lg, v, e = N.root_inference_fn(net, obs)
    bits = torch.full((B,), (1 << 24) - 1, dtype=torch.int32, device="cuda")
    ws = M.SearchWorkspace(B, 50)
    rec = (ctypes.c_uint64 * (W * TMAX))()
    cnt = (ctypes.c_uint32 * W)()
    for r in range(4):   # warm launches, then one recorded launch (counts reset before it)
        M.gumbel_muzero_policy(net, lg, v, e, bits, 50, 25, 1.0, seed=r, workspace=ws)
        torch.cuda.synchronize()
        fn(rec, cnt, 1)
    M.gumbel_muzero_policy(net, lg, v, e, bits, 50, 25, 1.0, seed=9, workspace=ws)
    torch.cuda.synchronize()
    fn(rec, cnt, 1)
    recs = np.frombuffer(rec, dtype=np.uint64).reshape(W, TMAX)
    segs = [segments([int(x) for x in recs[w]], int(cnt[w])) for w in range(W)]
    t0 = min(s[0][0] for s in segs if s)
    t1 = max(s[-1][1] for s in segs if s)
    clk = [clock_ghz([int(x) for x in recs[w]], int(cnt[w])) for w in range(W)]
    print(f"B={B}: one simulation of workgroup 0 spans {t1 - t0} cycles at {np.mean(clk):.3f} GHz "
          f"({(t1 - t0) / np.mean(clk) / 1e3:.1f} us); records per wave {list(cnt)}")
    tot_idle = defaultdict(float)
    for simd in range(4):
        a, b = segs[simd], segs[simd + 4]
        cuts = sorted({t for s in a + b for t in (s[0], s[1])} | {t0, t1})
        fed = 0
        idle = defaultdict(float)

        def cat_at(ss, t):
            for s in ss:
                if s[0] <= t < s[1]:
                    return s[2]
            return "-"
        for u, v_ in zip(cuts[:-1], cuts[1:]):
            m = (u + v_) / 2
            ca, cb = cat_at(a, m), cat_at(b, m)
            if ca == "mfma" or cb == "mfma":
                fed += v_ - u
            else:
                idle[f"{ca}|{cb}"] += v_ - u
        span = t1 - t0
        print(f"SIMD {simd}: pipe fed (a wave in an MFMA loop) {fed} of {span} cycles = {fed / span:.3f}")
        for k, x in sorted(idle.items(), key=lambda kv: -kv[1])[:8]:
            print(f"    idle while old|young = {k:>12}: {x:8.0f} cycles")
            tot_idle[k] += x / 4
    print("mean over SIMDs, idle cycles by (old wave | young wave) activity:")
    for k, x in sorted(tot_idle.items(), key=lambda kv: -kv[1])[:12]:
        print(f"    {k:>14}: {x:8.0f}")
    # per-wave totals
    print("per-wave cycles by category:")
    for w in range(W):
        d = defaultdict(int)
        for s in segs[w]:
            d[s[2]] += s[1] - s[0]
        print(f"  wave {w}: " + " ".join(f"{k}={d[k]}" for k in CATS if d[k]))
    np.save(os.path.join("gpurun_out", "timeline.npy"), recs[:, :max(cnt)])


if __name__ == "__main__":
    main()
