"""Per-phase shader-clock shares of the DOG actor kernel k_dog_play (diagnostic build with -DMUZ_DOG_STAMPS), and the
cycles of each physical wave's check passes (dog_checks_play: wave w runs check waves w and w + 4 of the 7).

    make -C exploring-muzero-on-dog_amd/csrc BUILD=/tmp/build_dogst EXTRA=-DMUZ_DOG_STAMPS OUT=../variants/libmuz_dogst.so
    MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_dogst.so python profiles/diag_dog_play_stamps.py

Thread 0 of every workgroup (one game) stamps each phase of every turn; cycles per game-turn.  (Round 4's
r4c_dog_stamps_*.log came from this script under the name diag_dog_stamps.py, since reused for the search stamps.)"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import dog as DG  # noqa: E402
from exploring_muzero_on_dog_amd import lib as L  # noqa: E402

CATS = ["reset", "base checks + barrier", "mask words + choice", "env_step", "barrier", "deal"]
CHECK_WAVES = ["swap 0-63 | hot-7 0-63", "swap 64-127 | hot-7 64-119", "swap 128-191 | normal + -4", "swap 192-223 | -"]
if os.environ.get("MUZ_DOG_PAIRING", "0") == "1":   # a -DMUZ_DOG_PAIRING=1 build (env_dog.hip dog_checks_play)
    CHECK_WAVES = ["swap 0-63 | swap 128-191", "swap 64-127 | swap 192-223", "hot-7 0-63 | normal + -4", "hot-7 64-119 | -"]


def main():
    lib = L.load()
    fn, fw = lib.muz_diag_dog_stamps, lib.muz_diag_dog_wave_stamps
    for f in (fn, fw):
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    B, T, launches = 1024, 16, 20
    rp = DG.RandomPlay(B, seed=4, fused=True)
    steps = torch.zeros(B, dtype=torch.int32, device="cuda")
    rp.play(T, steps, auto_reset=True)
    torch.cuda.synchronize()
    buf, wb = (ctypes.c_uint64 * 8)(), (ctypes.c_uint64 * 24)()
    fn(buf, 1)
    fw(wb, 1)
    for _ in range(launches):
        rp.play(T, steps, auto_reset=True)
    torch.cuda.synchronize()
    fn(buf, 0)
    fw(wb, 0)
    tot = sum(buf[i] for i in range(6))
    turns = B * T * launches
    print(f"B={B}: {tot / turns:.0f} cycles per game-turn (thread 0 of each game's workgroup)")
    for i, c in enumerate(CATS):
        print(f"{c:>24}: {100.0 * buf[i] / tot:6.2f} %   {buf[i] / turns:8.0f} cycles/turn")
    for w in range(4):
        print(f"  wave {w}: setup before the passes {wb[w] / turns:7.0f} cycles/turn, closing-barrier wait "
              f"{wb[4 + w] / turns:7.0f} cycles/turn")
    print("check passes per physical wave (cycles per turn over all turns; cycles per pass that ran a check; share run):")
    for w in range(4):
        for p in range(2):
            cyc, ran = wb[8 + 4 * p + w], wb[16 + 4 * p + w]
            name = CHECK_WAVES[w].split(" | ")[p]
            if name == "-":
                continue
            print(f"  wave {w} pass {p} ({name:>14}): {cyc / turns:7.0f} cycles/turn, "
                  f"{(cyc / ran if ran else 0):7.0f} per run pass, ran in {100.0 * ran / turns:5.1f} % of turns")


if __name__ == "__main__":
    main()
