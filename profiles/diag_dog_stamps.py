"""Per-phase shader-clock shares of the DOG actor kernel k_dog_play (diagnostic build with -DMUZ_DOG_STAMPS).

    make -C exploring-muzero-on-dog_amd/csrc BUILD=/tmp/build_dogst EXTRA=-DMUZ_DOG_STAMPS OUT=../variants/libmuz_dogst.so
    MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_dogst.so python profiles/diag_dog_stamps.py

Thread 0 of every workgroup (one game) stamps each phase of every turn; cycles per game-turn."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import dog as DG  # noqa: E402
from exploring_muzero_on_dog_amd import lib as L  # noqa: E402

CATS = ["reset", "base checks + barrier", "mask words + choice", "env_step (lane 0)", "barrier", "deal"]


def main():
    lib = L.load()
    fn = lib.muz_diag_dog_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    B, T, launches = 1024, 16, 20
    rp = DG.RandomPlay(B, seed=4, fused=True)
    steps = torch.zeros(B, dtype=torch.int32, device="cuda")
    rp.play(T, steps, auto_reset=True)
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * 8)()
    fn(buf, 1)
    for _ in range(launches):
        rp.play(T, steps, auto_reset=True)
    torch.cuda.synchronize()
    fn(buf, 0)
    tot = sum(buf[i] for i in range(6))
    turns = B * T * launches
    print(f"B={B}: {tot / turns:.0f} cycles per game-turn (thread 0 of each game's workgroup)")
    for i, c in enumerate(CATS):
        print(f"{c:>24}: {100.0 * buf[i] / tot:6.2f} %   {buf[i] / turns:8.0f} cycles/turn")


if __name__ == "__main__":
    main()
