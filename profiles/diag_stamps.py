"""Per-phase cycle breakdown of the Gumbel-search kernel (diagnostic build, never the timed one).

    make -C exploring-muzero-on-dog_amd/csrc DIAG=1 OUT=../libmuz_diag.so
    MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/libmuz_diag.so python profiles/diag_stamps.py

Thread 0 of every workgroup stamps s_memtime after each phase; totals are summed over workgroups.
Only the SHARES are meaningful (stamps add waits of their own)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
from exploring_muzero_on_dog_amd import detmadn as E  # noqa: E402
from exploring_muzero_on_dog_amd import game_agent as GA  # noqa: E402
from exploring_muzero_on_dog_amd import lib as L  # noqa: E402
from exploring_muzero_on_dog_amd import nets as N  # noqa: E402

PHASES = ["loop-top", "select", "gather", "dynamics", "emb-write", "prediction", "expand+backup", "-"]


def main():
    lib = L.load()
    fn = lib.muz_diag_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    C = E.num_channels(2)
    net = N.DeviceNet(N.init_muzero_params(0, C), C)
    batch = int(os.environ.get("BATCH", "4096"))
    eng = GA.SelfPlayEngine(net, batch, num_players=2, max_steps=500, num_simulations=50, max_depth=25)
    eng.play(1)
    buf = (ctypes.c_uint64 * 8)()
    fn(buf, 1)
    eng.play(2)
    fn(buf, 0)
    tot = sum(buf[i] for i in range(7))
    print(f"batch {batch}, stats {eng.last_stats}")
    for i in range(7):
        print(f"{PHASES[i]:>14}: {100.0 * buf[i] / tot:6.2f} %  ({buf[i] / 1e9:.3f} Gcycles)")


if __name__ == "__main__":
    main()
