"""Host AddressSanitizer + UBSan run of the C++ that executes on the host (VERDICT r5 "missing" 5): the CPU restatements
bench.py's cpu_baseline legs run in the bench process (oracle/cpu_*.cpp, cpu_search.hpp -- det, classic and DOG
self-play with their networks and searches, DOG random play, the env benches on OpenMP threads) and libmuz.so's
host-only TicTacToe engine (csrc/tictactoe.cpp), built as one sanitized executable by `make -C oracle asan`.  The
networks' parameters come from the oracles' initialisers through a small binary file."""
import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_asan", "asan_check")


def _write(path, params):
    with open(path, "wb") as f:
        f.write(struct.pack("<i", len(params)))
        for k, v in params.items():
            b = k.encode()
            a = np.ascontiguousarray(v, np.float32).ravel()
            f.write(struct.pack("<i", len(b)) + b + struct.pack("<q", a.size))
            f.write(a.tobytes())


@pytest.mark.timeout(900)
def test_host_code_clean_under_asan_and_ubsan(tmp_path):
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "asan"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    from oracle import classic_nets as CN
    from oracle import dog_muzero as DM
    from oracle import nets as ON
    files = [str(tmp_path / n) for n in ("det.bin", "classic.bin", "dog.bin")]
    _write(files[0], ON.init_params(34, seed=1, randomize_affine=True))
    _write(files[1], CN.init_params(11, seed=2, randomize_affine=True))
    _write(files[2], DM.init_params(seed=3, randomize_affine=True))
    env = dict(os.environ, OMP_NUM_THREADS="2", ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    p = subprocess.run([EXE] + files, capture_output=True, text=True, timeout=800, env=env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    assert "AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-4000:]
    assert "all host paths ran clean" in p.stdout
