"""libmuz.so loads and exports exactly what include/muz.h declares (CPU only: no compute calls)."""
import ctypes
import os
import re

import muzpkg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "muz.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(muz_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    names = declared_functions()
    assert "muz_detmadn_step" in names and "muz_version" in names


def test_library_exports_every_declared_symbol():
    from exploring_muzero_on_dog_amd import lib as L
    assert os.path.exists(L.LIB_PATH), "libmuz.so not built"
    so = ctypes.CDLL(L.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(so, n)]
    assert not missing, missing
    # the python binding covers every declared symbol with a signature
    assert set(declared_functions()) <= set(L.SIGNATURES), set(declared_functions()) - set(L.SIGNATURES)


def test_library_is_gfx950_code():
    from exploring_muzero_on_dog_amd import lib as L
    data = open(L.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data   # offload bundle entry of the fat binary


def test_version_string_without_gpu():
    from exploring_muzero_on_dog_amd import lib as L
    so = L.load()
    assert so.muz_version().startswith(b"libmuz")
    assert so.muz_error_string(L.MUZ_E_INVALID) == b"invalid argument"
