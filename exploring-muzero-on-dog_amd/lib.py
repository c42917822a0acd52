"""ctypes binding of libmuz.so (C ABI declared in include/muz.h).

No torch types cross the boundary: callers pass raw device pointers
(``tensor.data_ptr()``) and a ``hipStream_t`` (``torch.cuda.current_stream().cuda_stream``).
There is deliberately no CPU fallback: if the library is missing this module raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmuz.so")

c_i8p = ctypes.POINTER(ctypes.c_int8)
c_u8p = ctypes.POINTER(ctypes.c_uint8)
vp = ctypes.c_void_p

MUZ_OK = 0
MUZ_E_BASE = 10000
MUZ_E_INVALID = MUZ_E_BASE + 1
MUZ_E_UNSUPPORTED = MUZ_E_BASE + 2


class MuzRules(ctypes.Structure):
    _fields_ = [
        ("num_players", ctypes.c_int32),
        ("distance", ctypes.c_int32),
        ("layout", ctypes.c_int32 * 4),
        ("starting_player", ctypes.c_int32),
        ("enable_teams", ctypes.c_int32),
        ("enable_initial_free_pin", ctypes.c_int32),
        ("enable_circular_board", ctypes.c_int32),
        ("enable_start_blocking", ctypes.c_int32),
        ("enable_jump_in_goal_area", ctypes.c_int32),
        ("enable_friendly_fire", ctypes.c_int32),
        ("enable_start_on_1", ctypes.c_int32),
        ("enable_bonus_turn_on_6", ctypes.c_int32),
        ("must_traverse_start", ctypes.c_int32),
    ]


class MuzDetSoA(ctypes.Structure):
    _fields_ = [
        ("board", vp),
        ("pins", vp),
        ("current_player", vp),
        ("reward", vp),
        ("done", vp),
        ("action_set", vp),
        ("stride", ctypes.c_int32),
    ]


# name -> (restype, argtypes).  Kept in sync with include/muz.h (tests/test_capi.py checks it).
SIGNATURES = {
    "muz_version": (ctypes.c_char_p, []),
    "muz_error_string": (ctypes.c_char_p, [ctypes.c_int]),
    "muz_detmadn_reset": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, ctypes.c_int32, vp]),
    "muz_detmadn_legal": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, ctypes.c_int32, vp]),
    "muz_detmadn_step": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, vp, vp, vp, ctypes.c_int32, vp]),
    "muz_detmadn_step_pin_move": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, vp, vp, vp,
                                                 ctypes.c_int32, vp]),
    "muz_detmadn_nostep": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, vp, ctypes.c_int32, vp]),
    "muz_detmadn_encode_f32": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, ctypes.c_int32, vp]),
    "muz_detmadn_encode_i8": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, ctypes.c_int32, vp]),
}

_lib = None


class MuzError(RuntimeError):
    pass


def load():
    """Load libmuz.so (raises if it was not built -- there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MuzError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    # torch must own the HIP runtime first so both share one libamdhip64.so.7 instance.
    import torch  # noqa: F401
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str = ""):
    if rc != MUZ_OK:
        msg = load().muz_error_string(rc).decode()
        raise MuzError(f"{what} failed: {msg} (code {rc})")


def stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())
