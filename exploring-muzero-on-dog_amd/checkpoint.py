"""Checkpoint I/O (SURVEY §8f "next" 4): the reference's Flax parameter trees <-> this engine's flat
path-named dicts.

* ``load_flax_msgpack`` / ``save_flax_msgpack``: the byte format of ``flax.serialization.to_bytes`` /
  ``from_bytes`` (TicTacToe/train.py:202-209, TicTacToe/eval.py:13-26 use it for their ``.params``
  files): a msgpack map of the state dict, every array as msgpack ext type 1 holding
  ``(shape, dtype name, C-order bytes)``.  Decoding executes nothing from the file (plain msgpack).
* ``flatten`` / ``unflatten``: nested dict <-> ``"a/b/c"`` names.
* ``muzero_tree_to_flat`` / ``flat_to_muzero_tree``: init_muzero_params' layout
  (muzero_deterministic_madn.py:706-748: ``{"representation": {"params": ...}, "dynamics": ...,
  "prediction": ...}``) <-> the names of nets.param_shapes, which nets.DeviceNet packs for the kernels.
* ``save_flat`` / ``load_flat``: safetensors files of a flat dict (this engine's own checkpoints).

The reference's det / classic MuZero checkpoints are pickles of jax arrays (train_with_reward.py:300-305);
they are not read here (unpickling executes code) -- convert them once with flax.serialization.to_bytes.
"""
from __future__ import annotations

import msgpack
import numpy as np

_EXT_NDARRAY = 1
_EXT_NPSCALAR = 3
NETS = ("representation", "dynamics", "prediction")


def _ext_hook(code, payload):
    if code == _EXT_NDARRAY:
        shape, dtype, buf = msgpack.unpackb(payload, raw=False)
        return np.frombuffer(buf, dtype=np.dtype(dtype)).reshape(shape).copy()
    if code == _EXT_NPSCALAR:
        shape, dtype, buf = msgpack.unpackb(payload, raw=False)
        return np.frombuffer(buf, dtype=np.dtype(dtype))[0]
    return msgpack.ExtType(code, payload)


def _default(obj):
    if isinstance(obj, np.ndarray):
        arr = np.ascontiguousarray(obj)
        return msgpack.ExtType(_EXT_NDARRAY, msgpack.packb((arr.shape, arr.dtype.name, arr.tobytes("C")),
                                                           use_bin_type=True))
    if isinstance(obj, np.generic):
        return msgpack.ExtType(_EXT_NPSCALAR, msgpack.packb(((), obj.dtype.name, obj.tobytes()), use_bin_type=True))
    raise TypeError(f"cannot serialise {type(obj)}")


def load_flax_msgpack(src) -> dict:
    """flax.serialization.msgpack_restore of a ``.params`` file (path or bytes) -> nested dict of arrays."""
    data = src if isinstance(src, (bytes, bytearray)) else open(src, "rb").read()
    return msgpack.unpackb(data, ext_hook=_ext_hook, raw=False, strict_map_key=False)


loads_flax_msgpack = load_flax_msgpack


def dumps_flax_msgpack(tree: dict) -> bytes:
    """flax.serialization.msgpack_serialize of a nested dict of arrays."""
    return msgpack.packb(tree, default=_default, strict_types=True)


def save_flax_msgpack(path: str, tree: dict):
    with open(path, "wb") as f:
        f.write(dumps_flax_msgpack(tree))


def flatten(tree: dict, prefix: str = "") -> dict:
    out = {}
    for k, v in tree.items():
        name = f"{prefix}/{k}" if prefix else str(k)
        if isinstance(v, dict):
            out.update(flatten(v, name))
        else:
            out[name] = v
    return out


def unflatten(flat: dict) -> dict:
    tree: dict = {}
    for name, v in flat.items():
        node = tree
        parts = name.split("/")
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = v
    return tree


def muzero_tree_to_flat(tree: dict) -> dict:
    """init_muzero_params layout -> nets.param_shapes names (``net/Layer/param``), float32."""
    flat = {}
    for net in NETS:
        sub = tree[net]["params"] if "params" in tree[net] else tree[net]
        for k, v in flatten(sub, net).items():
            flat[k] = np.asarray(v, np.float32)
    return flat


def muzero_tree_to_flat_any(tree: dict) -> dict:
    """muzero_tree_to_flat keeping the leaves as they are (torch tensors, e.g. a learner's live parameters,
    stay torch tensors)."""
    flat = {}
    for net in NETS:
        sub = tree[net]["params"] if "params" in tree[net] else tree[net]
        flat.update(flatten(sub, net))
    return flat


def flat_to_muzero_tree(flat: dict) -> dict:
    tree = unflatten(flat)
    return {net: {"params": tree[net]} for net in NETS}


def save_flat(path: str, flat: dict):
    from safetensors.numpy import save_file
    save_file({k: np.ascontiguousarray(v) for k, v in flat.items()}, path)


def load_flat(path: str) -> dict:
    from safetensors.numpy import load_file
    return load_file(path)
