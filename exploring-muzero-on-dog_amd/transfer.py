"""Actors -> learner trajectory transfer and learner -> actors weight broadcast.

The north star places one self-play actor per GPU and a single learner rank that receives every actor's
finished games over RCCL (xGMI point-to-point links), into a device-resident replay ring.  The
reference has no such path: its actors are the same process as the learner, and finished games go
device -> host with ``np.array`` and are copied slot by slot (vec_replay_buffer.py:36-61).

* ``pack(buffers)``: an actor packs its games' ``[0, idx)`` steps into contiguous rows on its GPU
  (``muz_traj_offsets`` + ``muz_traj_pack``): no padding to T crosses the link.
* ``gather_packed(packed, dst)``: the packed rows of every rank arrive at rank ``dst`` -- one
  ``all_gather`` of (games, rows) per rank, then ``batch_isend_irecv`` of each field (one message per
  field and actor; each actor drives its own xGMI link to the learner, so the transfers run link-parallel).
* ``VectorizedReplayBuffer.save_packed`` (replay.py) writes received rows into the ring directly
  (``muz_ring_save_packed``).
* ``broadcast_weights(net, src)``: the packed fp32 weight arena is ONE tensor, so a parameter update is
  one ``broadcast``; receivers re-derive their FiLM tables (``net.prepare()``).
* ``deliver_to_learner`` / ``publish_weights``: config (e)'s two exchanges per iteration as bench.py's train
  workload (and its multi-rank tests) run them -- every actor's packed games into the learner's ring, the learner's
  new weights back to every rank.

``gather_packed`` / ``broadcast_weights`` are backend-agnostic (RCCL for device tensors, gloo for CPU
tensors in the multi-process tests).
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from . import lib as _L

CELLS = 56


def fields(obs_channels: int, num_actions: int, chance: bool):
    """(name, dtype, per-row shape) of a packed game store, in transfer order."""
    f = [("obs", torch.int8, (obs_channels, CELLS)), ("act", torch.int32, ()), ("rew", torch.int32, ()),
         ("val", torch.float32, ()), ("pol", torch.float32, (num_actions,)), ("mask", torch.float32, ()),
         ("player", torch.int32, ()), ("team", torch.int32, ()), ("discount", torch.int32, ())]
    if chance:
        f += [("dice", torch.int32, ()), ("dice_dist", torch.float32, (6,))]
    return f


def traj_struct(rows: dict, max_steps: int = 0) -> _L.MuzTraj:
    t = _L.MuzTraj()
    for k in ("obs", "act", "rew", "val", "pol", "mask", "player", "team", "discount", "idx"):
        setattr(t, k, rows[k].data_ptr() if rows.get(k) is not None and rows[k].numel() else 0)
    t.max_steps = int(max_steps)
    return t


def chance_struct(rows: dict):
    if "dice" not in rows:
        return None
    c = _L.MuzTrajChance()
    c.dice = rows["dice"].data_ptr() if rows["dice"].numel() else 0
    c.dice_dist = rows["dice_dist"].data_ptr() if rows["dice_dist"].numel() else 0
    return c


def pack(buffers: dict) -> dict:
    """Self-play buffers ([n, T] layout, game_agent / game_agent_stochastic) -> packed rows on the same
    device: every field [R, ...] with R = sum(idx), plus ``idx`` [n] and ``row_offset`` [n] (int64)."""
    n, T = buffers["act"].shape
    C, A = buffers["obs"].shape[2], buffers["pol"].shape[2]
    dev = buffers["act"].device
    chance = "dice" in buffers
    lib, s = _L.load(), _L.stream_ptr()
    off = torch.empty((n,), dtype=torch.int64, device=dev)
    tot = torch.empty((1,), dtype=torch.int64, device=dev)
    _L.check(lib.muz_traj_offsets(_L.ptr(buffers["idx"]), n, _L.ptr(off), _L.ptr(tot), s), "muz_traj_offsets")
    R = int(tot.item())
    out = {name: torch.empty((R,) + shp, dtype=dt, device=dev) for name, dt, shp in fields(C, A, chance)}
    out["idx"] = torch.empty((n,), dtype=torch.int32, device=dev)
    out["row_offset"] = off
    src_ch, dst_ch = chance_struct(buffers), chance_struct(out)
    _L.check(lib.muz_traj_pack(traj_struct(buffers, T), None if src_ch is None else ctypes.byref(src_ch), _L.ptr(off),
                               n, C, A, traj_struct(out), None if dst_ch is None else ctypes.byref(dst_ch), s),
             "muz_traj_pack")
    return out


def dog_fields():
    """(name, dtype, per-row shape) of packed DOG actor records (dog.DogTrajectory), in transfer order."""
    return [("act", torch.int32, ()), ("player", torch.int32, ()), ("reward", torch.int32, ()),
            ("legal", torch.int32, ()), ("done", torch.uint8, ())]


def gather_packed(packed: dict, obs_channels: int = 0, num_actions: int = 0, chance: bool = False, dst: int = 0,
                  group=None, spec: list | None = None) -> list | None:
    """Every rank's packed games -> rank ``dst`` (a list indexed by source rank, its own included);
    None on the other ranks.  Tensors stay on their device (RCCL) or CPU (gloo).  ``spec`` overrides the
    field list (dog_fields() for DOG actor records); by default the det / classic trajectory fields."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = packed["idx"].device
    meta = torch.tensor([packed["idx"].shape[0], packed["act"].shape[0]], dtype=torch.int64, device=dev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    spec = fields(obs_channels, num_actions, chance) if spec is None else spec
    order = [("idx", torch.int32, None), ("row_offset", torch.int64, None)] + spec
    ops, result = [], None
    if rank == dst:
        result = []
        for r in range(world):
            n, R = (int(x) for x in metas[r].tolist())
            if r == dst:
                result.append(packed)
                continue
            got = {}
            for name, dt, shp in order:
                t = torch.empty((n,) if shp is None else (R,) + shp, dtype=dt, device=dev)
                got[name] = t
                if t.numel():
                    ops.append(dist.P2POp(dist.irecv, t, dist.get_global_rank(group, r) if group else r, group))
            result.append(got)
    else:
        for name, _, _ in order:
            t = packed[name].contiguous()
            if t.numel():
                ops.append(dist.P2POp(dist.isend, t, dist.get_global_rank(group, dst) if group else dst, group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return result


def empty_packed(obs_channels: int, num_actions: int, device, chance: bool = False) -> dict:
    """A rank's packed store without games (the learner's own part of a gather, or an actor with none)."""
    z = {name: torch.empty((0,) + shp, dtype=dt, device=device) for name, dt, shp in fields(obs_channels, num_actions,
                                                                                           chance)}
    z["idx"] = torch.empty((0,), dtype=torch.int32, device=device)
    z["row_offset"] = torch.empty((0,), dtype=torch.int64, device=device)
    return z


def deliver_to_learner(packed: dict | None, ring, obs_channels: int, num_actions: int, learner_rank: int,
                       chance: bool = False, group=None, device=None) -> int:
    """One iteration's finished games of every actor rank -> the learner rank's replay ring (config (e): the
    reference's ``replay.save_games_from_buffers(buffers)`` after ``play_n_games_v3``, MuZero_DOG/train.py:255-268,
    train_with_reward.py:255-268, with the actors on other GPUs).  A collective over all ranks of ``group``: each actor
    passes its ``pack``ed rows, the learner passes None (its own part is empty) and its ring (any object with
    ``save_packed``); the learner writes every actor's rows in rank order.  Returns the number of games the learner
    saved (0 on an actor)."""
    rank = dist.get_rank(group)
    if rank == learner_rank:
        if device is None:
            device = getattr(ring, "device", "cpu")
        packed = empty_packed(obs_channels, num_actions, device, chance)
    elif packed is None:
        raise ValueError("an actor rank must pass its packed games")
    got = gather_packed(packed, obs_channels, num_actions, chance, dst=learner_rank, group=group)
    if got is None:
        return 0
    n = 0
    for r, p in enumerate(got):
        if r != learner_rank and p["idx"].shape[0]:
            ring.save_packed(p)
            n += int(p["idx"].shape[0])
    return n


def publish_weights(net, learner, learner_rank: int, group=None, async_op: bool = False):
    """The learner's new parameters -> every rank's self-play network (MuZero_DOG/train.py:276, where the next
    play_n_games_v3 simply reads the updated ``params``): the learner rank packs them into its arena
    (``learner.push_to(net)``), then one broadcast of the arena.  ``async_op``: returns the broadcast's handle
    (``_WeightUpdate``; the overlapped loop waits on it before the next self-play call)."""
    if dist.get_rank(group) == learner_rank:
        learner.push_to(net)
    if async_op:
        return broadcast_weights_async(net, src=learner_rank, group=group)
    broadcast_weights(net, src=learner_rank, group=group)
    return None


def broadcast_weights(net, src: int = 0, group=None):
    """Learner -> actors parameter update: one broadcast of the packed weight arena, then the derived
    FiLM tables are rebuilt on every rank."""
    dist.broadcast(net.buffer, src=src, group=group)
    if hasattr(net, "prepare"):
        net.prepare()


class _WeightUpdate:
    """Handle of an asynchronous weight broadcast: wait() completes it and, on a receiving rank, rebuilds the
    derived FiLM tables (net.prepare) so the next self-play launch sees the new weights."""

    def __init__(self, work, net, receiver):
        self.work, self.net, self.receiver = work, net, receiver

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
            if self.receiver and hasattr(self.net, "prepare"):
                self.net.prepare()
            # RCCL's work.wait() only orders the CURRENT stream after the broadcast (and prepare() is queued on
            # it), while self-play and the learner run on streams of their own: block the host until the arena
            # and its FiLM tables are final, so no later launch on any stream reads a half-received arena (an
            # actor) or overwrites one the broadcast is still sending (the learner's next push_to).
            buf = getattr(self.net, "buffer", None)
            if isinstance(buf, torch.Tensor) and buf.is_cuda:
                torch.cuda.current_stream(buf.device).synchronize()


def broadcast_weights_async(net, src: int = 0, group=None) -> _WeightUpdate:
    """broadcast_weights with ``async_op=True`` (pipeline.run_overlapped): the learner goes on training while
    the arena travels; an actor calls wait() before its next self-play call.  The source must not repack its
    arena before its own handle's wait()."""
    work = dist.broadcast(net.buffer, src=src, group=group, async_op=True)
    return _WeightUpdate(work, net, dist.get_rank(group) != src)
