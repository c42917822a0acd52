"""Device-resident replay ring (host mirror of MuZero_det_MADN/vec_replay_buffer.py:9-264).

``VectorizedReplayBuffer`` keeps the reference's constructor, attributes (``position``, ``size``,
``bootstrap_value_target``) and methods:

* ``save_games_from_buffers(buffers)`` takes the self-play buffer dict (device tensors, as returned by
  ``game_agent.SelfPlayEngine.play``) and copies every game with ``idx > 0`` into the next ring slots
  ON DEVICE (``muz_ring_save``): no host round trip of the trajectories;
* ``sample_batch()`` draws the episode / start indices exactly like the reference (numpy legacy
  ``randint`` calls in the same order, from ``rng`` -- the ``np.random`` module by default, as in the
  reference, or a seeded ``np.random.RandomState``), then gathers the batch and computes the value
  targets on device (``muz_ring_sample``).  The result is a dict of device tensors with the reference's
  keys and shapes.

Storage: observations int8 (the encoder's values are 0..4), everything else as in the reference, all
in HBM: capacity 20000 x T 550 x C 34 needs 21 GB instead of the reference's 84 GB host fp32 array.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import lib as _L

GAMMA = 0.997
TERMINAL_RATIO = 0.25
CELLS = 56


class VectorizedReplayBuffer:
    def __init__(self, capacity: int, batch_size: int, unroll_steps: int, td_steps: int, obs_shape=(14, 56),
                 action_dim=24, max_episode_length=500, bootstrap_value_target=True, device="cuda", rng=None):
        C, W = obs_shape
        if W != CELLS:
            raise ValueError("observations must be [C, 56]")
        if td_steps > max_episode_length:
            raise ValueError("td_steps > max_episode_length")
        self.capacity, self.batch_size = int(capacity), int(batch_size)
        self.unroll_steps, self.td_steps = int(unroll_steps), int(td_steps)
        self.obs_shape, self.action_dim = (int(C), CELLS), int(action_dim)
        self.max_episode_length = int(max_episode_length)
        self.bootstrap_value_target = bool(bootstrap_value_target)
        self.position = 0
        self.size = 0
        self.rng = np.random if rng is None else rng
        self.device = torch.device(device)
        cap, T = self.capacity, self.max_episode_length
        z = dict(device=self.device)
        self.observations = torch.zeros((cap, T, C, CELLS), dtype=torch.int8, **z)
        self.actions = torch.zeros((cap, T), dtype=torch.int32, **z)
        self.rewards = torch.zeros((cap, T), dtype=torch.int32, **z)
        self.root_values = torch.zeros((cap, T), dtype=torch.float32, **z)
        self.child_visits = torch.zeros((cap, T, self.action_dim), dtype=torch.float32, **z)
        self.masks = torch.zeros((cap, T), dtype=torch.float32, **z)
        self.players = torch.zeros((cap, T), dtype=torch.int32, **z)
        self.teams = torch.zeros((cap, T), dtype=torch.int32, **z)
        self.discounts = torch.zeros((cap, T), dtype=torch.int32, **z)
        self.episode_lengths = torch.zeros((cap,), dtype=torch.int32, **z)
        # host copy of the lengths: the index draws need them (the reference reads its own array)
        self._ep_len_host = np.zeros(cap, np.int32)
        # 0.997 ** n as NumPy evaluates GAMMA ** int_array (float64 pow), n = 0..T
        self.gamma_pow = torch.from_numpy(np.power(GAMMA, np.arange(T + 1).astype(np.float64))).to(self.device)
        self._count = torch.zeros((1,), dtype=torch.int32, **z)

    def ring(self) -> _L.MuzRing:
        r = _L.MuzRing()
        r.obs, r.act, r.rew = self.observations.data_ptr(), self.actions.data_ptr(), self.rewards.data_ptr()
        r.val, r.pol, r.mask = self.root_values.data_ptr(), self.child_visits.data_ptr(), self.masks.data_ptr()
        r.player, r.team, r.discount = self.players.data_ptr(), self.teams.data_ptr(), self.discounts.data_ptr()
        r.ep_len = self.episode_lengths.data_ptr()
        r.capacity, r.max_steps = self.capacity, self.max_episode_length
        r.obs_channels, r.num_actions = self.obs_shape[0], self.action_dim
        r.won_if_positive = 0
        return r

    def _chance(self, b: dict):
        return None

    def _extra_outputs(self, B, K, z):
        return {}

    @staticmethod
    def _traj(b: dict) -> _L.MuzTraj:
        t = _L.MuzTraj()
        for k in ("obs", "act", "rew", "val", "pol", "mask", "player", "team", "discount", "idx"):
            setattr(t, k, b[k].data_ptr())
        t.max_steps = b["act"].shape[1]
        return t

    # dtype of each trajectory field in the device ring / muz_traj (obs: int8 values 0..4)
    TRAJ_DTYPES = {"obs": torch.int8, "act": torch.int32, "rew": torch.int32, "val": torch.float32,
                   "pol": torch.float32, "mask": torch.float32, "player": torch.int32, "team": torch.int32,
                   "discount": torch.int32, "idx": torch.int32}

    def stage(self, all_buffers: dict) -> dict:
        """Host trajectories (the reference's NumPy / jnp buffer dict, obs fp32) -> device tensors.

        Each host field is converted to the ring's dtype on the host (observations to int8 after checking
        that every value is an integer in [-128, 127], so the conversion is exact), copied into pinned
        (page-locked) memory and sent with one asynchronous host->device copy on the current stream
        (hipMemcpyAsync; the pinned block is released once its copy has completed).  Fields already on
        the ring's device pass through (made contiguous if they are strided views)."""
        out = {}
        for k, v in all_buffers.items():
            want = self.TRAJ_DTYPES.get(k, None)
            if isinstance(v, torch.Tensor) and v.device == self.device:
                # the kernels read data_ptr() as a dense [n, T, ...] block: a strided view is made dense
                v = v if want is None or v.dtype == want or k == "obs" else v.to(want)
                out[k] = v.contiguous()
                continue
            a = v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
            if k == "obs" and a.dtype != np.int8:
                i8 = a.astype(np.int8)
                if not np.array_equal(i8.astype(a.dtype), a):
                    raise ValueError("observations must hold small integers to be stored as int8")
                a = i8
            t = torch.from_numpy(np.ascontiguousarray(a))
            if want is not None and t.dtype != want:
                t = t.to(want)
            out[k] = t.pin_memory().to(self.device, non_blocking=True)
        if out["obs"].dtype != torch.int8:
            # device fp32 observations (e.g. a torch re-implementation's buffers): exact int8 cast on device
            o = out["obs"]
            i8 = o.to(torch.int8)
            if not torch.equal(i8.to(o.dtype), o):
                raise ValueError("observations must hold small integers to be stored as int8")
            out["obs"] = i8
        return out

    def save_games_from_buffers(self, all_buffers: dict):
        """vec_replay_buffer.py:36-61 on device.  Device buffers (SelfPlayEngine) are saved in place; host
        buffers (NumPy, as the reference's callers hold them) go through pinned staging first (``stage``)."""
        b = all_buffers
        if any(not (isinstance(v, torch.Tensor) and v.device == self.device) for v in b.values()) or \
                b["obs"].dtype != torch.int8:
            b = self.stage(b)
        n = b["idx"].shape[0]
        if b["obs"].dtype != torch.int8 or tuple(b["obs"].shape[2:]) != self.obs_shape:
            raise ValueError("expected int8 observations of shape [n, T, C, 56]")
        slots = torch.empty((n,), dtype=torch.int32, device=self.device)
        ch = self._chance(b)
        _L.check(_L.load().muz_ring_save(self.ring(), self._traj(b), None if ch is None else ctypes.byref(ch), n,
                                         self.position, _L.ptr(slots), _L.ptr(self._count), _L.stream_ptr()),
                 "muz_ring_save")
        self._advance(slots, b["idx"])

    def save_packed(self, packed: dict):
        """Games packed by transfer.pack (possibly received from another rank by transfer.gather_packed)
        into the ring, with the same slot rule as save_games_from_buffers."""
        from .transfer import chance_struct, traj_struct
        n = packed["idx"].shape[0]
        if n == 0:
            return
        if tuple(packed["obs"].shape[1:]) != self.obs_shape or packed["pol"].shape[1] != self.action_dim:
            raise ValueError("packed games do not match the ring's observation / action shape")
        max_len = int(packed["idx"].max().item())
        if max_len > self.max_episode_length:
            raise ValueError("a packed game is longer than max_episode_length")
        slots = torch.empty((n,), dtype=torch.int32, device=self.device)
        ch = chance_struct(packed) if self._chance(packed) is not None else None
        _L.check(_L.load().muz_ring_save_packed(self.ring(), traj_struct(packed), None if ch is None else ctypes.byref(ch),
                                                _L.ptr(packed["row_offset"]), n, max_len, self.position,
                                                _L.ptr(slots), _L.ptr(self._count), _L.stream_ptr()),
                 "muz_ring_save_packed")
        self._advance(slots, packed["idx"])

    def _advance(self, slots, idx):
        count = int(self._count.item())
        sl = slots.cpu().numpy()
        lens = idx.cpu().numpy()
        keep = sl >= 0
        self._ep_len_host[sl[keep]] = lens[keep]
        self.position = (self.position + count) % self.capacity
        self.size = min(self.size + count, self.capacity)

    def draw_indices(self):
        """vec_replay_buffer.py:72-99: the reference's numpy draws, in its order."""
        n_terminal = int(self.batch_size * TERMINAL_RATIO)
        n_normal = self.batch_size - n_terminal
        r = self.rng
        ep_n = r.randint(0, self.size, size=n_normal)
        len_n = self._ep_len_host[ep_n]
        t_n = r.randint(0, (len_n - 1) + 1)
        ep_t = r.randint(0, self.size, size=n_terminal)
        len_t = self._ep_len_host[ep_t]
        max_k = np.minimum(self.unroll_steps - 1, len_t - 1)
        term_k = np.array([r.randint(0, int(m) + 1) for m in max_k])
        t_t = np.maximum(len_t - 1 - term_k, 0)
        return np.concatenate([ep_n, ep_t]).astype(np.int32), np.concatenate([t_n, t_t]).astype(np.int32)

    def sample_at(self, ep_indices, t_starts, out: dict | None = None) -> dict:
        """The deterministic part of sample_batch (vec_replay_buffer.py:101-264), on device.  `out`: the
        batch tensors to fill (same keys, shapes and dtypes as a returned batch, contiguous, on the ring's
        device) -- a learner's static graph inputs, so no copy follows."""
        B = len(ep_indices)
        K = self.unroll_steps + 1
        C, A = self.obs_shape[0], self.action_dim
        z = dict(device=self.device)
        if out is not None:
            ref = self._batch_spec(B, K, C, A)
            for k, (shape, dt) in ref.items():
                t = out.get(k)
                if t is None or tuple(t.shape) != shape or t.dtype != dt or not t.is_contiguous() \
                        or t.device.type != self.device.type or \
                        (self.device.index is not None and t.device.index != self.device.index):
                    raise ValueError(f"sample_at(out=): '{k}' must be a contiguous {dt} {shape} tensor on {self.device}")
        else:
            out = self._new_batch(B, K, C, A, z)
        s = _L.MuzSample()
        for k in self._batch_spec(B, K, C, A):
            setattr(s, k, out[k].data_ptr())
        ep, ts = self._stage_indices(ep_indices, t_starts)
        _L.check(_L.load().muz_ring_sample(self.ring(), _L.ptr(ep), _L.ptr(ts), B, self.unroll_steps, self.td_steps,
                                           int(self.bootstrap_value_target), _L.ptr(self.gamma_pow), s,
                                           _L.stream_ptr()), "muz_ring_sample")
        st = getattr(self, "_idx_stage", None)
        if st is not None and self.device.type == "cuda":
            # the slot is free again once this sample has read it (covers the pinned source and the device copy)
            ev = st["ev"][st["k"] ^ 1] = torch.cuda.Event()
            ev.record()
        return out

    def _batch_spec(self, B, K, C, A) -> dict:
        spec = getattr(self, "_spec", None)
        if spec is None or spec[0] != B:
            spec = self._spec = (B, {k: (tuple(v.shape), v.dtype)
                                     for k, v in self._new_batch(B, K, C, A, dict(device="meta")).items()})
        return spec[1]

    def _stage_indices(self, ep_indices, t_starts):
        """Episode / start indices to the device through a pinned double buffer (an async copy; a pageable
        source would make the copy wait for the stream to drain, serialising the host's next index draw with
        the previous learner step).  Slot k is reused only after the sample that read it two calls ago completed
        (the event sample_at records after its launch)."""
        B = len(ep_indices)
        if self.device.type != "cuda":
            return (torch.as_tensor(np.asarray(ep_indices, np.int32)).to(self.device),
                    torch.as_tensor(np.asarray(t_starts, np.int32)).to(self.device))
        st = getattr(self, "_idx_stage", None)
        if st is None or st["host"].shape[1] != 2 * B:
            st = self._idx_stage = {"host": torch.empty((2, 2 * B), dtype=torch.int32, pin_memory=True),
                                    "dev": torch.empty((2, 2 * B), dtype=torch.int32, device=self.device),
                                    "ev": [None, None], "k": 0}
        k = st["k"]
        st["k"] ^= 1
        if st["ev"][k] is not None:
            st["ev"][k].synchronize()
        h = st["host"][k].numpy()
        h[:B] = np.asarray(ep_indices, np.int32)
        h[B:] = np.asarray(t_starts, np.int32)
        d = st["dev"][k]
        d.copy_(st["host"][k], non_blocking=True)
        return d[:B], d[B:]

    def _new_batch(self, B, K, C, A, z) -> dict:
        out = {
            "observations": torch.empty((B, C, CELLS), dtype=torch.float32, **z),
            "actions": torch.empty((B, K - 1), dtype=torch.int32, **z),
            "rewards": torch.empty((B, K - 1), dtype=torch.int32, **z),
            "policies": torch.empty((B, K, A), dtype=torch.float32, **z),
            "values": torch.empty((B, K), dtype=torch.float32, **z),
            "masks": torch.empty((B, K), dtype=torch.float32, **z),
            "target_values": torch.empty((B, K), dtype=torch.float32, **z),
            "discount_targets": torch.empty((B, K - 1), dtype=torch.int32, **z),
        }
        out.update(self._extra_outputs(B, K, z))
        return out

    def sample_batch(self) -> dict:
        """vec_replay_buffer.py:63-264."""
        ep, t = self.draw_indices()
        return self.sample_at(ep, t)


class VectorizedReplayBufferStochastic(VectorizedReplayBuffer):
    """MuZero_Classic_MADN/vec_replay_buffer_stochastic.py:10-297 on device: the det ring plus the dice
    outcomes / distributions of each step; "game won" = final reward class > 0 (line 194); batches also
    carry dice_outcomes (die - 1) and dice_probs."""

    def __init__(self, capacity: int, batch_size: int, unroll_steps: int, td_steps: int, obs_shape=(11, 56),
                 action_dim=4, max_episode_length=500, bootstrap_value_target=True, device="cuda", rng=None):
        super().__init__(capacity, batch_size, unroll_steps, td_steps, obs_shape, action_dim, max_episode_length,
                         bootstrap_value_target, device, rng)
        self.actions.fill_(-1)
        cap, T = self.capacity, self.max_episode_length
        self.dice_outcomes = torch.full((cap, T), -1, dtype=torch.int32, device=self.device)
        self.dice_distributions = torch.zeros((cap, T, 6), dtype=torch.float32, device=self.device)

    def ring(self) -> _L.MuzRing:
        r = super().ring()
        r.won_if_positive = 1
        r.dice, r.dice_dist = self.dice_outcomes.data_ptr(), self.dice_distributions.data_ptr()
        return r

    TRAJ_DTYPES = dict(VectorizedReplayBuffer.TRAJ_DTYPES, dice=torch.int32, dice_dist=torch.float32)

    def _chance(self, b: dict):
        ch = _L.MuzTrajChance()
        ch.dice, ch.dice_dist = b["dice"].data_ptr(), b["dice_dist"].data_ptr()
        return ch

    def _extra_outputs(self, B, K, z):
        return {"dice_outcomes": torch.empty((B, K - 1), dtype=torch.int32, **z),
                "dice_probs": torch.empty((B, K - 1, 6), dtype=torch.float32, **z)}
