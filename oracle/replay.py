"""CPU oracle: the reference replay buffer (TEST INFRASTRUCTURE ONLY).

NumPy restatement of ``MuZero_det_MADN/vec_replay_buffer.py:9-264`` (``VectorizedReplayBuffer``):
``save_games_from_buffers`` (36-61) and ``sample_batch`` (63-264).  Only ``tests/`` use it.

The reference draws its sample indices from NumPy's legacy global generator (``np.random.randint``,
unseeded).  Here the generator is an argument with the same interface (``np.random.RandomState`` or
the ``np.random`` module itself), called in exactly the reference's order, so a seeded
``RandomState`` reproduces the reference's draws for the same seed.  Arithmetic of the targets is
float64 as in NumPy (GAMMA ** n, z * discount, bootstrap * discount) and rounded to float32 at the
end, where the reference's ``jnp.array`` conversion rounds it.

Parity status: restated from source; the reference has no tests for the buffer (parity unpinned
beyond this restatement).
"""
from __future__ import annotations

import numpy as np

GAMMA = 0.997
TERMINAL_RATIO = 0.25


class VectorizedReplayBuffer:
    """vec_replay_buffer.py:9-34 (obs kept as given; the device ring stores them int8)."""

    def __init__(self, capacity, batch_size, unroll_steps, td_steps, obs_shape=(14, 56), action_dim=24,
                 max_episode_length=500, bootstrap_value_target=True, rng=None):
        self.capacity = capacity
        self.batch_size = batch_size
        self.unroll_steps = unroll_steps
        self.td_steps = td_steps
        self.obs_shape = tuple(obs_shape)
        self.action_dim = action_dim
        self.max_episode_length = max_episode_length
        T = max_episode_length
        self.observations = np.zeros((capacity, T, *self.obs_shape), dtype=np.float32)
        self.actions = np.zeros((capacity, T), dtype=np.int32)
        self.rewards = np.zeros((capacity, T), dtype=np.int32)
        self.root_values = np.zeros((capacity, T), dtype=np.float32)
        self.child_visits = np.zeros((capacity, T, action_dim), dtype=np.float32)
        self.masks = np.zeros((capacity, T), dtype=np.float32)
        self.players = np.zeros((capacity, T), dtype=np.int32)
        self.teams = np.zeros((capacity, T), dtype=np.int32)
        self.episode_lengths = np.zeros(capacity, dtype=np.int32)
        self.discounts = np.zeros((capacity, T), dtype=np.int32)
        self.position = 0
        self.size = 0
        self.bootstrap_value_target = bootstrap_value_target
        self.rng = np.random if rng is None else rng

    def save_games_from_buffers(self, b):
        """vec_replay_buffer.py:36-61: games with idx > 0 go to consecutive ring slots."""
        lengths = np.asarray(b["idx"])
        for i in range(lengths.shape[0]):
            pos = self.position
            L = int(lengths[i])
            if L == 0:
                continue
            self.observations[pos, :L] = np.asarray(b["obs"][i, :L])
            self.actions[pos, :L] = np.asarray(b["act"][i, :L])
            self.rewards[pos, :L] = np.asarray(b["rew"][i, :L])
            self.root_values[pos, :L] = np.asarray(b["val"][i, :L])
            self.child_visits[pos, :L] = np.asarray(b["pol"][i, :L])
            self.masks[pos, :L] = np.asarray(b["mask"][i, :L])
            self.players[pos, :L] = np.asarray(b["player"][i, :L])
            self.teams[pos, :L] = np.asarray(b["team"][i, :L])
            self.discounts[pos, :L] = np.asarray(b["discount"][i, :L])
            self.episode_lengths[pos] = L
            self.position = (pos + 1) % self.capacity
            self.size = min(self.size + 1, self.capacity)

    def draw_indices(self):
        """The random part of sample_batch (vec_replay_buffer.py:72-99), in the reference's call order."""
        n_terminal = int(self.batch_size * TERMINAL_RATIO)
        n_normal = self.batch_size - n_terminal
        r = self.rng
        ep_n = r.randint(0, self.size, size=n_normal)
        len_n = self.episode_lengths[ep_n]
        t_n = r.randint(0, (len_n - 1) + 1)
        ep_t = r.randint(0, self.size, size=n_terminal)
        len_t = self.episode_lengths[ep_t]
        max_k = np.minimum(self.unroll_steps - 1, len_t - 1)
        term_k = np.array([r.randint(0, int(m) + 1) for m in max_k])
        t_t = np.maximum(len_t - 1 - term_k, 0)
        return np.concatenate([ep_n, ep_t]), np.concatenate([t_n, t_t])

    def sample_at(self, ep_indices, t_starts):
        """The deterministic part of sample_batch (vec_replay_buffer.py:101-264) for given indices."""
        return self._sample_common(ep_indices, t_starts, won=lambda fr: fr == 2)

    def _sample_common(self, ep_indices, t_starts, won):
        K = self.unroll_steps + 1
        TD = self.td_steps
        B = ep_indices.shape[0]
        ep_lengths = self.episode_lengths[ep_indices]
        root_obs = self.observations[ep_indices, t_starts]
        final = ep_lengths - 1
        final_rewards = self.rewards[ep_indices, final]
        final_players = self.players[ep_indices, final]
        final_teams = self.teams[ep_indices, final]
        seq = t_starts[:, None] + np.arange(K)[None, :]
        valid = seq < ep_lengths[:, None]
        seqc = np.minimum(seq, ep_lengths[:, None] - 1)
        epb = np.broadcast_to(ep_indices[:, None], (B, K))
        actions = self.actions[epb[:, :-1], seqc[:, :-1]]
        rewards = self.rewards[epb[:, :-1], seqc[:, :-1]]
        policies = self.child_visits[epb, seqc]
        values = self.root_values[epb, seqc]
        masks = self.masks[epb, seqc]
        discount_targets = self.discounts[epb[:, :-1], seqc[:, :-1]]
        seq_players = self.players[epb, seqc]
        seq_teams = self.teams[epb, seqc]
        won = won(final_rewards[:, None])
        single = seq_teams == -1
        z = np.where(won, np.where(single, np.where(final_players[:, None] == seq_players, 1.0, -1.0),
                                   np.where(final_teams[:, None] == seq_teams, 1.0, -1.0)), 0.0)
        steps_until_end = ep_lengths[:, None] - 1 - seq
        boot_from_value = steps_until_end >= TD
        boot_idx = np.minimum(seq + TD, ep_lengths[:, None] - 1)
        boot_raw = self.root_values[epb, boot_idx]
        boot_players = self.players[epb, boot_idx]
        boot_teams = self.teams[epb, boot_idx]
        same = np.where(seq_teams != -1, seq_teams == boot_teams, seq_players == boot_players)
        boot = np.where(same, boot_raw, -boot_raw)
        z = z * GAMMA ** np.maximum(steps_until_end, 0)
        target = np.where((z == 0) | (boot_from_value & self.bootstrap_value_target),
                          boot * (GAMMA ** np.minimum(TD, steps_until_end)), z)
        target = np.clip(target, -1.0, 1.0)
        return {
            "observations": root_obs.astype(np.float32),
            "actions": np.where(valid[:, :-1], actions, 0).astype(np.int32),
            "rewards": np.where(valid[:, :-1], rewards, 1).astype(np.int32),
            "policies": np.where(valid[:, :, None], policies, 0.0).astype(np.float32),
            "values": np.where(valid, values, 0.0).astype(np.float32),
            "masks": np.where(valid, masks, 0.0).astype(np.float32),
            "target_values": np.where(valid, target, 0.0).astype(np.float32),
            "discount_targets": np.where(valid[:, :-1], discount_targets, 1).astype(np.int32),
        }

    def sample_batch(self):
        """vec_replay_buffer.py:63-264."""
        ep, t = self.draw_indices()
        return self.sample_at(ep, t)


class VectorizedReplayBufferStochastic(VectorizedReplayBuffer):
    """MuZero_Classic_MADN/vec_replay_buffer_stochastic.py:10-297: the det buffer plus dice outcomes and
    dice distributions, "game won" = final reward class > 0 (line 194, a quirk kept as is), and the
    batch keys dice_outcomes (die - 1, padding 0) / dice_probs (padding uniform)."""

    def __init__(self, capacity, batch_size, unroll_steps, td_steps, obs_shape=(11, 56), action_dim=4,
                 max_episode_length=500, bootstrap_value_target=True, rng=None):
        super().__init__(capacity, batch_size, unroll_steps, td_steps, obs_shape, action_dim, max_episode_length,
                         bootstrap_value_target, rng)
        self.actions[:] = -1
        self.dice_outcomes = np.full((capacity, max_episode_length), -1, dtype=np.int32)
        self.dice_distributions = np.zeros((capacity, max_episode_length, 6), dtype=np.float32)

    def save_games_from_buffers(self, b):
        lengths = np.asarray(b["idx"])
        pos0 = self.position
        slots = []
        for i in range(lengths.shape[0]):
            if int(lengths[i]) > 0:
                slots.append((i, (pos0 + len(slots)) % self.capacity))
        super().save_games_from_buffers(b)
        for i, pos in slots:
            L = int(lengths[i])
            self.dice_outcomes[pos, :L] = np.asarray(b["dice"][i, :L])
            self.dice_distributions[pos, :L] = np.asarray(b["dice_dist"][i, :L])

    def sample_at(self, ep_indices, t_starts):
        out = self._sample_common(ep_indices, t_starts, won=lambda fr: fr > 0)
        K = self.unroll_steps + 1
        ep_lengths = self.episode_lengths[ep_indices]
        seq = t_starts[:, None] + np.arange(K)[None, :]
        valid = seq < ep_lengths[:, None]
        seqc = np.minimum(seq, ep_lengths[:, None] - 1)
        epb = np.broadcast_to(ep_indices[:, None], seq.shape)
        dice = self.dice_outcomes[epb[:, :-1], seqc[:, :-1]]
        dice = np.where(valid[:, :-1], dice, 0)
        probs = np.where(valid[:, :-1, None], self.dice_distributions[epb[:, :-1], seqc[:, :-1]],
                         np.full(6, 1.0 / 6.0, dtype=np.float32))
        out["dice_outcomes"] = np.maximum(dice - 1, 0).astype(np.int32)
        out["dice_probs"] = probs.astype(np.float32)
        return out
