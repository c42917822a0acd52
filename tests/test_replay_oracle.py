"""The replay-buffer oracle (oracle/replay.py) on hand-built episodes (CPU)."""
import numpy as np

from oracle.replay import GAMMA, VectorizedReplayBuffer


def make_buffers(lengths, T, C=18, A=24, seed=0, winner_reward=True):
    """Synthetic play_batch_of_games buffers: 2-player games, alternating players, last step won."""
    rng = np.random.default_rng(seed)
    n = len(lengths)
    b = {
        "obs": rng.integers(0, 5, (n, T, C, 56)).astype(np.int8),
        "act": rng.integers(-1, A, (n, T)).astype(np.int32),
        "rew": np.ones((n, T), np.int32),
        "val": rng.uniform(-1, 1, (n, T)).astype(np.float32),
        "pol": rng.dirichlet(np.ones(A), (n, T)).astype(np.float32),
        "mask": rng.integers(0, 2, (n, T)).astype(np.float32),
        "player": (np.arange(T)[None, :] % 2).repeat(n, 0).astype(np.int32),
        "team": -np.ones((n, T), np.int32),
        "discount": rng.integers(0, 3, (n, T)).astype(np.int32),
        "idx": np.asarray(lengths, np.int32),
    }
    for i, L in enumerate(lengths):
        if L > 0 and winner_reward and i % 3 != 2:
            b["rew"][i, L - 1] = 2
    return b


def test_save_ring_semantics():
    rb = VectorizedReplayBuffer(5, 8, 3, 4, obs_shape=(18, 56), max_episode_length=20)
    b = make_buffers([3, 0, 7, 2], 20)
    rb.save_games_from_buffers(b)
    assert (rb.position, rb.size) == (3, 3)
    assert rb.episode_lengths[:3].tolist() == [3, 7, 2]
    assert np.array_equal(rb.observations[1, :7], b["obs"][2, :7].astype(np.float32))
    rb.save_games_from_buffers(make_buffers([4, 5, 6], 20, seed=1))   # wraps: slots 3, 4, 0
    assert (rb.position, rb.size) == (1, 5)
    assert rb.episode_lengths.tolist() == [6, 7, 2, 4, 5]


def test_sample_targets_hand_checked():
    T, K, TD = 30, 4, 5
    rb = VectorizedReplayBuffer(4, 4, K - 1, TD, obs_shape=(18, 56), max_episode_length=T,
                                bootstrap_value_target=False)
    b = make_buffers([12], T)
    rb.save_games_from_buffers(b)
    L = 12
    out = rb.sample_at(np.array([0, 0]), np.array([0, 10]))
    winner = int(b["player"][0, L - 1])
    # start 0: every step is > TD from the end but z != 0 and bootstrap disabled -> discounted z
    for k in range(K):
        z = (1.0 if b["player"][0, k] == winner else -1.0) * GAMMA ** (L - 1 - k)
        assert np.isclose(out["target_values"][0, k], np.float32(z), atol=0, rtol=0)
    # start 10: k = 0, 1 valid, k >= 2 padded
    assert out["masks"][1, 2:].tolist() == [0.0, 0.0]
    assert out["rewards"][1, 2:].tolist() == [1]
    assert out["discount_targets"][1, 2:].tolist() == [1]
    assert np.all(out["policies"][1, 2:] == 0)
    assert out["target_values"][1, 2:].tolist() == [0.0, 0.0]


def test_sample_bootstrap_and_flip():
    T, TD = 40, 3
    rb = VectorizedReplayBuffer(2, 2, 2, TD, obs_shape=(18, 56), max_episode_length=T, bootstrap_value_target=True)
    b = make_buffers([30], T, winner_reward=False)          # no winner: z == 0 -> always bootstrap
    rb.save_games_from_buffers(b)
    out = rb.sample_at(np.array([0]), np.array([5]))
    for k in range(3):
        t = 5 + k
        bi = min(t + TD, 29)
        same = b["player"][0, t] == b["player"][0, bi]
        v = np.float64(b["val"][0, bi]) * (1 if same else -1) * GAMMA ** min(TD, 29 - t)
        assert out["target_values"][0, k] == np.float32(np.clip(v, -1, 1))


def test_draws_follow_the_reference_order():
    rb = VectorizedReplayBuffer(50, 16, 9, 50, obs_shape=(18, 56), max_episode_length=60,
                                rng=np.random.RandomState(123))
    rb.save_games_from_buffers(make_buffers(list(np.random.default_rng(3).integers(1, 60, 40)), 60))
    ep, t = rb.draw_indices()
    r = np.random.RandomState(123)
    ep_n = r.randint(0, 40, size=12)
    t_n = r.randint(0, rb.episode_lengths[ep_n])
    assert np.array_equal(ep[:12], ep_n) and np.array_equal(t[:12], t_n)
    assert np.all(t < rb.episode_lengths[ep])
