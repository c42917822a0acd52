"""Device replay ring (muz_ring_save / muz_ring_sample) vs the replay oracle (GPU).

Both sides get the same trajectories and the same seeded numpy draws; ring contents and every sampled
tensor must be identical (integers bit-exact, floats bit-exact: the targets are double-then-float on
both sides).  Covers zero-length games, ring wrap-around within one call and across calls, padding of
windows past the episode end, bootstrap on / off, and real self-play buffers."""
import numpy as np
import pytest
import torch

from oracle.replay import VectorizedReplayBuffer as OracleRB
from tests.test_replay_oracle import make_buffers

pytestmark = pytest.mark.gpu


def _R():
    from exploring_muzero_on_dog_amd import replay as R
    return R


def to_dev(b):
    return {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in b.items()}


def assert_ring_equal(dev, ora):
    assert (dev.position, dev.size) == (ora.position, ora.size)
    lens = dev.episode_lengths.cpu().numpy()
    assert np.array_equal(lens, ora.episode_lengths)
    obs = dev.observations.cpu().numpy()
    fields = [("actions", "actions"), ("rewards", "rewards"), ("root_values", "root_values"),
              ("child_visits", "child_visits"), ("masks", "masks"), ("players", "players"), ("teams", "teams"),
              ("discounts", "discounts")]
    host = {a: getattr(dev, a).cpu().numpy() for a, _ in fields}
    for s in range(ora.size):
        L = lens[s]
        assert np.array_equal(obs[s, :L].astype(np.float32), ora.observations[s, :L]), s
        for a, b in fields:
            assert np.array_equal(host[a][s, :L], getattr(ora, b)[s, :L]), (a, s)


def assert_sample_equal(d, o):
    for k, v in o.items():
        got = d[k].cpu().numpy()
        assert got.dtype == v.dtype, k
        assert np.array_equal(got, v), (k, np.argwhere(got != v)[:5])


@pytest.mark.parametrize("boot", [False, True])
def test_ring_save_and_sample_synthetic(cuda, boot):
    R = _R()
    T, C, cap = 64, 18, 23
    dev = R.VectorizedReplayBuffer(cap, 96, 10, 7, obs_shape=(C, 56), max_episode_length=T,
                                   bootstrap_value_target=boot, rng=np.random.RandomState(5))
    ora = OracleRB(cap, 96, 10, 7, obs_shape=(C, 56), max_episode_length=T, bootstrap_value_target=boot,
                   rng=np.random.RandomState(5))
    rng = np.random.default_rng(11)
    for call in range(4):
        lengths = rng.integers(0, T + 1, 17 if call else 30)   # call 0 wraps inside one call (30 > 23)
        lengths[::5] = 0
        b = make_buffers(lengths, T, C=C, seed=call)
        b["team"][1::2] = (b["player"][1::2] % 2)                # some team-mode games
        dev.save_games_from_buffers(to_dev(b))
        ora.save_games_from_buffers(b)
        assert_ring_equal(dev, ora)
        for _ in range(3):
            assert_sample_equal(dev.sample_batch(), ora.sample_batch())


def test_ring_from_host_buffers_pinned_staging(cuda):
    """Reference-style host buffers (NumPy, fp32 observations, as play_n_games_v3's callers hold them) go
    through pinned staging + async host->device copies into the device ring: same ring as the oracle fed
    the same arrays; non-integral observations are refused (int8 storage would not be exact)."""
    R = _R()
    T, C, cap = 48, 18, 16
    dev = R.VectorizedReplayBuffer(cap, 64, 10, 7, obs_shape=(C, 56), max_episode_length=T,
                                   rng=np.random.RandomState(2))
    ora = OracleRB(cap, 64, 10, 7, obs_shape=(C, 56), max_episode_length=T, rng=np.random.RandomState(2))
    rng = np.random.default_rng(4)
    for call in range(3):
        b = make_buffers(rng.integers(0, T + 1, 11), T, C=C, seed=10 + call)
        host = dict(b, obs=b["obs"].astype(np.float32))          # the reference's fp32 observations
        dev.save_games_from_buffers(host)
        ora.save_games_from_buffers(b)
        assert_ring_equal(dev, ora)
        assert_sample_equal(dev.sample_batch(), ora.sample_batch())
    bad = make_buffers(np.array([5, 7]), T, C=C, seed=99)
    bad["obs"] = bad["obs"].astype(np.float32) + 0.5
    with pytest.raises(ValueError):
        dev.save_games_from_buffers(bad)


def test_ring_with_selfplay_buffers(cuda):
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import nets as N
    R = _R()
    C = E.num_channels(4)
    net = N.DeviceNet(N.init_muzero_params(0, C), C)
    eng = GA.SelfPlayEngine(net, 40, num_players=4, max_steps=80, num_simulations=8, max_depth=6)
    bufs = eng.play(seed=3)
    host = {k: v.cpu().numpy() for k, v in bufs.items()}
    dev = R.VectorizedReplayBuffer(64, 128, 10, 50, obs_shape=(C, 56), max_episode_length=80,
                                   rng=np.random.RandomState(1))
    ora = OracleRB(64, 128, 10, 50, obs_shape=(C, 56), max_episode_length=80, rng=np.random.RandomState(1))
    for _ in range(2):
        dev.save_games_from_buffers(bufs)
        ora.save_games_from_buffers(host)
    assert_ring_equal(dev, ora)
    assert_sample_equal(dev.sample_batch(), ora.sample_batch())


def test_stochastic_ring_with_classic_selfplay(cuda):
    """vec_replay_buffer_stochastic.py: dice outcomes / distributions, the `final reward class > 0` rule."""
    from oracle import classic_madn as cm
    from oracle import classic_nets as CN
    from oracle.replay import VectorizedReplayBufferStochastic as OracleRBS
    from exploring_muzero_on_dog_amd import game_agent_stochastic as GS
    from exploring_muzero_on_dog_amd import stochastic as S
    R = _R()
    C = cm.num_channels(4)
    net = S.DeviceClassicNet(CN.init_params(C, seed=4), C)
    eng = GS.StochasticSelfPlayEngine(net, 24, max_steps=90, num_simulations=8, max_depth=6)
    bufs = eng.play(seed=9)
    host = {k: v.cpu().numpy() for k, v in bufs.items()}
    dev = R.VectorizedReplayBufferStochastic(30, 64, 10, 20, obs_shape=(C, 56), max_episode_length=90,
                                             rng=np.random.RandomState(2))
    ora = OracleRBS(30, 64, 10, 20, obs_shape=(C, 56), max_episode_length=90, rng=np.random.RandomState(2))
    for _ in range(2):                                          # 48 games into 30 slots: wraps
        dev.save_games_from_buffers(bufs)
        ora.save_games_from_buffers(host)
    assert_ring_equal(dev, ora)
    assert np.array_equal(dev.dice_outcomes.cpu().numpy()[:, :90][ora.episode_lengths[:, None] > np.arange(90)],
                          ora.dice_outcomes[ora.episode_lengths[:, None] > np.arange(90)])
    for _ in range(2):
        assert_sample_equal(dev.sample_batch(), ora.sample_batch())


def _host_pack(host, T):
    """NumPy reference of transfer.pack: rows [0, idx) of every game, concatenated in game order."""
    lens = host["idx"]
    out = {k: np.concatenate([host[k][g, :lens[g]] for g in range(len(lens))]) for k in host if k != "idx"}
    out["idx"] = lens
    out["row_offset"] = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    return out


def _assert_rings_identical(a, b):
    assert (a.position, a.size) == (b.position, b.size)
    for k in ("observations", "actions", "rewards", "root_values", "child_visits", "masks", "players", "teams",
              "discounts", "episode_lengths") + (("dice_outcomes", "dice_distributions") if hasattr(a, "dice_outcomes")
                                                  else ()):
        assert torch.equal(getattr(a, k), getattr(b, k)), k


def test_pack_and_save_packed_det(cuda):
    """transfer.pack == NumPy packing, and a ring fed with packed rows == a ring fed with the buffers."""
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import nets as N
    from exploring_muzero_on_dog_amd import transfer as TR
    R = _R()
    C = E.num_channels(4)
    net = N.DeviceNet(N.init_muzero_params(0, C), C)
    eng = GA.SelfPlayEngine(net, 40, num_players=4, max_steps=80, num_simulations=8, max_depth=6)
    bufs = eng.play(seed=5)
    packed = TR.pack(bufs)
    want = _host_pack({k: v.cpu().numpy() for k, v in bufs.items()}, 80)
    for k, v in want.items():
        assert np.array_equal(packed[k].cpu().numpy(), v), k
    a = R.VectorizedReplayBuffer(50, 64, 10, 20, obs_shape=(C, 56), max_episode_length=80)
    b = R.VectorizedReplayBuffer(50, 64, 10, 20, obs_shape=(C, 56), max_episode_length=80)
    for _ in range(2):                                           # 80 games into 50 slots: wraps
        a.save_games_from_buffers(bufs)
        b.save_packed(packed)
    _assert_rings_identical(a, b)


def test_pack_and_save_packed_classic_dice(cuda):
    from oracle import classic_nets as CN
    from exploring_muzero_on_dog_amd import classic as CL
    from exploring_muzero_on_dog_amd import game_agent_stochastic as GS
    from exploring_muzero_on_dog_amd import stochastic as S
    from exploring_muzero_on_dog_amd import transfer as TR
    R = _R()
    C = CL.num_channels(4)
    net = S.DeviceClassicNet(CN.init_params(C, seed=4), C)
    eng = GS.StochasticSelfPlayEngine(net, 24, max_steps=90, num_simulations=8, max_depth=6)
    bufs = eng.play(seed=2)
    packed = TR.pack(bufs)
    want = _host_pack({k: v.cpu().numpy() for k, v in bufs.items()}, 90)
    for k, v in want.items():
        assert np.array_equal(packed[k].cpu().numpy(), v), k
    a = R.VectorizedReplayBufferStochastic(30, 64, 10, 20, obs_shape=(C, 56), max_episode_length=90)
    b = R.VectorizedReplayBufferStochastic(30, 64, 10, 20, obs_shape=(C, 56), max_episode_length=90)
    for _ in range(2):
        a.save_games_from_buffers(bufs)
        b.save_packed(packed)
    _assert_rings_identical(a, b)
