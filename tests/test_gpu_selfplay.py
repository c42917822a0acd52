"""Native self-play loop (muz_detmadn_selfplay) vs the CPU restatement of game_agent.py (GPU).

The oracle self-play is driven by the GPU network kernels (root + recurrent inference) and the
same counter-based Gumbel noise, so the comparison covers the bookkeeping, the env transitions,
the compaction and the search; network arithmetic itself is covered by test_gpu_nets.py."""
import numpy as np
import pytest
import torch

from oracle import detmadn as dm
from oracle import nets as ON
from oracle import selfplay as OS
from tests._parity import selfplay_parity

pytestmark = pytest.mark.gpu


def _mods():
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import nets as N
    return GA, N


def gpu_fns(N, net):
    def root(params, obs):
        lg, v, e = N.root_inference_fn(net, torch.from_numpy(obs).cuda())
        return lg.cpu().numpy(), v.cpu().numpy(), e.cpu().numpy()

    def rec(params, action, emb):
        r, d, lg, v, ne = N.recurrent_inference_fn(net, torch.from_numpy(np.asarray(action, np.int32)).cuda(),
                                                   torch.from_numpy(np.ascontiguousarray(emb)).cuda())
        return r.cpu().numpy(), d.cpu().numpy(), lg.cpu().numpy(), v.cpu().numpy(), ne.cpu().numpy()
    return root, rec


@pytest.mark.parametrize("P,n,S,D,T,temp", [(2, 24, 8, 8, 400, 1.0), (4, 8, 6, 4, 700, 0.5)])
def test_selfplay_matches_oracle(cuda, P, n, S, D, T, temp):
    GA, N = _mods()
    C = dm.num_channels(P)
    params = ON.init_params(C, seed=31, randomize_affine=True)
    net = N.DeviceNet(params, C)
    eng = GA.SelfPlayEngine(net, n, num_players=P, max_steps=T, num_simulations=S, max_depth=D)
    seed = 1234
    buf = {k: v.cpu().numpy() for k, v in eng.play(seed, temp).items()}
    envs = [dm.env_reset(num_players=P, **dm.SELFPLAY_RULES) for _ in range(n)]
    root, rec = gpu_fns(N, net)
    ref, steps = OS.play_batch_of_games(params, root, rec, envs, S, D, T, temp, seed)
    diverged = selfplay_parity(f"det self-play P{P} n{n} S{S} D{D} T{temp}", buf, ref,
                               ("act", "rew", "player", "team", "discount", "mask", "obs"))
    if not diverged:
        assert eng.last_turns == steps
        assert np.array_equal(buf["idx"], ref["idx"])


def test_selfplay_default_config_runs_and_is_deterministic(cuda):
    """config (b) shape at a small batch: 2 players, S=50, D=25; two calls with one seed are identical."""
    GA, N = _mods()
    C = dm.num_channels(2)
    net = N.DeviceNet(N.init_muzero_params(2, C), C)
    eng = GA.SelfPlayEngine(net, 64, num_players=2, max_steps=500, num_simulations=50, max_depth=25)
    b1 = {k: v.clone() for k, v in eng.play(7).items()}
    b2 = eng.play(7)
    for k in b1:
        assert torch.equal(b1[k], b2[k]), k
    idx = b1["idx"].cpu().numpy()
    assert (idx > 0).all() and (idx <= 500).all()
    mask = b1["mask"].cpu().numpy()
    act = b1["act"].cpu().numpy()
    T = np.arange(500)[None, :]
    assert ((act >= 0) == (mask > 0))[T < idx[:, None]].all()
    pol = b1["pol"].cpu().numpy()
    s = pol.sum(-1)
    assert np.allclose(s[mask > 0], 1.0, atol=1e-5)


@pytest.mark.parametrize("P,games,lanes,T", [(2, 40, 16, 300), (4, 37, 8, 60)])
def test_stream_equals_batch(cuda, P, games, lanes, T):
    """muz_detmadn_selfplay_stream: `games` games through `lanes` refilled lanes give exactly the
    trajectories of one muz_detmadn_selfplay batch of `games` (noise keyed by game and own step;
    T = 60 truncates most 4p games at max_steps)."""
    GA, N = _mods()
    C = dm.num_channels(P)
    net = N.DeviceNet(N.init_muzero_params(3, C), C)
    batch = GA.SelfPlayEngine(net, games, num_players=P, max_steps=T, num_simulations=8, max_depth=6)
    want = {k: v.clone() for k, v in batch.play(99, 1.0).items()}
    eng = GA.SelfPlayEngine(net, lanes, num_players=P, max_steps=T, num_simulations=8, max_depth=6)
    got = eng.play_stream(games, 99, 1.0)
    for k in want:
        assert torch.equal(got[k], want[k]), k
    st = eng.last_stats
    assert st["searches"] == batch.last_stats["searches"]
    assert st["turns"] >= batch.last_stats["turns"]
