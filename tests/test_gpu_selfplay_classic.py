"""Native Stochastic-MuZero self-play (muz_classic_selfplay) vs the CPU restatement of
game_agent_stochastic.py (GPU).

The oracle loop is driven by the GPU network kernels and the same counter RNG (die uniforms, tie-break
uniforms, final Gumbel draws); the root Dirichlet fraction is 0 on both sides (the engine's Gamma
sampler is not restated), so everything else -- dice, env transitions, compaction, search, records --
is compared exactly."""
import numpy as np
import pytest
import torch

from oracle import classic_madn as cm
from oracle import classic_nets as CN
from oracle import selfplay as OS
from tests._parity import selfplay_parity

pytestmark = pytest.mark.gpu


def _mods():
    from exploring_muzero_on_dog_amd import game_agent_stochastic as GS
    from exploring_muzero_on_dog_amd import stochastic as S
    return GS, S


def gpu_fns(S, net):
    def root(params, obs):
        return tuple(t.cpu().numpy() for t in S.root_inference_fn(net, torch.from_numpy(obs).cuda()))

    def dec(params, action, emb):
        return tuple(t.cpu().numpy() for t in S.decision_recurrent_fn(
            net, torch.from_numpy(np.asarray(action, np.int32)).cuda(), torch.from_numpy(np.ascontiguousarray(emb)).cuda()))

    def cha(params, chance, after):
        return tuple(t.cpu().numpy() for t in S.chance_recurrent_fn(
            net, torch.from_numpy(np.asarray(chance, np.int32)).cuda(), torch.from_numpy(np.ascontiguousarray(after)).cuda()))
    return root, dec, cha


@pytest.mark.parametrize("n,Ssim,D,T,temp", [(12, 8, 6, 120, 1.0), (6, 16, 10, 90, 0.6)])
def test_classic_selfplay_matches_oracle(cuda, n, Ssim, D, T, temp):
    GS, S = _mods()
    C = cm.num_channels(4)
    params = CN.init_params(C, seed=13, randomize_affine=True)
    net = S.DeviceClassicNet(params, C)
    eng = GS.StochasticSelfPlayEngine(net, n, max_steps=T, num_simulations=Ssim, max_depth=D)
    seed = 4242
    buf = {k: v.cpu().numpy() for k, v in eng.play(seed, temp, dirichlet_fraction=0.0).items()}
    envs = [cm.env_reset(num_players=4, **cm.SELFPLAY_RULES) for _ in range(n)]
    root, dec, cha = gpu_fns(S, net)
    ref, steps = OS.play_batch_of_games_stochastic(params, root, dec, cha, envs, Ssim, D, T, temp, seed)
    diverged = selfplay_parity(f"classic self-play n{n} S{Ssim} D{D} T{temp}", buf, ref,
                               ("act", "rew", "player", "team", "discount", "mask", "dice", "obs", "dice_dist"))
    if not diverged:
        assert eng.last_turns == steps
        assert np.array_equal(buf["idx"], ref["idx"])


def test_classic_selfplay_config_c_shape_runs(cuda):
    """config (c) at a small batch: 4 players in teams, dice rethrow, S=50; deterministic per seed."""
    GS, S = _mods()
    C = cm.num_channels(4)
    net = S.DeviceClassicNet(CN.init_params(C, seed=2), C)
    eng = GS.StochasticSelfPlayEngine(net, 48, max_steps=300, num_simulations=50, max_depth=25)
    b1 = {k: v.clone() for k, v in eng.play(3).items()}
    b2 = eng.play(3)
    for k in b1:
        assert torch.equal(b1[k], b2[k]), k
    idx = b1["idx"].cpu().numpy()
    mask = b1["mask"].cpu().numpy()
    act = b1["act"].cpu().numpy()
    live = np.arange(300)[None, :] < idx[:, None]
    assert ((act >= 0) == (mask > 0))[live].all()
    assert np.allclose(b1["pol"].cpu().numpy().sum(-1)[mask > 0], 1.0, atol=1e-5)
    dice = b1["dice"].cpu().numpy()
    assert ((dice >= 1) & (dice <= 6))[live].all()
    assert np.allclose(b1["dice_dist"].cpu().numpy().sum(-1)[live], 1.0, atol=1e-5)


@pytest.mark.parametrize("games,lanes,T", [(30, 12, 200), (25, 8, 40)])
def test_classic_stream_equals_batch(cuda, games, lanes, T):
    """muz_classic_selfplay_stream == muz_classic_selfplay on a batch of `games` (dice, Dirichlet, tie-break
    and final noise keyed by game number and own step)."""
    from oracle import classic_nets as CN
    from exploring_muzero_on_dog_amd import classic as CL
    from exploring_muzero_on_dog_amd import game_agent_stochastic as GS
    from exploring_muzero_on_dog_amd import stochastic as S
    C = CL.num_channels(4)
    net = S.DeviceClassicNet(CN.init_params(C, seed=12), C)
    batch = GS.StochasticSelfPlayEngine(net, games, max_steps=T, num_simulations=6, max_depth=5)
    want = {k: v.clone() for k, v in batch.play(31, 1.0).items()}
    eng = GS.StochasticSelfPlayEngine(net, lanes, max_steps=T, num_simulations=6, max_depth=5)
    got = eng.play_stream(games, 31, 1.0)
    for k in want:
        assert torch.equal(got[k], want[k]), k
    assert eng.last_stats["searches"] == batch.last_stats["searches"]
