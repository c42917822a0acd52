"""The reference-signature entry points (GPU): play_n_games_v3 / run_muzero_mcts of MuZero_det_MADN and
their classic (Stochastic MuZero) counterparts take init_muzero_params' nested Flax dict and a PRNG key,
and return exactly what the device-native engine returns for the same weights and seed."""
import numpy as np
import pytest
import torch

from oracle import classic_madn as cm
from oracle import detmadn as dm

pytestmark = pytest.mark.gpu


def _m():
    from exploring_muzero_on_dog_amd import checkpoint as CK
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import game_agent_stochastic as GS
    from exploring_muzero_on_dog_amd import mcts as M
    from exploring_muzero_on_dog_amd import nets as N
    from exploring_muzero_on_dog_amd import stochastic as ST
    return CK, GA, GS, M, N, ST


@pytest.mark.parametrize("P", [2, 4])
def test_det_play_n_games_v3_reference_signature(cuda, P):
    CK, GA, GS, M, N, ST = _m()
    C = dm.num_channels(P)
    flat = N.init_muzero_params(3, C)
    tree = CK.flat_to_muzero_tree(flat)
    got = GA.play_n_games_v3(tree, np.array([0, 77], np.uint32), (C, 56), 24, 8, 4, 120, 1.0)
    eng = GA.SelfPlayEngine(N.DeviceNet(flat, C), 24, num_players=P, max_steps=120, num_simulations=8, max_depth=4)
    want = GA.reference_buffers(eng.play(77, 1.0), GA.REFERENCE_DTYPES)
    assert set(got) == set(GA.REFERENCE_DTYPES)
    # rows at or past idx hold the reference's initial values (game_agent.py:158-169: zeros, team -1)
    past = torch.arange(120, device="cuda")[None, :] >= got["idx"][:, None].long()
    assert bool(past.any()) or P == 4            # (4-player games usually run the whole 120 records)
    assert bool((got["team"][past] == -1).all()) and not bool(got["act"][past].any())
    assert not bool(got["obs"][past].any()) and not bool(got["pol"][past].any())
    for k, v in got.items():
        assert v.dtype == GA.REFERENCE_DTYPES[k], k
        assert tuple(v.shape) == tuple(want[k].shape), k
        assert torch.equal(v, want[k].to(v.dtype)), k
    assert got["obs"].dtype == torch.float32 and tuple(got["obs"].shape) == (24, 120, C, 56)
    keep = {k: v.clone() for k, v in got.items()}
    again = GA.play_n_games_v3(tree, 77, (C, 56), 24, 8, 4, 120, 1.0)   # int key == uint32[2] key (0, 77)
    assert torch.equal(again["act"], got["act"])
    GA.play_n_games_v3(tree, 78, (C, 56), 24, 8, 4, 120, 1.0)           # fresh copies: no aliasing of the engine
    assert all(torch.equal(keep[k], got[k]) for k in keep)


def test_det_run_muzero_mcts_reference_signature(cuda):
    CK, GA, GS, M, N, ST = _m()
    from tests.test_gpu_nets import random_obs
    C = dm.num_channels(2)
    flat = N.init_muzero_params(4, C)
    tree = CK.flat_to_muzero_tree(flat)
    obs, envs = random_obs("selfplay_2p", 40, 3)
    valid = np.stack([dm.valid_action(e).flatten() for e in envs])
    keep = valid.any(1)
    obs, valid = obs[keep], valid[keep]
    pol, rv = M.run_muzero_mcts(tree, 1234, obs, ~valid, 16, 8, 1.0)
    bits = torch.from_numpy((valid.astype(np.int64) << np.arange(24)).sum(1).astype(np.int32))
    pol2, rv2 = M.muzero_mcts(N.DeviceNet(flat, C), torch.from_numpy(obs).cuda(), bits, 16, 8, 1.0, seed=1234)
    assert torch.equal(pol.action, pol2.action) and torch.equal(pol.action_weights, pol2.action_weights)
    assert torch.equal(rv, rv2)
    ga = pol.action.cpu().numpy()
    assert valid[np.arange(len(ga)), ga].all()


def test_classic_reference_signatures(cuda):
    CK, GA, GS, M, N, ST = _m()
    C = cm.num_channels(4)
    flat = ST.init_classic_params(C, seed=6)
    tree = CK.flat_to_muzero_tree(flat)
    got = GS.play_n_games_v3(tree, 55, (C, 56), 12, 8, 4, 80, 1.0)
    eng = GS.StochasticSelfPlayEngine(ST.DeviceClassicNet(flat, C), 12, max_steps=80, num_simulations=8, max_depth=4)
    want = GA.reference_buffers(eng.play(55, 1.0), dict(GA.REFERENCE_DTYPES, dice=torch.int32,
                                                         dice_dist=torch.float32))
    past = torch.arange(80, device="cuda")[None, :] >= got["idx"][:, None].long()
    assert bool((got["team"][past] == -1).all()) and not bool(got["dice_dist"][past].any())
    for k, v in got.items():
        assert torch.equal(v, want[k].to(v.dtype)), k
    assert got["obs"].dtype == torch.float32
    from tests.test_gpu_stochastic import random_classic_states
    obs, envs = random_classic_states(32, 4)
    valid = np.stack([cm.valid_action(e) for e in envs])
    keep = valid.any(1)
    obs, valid = obs[keep], valid[keep]
    pol, rv = ST.run_stochastic_muzero_mcts(tree, 9, obs, ~valid, 16, 8, 1.0)
    bits = torch.from_numpy((valid.astype(np.int64) << np.arange(4)).sum(1).astype(np.int32))
    a2, w2, v2 = ST.stochastic_muzero_mcts(ST.DeviceClassicNet(flat, C), torch.from_numpy(obs).cuda(), bits, 16, 8, 1.0,
                                           seed=9)
    assert torch.equal(pol.action, a2) and torch.equal(pol.action_weights, w2) and torch.equal(rv, v2)


def test_play_n_games_v3_keeps_its_engine_across_weight_updates(cuda):
    """A test_training-style loop hands play_n_games_v3 new weights every iteration: the engine (state, workspace,
    GB-scale buffers) is reused and the new weights are the ones played (the cache used to miss)."""
    CK, GA, GS, M, N, ST = _m()
    C = dm.num_channels(2)
    tree1 = CK.flat_to_muzero_tree(N.init_muzero_params(3, C))
    tree2 = CK.flat_to_muzero_tree(N.init_muzero_params(4, C))
    GA.play_n_games_v3(tree1, 5, (C, 56), 16, 8, 4, 60, 1.0)
    eng1 = next(iter(GA._ENGINE_CACHE.values()))
    got = {k: v.clone() for k, v in GA.play_n_games_v3(tree2, 5, (C, 56), 16, 8, 4, 60, 1.0).items()}
    assert next(iter(GA._ENGINE_CACHE.values())) is eng1
    GA._ENGINE_CACHE.clear()
    N._NET_CACHE.clear()
    want = GA.play_n_games_v3(tree2, 5, (C, 56), 16, 8, 4, 60, 1.0)    # a fresh engine on tree2
    for k in ("act", "val", "pol", "idx"):
        assert torch.equal(got[k], want[k]), k


def test_learner_tree_version_drives_the_weight_cache(cuda):
    """The learner's live tree is fingerprinted by its update count (training.OptState.version), not its norms."""
    from exploring_muzero_on_dog_amd import training as T
    from exploring_muzero_on_dog_amd import learner as LR
    CK, GA, GS, M, N, ST = _m()
    C = dm.num_channels(2)
    opt = T.Optimizer(LR.Learner, 2, 0.005, 10, (), graph=False).init(N.init_muzero_params(3, C))
    f0 = N.params_fingerprint(opt.tree)
    assert f0 == (("version", 0),)
    net0 = N.as_device_net(opt.tree, C)
    assert N.as_device_net(opt.tree, C) is net0
    opt.version += 1                           # what train_step does after every learner step
    assert N.params_fingerprint(opt.tree) != f0
    assert N.as_device_net(opt.tree, C) is net0   # re-packed into the same live DeviceNet
