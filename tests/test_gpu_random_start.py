"""env_reset's random starting player (starting_player < 0 or >= P: deterministic_madn.py:60-62, classic_madn.py:70-72,
dog.py:102-104) on the device against the oracles.  The reference draws the seat with jax threefry from the reset
seed, which is not restated: the engine draws it from its counter RNG (csrc/rng.hpp start_seat, oracle start_seat),
so WHICH seat a seed gives is parity-unpinned; the rest of the reset and the uniform spread over seats are checked."""
import numpy as np
import pytest
import torch

from oracle import classic_madn as cm
from oracle import detmadn as dm
from oracle import dog as dg
from tests.dog_states import RULE_SETS, diff

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("P,sp", [(2, -1), (3, 7), (4, -1)])
def test_det_random_start_matches_oracle(cuda, P, sp):
    from exploring_muzero_on_dog_amd import detmadn as E
    seeds = np.random.default_rng(P).integers(0, 2**31, 400)
    gpu = E.env_reset(400, num_players=P, starting_player=sp, seeds=seeds, **dm.SELFPLAY_RULES)
    cp = gpu.current_player.cpu().numpy()
    pins = gpu.pins.cpu().numpy().T.reshape(400, P, 4)
    for b, s in enumerate(seeds):
        e = dm.env_reset(num_players=P, starting_player=sp, seed=int(s), **dm.SELFPLAY_RULES)
        assert cp[b] == e.current_player and np.array_equal(pins[b], e.pins), b
    assert set(cp.tolist()) == set(range(P))                 # every seat starts some game
    fixed = E.env_reset(8, num_players=P, starting_player=1, seeds=seeds[:8], **dm.SELFPLAY_RULES)
    assert (fixed.current_player.cpu().numpy() == 1).all()   # a valid seat ignores the seeds
    from exploring_muzero_on_dog_amd import lib as L
    with pytest.raises(L.MuzError):                          # no seed: the unseeded reset cannot draw
        E.env_reset(8, num_players=P, starting_player=sp, **dm.SELFPLAY_RULES)


def test_classic_random_start_matches_oracle(cuda):
    from exploring_muzero_on_dog_amd import classic as CL
    seeds = np.random.default_rng(9).integers(0, 2**31, 300)
    gpu = CL.env_reset(300, num_players=4, starting_player=-1, seeds=seeds, enable_teams=True)
    cp = gpu.current_player.cpu().numpy()
    for b, s in enumerate(seeds):
        assert cp[b] == cm.env_reset(num_players=4, starting_player=-1, seed=int(s), enable_teams=True).current_player
    assert set(cp.tolist()) == {0, 1, 2, 3}


def test_dog_random_start_matches_oracle(cuda):
    from exploring_muzero_on_dog_amd import dog as D
    kw = dict(RULE_SETS["selfplay_4p_teams"])
    kw.pop("num_players")
    n, seed = 96, 31
    gpu = D.env_reset(n, num_players=4, starting_player=-1, seed=seed, **kw)
    envs = [dg.env_reset(4, starting_player=-1, start_key=dg.engine_start_key(seed, g),
                         shuffle_keys=dg.engine_shuffle_keys(seed, g), **kw) for g in range(n)]
    assert diff(D.to_host(gpu), envs) is None
    assert len({e.round_starter for e in envs}) == 4          # the first deal's round starter is the drawn seat


def test_selfplay_rejects_random_start(cuda):
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import lib as L
    from exploring_muzero_on_dog_amd import nets as N
    from oracle import nets as ON
    C = dm.num_channels(2)
    net = N.DeviceNet(ON.init_params(C, seed=1), C)
    with pytest.raises(L.MuzError):
        GA.SelfPlayEngine(net, 8, num_players=2, max_steps=8, num_simulations=2, max_depth=2,
                          starting_player=-1).play(1, 1.0)
