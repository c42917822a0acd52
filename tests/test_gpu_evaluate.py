"""Evaluation harness (evaluate_agent.py) on the GPU: the random baseline is fair, the MuZero seat plays
legal games to the end, and results are reproducible."""
import pytest

from oracle import nets as ON

pytestmark = pytest.mark.gpu


def test_random_baseline_is_fair(cuda):
    from exploring_muzero_on_dog_amd import evaluate as EV
    r = EV.play_vs_random(None, 1024, seed=3)
    assert r["finished"] == 1024
    # teams: seats 0 and 2 win together; with random play both teams win about half of the games
    assert r["seat_wins"][0] == r["seat_wins"][2] and r["seat_wins"][1] == r["seat_wins"][3]
    assert abs(r["wins"] / 1024 - 0.5) < 0.07, r


def test_muzero_seat_vs_random(cuda):
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import evaluate as EV
    from exploring_muzero_on_dog_amd import nets as N
    C = E.num_channels(4)
    net = N.DeviceNet(ON.init_params(C, seed=1), C)
    a = EV.play_vs_random(net, 128, num_simulations=8, max_depth=6, seed=5)
    b = EV.play_vs_random(net, 128, num_simulations=8, max_depth=6, seed=5)
    assert a == b and a["finished"] == 128 and sum(a["seat_wins"]) > 0
    z = EV.compare_agents_statistically(net, None, 128, batch_size=128, num_simulations=8, max_depth=6)
    assert 0.0 <= z["p"] <= 1.0
