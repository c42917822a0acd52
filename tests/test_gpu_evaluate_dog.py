"""DOG evaluation harness on the GPU (MuZero_DOG/evaluate_agent.py; VERDICT r5 "missing" 2): evaluate_agent_parallel
with random seats and with the DOG slice's MuZero seats -- reproducible, one winning team per finished game, the
progress table -- and the reference's rule-based agent rejected (it cannot run on the 806-action mask).  Win-rate
parity is unpinned (the reference's DOG networks and inference functions are `pass`); the table goes to
gpurun_out/parity.log."""
import numpy as np
import pytest

from tests._parity import log

pytestmark = pytest.mark.gpu


def _check_table(r, n):
    w = r["wins_per_player"]
    assert w[0] == w[2] and w[1] == w[3]          # teams: seats 0 & 2 win together, 1 & 3 together
    assert w[0] + w[1] == r["finished"] <= n      # one winning team per finished game
    assert len(r["average_progress"]) == 4 and all(len(x) == 4 for x in r["average_progress"])


def test_dog_random_seats_reproducible(cuda):
    from exploring_muzero_on_dog_amd import evaluate as EV
    B = 32
    a = EV.evaluate_agent_parallel_dog(["random_agent"] * 4, batch_size=B, seed=3)
    b = EV.evaluate_agent_parallel_dog(["random_agent"] * 4, batch_size=B, seed=3)
    assert a["winners"] == b["winners"] and a["average_progress"] == b["average_progress"]
    _check_table(a, 4 * B)
    assert a["finished"] > 0
    log(f"DOG eval random vs random ({4 * B} games, {a['turns']} turns): finished {a['finished']}, winners "
        f"{a['winners']}, progress per player {np.round(a['progress_per_player'], 2).tolist()}")


def test_dog_muzero_seats_play_legal_games(cuda):
    from exploring_muzero_on_dog_amd import evaluate as EV
    from exploring_muzero_on_dog_amd import muzero_dog as MD
    params = MD.init_muzero_params(4)
    kw = dict(batch_size=3, num_simulations=4, max_depth=4, seed=6, max_turns=400)
    a = EV.evaluate_agent_parallel_dog([params, "random_agent", None, "random_agent"], **kw)
    b = EV.evaluate_agent_parallel_dog([params, "random_agent", None, "random_agent"], **kw)
    assert a["winners"] == b["winners"] and a["average_progress"] == b["average_progress"]
    _check_table(a, 12)
    log(f"DOG eval MuZero seats 0 & 2 (S 4, D 4) vs random (12 games, <= 400 turns): finished {a['finished']}, "
        f"winners {a['winners']}")


def test_dog_rule_based_agent_rejected(cuda):
    from exploring_muzero_on_dog_amd import evaluate as EV
    with pytest.raises(ValueError, match="cannot run"):
        EV.evaluate_agent_parallel_dog(["rule_based_agent", "random_agent"] * 2, batch_size=1)
