"""calculate_progress (evaluate_agent.py:129-195) in torch against the NumPy restatement, on CPU tensors."""
import numpy as np
import pytest

from oracle import detmadn as dm
from oracle import evaluate as OE
from tests._detmadn_util import RULE_SETS, random_play_transitions


@pytest.mark.parametrize("rule_set", ["selfplay_4p_teams", "selfplay_2p", "exotic_4p"])
def test_calculate_progress_matches_oracle(rule_set):
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import evaluate as EV
    kw = RULE_SETS[rule_set]
    envs = []
    for _, batch in random_play_transitions(rule_set, 8, 3, max_plies=400, p_illegal=0.0):
        envs.extend(e for _, e, _, _ in batch[::3])
    envs = envs[::5]
    rules = E.make_rules(kw["num_players"], **{k: v for k, v in kw.items() if k != "num_players"})
    st = E.state_from_host(np.stack([e.pins for e in envs]), [e.current_player for e in envs], rules,
                           action_set=np.stack([e.action_set for e in envs]), board=np.stack([e.board for e in envs]),
                           device="cpu")
    got = EV.calculate_progress(st, kw["must_traverse_start"]).numpy()
    want = np.array([[OE.calculate_progress(e, p) for p in range(e.num_players)] for e in envs])
    assert np.array_equal(got, want)
    assert (want > 0).any()


def test_manual_get_winner_matches_host_winners():
    import torch
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import evaluate as EV
    kw = RULE_SETS["selfplay_4p_teams"]
    rules = E.make_rules(4, **{k: v for k, v in kw.items() if k != "num_players"})
    goals = np.arange(40, 56).reshape(4, 4)
    cases = [[goals[0], goals[1], goals[2], [-1] * 4], [goals[0], goals[1], goals[2], goals[3]],
             [goals[0], [-1] * 4, goals[2], [-1] * 4], [[-1] * 4, goals[1], [5, -1, -1, -1], goals[3]]]
    pins = np.array(cases, np.int8)
    st = E.state_from_host(pins, [0] * 4, rules, device="cpu")
    got = EV.winners(st, True).numpy()
    for g, p in enumerate(pins):
        e = dm.env_reset(num_players=4, **dm.SELFPLAY_RULES)
        e = e.replace(pins=p, board=dm.set_pins_on_board(e.board, p))
        assert np.array_equal(got[g], OE.manual_get_winner(e)), g


def test_classic_rule_based_scores_crafted_state():
    """do_rule_based of the classic eval loop (evaluate_agent_stochastic.py:806-866) on a crafted state: pin 1 enters
    the goal (+5), pin 2 hits an opponent (+2.5), the two home pins score the out-of-home bonus (3.0 with >= 2 at home)
    but are illegal with a 3; the sampled pin is always a legal one."""
    from oracle import classic_madn as cm
    rules = dict(enable_teams=True, enable_initial_free_pin=False, enable_circular_board=False,
                 enable_friendly_fire=True, enable_start_blocking=False, enable_jump_in_goal_area=True,
                 enable_start_on_1=True, enable_bonus_turn_on_6=True, must_traverse_start=False,
                 enable_dice_rethrow=False)
    e = cm.env_reset(num_players=4, **rules)
    pins = -np.ones((4, 4), np.int8)
    pins[0] = [-1, 38, 5, -1]
    pins[1, 0] = 8
    e = e.replace(pins=pins, board=cm.set_pins_on_board(-np.ones_like(e.board), pins), die=3)
    sc, va = OE.classic_rule_based_scores(e)
    assert sc.tolist() == [3.0, 5.0, 2.5, 3.0]
    assert va.tolist() == [False, True, True, False]
    picks = {OE.classic_rule_based_action(e, 1, g, 0) for g in range(64)}
    assert picks <= {1, 2} and 1 in picks
    assert {OE.classic_random_action(e, 1, g, 0) for g in range(64)} == {1, 2}
