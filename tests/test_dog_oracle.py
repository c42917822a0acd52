"""DOG oracle self-consistency (CPU): the broadcast hot-7 legality equals the scalar restatement that the
golden vectors pin, the engine's deal keys are deterministic and shuffle like the reference's argsort,
and seeded random play conserves the cards."""
import numpy as np
import pytest

from oracle import dog as dg
from tests.dog_states import RULE_SETS, random_state, reset


@pytest.mark.parametrize("rule_set", sorted(RULE_SETS))
def test_val_action_7_all_matches_scalar(rule_set):
    rng = np.random.default_rng(3)
    for g in range(40):
        env = random_state(rng, RULE_SETS[rule_set], 11, g)
        got = dg.val_action_7_all(env)
        want = np.array([dg.val_action_7(env, d) for d in dg.DISTS_7_4])
        assert np.array_equal(got, want), (g, np.flatnonzero(got != want))


def test_engine_shuffle_keys_deterministic():
    kw = RULE_SETS["selfplay_4p_teams"]
    a, b, c = reset(kw, 5, 0), reset(kw, 5, 0), reset(kw, 5, 1)
    assert np.array_equal(a.hands, b.hands) and not np.array_equal(a.hands, c.hands)
    assert a.hands.sum() == 24 and a.deck.sum() == 110 - 24 and a.deal == 1 and a.phase == 1
    k = dg.engine_shuffle_keys(5, 0)(a)
    assert k.dtype == np.float32 and k.shape == (120,) and (k >= 0).all() and (k < 1).all()
    assert len(np.unique(k)) > 110


@pytest.mark.parametrize("rule_set", ["selfplay_4p_teams", "default_2p"])
def test_oracle_random_play_conserves_cards(rule_set):
    """Cards only move deck -> hands -> table; a reset_deck refills.  Track the table pile."""
    kw = RULE_SETS[rule_set]
    env = reset(kw, 9, 0)
    keys = dg.engine_shuffle_keys(9, 0)
    played = 0
    for t in range(300):
        if env.done:
            break
        m = dg.valid_actions(env)
        a = dg.engine_random_action(m, 9, 0, t)
        before = env.hands.astype(np.int64).sum() + env.deck.astype(np.int64).sum()
        if a < 0:
            env, r, _ = dg.no_step(env, keys)
            continue
        deal0 = env.deal
        env, r, _ = dg.env_step(env, a, keys)
        assert r >= 0, "a legal action is never refused"
        after = env.hands.astype(np.int64).sum() + env.deck.astype(np.int64).sum()
        if env.deal == deal0 and a < 792:
            assert after == before - 1
            played += 1
    assert played > 50
