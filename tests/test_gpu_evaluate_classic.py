"""Classic-MADN evaluation harness on the GPU (MuZero_Classic_MADN/evaluate_agent_stochastic.py):
the agents' kernel (muz_classic_policy_action: the random and the rule-based agent of play_eval_loop_jitted) equals
oracle/evaluate.py's restatement on 2 rule sets, random vs random is fair, the rule-based team against random seats
(the table goes to gpurun_out/parity.log), the Stochastic MuZero seats play legal games to the end reproducibly, and
test_agent_vs_random / compare_agents_statistically run end to end.  Win-rate parity is unpinned (the reference's
trained classic params are a pickle that is not in the repository)."""
import numpy as np
import pytest
import torch

from oracle import classic_madn as cm
from tests._parity import log

pytestmark = pytest.mark.gpu

EVAL_RULES = dict(enable_teams=True, enable_initial_free_pin=True, enable_circular_board=False,
                  enable_friendly_fire=True, enable_start_blocking=False, enable_jump_in_goal_area=True,
                  enable_start_on_1=True, enable_bonus_turn_on_6=True, must_traverse_start=False,
                  enable_dice_rethrow=False)
RULE_SETS = {
    "eval_4p_teams": dict(num_players=4, **EVAL_RULES),        # evaluate_agent_stochastic.py:938-948
    "exotic_4p": dict(num_players=4, enable_teams=False, enable_initial_free_pin=True, enable_circular_board=True,
                      enable_start_blocking=True, enable_jump_in_goal_area=False, enable_friendly_fire=True,
                      enable_start_on_1=False, enable_bonus_turn_on_6=True, enable_dice_rethrow=True,
                      must_traverse_start=True),
}


def _states(kw, n, seed):
    """Seeded random classic play (die thrown every ply), states sampled after their throw."""
    rng = np.random.default_rng(seed)
    envs = [cm.env_reset(**kw) for _ in range(32)]
    out = []
    for _ in range(300):
        nxt = []
        for e in envs:
            if e.done:
                nxt.append(e)
                continue
            e = cm.throw_die(e, float(rng.random()))
            out.append(e)
            va = cm.valid_action(e)
            e = cm.env_step(e, int(rng.choice(np.flatnonzero(va))))[0] if va.any() else cm.no_step(e)[0]
            nxt.append(e)
        envs = nxt
    pick = rng.choice(len(out), size=min(n, len(out)), replace=False)
    return [out[i] for i in pick]


@pytest.mark.parametrize("rule_set", sorted(RULE_SETS))
def test_classic_policy_kernel_matches_oracle(cuda, rule_set):
    from exploring_muzero_on_dog_amd import classic as CL
    from exploring_muzero_on_dog_amd import evaluate as EV
    from oracle import evaluate as OE
    kw = RULE_SETS[rule_set]
    envs = _states(kw, 512, 3)
    rules = CL.make_rules(num_players=4, starting_player=0, **{k: v for k, v in kw.items() if k != "num_players"})
    st = CL.state_from_host(pins=np.stack([e.pins for e in envs]), current_player=[e.current_player for e in envs],
                            rules=rules, die=np.array([e.die for e in envs], np.int8),
                            done=np.array([e.done for e in envs], np.uint8), board=np.stack([e.board for e in envs]))
    bits = CL.legal_bits(st)
    gid = torch.arange(len(envs), dtype=torch.int32, device="cuda") + 77
    hits = 0
    for turn in (0, 9):
        ra = EV.classic_policy_action(st, bits, "random_agent", 5, turn, game_id=gid).cpu().numpy()
        rb = EV.classic_policy_action(st, bits, "rule_based_agent", 5, turn, game_id=gid).cpu().numpy()
        want_r = [OE.classic_random_action(e, 5, 77 + i, turn) for i, e in enumerate(envs)]
        want_b = [OE.classic_rule_based_action(e, 5, 77 + i, turn) for i, e in enumerate(envs)]
        assert ra.tolist() == want_r
        assert rb.tolist() == want_b
        va = np.stack([cm.valid_action(e) for e in envs])
        assert all(va[i, a] for i, a in enumerate(rb) if a >= 0)
        assert all((a < 0) == (not va[i].any()) for i, a in enumerate(rb))
        hits += sum(float(OE.classic_rule_based_scores(e)[0].max()) > 0 for e in envs)
    assert hits > 0   # the bonuses are exercised


def test_classic_random_is_fair_and_rule_based_table(cuda):
    from exploring_muzero_on_dog_amd import evaluate as EV
    B = 128
    n = 4 * B
    rr = EV.evaluate_agent_parallel_classic(["random_agent"] * 4, batch_size=B, seed=1)
    w = rr["wins_per_player"]
    assert rr["finished"] == n
    assert w[0] == w[2] and w[1] == w[3] and w[0] + w[1] == n      # teams: one team wins every finished game
    assert abs(w[0] / n - 0.5) < 4 * (0.25 / n) ** 0.5, w          # fair within 4 sigma of the binomial
    log(f"classic eval random vs random ({n} games, 4 x {B} per starting player): winners {rr['winners']}, "
        f"progress {np.round(rr['average_progress'], 2).tolist()}")
    tab = {}
    for name, seats in (("rule seats 0&2", ["rule_based_agent", "random_agent"] * 2),
                        ("rule seats 1&3", ["random_agent", "rule_based_agent"] * 2)):
        r = EV.evaluate_agent_parallel_classic(seats, batch_size=B, seed=2)
        assert r["finished"] == n
        wp = r["wins_per_player"]
        rule_share = (wp[0] if seats[0] == "rule_based_agent" else wp[1]) / n
        tab[name] = rule_share
        log(f"classic eval {name} vs random ({n} games): winners {r['winners']}, wins per player {wp}, rule-based "
            f"team share {rule_share:.3f}, progress per player {np.round(r['progress_per_player'], 2).tolist()}")
    # the rule-based agent of play_eval_loop_jitted prefers goal entries, leaving home and hits: it beats random seats
    assert min(tab.values()) > 0.5 + 3 * (0.25 / n) ** 0.5, tab


def test_classic_muzero_seats_reproducible_and_vs_random(cuda):
    from exploring_muzero_on_dog_amd import classic as CL
    from exploring_muzero_on_dog_amd import evaluate as EV
    from oracle import classic_nets as CN
    C = CL.num_channels(4)
    params = CN.init_params(C, seed=3)
    kw = dict(batch_size=6, num_simulations=8, max_depth=6, seed=4)
    a = EV.evaluate_agent_parallel_classic([params, "random_agent", None, "rule_based_agent"], **kw)
    b = EV.evaluate_agent_parallel_classic([params, "random_agent", None, "rule_based_agent"], **kw)
    assert a["winners"] == b["winners"] and a["average_progress"] == b["average_progress"]
    w = a["wins_per_player"]
    assert a["finished"] == 24 and w[0] == w[2] and w[1] == w[3] and w[0] + w[1] == 24   # teams: 2 winners a game
    r1 = EV.play_vs_random_classic(params, 32, num_simulations=8, max_depth=6, seed=9)
    r2 = EV.play_vs_random_classic(params, 32, num_simulations=8, max_depth=6, seed=9)
    assert r1 == r2 and r1["finished"] == 32 and r1["seat_wins"][0] == r1["seat_wins"][2]
    z = EV.compare_agents_statistically_classic("rule_based_agent", "random_agent", 256, batch_size=128)
    assert 0.0 <= z["p"] <= 1.0 and z["winrate1"] > z["winrate2"], z
    log(f"classic test_agent_vs_random: rule-based {z['winrate1']:.3f}, random {z['winrate2']:.3f} of 256 games "
        f"(seat 0 + partner vs random), z {z['z']:.2f}, p {z['p']:.2e}")
