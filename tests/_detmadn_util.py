"""Test helpers: seeded random play with the CPU oracle, and oracle<->SoA conversion."""
import numpy as np

from oracle import detmadn as dm

RULE_SETS = {
    # config (b): game_agent.py:12-22 rules at 2 players (teams forced off)
    "selfplay_2p": dict(num_players=2, **dm.SELFPLAY_RULES),
    # training rules: 4 players, teams
    "selfplay_4p_teams": dict(num_players=4, **dm.SELFPLAY_RULES),
    # every optional branch switched on (circular, start blocking, friendly fire, must traverse, no jump)
    "exotic_4p": dict(num_players=4, enable_teams=False, enable_initial_free_pin=True, enable_circular_board=True,
                      enable_start_blocking=True, enable_jump_in_goal_area=False, enable_friendly_fire=True,
                      enable_start_on_1=False, enable_bonus_turn_on_6=True, must_traverse_start=True),
    "exotic_2p": dict(num_players=2, enable_teams=False, enable_initial_free_pin=False, enable_circular_board=False,
                      enable_start_blocking=True, enable_jump_in_goal_area=False, enable_friendly_fire=False,
                      enable_start_on_1=True, enable_bonus_turn_on_6=False, must_traverse_start=True),
}


def random_play_transitions(rule_set, n_games, seed, max_plies=600, p_illegal=0.1):
    """Yield (ply, list_of(env, kind, action)) for lockstep checking.

    kind = 'step' (action index, possibly illegal) or 'nostep' (no legal move)."""
    kw = RULE_SETS[rule_set]
    rng = np.random.default_rng(seed)
    envs = [dm.env_reset(**kw) for _ in range(n_games)]
    for ply in range(max_plies):
        batch = []
        for i, env in enumerate(envs):
            if env.done:
                continue
            va = dm.valid_action(env).flatten()
            if va.any():
                if rng.random() < p_illegal:
                    a = int(rng.integers(0, 24))
                else:
                    a = int(rng.choice(np.flatnonzero(va)))
                batch.append((i, env, "step", a))
            else:
                batch.append((i, env, "nostep", -1))
        if not batch:
            return
        yield ply, batch
        for i, env, kind, a in batch:
            if kind == "step":
                envs[i] = dm.env_step(env, dm.map_action(a))[0]
            else:
                envs[i] = dm.no_step(env)[0]


def legal_bits_oracle(env):
    va = dm.valid_action(env).flatten()
    return int(sum(1 << i for i in range(24) if va[i]))
