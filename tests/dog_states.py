"""Random DOG states for the oracle / GPU lockstep tests (test helper, not a test module).

``random_state`` scatters pins over home, the track and the player's own goal (distinct cells), deals
random hands and picks the turn bookkeeping at random, so that one ply reaches captures, hot-7 path
hits, goal entries, finished players (team substitution) and game ends without playing hundreds of
plies first.  ``RULE_SETS`` are the configurations the tests sweep."""
import numpy as np

from oracle import dog as dg

RULE_SETS = {
    # config (d): MuZero_DOG/game_agent.py:12-23, 4 players in teams (swap phase on)
    "selfplay_4p_teams": dict(num_players=4, **dg.SELFPLAY_RULES),
    # env_reset defaults (dog.py:83-100), 2 players -- the setting of DOG/test.py
    "default_2p": dict(num_players=2, **dg.DEFAULT_RULES),
    "exotic_3p": dict(num_players=3, enable_teams=False, enable_initial_free_pin=True, enable_circular_board=False,
                      enable_start_blocking=True, enable_jump_in_goal_area=False, enable_friendly_fire=False,
                      must_traverse_start=False),
    "exotic_4p": dict(num_players=4, enable_teams=True, enable_initial_free_pin=False, enable_circular_board=False,
                      enable_start_blocking=False, enable_jump_in_goal_area=True, enable_friendly_fire=True,
                      must_traverse_start=False),
}


def reset(kw, seed, game):
    return dg.env_reset(shuffle_keys=dg.engine_shuffle_keys(seed, game), **kw)


def random_state(rng, kw, seed, game):
    env = reset(kw, seed, game)
    P = env.num_players
    pins = -np.ones((P, 4), np.int32)
    used = set()
    for p in range(P):
        goal_free = list(env.goal[p])
        for k in range(4):
            u = rng.random()
            if u < 0.2:
                continue
            if u < 0.45 and goal_free:
                cell = int(goal_free.pop(int(rng.integers(0, len(goal_free)))))
            else:
                free = [c for c in range(40) if c not in used]
                cell = int(free[int(rng.integers(0, len(free)))])
            used.add(cell)
            pins[p, k] = cell
    board = dg.set_pins_on_board(-np.ones(56, np.int8), pins)
    hands = rng.integers(0, 3, (P, 14)).astype(np.int8) * (rng.random((P, 14)) < 0.35)
    hands[rng.random(P) < 0.15] = 0                                  # some players out of cards
    deck = np.clip(8 - hands.sum(0), 0, 8).astype(np.int8)
    deck[rng.random(14) < 0.5] = 0                                    # thin deck -> reset_deck paths
    teams4 = env.rules["enable_teams"] and P == 4
    phase = int(teams4 and rng.random() < 0.25)
    return env.replace(pins=pins, board=board, hands=hands.astype(np.int8), deck=deck,
                       current_player=int(rng.integers(0, P)), round_starter=int(rng.integers(0, P)), phase=phase,
                       hand_size=int(rng.integers(2, 7)), deal=int(rng.integers(0, 9)),
                       swap_choices=np.full(4, -1, np.int8))


def fields_of(envs):
    """Host SoA dict for exploring_muzero_on_dog_amd.dog.state_from_host."""
    return dict(board=np.stack([e.board for e in envs]), pins=np.stack([e.pins for e in envs]),
                deck=np.stack([e.deck for e in envs]), hands=np.stack([e.hands for e in envs]),
                swap_choices=np.stack([e.swap_choices for e in envs]),
                current_player=np.array([e.current_player for e in envs]),
                round_starter=np.array([e.round_starter for e in envs]), phase=np.array([e.phase for e in envs]),
                hand_size=np.array([e.hand_size for e in envs]), reward=np.array([e.reward for e in envs]),
                done=np.array([e.done for e in envs], np.uint8), deal=np.array([e.deal for e in envs]))


def diff(host, envs):
    """First mismatch between a device host view (dog.to_host) and oracle states, or None."""
    for b, e in enumerate(envs):
        want = dict(board=e.board, pins=e.pins, deck=e.deck, hands=e.hands, swap_choices=e.swap_choices,
                    current_player=e.current_player, round_starter=e.round_starter, phase=e.phase,
                    hand_size=e.hand_size, reward=e.reward, done=int(e.done), deal=e.deal)
        for k, v in want.items():
            if not np.array_equal(np.asarray(host[k][b]).astype(np.int64), np.asarray(v).astype(np.int64)):
                return b, k, np.asarray(host[k][b]).tolist(), np.asarray(v).tolist()
    return None
