"""CPU oracle for the evaluation harness of MuZero_det_MADN/evaluate_agent.py (TEST INFRASTRUCTURE ONLY).

  rule_based_action   do_rule_based (evaluate_agent.py:777-864; scores restated with their quirks: the
                      base score jnp.repeat(abundance, 4)[a] = abundance[a // 4], landing cells from
                      cur + jnp.arange(6), the unsubstituted current player) + jax.random.categorical as
                      argmax(logits + Gumbel) with the engine's counter Gumbel draw
  random_action       do_random (770-775) the same way over 0 / -1e9 logits
  calculate_progress  calculate_progress (129-195): rotated pin positions, sorted, greedily matched to the
                      rotated goal cells 40..43 by repeated masked argmin of |pin - goal|
  manual_get_winner   16-45
  classic_*           the classic agents of MuZero_Classic_MADN/evaluate_agent_stochastic.py play_eval_loop_jitted:
                      do_random (800-804) and do_rule_based (806-866: per pin, the landing cell of cur + die of the
                      UNSUBSTITUTED current player, goal 5 / out 3 or 2 / hit 2.5, base 0, temperature 0.25), sampled
                      with the first 4 of the same counter Gumbel draws
Parity of the random SOURCE is unpinned (the reference draws with jax threefry); given the draws the
restatement is exact.
"""
from __future__ import annotations

import numpy as np

from oracle import detmadn as dm
from oracle.dog import M64, _game_key, _mix64, _u24

F32 = np.float32
POLICY_STREAM = 0x9011C7A6E47
TINY = np.finfo(np.float32).tiny
RULE_AGENT = dict(temperature=0.25, goal_bonus=5.0, out_many=3.0, out_few=2.0, hit_bonus=2.0)   # 777-864


def policy_gumbel(seed, game, turn):
    key = _game_key(seed ^ POLICY_STREAM, game, turn)
    out = np.empty(24, F32)
    for a in range(24):
        u = max(F32(_u24(_mix64(key ^ (((a + 1) * 0xD6E8FEB86659FD93) & M64)))), F32(TINY))
        out[a] = -np.log(-np.log(F32(u)))
    return out


def random_action(env, seed, game, turn):
    va = dm.valid_action(env).flatten()
    if not va.any():
        return -1
    logits = np.where(va, F32(0.0), F32(-1e9)).astype(F32)
    return int(np.argmax((logits + policy_gumbel(seed, game, turn)).astype(F32)))


def rule_based_scores(env, agent=RULE_AGENT):
    """The rule-based agent's per-action scores (24,) before masking."""
    va = dm.valid_action(env).flatten()
    cp = env.current_player
    P = env.num_players
    bs = env.board_size
    cur = env.pins[cp].astype(np.int64)[:, None]
    moved = cur + np.arange(6)[None, :]
    fitted = moved % bs
    x = moved - int(env.target[cp]) - int(env.rules["must_traverse_start"])
    goal = env.goal[cp].astype(np.int64)
    gx = goal[np.clip(np.where(x - 1 < 0, x - 1 + 4, x - 1), 0, 3)]
    new = np.where(cur < 0, int(env.start[cp]),
                   np.where(cur >= bs, moved, np.where((4 >= x) & (x > 0) & (cur <= int(env.target[cp])), gx, fitted)))
    opp = np.ones((P, 4), bool)
    opp[cp] = False
    if env.rules["enable_teams"]:
        opp[(cp + 2) % 4] = False
    opp_pins = np.where(opp, env.pins, -1).flatten()
    home = int((env.pins[cp] < 0).sum())
    counts = va.reshape(4, 6).sum(0).astype(F32)
    abund = (counts / max(F32(counts.sum()), F32(1.0))).astype(F32)
    base = np.repeat(abund, 4)
    gb = np.where(np.isin(new, goal) & (cur < bs), F32(agent["goal_bonus"]), F32(0.0)).flatten()
    ob = np.where((cur < 0) & (new == int(env.start[cp])), F32(agent["out_many"] if home >= 2 else agent["out_few"]),
                  F32(0.0)).flatten()
    hb = np.where((new != cur) & np.isin(new, opp_pins), F32(agent["hit_bonus"]), F32(0.0)).flatten()
    return (((base + gb).astype(F32) + ob).astype(F32) + hb).astype(F32), va


def rule_based_action(env, seed, game, turn, agent=RULE_AGENT):
    sc, va = rule_based_scores(env, agent)
    if not va.any():
        return -1
    logits = np.where(va, (sc / F32(agent["temperature"])).astype(F32), F32(-np.inf))
    return int(np.argmax((logits + policy_gumbel(seed, game, turn)).astype(F32)))


def calculate_progress(env, player_idx):
    bs = env.board_size
    distance = bs // env.num_players
    pins = env.pins[player_idx].astype(np.int64)
    goals = env.goal[player_idx].astype(np.int64)
    trav = int(env.rules["must_traverse_start"])
    rot = np.where(pins < 0, pins - 5, np.where(pins < bs, (pins - distance * player_idx) % bs - trav,
                                                 bs + (pins - goals[0])))
    rg = np.arange(bs, bs + 4)
    sp = np.sort(rot)
    dmat = np.abs(sp[:, None] - rg[None, :]).astype(np.float64)
    mask = np.ones((4, 4), bool)
    total = 0.0
    for _ in range(4):
        flat = int(np.argmin(np.where(mask, dmat, np.inf)))
        r, c = flat // 4, flat % 4
        total += dmat[r, c]
        mask[r, :] = False
        mask[:, c] = False
    return np.float32(total)


def manual_get_winner(env):
    done = np.array([dm.is_player_done(env.num_players, env.board, env.goal, p) for p in range(4)])
    if not env.rules["enable_teams"]:
        return done
    t0, t1 = done[0] & done[2], done[1] & done[3]
    if (t0 & t1) or not (t0 | t1):
        return np.zeros(4, bool)
    return np.array([True, False, True, False]) if t0 else np.array([False, True, False, True])


# ---- classic MADN agents (MuZero_Classic_MADN/evaluate_agent_stochastic.py) -------------------------------------
CLASSIC_RULE_AGENT = dict(temperature=0.25, goal_bonus=5.0, out_many=3.0, out_few=2.0, hit_bonus=2.5)   # 806-866


def classic_random_action(env, seed, game, turn):
    """do_random (evaluate_agent_stochastic.py:800-804) over the 4 pins."""
    from oracle import classic_madn as cm
    va = cm.valid_action(env)
    if not va.any():
        return -1
    logits = np.where(va, F32(0.0), F32(-1e9)).astype(F32)
    return int(np.argmax((logits + policy_gumbel(seed, game, turn)[:4]).astype(F32)))


def classic_rule_based_scores(env, agent=CLASSIC_RULE_AGENT):
    """do_rule_based (806-866): the score (4,) of every pin before masking, and the legal mask."""
    from oracle import classic_madn as cm
    va = cm.valid_action(env)
    cp = env.current_player
    P = env.num_players
    bs = env.board_size
    cur = env.pins[cp].astype(np.int64)
    moved = cur + int(env.die)
    fitted = moved % bs
    x = moved - int(env.target[cp]) - int(env.rules["must_traverse_start"])
    goal = env.goal[cp].astype(np.int64)
    gx = goal[np.clip(np.where(x - 1 < 0, x - 1 + 4, x - 1), 0, 3)]
    start = int(env.start[cp])
    new = np.where(cur < 0, start,
                   np.where(cur >= bs, moved, np.where((4 >= x) & (x > 0) & (cur <= int(env.target[cp])), gx, fitted)))
    opp = np.ones((P, 4), bool)
    opp[cp] = False
    if env.rules["enable_teams"]:
        opp[(cp + 2) % 4] = False
    opp_pins = np.where(opp, env.pins, -1).flatten()
    home = int((cur < 0).sum())
    gb = np.where(np.isin(new, goal) & (cur < bs), F32(agent["goal_bonus"]), F32(0.0))
    ob = np.where((cur < 0) & (new == start), F32(agent["out_many"] if home >= 2 else agent["out_few"]), F32(0.0))
    hb = np.where((new != cur) & np.isin(new, opp_pins), F32(agent["hit_bonus"]), F32(0.0))
    return (((np.zeros(4, F32) + gb).astype(F32) + ob).astype(F32) + hb).astype(F32), va


def classic_rule_based_action(env, seed, game, turn, agent=CLASSIC_RULE_AGENT):
    sc, va = classic_rule_based_scores(env, agent)
    if not va.any():
        return -1
    logits = np.where(va, (sc / F32(agent["temperature"])).astype(F32), F32(-np.inf))
    return int(np.argmax((logits + policy_gumbel(seed, game, turn)[:4]).astype(F32)))
