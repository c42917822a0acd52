"""Evaluation harness for det-MADN agents (SURVEY §8f "next" 3; MuZero_det_MADN/evaluate_agent.py).

  test_agent_vs_random          evaluate_agent.py:383-472: the agent plays seat 0 (and seat 2, its
                                partner, when teams are on) with a temperature-0 Gumbel search; the other
                                seats play uniformly random legal moves (multiactor_step_with_random_agent_v2,
                                474-646); no-move turns apply no_step; wins are counted at seat 0
                                (manual_get_winner 16-45); at most 2000 turns.
  compare_agents_statistically  648-713: both agents against random opponents, two-proportion z-test.

Everything runs batched on the GPU: one legal-mask launch per turn, the agent's games go through
encode -> root inference -> muz_gumbel_search as one sub-batch, the random seats draw from the legal
bitmask on the device, and env_step / no_step run on sub-batches of the SoA state.  Differences from the
reference, on purpose: the starting player cycles over the games (game % P) instead of a jax random draw,
and the random seats use torch's generator (the reference's jax keys are not restated).
"""
from __future__ import annotations

import math

import torch

from . import detmadn as E
from . import mcts as M
from . import nets as N

# MuZero_det_MADN/evaluate_agent.py uses the game_agent.py rules
RULES = dict(E.SELFPLAY_RULES)


def _sub(env: E.DetMADNState, idx: torch.Tensor) -> E.DetMADNState:
    return E.DetMADNState(env.board[:, idx].contiguous(), env.pins[:, idx].contiguous(),
                          env.current_player[idx].contiguous(), env.reward[idx].contiguous(),
                          env.done[idx].contiguous(), env.action_set[:, idx].contiguous(), env.rules, env.num_players)


def _put(env: E.DetMADNState, idx: torch.Tensor, sub: E.DetMADNState):
    env.board[:, idx] = sub.board
    env.pins[:, idx] = sub.pins
    env.current_player[idx] = sub.current_player
    env.reward[idx] = sub.reward
    env.done[idx] = sub.done
    env.action_set[:, idx] = sub.action_set


def random_legal(bits: torch.Tensor, gen: torch.Generator) -> torch.Tensor:
    """A uniformly random set bit of each 24-bit legal mask (jax.random.categorical over valid actions)."""
    mask = E.bits_to_mask(bits).reshape(bits.shape[0], -1).float()
    u = torch.rand(mask.shape, generator=gen, device=bits.device)
    return torch.argmax(torch.where(mask > 0, u, torch.full_like(u, -1.0)), dim=1).to(torch.int32)


def winners(env: E.DetMADNState, teams: bool) -> torch.Tensor:
    """manual_get_winner (evaluate_agent.py:16-45) -> bool [B, P]: players whose goal is full, or the
    finished team (and nobody when both or neither team is done)."""
    P = env.num_players
    pins = env.pins_bp().long()
    done_p = (pins >= 40).all(dim=2)                       # a player's pins only enter its own goal cells
    if not (teams and P == 4):
        return done_p
    t0 = done_p[:, 0] & done_p[:, 2]
    t1 = done_p[:, 1] & done_p[:, 3]
    ok = t0 ^ t1
    w = torch.zeros_like(done_p)
    w[:, 0] = w[:, 2] = ok & t0
    w[:, 1] = w[:, 3] = ok & t1
    return w


@torch.no_grad()
def play_vs_random(net: N.DeviceNet | None, num_games: int, num_players: int = 4, num_simulations: int = 50,
                   max_depth: int = 25, seed: int = 42, max_turns: int = 2000, rules: dict | None = None,
                   device="cuda") -> dict:
    """One batch of games, agent at seat 0 (+2 with teams), random elsewhere.  ``net=None`` makes the
    agent random too (the baseline).  Returns wins at seat 0, per-seat wins and pins in goal."""
    r = dict(RULES if rules is None else rules)
    teams = bool(r.get("enable_teams", False)) and num_players == 4
    P = num_players
    env = E.env_reset(num_games, num_players=P, device=device, **r)
    # starting player = game % P: re-run the reset per starting player on the matching games
    for sp in range(1, P):
        idx = torch.arange(sp, num_games, P, device=device)
        if idx.numel():
            sub = E.env_reset(idx.numel(), num_players=P, starting_player=sp, device=device, **r)
            _put(env, idx, sub)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    ws = M.SearchWorkspace(num_games, num_simulations, device) if net is not None else None
    for turn in range(max_turns):
        active = env.done == 0
        if not bool(active.any()):
            break
        bits = E.legal_bits(env)
        cp = env.current_player.long()
        agent_seat = (cp == 0) | ((cp == 2) & teams)
        has = bits != 0
        act = torch.zeros(num_games, dtype=torch.int32, device=device)
        mover = active & has
        ag = (mover & agent_seat).nonzero().flatten() if net is not None else mover.new_zeros(0, dtype=torch.long)
        rd = (mover & ~agent_seat).nonzero().flatten() if net is not None else mover.nonzero().flatten()
        if ag.numel():
            sub = _sub(env, ag)
            obs = E.encode_board(sub)
            out, _ = M.muzero_mcts(net, obs, bits[ag], num_simulations, max_depth, 0.0, seed=seed, turn=turn,
                                       workspace=ws)
            act[ag] = out.action
        if rd.numel():
            act[rd] = random_legal(bits[rd], gen)
        step = mover.nonzero().flatten()
        if step.numel():
            sub = _sub(env, step)
            E.env_step(sub, act[step])
            _put(env, step, sub)
        nos = (active & ~has).nonzero().flatten()
        if nos.numel():
            sub = _sub(env, nos)
            E.no_step(sub)
            _put(env, nos, sub)
    w = winners(env, teams)
    in_goal = (env.pins_bp().long() >= 40).sum(dim=2).float().mean(dim=0)
    return {"games": num_games, "wins": int(w[:, 0].sum()), "seat_wins": w.sum(dim=0).tolist(),
            "finished": int(env.done.sum()), "pins_in_goal": in_goal.tolist()}


def test_agent_vs_random(net: N.DeviceNet | None, num_games: int, batch_size: int = 1024, seed: int = 42,
                         **kw) -> tuple:
    """evaluate_agent.py:383-472 -> (wins at seat 0, mean pins in goal per seat)."""
    wins, prog, done = 0, None, 0
    for b in range(0, num_games, batch_size):
        r = play_vs_random(net, min(batch_size, num_games - b), seed=seed + b, **kw)
        wins += r["wins"]
        p = torch.tensor(r["pins_in_goal"]) * r["games"]
        prog = p if prog is None else prog + p
        done += r["games"]
    return wins, (prog / max(done, 1)).tolist()


def z_test(wins1: int, wins2: int, n: int) -> dict:
    """The two-proportion z-test of compare_agents_statistically (evaluate_agent.py:680-693)."""
    w1, w2 = wins1 / n, wins2 / n
    se = math.sqrt(w1 * (1 - w1) / n + w2 * (1 - w2) / n)
    if se > 0:
        z = (w1 - w2) / se
        p = 2 * (1 - 0.5 * (1 + math.erf(abs(z) / math.sqrt(2))))
    else:
        z, p = 0.0, 1.0
    return {"winrate1": w1, "winrate2": w2, "z": z, "p": p, "significant": abs(z) > 1.96}


def compare_agents_statistically(net1, net2, num_games: int = 1000, batch_size: int = 1024, seed: int = 42, **kw):
    """evaluate_agent.py:648-713: each agent against random opponents on the same seeds, then z_test."""
    w1, _ = test_agent_vs_random(net1, num_games, batch_size, seed, **kw)
    w2, _ = test_agent_vs_random(net2, num_games, batch_size, seed, **kw)
    return z_test(w1, w2, num_games)
