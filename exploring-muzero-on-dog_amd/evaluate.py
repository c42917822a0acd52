"""Evaluation harness for det-MADN agents (SURVEY §8f "next" 3; MuZero_det_MADN/evaluate_agent.py).

  test_agent_vs_random          evaluate_agent.py:383-472: the agent plays seat 0 (and seat 2, its
                                partner, when teams are on) with a temperature-0 Gumbel search; the other
                                seats play uniformly random legal moves (multiactor_step_with_random_agent_v2,
                                474-646); no-move turns apply no_step; wins are counted at seat 0
                                (manual_get_winner 16-45); at most 2000 turns.
  compare_agents_statistically  648-713: both agents against random opponents, two-proportion z-test.
  evaluate_agent_parallel       253-311 + play_n_games_for_eval_jitted / play_eval_loop_jitted 715-960: four
                                seats, each a MuZero agent (a DeviceNet, or None = randomly initialised
                                params), 'rule_based_agent' or 'random_agent'; batch_size games per starting
                                player; winners and calculate_progress (129-195) per starting player.
  policy_action                 the random agent (770-775) and the rule-based agent (777-864) as one device
                                kernel (muz_detmadn_policy_action), sampling by Gumbel-max on the counter RNG.

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
from . import lib as _L
from . import mcts as M
from . import nets as N

# evaluate_agent.py:777-864 (the variant evaluate_agent_parallel runs); 509-603 uses 0.5 / 5 / 3 / 1.5 / 2.5
RULE_AGENT = dict(temperature=0.25, goal_bonus=5.0, out_many=3.0, out_few=2.0, hit_bonus=2.0)

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


# ---- four seats: evaluate_agent_parallel (evaluate_agent.py:253-311, 715-960) ----------------------------
def policy_action(env: E.DetMADNState, legal: torch.Tensor, mode: str, seed: int, turn: int, agent: dict | None = None,
                  game_id: torch.Tensor | None = None) -> torch.Tensor:
    """The random ('random_agent') or rule-based ('rule_based_agent') action of every game (int32 [B], -1
    without a legal action), one launch over the batch (muz_detmadn_policy_action)."""
    m = {"random_agent": 0, "rule_based_agent": 1}[mode]
    a = dict(RULE_AGENT if agent is None else agent)
    ag = _L.MuzRuleAgent(a["temperature"], a["goal_bonus"], a["out_many"], a["out_few"], a["hit_bonus"])
    out = torch.empty((env.batch,), dtype=torch.int32, device=env.board.device)
    gid = None if game_id is None else game_id.to(device=out.device, dtype=torch.int32).contiguous()
    _L.check(_L.load().muz_detmadn_policy_action(env.rules, env.soa(), _L.ptr(legal.contiguous()), m, ag,
                                                 int(seed) & ((1 << 64) - 1), int(turn), _L.ptr(gid), _L.ptr(out),
                                                 env.batch, _L.stream_ptr()), "muz_detmadn_policy_action")
    return out


def _seats(rules, P):
    """Seat (start cell / 10) of each player after env_reset's layout fix-up (deterministic_madn.py:70-74)."""
    lay = [bool(rules.layout[i]) for i in range(4)]
    if sum(lay) != P or (all(lay) and P < 4):
        lay = [i < P for i in range(4)]
    return [i for i in range(4) if lay[i]]


def calculate_progress(env: E.DetMADNState, must_traverse_start: bool = False) -> torch.Tensor:
    """calculate_progress (evaluate_agent.py:129-195) for every game and player -> float32 [B, P]: pins rotated
    to the player's view (home -> pin - 5, track -> (pin - (40 // P) * p) % 40 - traverse, goal -> 40 + offset),
    sorted, and greedily matched to the goal cells 40..43 (repeated masked argmin of |pin - goal|, first index
    on ties).  Note the reference's distance = board_size // num_players (20 at two players, as written)."""
    P = env.num_players
    pins = env.pins_bp().long()                                           # [B, P, 4]
    seats = torch.tensor(_seats(env.rules, P), device=pins.device)
    p_idx = torch.arange(P, device=pins.device)[None, :, None]
    g0 = (40 + 4 * seats)[None, :, None]
    rot = torch.where(pins < 0, pins - 5,
                      torch.where(pins < 40, torch.remainder(pins - (40 // P) * p_idx, 40) - int(must_traverse_start),
                                  40 + (pins - g0)))
    sp = torch.sort(rot, dim=2).values
    dmat = (sp[..., :, None] - (40 + torch.arange(4, device=pins.device))).abs().double()   # [B, P, 4, 4]
    mask = torch.ones_like(dmat, dtype=torch.bool)
    total = torch.zeros(dmat.shape[:2], dtype=torch.float64, device=pins.device)
    inf = torch.full_like(dmat, float("inf"))
    for _ in range(4):
        flat = torch.where(mask, dmat, inf).flatten(2).argmin(dim=2)     # first minimum
        r, c = flat // 4, flat % 4
        total += dmat.flatten(2).gather(2, flat[..., None])[..., 0]
        rows = torch.arange(4, device=pins.device)
        mask &= ~(rows[None, None, :, None] == r[..., None, None])
        mask &= ~(rows[None, None, None, :] == c[..., None, None])
    return total.float()


@torch.no_grad()
def evaluate_agent_parallel(agents, batch_size: int = 20, num_simulations: int = 100, max_depth: int = 50,
                            temperature: float = 0.0, seed: int = 0, rules: dict | None = None, max_turns: int = 2000,
                            rule_agent: dict | None = None, device="cuda") -> dict:
    """evaluate_agent_parallel (evaluate_agent.py:253-311): `agents` = the four seats (player indices 0-3),
    each a DeviceNet, None (a MuZero agent with randomly initialised params), 'rule_based_agent' or
    'random_agent'.  4 x batch_size games, block i started by player i (jnp.repeat(arange(4), batch_size)),
    at most 2000 turns; MuZero seats search with S / D / temperature (evaluate_agent.py:938-940 defaults).
    Returns winners[start][player] and average_progress[start][player] as the reference prints them, plus
    their totals (wins per player, progress per player = column sum / 4)."""
    r = dict(RULES if rules is None else rules)
    P = 4
    C = E.num_channels(P)
    nets = []
    for i, a in enumerate(agents):
        if a is None:
            nets.append(N.DeviceNet(N.init_muzero_params(1_000_003 * (seed + 1) + i, C), C, device=device))
        elif isinstance(a, str):
            if a not in ("rule_based_agent", "random_agent"):
                raise ValueError(f"unknown agent {a!r}")
            nets.append(a)
        else:
            nets.append(N.as_device_net(a, C, device=device))
    n = 4 * batch_size
    env = E.env_reset(n, num_players=P, device=device, **r)
    for sp in range(1, 4):
        idx = torch.arange(sp * batch_size, (sp + 1) * batch_size, device=device)
        _put(env, idx, E.env_reset(batch_size, num_players=P, starting_player=sp, device=device, **r))
    gid = torch.arange(n, device=device, dtype=torch.int32)
    ws = M.SearchWorkspace(n, num_simulations, device) if any(not isinstance(x, str) for x in nets) else None
    for turn in range(max_turns):
        active = env.done == 0
        if not bool(active.any()):
            break
        bits = E.legal_bits(env)
        cp = env.current_player.long()
        has = bits != 0
        mover = active & has
        act = torch.full((n,), -1, dtype=torch.int32, device=device)
        for s, a in enumerate(nets):
            sel = mover & (cp == s)
            if not bool(sel.any()):
                continue
            if isinstance(a, str):
                pa = policy_action(env, bits, a, seed, turn, rule_agent, gid)
                act = torch.where(sel, pa, act)
            else:
                idx = sel.nonzero().flatten()
                sub = _sub(env, idx)
                out, _ = M.muzero_mcts(a, E.encode_board(sub), bits[idx], num_simulations, max_depth, temperature,
                                       seed=seed, turn=turn, workspace=ws)
                act[idx] = out.action
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
    w = winners(env, bool(r.get("enable_teams", False))) & (env.done != 0)[:, None]
    prog = calculate_progress(env, bool(r.get("must_traverse_start", False)))
    win_tab = w.long().reshape(4, batch_size, P).sum(dim=1)
    prog_tab = prog.reshape(4, batch_size, P).mean(dim=1)
    return {"games": n, "winners": win_tab.tolist(), "average_progress": prog_tab.tolist(),
            "wins_per_player": win_tab.sum(dim=0).tolist(), "progress_per_player": (prog_tab.sum(dim=0) / 4).tolist(),
            "finished": int((env.done != 0).sum()), "final_state": env}


# ---- classic MADN: MuZero_Classic_MADN/evaluate_agent_stochastic.py ------------------------------------------------
# evaluate_agent_stochastic.py:938-948 (the keys it leaves out take env_reset's defaults: no dice rethrow)
CLASSIC_RULES = dict(enable_teams=True, enable_initial_free_pin=True, enable_circular_board=False,
                     enable_friendly_fire=True, enable_start_blocking=False, enable_jump_in_goal_area=True,
                     enable_start_on_1=True, enable_bonus_turn_on_6=True, must_traverse_start=False,
                     enable_dice_rethrow=False)
# do_rule_based of play_eval_loop_jitted (806-866); NUM_SIMULATIONS / MAX_DEPTH / TEMPERATURE of 950-952
CLASSIC_RULE_AGENT = dict(temperature=0.25, goal_bonus=5.0, out_many=3.0, out_few=2.0, hit_bonus=2.5)
CLASSIC_SIMULATIONS, CLASSIC_DEPTH = 75, 50


def classic_policy_action(env, legal: torch.Tensor, mode: str, seed: int, turn: int, agent: dict | None = None,
                          game_id: torch.Tensor | None = None) -> torch.Tensor:
    """The classic random ('random_agent', do_random 800-804) or rule-based ('rule_based_agent', do_rule_based
    806-866) pin of every game for the die in the state (int32 [B], -1 without a legal pin), one launch
    (muz_classic_policy_action)."""
    m = {"random_agent": 0, "rule_based_agent": 1}[mode]
    a = dict(CLASSIC_RULE_AGENT if agent is None else agent)
    ag = _L.MuzRuleAgent(a["temperature"], a["goal_bonus"], a["out_many"], a["out_few"], a["hit_bonus"])
    out = torch.empty((env.batch,), dtype=torch.int32, device=env.board.device)
    gid = None if game_id is None else game_id.to(device=out.device, dtype=torch.int32).contiguous()
    _L.check(_L.load().muz_classic_policy_action(env.rules, env.soa(), _L.ptr(legal.contiguous()), m, ag,
                                                 int(seed) & ((1 << 64) - 1), int(turn), _L.ptr(gid), _L.ptr(out),
                                                 env.batch, _L.stream_ptr()), "muz_classic_policy_action")
    return out


def _csub(env, idx: torch.Tensor):
    from . import classic as CL
    return CL.ClassicMADNState(env.board[:, idx].contiguous(), env.pins[:, idx].contiguous(),
                               env.current_player[idx].contiguous(), env.reward[idx].contiguous(),
                               env.done[idx].contiguous(), env.die[idx].contiguous(), env.rules, env.num_players)


def _cput(env, idx: torch.Tensor, sub):
    env.board[:, idx] = sub.board
    env.pins[:, idx] = sub.pins
    env.current_player[idx] = sub.current_player
    env.reward[idx] = sub.reward
    env.done[idx] = sub.done
    env.die[idx] = sub.die


def _classic_turn(env, seats, gid, turn, seed, gen, num_simulations, max_depth, temperature, rule_agent, ws,
                  throw=True):
    """One turn of every unfinished game (play_eval_loop_jitted's body_fn, 754-900): throw_die (its dice_probabilities,
    soft lock aware), then per game the agent of its current player -- a stochastic MuZero search ('mcts': a
    DeviceClassicNet), 'random_agent' or 'rule_based_agent' -- and env_step, or no_step without a legal pin."""
    from . import classic as CL
    from . import stochastic as ST
    n = env.batch
    active = env.done == 0
    if throw:
        # the uniform draws of the die: torch's generator (the reference's jax key is not restated)
        CL.throw_die(env, torch.rand((n,), generator=gen, device=env.board.device))
    bits = CL.legal_bits(env)
    cp = env.current_player.long()
    has = (bits & 15) != 0
    mover = active & has
    act = torch.full((n,), -1, dtype=torch.int32, device=env.board.device)
    for s, a in enumerate(seats):
        sel = mover & (cp == s)
        if not bool(sel.any()):
            continue
        if isinstance(a, str):
            act = torch.where(sel, classic_policy_action(env, bits, a, seed, turn, rule_agent, gid), act)
        else:
            idx = sel.nonzero().flatten()
            sub = _csub(env, idx)
            out = ST.stochastic_muzero_mcts(a, CL.encode_board(sub), bits[idx], num_simulations, max_depth,
                                            temperature, seed=seed, turn=turn, game_id=gid[idx], workspace=ws)
            act[idx] = out[0]
    step = mover.nonzero().flatten()
    if step.numel():
        sub = _csub(env, step)
        CL.env_step(sub, act[step])
        _cput(env, step, sub)
    nos = (active & ~has).nonzero().flatten()
    if nos.numel():
        sub = _csub(env, nos)
        CL.no_step(sub)
        _cput(env, nos, sub)
    return bool(active.any())


def _classic_seat(a, C, i, seed, device):
    from . import stochastic as ST
    if a is None:     # a Stochastic MuZero agent with randomly initialised params
        return ST.DeviceClassicNet(ST.init_classic_params(C, seed=1_000_003 * (seed + 1) + i), C, device=device)
    if isinstance(a, str):
        if a not in ("rule_based_agent", "random_agent"):
            raise ValueError(f"unknown agent {a!r}")
        return a
    return ST.as_device_classic_net(a, C, device=device)


@torch.no_grad()
def evaluate_agent_parallel_classic(agents, batch_size: int = 150, num_simulations: int = CLASSIC_SIMULATIONS,
                                    max_depth: int = CLASSIC_DEPTH, temperature: float = 0.0, seed: int = 0,
                                    rules: dict | None = None, max_turns: int = 2000, rule_agent: dict | None = None,
                                    device="cuda") -> dict:
    """evaluate_agent_parallel (evaluate_agent_stochastic.py:253-315) with play_n_games_for_eval_jitted /
    play_eval_loop_jitted (717-936): `agents` = the four seats, each a DeviceClassicNet / Flax params (Stochastic
    MuZero, temperature 0, S 75, D 50), None (randomly initialised params), 'rule_based_agent' or 'random_agent';
    4 x batch_size games, block i started by player i; the die thrown every turn; at most 2000 turns.  Returns
    winners[start][player] and average_progress[start][player] as the reference prints them, and their totals."""
    from . import classic as CL
    from . import stochastic as ST
    r = dict(CLASSIC_RULES if rules is None else rules)
    P = 4
    C = CL.num_channels(P)
    seats = [_classic_seat(a, C, i, seed, device) for i, a in enumerate(agents)]
    n = 4 * batch_size
    env = CL.env_reset(n, num_players=P, device=device, **r)
    for sp in range(1, 4):
        idx = torch.arange(sp * batch_size, (sp + 1) * batch_size, device=device)
        _cput(env, idx, CL.env_reset(batch_size, num_players=P, starting_player=sp, device=device, **r))
    gid = torch.arange(n, device=device, dtype=torch.int32)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    ws = None
    if any(not isinstance(x, str) for x in seats):
        ws = torch.empty((_L.load().muz_stochastic_workspace_bytes(n, num_simulations),), dtype=torch.uint8,
                         device=device)
    for turn in range(max_turns):
        if not _classic_turn(env, seats, gid, turn, seed, gen, num_simulations, max_depth, temperature, rule_agent,
                             ws):
            break
    w = winners(env, bool(r.get("enable_teams", False))) & (env.done != 0)[:, None]
    prog = calculate_progress(env, bool(r.get("must_traverse_start", False)))
    win_tab = w.long().reshape(4, batch_size, P).sum(dim=1)
    prog_tab = prog.reshape(4, batch_size, P).mean(dim=1)
    return {"games": n, "winners": win_tab.tolist(), "average_progress": prog_tab.tolist(),
            "wins_per_player": win_tab.sum(dim=0).tolist(), "progress_per_player": (prog_tab.sum(dim=0) / 4).tolist(),
            "finished": int((env.done != 0).sum()), "final_state": env}


@torch.no_grad()
def play_vs_random_classic(agent, num_games: int, num_simulations: int = CLASSIC_SIMULATIONS,
                           max_depth: int = CLASSIC_DEPTH, seed: int = 42, max_turns: int = 2000,
                           rules: dict | None = None, device="cuda") -> dict:
    """One batch of test_agent_vs_random (evaluate_agent_stochastic.py:387-476): the agent at seat 0 (+ seat 2, its
    partner, with teams) -- a Stochastic MuZero searching at temperature 0 (multiactor_step_with_random_agent_v2,
    478-650), or 'rule_based_agent' / 'random_agent' -- the other seats random; a random starting player per game
    (env_reset's seed); wins counted at seat 0.  The die is thrown every turn as play_eval_loop_jitted does: the v2
    step as written never throws it, so its games keep env_reset's die 0, have no legal pin and end only at
    MAX_STEPS (oracle/classic_madn.py: valid_action of a fresh state with die 0 is all False)."""
    from . import classic as CL
    r = dict(CLASSIC_RULES if rules is None else rules)
    P = 4
    C = CL.num_channels(P)
    teams = bool(r.get("enable_teams", False))
    ag = _classic_seat(agent, C, 0, seed, device)
    seats = [ag, "random_agent", ag if teams else "random_agent", "random_agent"]
    g = torch.Generator().manual_seed(seed)
    seeds = torch.randint(0, 1_000_000, (num_games,), generator=g).tolist()
    env = CL.env_reset(num_games, num_players=P, starting_player=-1, device=device, seeds=seeds, **r)
    env.rules = CL.make_rules(P, starting_player=0, **r)   # (the seat is in the state now; the kernels take 0..P-1)
    gid = torch.arange(num_games, device=device, dtype=torch.int32)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    ws = None
    if not isinstance(ag, str):
        ws = torch.empty((_L.load().muz_stochastic_workspace_bytes(num_games, num_simulations),), dtype=torch.uint8,
                         device=device)
    for turn in range(max_turns):
        if not _classic_turn(env, seats, gid, turn, seed, gen, num_simulations, max_depth, 0.0, None, ws):
            break
    w = winners(env, teams) & (env.done != 0)[:, None]
    prog = calculate_progress(env, bool(r.get("must_traverse_start", False)))
    return {"games": num_games, "wins": int(w[:, 0].sum()), "seat_wins": w.sum(dim=0).tolist(),
            "finished": int((env.done != 0).sum()), "progress": prog.mean(dim=0).tolist()}


def test_agent_vs_random_classic(agent, num_games: int, batch_size: int = 100, seed: int = 42, **kw) -> tuple:
    """test_agent_vs_random (evaluate_agent_stochastic.py:387-476) -> (wins at seat 0, mean final pin distance per
    seat over the batches)."""
    wins, prog, nb = 0, None, 0
    for b in range(0, num_games, batch_size):
        r = play_vs_random_classic(agent, min(batch_size, num_games - b), seed=seed + b, **kw)
        wins += r["wins"]
        p = torch.tensor(r["progress"])
        prog = p if prog is None else prog + p
        nb += 1
    return wins, (prog / max(nb, 1)).tolist()


def compare_agents_statistically_classic(agent1, agent2, num_games: int = 1000, batch_size: int = 100,
                                         seed: int = 42, **kw) -> dict:
    """compare_agents_statistically (evaluate_agent_stochastic.py:652-717): both agents against random opponents on
    the same seeds, then the two-proportion z-test."""
    w1, _ = test_agent_vs_random_classic(agent1, num_games, batch_size, seed, **kw)
    w2, _ = test_agent_vs_random_classic(agent2, num_games, batch_size, seed, **kw)
    return z_test(w1, w2, num_games)


# ---- DOG: MuZero_DOG/evaluate_agent.py --------------------------------------------------------------------------
# evaluate_agent.py:530-541; NUM_SIMULATIONS / MAX_DEPTH 544-545, TEMPERATURE 0.20 (552: the value the script runs with)
DOG_RULES = dict(enable_teams=True, enable_initial_free_pin=False, enable_circular_board=True, enable_friendly_fire=True,
                 enable_start_blocking=True, enable_jump_in_goal_area=False, must_traverse_start=True,
                 disable_swapping=False, disable_hot_seven=False, disable_joker=False)
DOG_SIMULATIONS, DOG_DEPTH, DOG_TEMPERATURE = 100, 50, 0.2


def _dog_seat(a, i, seed, device):
    from . import muzero_dog as MD
    if a is None:     # a MuZero agent with randomly initialised params (the DOG slice's networks)
        return MD.DeviceDogNet(MD.init_muzero_params(1_000_003 * (seed + 1) + i), device=device)
    if isinstance(a, str):
        if a == "rule_based_agent":
            # do_rule_based (evaluate_agent.py:403-480) is det-MADN's agent copied: valid_mask.reshape(4, 6) of the
            # 806-action DOG mask cannot run, so the reference has no DOG rule-based agent to restate
            raise ValueError("MuZero_DOG/evaluate_agent.py's rule-based agent reshapes the 806-action mask to (4, 6) "
                             "and cannot run; use 'random_agent' or a MuZero agent")
        if a != "random_agent":
            raise ValueError(f"unknown agent {a!r}")
        return a
    return MD.as_device_net(a, device=device)


@torch.no_grad()
def evaluate_agent_parallel_dog(agents, batch_size: int = 20, num_simulations: int = DOG_SIMULATIONS,
                                max_depth: int = DOG_DEPTH, temperature: float = DOG_TEMPERATURE, seed: int = 0,
                                rules: dict | None = None, max_turns: int = 2000, device="cuda") -> dict:
    """evaluate_agent_parallel (MuZero_DOG/evaluate_agent.py:255-313) with play_n_games_for_eval_jitted /
    play_eval_loop_jitted (315-527): `agents` = the four seats, each the DOG slice's MuZero (a DeviceDogNet or its
    flat params; None = randomly initialised params; run_muzero_mcts at A = 806, S 100, D 50, temperature 0.2) or
    'random_agent' (do_random: a uniform legal action); 4 x batch_size games, block i started by player i, at most
    2000 turns; a game without a legal action applies no_step.  Every game steps in its own lane each turn (a finished
    game's lane applies no_step, which leaves its pins alone), so a game's deals are keyed by its own index.  Returns
    winners[start][player] and average_progress[start][player] as the reference prints them, and their totals.
    Win-rate parity is unpinned: the reference's DOG networks and inference functions are `pass`."""
    from . import dog as DOG
    from . import muzero_dog as MD
    r = dict(DOG_RULES if rules is None else rules)
    P = 4
    seats = [_dog_seat(a, i, seed, device) for i, a in enumerate(agents)]
    n = 4 * batch_size
    env = DOG.env_reset(n, num_players=P, seed=seed, device=device, **r)
    for sp in range(1, 4):   # block sp started by player sp (its deals keyed by seed + sp)
        blk = DOG.env_reset(batch_size, num_players=P, starting_player=sp, seed=seed + sp, device=device, **r)
        sl = slice(sp * batch_size, (sp + 1) * batch_size)
        for k in ("board", "pins", "deck", "hands", "swap_choices"):
            getattr(env, k)[:, sl] = getattr(blk, k)
        for k in ("current_player", "round_starter", "phase", "hand_size", "reward", "done", "deal"):
            getattr(env, k)[sl] = getattr(blk, k)
    ws = MD.SearchWorkspace(n, num_simulations, device) if any(not isinstance(x, str) for x in seats) else None
    for turn in range(max_turns):
        active = env.done == 0
        if not bool(active.any()):
            break
        legal = DOG.legal_mask(env)
        has = (legal != 0).any(dim=1)
        mover = active & has
        cp = env.current_player.long()
        act = torch.full((n,), -1, dtype=torch.int32, device=device)
        for s, a in enumerate(seats):
            sel = mover & (cp == s)
            if not bool(sel.any()):
                continue
            if isinstance(a, str):
                act = torch.where(sel, DOG.random_action(legal, seed=seed, turn=turn), act)
            else:
                idx = sel.nonzero().flatten()
                sub = DOG.DOGState(*(getattr(env, k)[:, idx].contiguous() if getattr(env, k).dim() == 2 else
                                     getattr(env, k)[idx].contiguous()
                                     for k in ("board", "pins", "deck", "hands", "swap_choices", "current_player",
                                               "round_starter", "phase", "hand_size", "reward", "done", "deal")),
                                   rules=env.rules, num_players=P, seed=env.seed)
                lg, v, e = MD.root_inference_fn(a, MD.encode_board(sub), scratch=ws.scratch)
                pol, _ = MD.gumbel_muzero_policy(a, lg, v, e, legal[idx], num_simulations, max_depth, temperature,
                                                 seed=seed, turn=turn, workspace=ws)
                act[idx] = pol.action
        act = torch.where(active, act, torch.full_like(act, -1))
        DOG.env_step(env, act)   # negative: no_step (a game without a legal action, or a finished one)
    w = winners(env, bool(r.get("enable_teams", False))) & (env.done != 0)[:, None]
    prog = calculate_progress(env, bool(r.get("must_traverse_start", False)))
    win_tab = w.long().reshape(4, batch_size, P).sum(dim=1)
    prog_tab = prog.reshape(4, batch_size, P).mean(dim=1)
    return {"games": n, "winners": win_tab.tolist(), "average_progress": prog_tab.tolist(),
            "wins_per_player": win_tab.sum(dim=0).tolist(), "progress_per_player": (prog_tab.sum(dim=0) / 4).tolist(),
            "finished": int((env.done != 0).sum()), "turns": turn + 1, "final_state": env}
