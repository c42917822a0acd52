"""CPU oracle: batched self-play bookkeeping of MuZero_det_MADN/game_agent.py:50-183 (TEST INFRASTRUCTURE ONLY).

Drives the env oracle (oracle/detmadn.py) and a Gumbel search (oracle/mctx_gumbel.py) with
injected networks, and records the same buffers as play_batch_of_games_jitted.  The per-move
Gumbel noise follows the engine's counter RNG (``gumbel_noise``) so that both sides see the same
noise; the reference draws it with jax threefry (parity of the noise source: unpinned).
"""
from __future__ import annotations

import numpy as np

from oracle import detmadn as dm
from oracle import mctx_gumbel as G

M64 = (1 << 64) - 1
TINY = np.finfo(np.float32).tiny


def _mix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def gumbel_noise(seed, gid, turn, A=24, scale=1.0):
    """Counter-based Gumbel draw of the engine (csrc/search.hip:gumbel_noise): -log(-log(U[tiny,1)))."""
    out = np.empty(A, np.float32)
    for a in range(A):
        h = _mix64((seed & M64) ^ _mix64(((gid & 0xFFFFFFFF) << 32) | (turn & 0xFFFFFFFF))
                   ^ (((a + 1) * 0xD6E8FEB86659FD93) & M64))
        u = np.float32((h >> 40) * (1.0 / 16777216.0))
        u = max(u, np.float32(TINY))
        out[a] = np.float32(scale) * (-np.log(-np.log(np.float32(u))))
    return out.astype(np.float32)


def play_batch_of_games(params, root_fn, recurrent_fn, envs, num_simulations, max_depth, max_steps, temp, seed):
    """game_agent.py:50-183 over a list of oracle envs.  root_fn(params, obs[B,C,56]) -> (logits, value, emb)."""
    n = len(envs)
    P = envs[0].num_players
    C = dm.num_channels(P)
    T = max_steps
    teams = envs[0].rules["enable_teams"]
    buf = {
        "obs": np.zeros((n, T, C, 56), np.int8), "act": np.zeros((n, T), np.int32),
        "rew": np.zeros((n, T), np.int32), "val": np.zeros((n, T), np.float32),
        "pol": np.zeros((n, T, 24), np.float32), "mask": np.zeros((n, T), np.float32),
        "player": np.zeros((n, T), np.int32), "team": np.full((n, T), -1, np.int32),
        "discount": np.zeros((n, T), np.int32), "idx": np.zeros(n, np.int32),
        # test instrumentation: smallest relative top-2 gap of any argmax decision of the turn's search
        # (inf on no-move turns), see mctx_gumbel.top2_margin
        "margin": np.full((n, T), np.inf),
        "gain": np.zeros((n, T)),          # Q-rescale gain of the turn's action weights (test instrumentation)
    }
    dones = np.zeros(n, bool)
    step = 0
    while (~dones).any() and step < max_steps:
        search, nomove = [], []
        for i in range(n):
            if dones[i]:
                continue
            va = dm.valid_action(envs[i]).flatten()
            (search if va.any() else nomove).append((i, va))
        if search:
            obs = np.stack([dm.encode_board(envs[i]) for i, _ in search]).astype(np.float32)
            invalid = np.stack([~va for _, va in search])
            gum = np.stack([gumbel_noise(seed, i, step, scale=temp) for i, _ in search])
            lg, v, e = root_fn(params, obs)
            trace = {}
            act, w, rv, _ = G.gumbel_muzero_policy(params, lg, v, e, recurrent_fn, num_simulations, invalid, gum,
                                                   max_depth=max_depth, trace=trace)
            for k, (i, _) in enumerate(search):
                env = envs[i]
                t = buf["idx"][i]
                buf["margin"][i, t] = trace["margin"][k]
                buf["gain"][i, t] = trace["gain"][k]
                cpb = env.current_player
                teamb = cpb % 2 if teams else -1
                nxt, r, nd = dm.env_step(env, dm.map_action(int(act[k])))
                nteam = nxt.current_player % 2 if teams else -1
                buf["obs"][i, t] = obs[k].astype(np.int8)
                buf["act"][i, t] = act[k]
                buf["rew"][i, t] = 2 if (nd and r > 0) else (0 if (nd and r < 0) else 1)
                buf["val"][i, t] = rv[k]
                buf["pol"][i, t] = w[k]
                buf["mask"][i, t] = 1.0
                buf["player"][i, t] = cpb
                buf["team"][i, t] = teamb
                buf["discount"][i, t] = 1 if nd else ((2 if teamb == nteam else 0) if teams
                                                      else (2 if cpb == nxt.current_player else 0))
                buf["idx"][i] = t + 1
                envs[i] = nxt
                dones[i] = nd
        for i, _ in nomove:
            env = envs[i]
            t = buf["idx"][i]
            buf["act"][i, t] = -1
            buf["rew"][i, t] = 1
            buf["player"][i, t] = env.current_player
            buf["team"][i, t] = env.current_player % 2 if teams else -1
            buf["discount"][i, t] = 1
            buf["idx"][i] = t + 1
            envs[i], _, nd = dm.no_step(env)
            dones[i] = nd
        step += 1
    return buf, step


# ---------------------------------------------------------------------------------------------------
# Stochastic MuZero self-play for classic MADN (MuZero_Classic_MADN/game_agent_stochastic.py:52-218)
DIE_STREAM = 0xD1CE5EEDF00D
GUMBEL_STREAM = 0xC2B2AE3D27D4EB4F


def die_uniform(seed, g, turn):
    """csrc/selfplay_classic.hip:die_uniform."""
    h = _mix64(((seed ^ DIE_STREAM) & M64) ^ _mix64(((g & 0xFFFFFFFF) << 32) | (turn & 0xFFFFFFFF)))
    return np.float32((h >> 40) * (1.0 / 16777216.0))


def play_batch_of_games_stochastic(params, root_fn, decision_fn, chance_fn, envs, num_simulations, max_depth,
                                   max_steps, temp, seed, dirichlet_fraction=0.0, time_budget=None):
    """game_agent_stochastic.py:52-218 over a list of oracle classic envs.  The root Dirichlet noise is
    only supported with dirichlet_fraction 0 here (the engine's Gamma sampler is not restated).  With
    `time_budget` (seconds) the loop also stops once that much wall time has passed (bench.py's CPU sample)."""
    import time as _time
    _t0 = _time.perf_counter()
    from oracle import classic_madn as cm
    from oracle import mctx_stochastic as MS
    assert dirichlet_fraction == 0.0
    n = len(envs)
    P = envs[0].num_players
    C = cm.num_channels(P)
    T = max_steps
    teams = envs[0].rules["enable_teams"]
    buf = {
        "obs": np.zeros((n, T, C, 56), np.int8), "act": np.zeros((n, T), np.int32), "rew": np.zeros((n, T), np.int32),
        "val": np.zeros((n, T), np.float32), "pol": np.zeros((n, T, 4), np.float32), "mask": np.zeros((n, T), np.float32),
        "dice": np.zeros((n, T), np.int32), "dice_dist": np.zeros((n, T, 6), np.float32),
        "player": np.zeros((n, T), np.int32), "team": np.full((n, T), -1, np.int32),
        "discount": np.zeros((n, T), np.int32), "idx": np.zeros(n, np.int32),
        "margin": np.full((n, T), np.inf),   # test instrumentation, as in play_batch_of_games
    }
    dones = np.zeros(n, bool)
    step = 0
    while (~dones).any() and step < max_steps:
        if time_budget is not None and _time.perf_counter() - _t0 > time_budget:
            break
        search, nomove = [], []
        for i in range(n):
            if dones[i]:
                continue
            envs[i] = cm.throw_die(envs[i], float(die_uniform(seed, i, step)))
            va = cm.valid_action(envs[i])
            (search if va.any() else nomove).append((i, va))
        if search:
            obs = np.stack([cm.encode_board(envs[i]) for i, _ in search]).astype(np.float32)
            invalid = np.stack([~va for _, va in search])
            gids = np.array([i for i, _ in search])
            gum = np.stack([gumbel_noise(seed ^ GUMBEL_STREAM, int(i), step, A=4) for i in gids])
            lg, v, e = root_fn(params, obs)
            trace = {}
            act, w, rv, _ = MS.stochastic_muzero_policy(params, lg, v, e, decision_fn, chance_fn, num_simulations,
                                                        invalid, np.zeros((len(search), 4), np.float32), gum,
                                                        max_depth=max_depth, temperature=temp, seed=seed, turn=step,
                                                        gids=gids, dirichlet_fraction=0.0, trace=trace)
            for k, (i, _) in enumerate(search):
                env = envs[i]
                t = buf["idx"][i]
                buf["margin"][i, t] = trace["margin"][k]
                cpb = env.current_player
                teamb = cpb % 2 if teams else -1
                nxt, r, nd = cm.env_step(env, int(act[k]))
                nteam = nxt.current_player % 2 if teams else -1
                buf["obs"][i, t] = obs[k].astype(np.int8)
                buf["act"][i, t] = act[k]
                buf["rew"][i, t] = 2 if (nd and r > 0) else (0 if (nd and r < 0) else 1)
                buf["val"][i, t] = rv[k]
                buf["pol"][i, t] = w[k]
                buf["mask"][i, t] = 1.0
                buf["dice"][i, t] = env.die
                buf["dice_dist"][i, t] = cm.dice_probabilities(nxt)
                buf["player"][i, t] = cpb
                buf["team"][i, t] = teamb
                buf["discount"][i, t] = 1 if nd else ((2 if teamb == nteam else 0) if teams
                                                      else (2 if cpb == nxt.current_player else 0))
                buf["idx"][i] = t + 1
                envs[i] = nxt
                dones[i] = nd
        for i, _ in nomove:
            env = envs[i]
            t = buf["idx"][i]
            nxt, _, nd = cm.no_step(env)
            buf["act"][i, t] = -1
            buf["rew"][i, t] = 1
            buf["dice"][i, t] = env.die
            buf["dice_dist"][i, t] = cm.dice_probabilities(nxt)
            buf["player"][i, t] = env.current_player
            buf["team"][i, t] = env.current_player % 2 if teams else -1
            buf["discount"][i, t] = 1
            buf["idx"][i] = t + 1
            envs[i] = nxt
            dones[i] = nd
        step += 1
    return buf, step
