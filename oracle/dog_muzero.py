"""CPU oracle of the DOG MuZero slice (TEST INFRASTRUCTURE ONLY).

The reference's DOG MuZero is a skeleton: ``RepresentationNetwork`` exists (MuZero_DOG/muzero_dog.py:25-83,
restated by oracle/nets.py with its LayerNorm head), while ``encode_board`` (DOG/dog.py:1264-1272),
``DynamicsNetwork`` / ``PredictionNetwork`` / ``root_inference_fn`` / ``recurrent_inference_fn``
(muzero_dog.py:85-99) and the self-play loop (MuZero_DOG/game_agent.py:52-57) are ``pass``.  SURVEY §8(d)
asks for "MCTS with the det-MADN-shaped nets at A=806"; this file defines the missing pieces the way the
device path (csrc/dog_muzero.hip, csrc/dog_search.hip) implements them:

* ``encode_board``: 34 channels x 56 cells, the det-MADN 4p encoding's shape (muzero_dog.py:34-35 slices 6
  spatial channels and 28 global features) -- DOG-specific content, defined here (parity unpinned);
* the networks: RepresentationNetwork (LayerNorm head) + DynamicsNetwork4 / PredictionNetwork4 of the det
  file at A = 806 (oracle/nets.py with ``head="layernorm"``);
* ``run_muzero_mcts``: mctx.gumbel_muzero_policy as muzero_dog.py:101-137 calls it (oracle/mctx_gumbel.py;
  at A = 806 its action sums follow the device search's lane order, mctx_gumbel.lane_tree_sum).

Parity status: the env transitions under it are pinned (oracle/dog.py); the encoding, the Dyn / Pred nets and
the search at A = 806 are UNPINNED (the reference has no code for them).
"""
from __future__ import annotations

import numpy as np

from . import dog as D
from . import nets as ON

NUM_ACTIONS = 806
NUM_CHANNELS = 34
CELLS = 56


def encode_board(env: D.State) -> np.ndarray:
    """DOG observation int[34, 56] from the current player's perspective (builder-defined; DOG/dog.py:1264-1272
    is ``pass``).  Spatial channels as det-MADN's encode_board (deterministic_madn.py:395-438): the track rolled
    by -10*cp and the goals by -4*cp, then
      0..3  pins of player (cp + r) % 4,  4 own team,  5 opponents;
    global features (broadcast over the 56 cells; the network reads cell 0):
      6..9    pins at home of player (cp + r) % 4
      10..23  card counts of the hand the mover plays from (dog.py sub_player: the partner's once cp is done)
      24..27  cards held by player (cp + r) % 4
      28 phase (1 = swap), 29 hand size of the next deal, 30 mover plays the partner's hand,
      31 cards left in the deck, 32 (round_starter - cp) % 4, 33 pins in goal of the mover's team."""
    P = env.num_players
    if P != 4:
        raise ValueError("the DOG MuZero slice plays 4-player DOG (config d)")
    cp = int(env.current_player)
    bs = env.board_size
    dist = bs // 4
    track = np.roll(env.board[:bs], -dist * cp)
    goals = np.roll(env.board[bs:env.total_board_size], -4 * cp)
    b = np.concatenate([track, goals]).astype(np.int32)
    rolled = (np.arange(4) + cp) % 4
    pc = (b[None, :] == rolled[:, None]).astype(np.int32)
    teams = bool(env.rules["enable_teams"])
    team = pc[0] + pc[2] if teams else pc[0]
    opp = pc[1] + pc[3] if teams else pc[1] + pc[2] + pc[3]
    sub = D.sub_player(env)
    pins = np.asarray(env.pins)
    hands = np.asarray(env.hands, np.int32)
    g = np.zeros(28, np.int32)
    g[0:4] = [(pins[p] == -1).sum() for p in rolled]
    g[4:18] = hands[sub]
    g[18:22] = [hands[p].sum() for p in rolled]
    g[22] = env.phase
    g[23] = env.hand_size
    g[24] = int(sub != cp)
    g[25] = int(np.asarray(env.deck, np.int32).sum())
    g[26] = (int(env.round_starter) - cp) % 4
    mates = [cp, (cp + 2) % 4] if teams else [cp]
    g[27] = sum(int((pins[p] >= bs).sum()) for p in mates)
    out = np.zeros((NUM_CHANNELS, CELLS), np.int32)
    out[0:4] = pc
    out[4] = team
    out[5] = opp
    out[6:] = g[:, None]
    return out


def init_params(seed: int = 0, randomize_affine: bool = False) -> dict:
    """Flat Flax-path parameters of the DOG slice: RepresentationNetwork (LayerNorm head) + Dyn4 / Pred4 at A=806."""
    return ON.init_params(NUM_CHANNELS, NUM_ACTIONS, seed=seed, randomize_affine=randomize_affine, head="layernorm")


def root_inference(params, obs):
    """root_inference_fn for the slice: RepresentationNetwork -> PredictionNetwork4 (A = 806)."""
    return ON.root_inference(params, obs)


def recurrent_inference(params, action, emb):
    """recurrent_inference_fn for the slice: DynamicsNetwork4 (one-hot 806) -> PredictionNetwork4."""
    return ON.recurrent_inference(params, action, emb)


def turn_record(env: D.State, action: int, weights, root_value: float, reward: int, done: bool, next_player: int):
    """One turn's row of the DOG self-play buffers (MuZero_DOG/game_agent.py:52-57 is ``pass``; the det loop it copies,
    MuZero_det_MADN/game_agent.py:64-141, defines it): ``env`` the state before the move, ``action`` < 0 a turn without
    a legal action (no_step), (reward, done, next_player) the step's result.  -> dict of the row's fields."""
    teams = bool(env.rules["enable_teams"])
    cp = int(env.current_player)
    team = cp % 2 if teams else -1
    if action < 0:       # do_skip (game_agent.py:112-116): zeros, act -1, value 0, mask 0, discount / reward class 1
        return dict(obs=np.zeros((NUM_CHANNELS, CELLS), np.int8), act=-1, rew=1, val=np.float32(0.0),
                    pol=np.zeros(NUM_ACTIONS, np.float32), mask=0.0, player=cp, team=team, discount=1)
    rew = 2 if (done and reward > 0) else (0 if (done and reward < 0) else 1)              # lines 95-99
    if done:
        disc = 1                                                                          # lines 102-109
    elif teams:
        disc = 2 if cp % 2 == next_player % 2 else 0
    else:
        disc = 2 if cp == next_player else 0
    return dict(obs=encode_board(env).astype(np.int8), act=int(action), rew=rew, val=np.float32(root_value),
                pol=np.asarray(weights, np.float32), mask=1.0, player=cp, team=team, discount=disc)
