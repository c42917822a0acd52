"""MuZero_DOG/game_agent.py on the GPU: DOG self-play with the MuZero policy of the DOG slice.

The reference's DOG self-play (``play_batch_of_games_jitted`` / ``play_n_games_v3``, MuZero_DOG/game_agent.py:52-65)
is ``pass``; its rules (``RULES``, game_agent.py:12-23) and the det-MADN loop it copies (MuZero_det_MADN/game_agent.py:
50-192: valid actions -> encode -> run_muzero_mcts -> env_step, or no_step without a legal move) define what it would
do.  ``DogSelfPlay`` runs that turn for a batch of games resident on the device -- muz_dog_legal, muz_dog_encode,
the root inference, the Gumbel search at A = 806 (k_dog_search) and muz_dog_step_restart, five launches per turn --
and restarts finished games in place so the batch stays full (config (d)'s actor).  Gumbel noise: the device stream
of (seed, game, turn); deals: the engine's counter keys.  Parity: followed turn by turn by oracle/dog.py +
oracle/mctx_gumbel.py driven by the same network kernels (tests/test_gpu_dog_muzero.py); unpinned beyond the env.
"""
from __future__ import annotations

import torch

from . import dog as DOG
from . import lib as _L
from . import muzero_dog as MD

RULES = dict(enable_teams=True, enable_initial_free_pin=False, enable_circular_board=True, enable_friendly_fire=True,
             enable_start_blocking=True, enable_jump_in_goal_area=False, must_traverse_start=True,
             disable_swapping=False, disable_hot_seven=False, disable_joker=False)


class DogSelfPlay:
    """A batch of 4-player DOG games played by the MuZero policy, state resident on the device."""

    def __init__(self, net: MD.DeviceDogNet, num_envs: int, num_simulations: int = 100, max_depth: int = 50,
                 temperature: float = 1.0, seed: int = 0, rules: dict | None = None, device="cuda"):
        self.net, self.B = net, int(num_envs)
        self.S, self.D, self.temp, self.seed = int(num_simulations), int(max_depth), float(temperature), int(seed)
        self.env = DOG.env_reset(self.B, num_players=4, seed=self.seed, device=device, **(rules or RULES))
        i32 = dict(dtype=torch.int32, device=device)
        self.words = torch.empty((self.B, DOG.MASK_WORDS), **i32)
        self.obs = torch.empty((self.B, MD.NUM_CHANNELS, 56), dtype=torch.float32, device=device)
        self.reward = torch.empty((self.B,), dtype=torch.int8, device=device)
        self.done = torch.empty((self.B,), dtype=torch.uint8, device=device)
        self.episodes = torch.zeros((self.B,), **i32)
        self.ws = MD.SearchWorkspace(self.B, self.S, device)
        self.turn_index = 0

    def turn(self):
        """One turn of every game: (action [B] (-1 = no_step), action_weights [B, 806], root_value [B])."""
        env = self.env
        DOG.legal_mask(env, out=self.words)
        MD.encode_board(env, out=self.obs)
        lg, v, e = MD.root_inference_fn(self.net, self.obs, self.ws.scratch)
        pol, rv = MD.gumbel_muzero_policy(self.net, lg, v, e, self.words, self.S, self.D, self.temp, seed=self.seed,
                                          turn=self.turn_index, workspace=self.ws)
        _L.check(_L.load().muz_dog_step_restart(env.rules, env.soa(), _L.ptr(pol.action), DOG.ctypes_u64(env.seed),
                                                _L.ptr(self.reward), _L.ptr(self.done), _L.ptr(self.episodes), self.B,
                                                _L.stream_ptr()), "muz_dog_step_restart")
        self.turn_index += 1
        return pol.action, pol.action_weights, rv

    def play(self, nturns: int):
        for _ in range(int(nturns)):
            self.turn()
        return self.B * int(nturns)
