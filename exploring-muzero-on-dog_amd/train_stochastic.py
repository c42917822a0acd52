"""The classic-MADN (Stochastic MuZero) learner script's entry points (MuZero_Classic_MADN/train_stochastic.py),
on the device engine.  Twin of train_with_reward.py:
  get_temperature(iteration, total_iterations)          :19-23
  balanced_loss(ce, is_rare, mask, n_valid, ...)        :25-31
  loss_fn_stochastic(params, batch)                     :34-181
  train_step(params, opt_state, batch)                  :183-199 -> (params, opt_state, losses)
  test_training(config, params=None, opt_state=None)    :201-355 -> (params, opt_state, times_per_iteration)
  RULES, TEMPERATURE_SCHEDULE, *_SCALING, config        :361-406
  learning_rate_schedule, optimizer                     :416-428
The bootstrap switch only fires when the run did not start on bootstrap targets (:289); self-play uses
game_agent_stochastic's RULES and 4 action slots.  Same by-design differences as train_with_reward.py.
"""
from __future__ import annotations

import os

import torch

from . import classic as E
from . import game_agent_stochastic as GS
from . import learner as LR
from . import replay as R
from . import stochastic as ST
from . import training as T

RULES = {                                   # :361-372
    'enable_teams': True,
    'enable_initial_free_pin': True,
    'enable_circular_board': False,
    'enable_friendly_fire': False,
    'enable_start_blocking': False,
    'enable_jump_in_goal_area': True,
    'enable_start_on_1': True,
    'enable_bonus_turn_on_6': True,
    'must_traverse_start': False,
    'enable_dice_rethrow': True,
}
TEMPERATURE_SCHEDULE = [2.0, 1.5, 1, 0.8, 0.7]
VALUE_SCALING = LR.CLASSIC_SCALING["value"]
POLICY_SCALING = LR.CLASSIC_SCALING["policy"]
CHANCE_SCALING = LR.CLASSIC_SCALING["chance"]
DISCOUNT_SCALING = LR.CLASSIC_SCALING["discount"]
REWARD_SCALING = LR.CLASSIC_SCALING["reward"]
config = {                                  # :380-406
    "seed": 8,
    "learning_rate": 0.005,
    "num_games_per_iteration": 1500,
    "iterations": 120,
    "Buffer_Capacity": 20000,
    "Buffer_batch_Size": 128,
    "unroll_steps": 10,
    "td_steps": 25,
    "max_episode_length": 800,
    "MCTS_simulations": 75,
    "MCTS_max_depth": 50,
    "Bootstrap_Value_Target": True,
    "Bootstrap_Switch_Iteration": 150,
    "Temperature_Schedule": TEMPERATURE_SCHEDULE,
    "train_steps_per_iteration": 2500,
    "rules": RULES,
    "Loss Scaling": {"value_loss": VALUE_SCALING, "policy_loss": POLICY_SCALING, "chance_loss": CHANCE_SCALING,
                     "discount_loss": DISCOUNT_SCALING, "reward_loss": REWARD_SCALING},
    "checkpoint_every": 100,
    "checkpoint_dir": os.path.join("MuZero_Classic_MADN", "models"),
}
LR_BOUNDARIES = LR.CLASSIC_LR_BOUNDARIES    # :416-423


def make_optimizer(cfg: dict) -> T.Optimizer:
    return T.Optimizer(LR.StochasticLearner, cfg["unroll_steps"], cfg["learning_rate"],
                       cfg["train_steps_per_iteration"], LR_BOUNDARIES)


optimizer = make_optimizer(config)


def learning_rate_schedule(step: int) -> float:
    return optimizer.schedule(step)


def get_temperature(iteration, total_iterations):
    return T.get_temperature(iteration, total_iterations, TEMPERATURE_SCHEDULE)


def balanced_loss(ce, is_rare, mask, n_valid, w_rare=1.0, w_common=0.1):
    """:25-31 on torch tensors (scalars for one step; learner.balanced_loss_steps batches the steps)."""
    masked_rare = mask * is_rare
    n_rare = torch.clamp(masked_rare.sum(), min=1.0)
    n_common = torch.clamp(n_valid - n_rare, min=1.0)
    return w_rare * (masked_rare * ce).sum() / n_rare + w_common * ((mask - masked_rare) * ce).sum() / n_common


def init_muzero_params(rng_key, input_shape) -> dict:
    """muzero_classic_madn.py:519-565: the Flax tree for an observation of ``input_shape`` = (C, 56)."""
    from . import checkpoint as CK
    from .nets import rng_key_to_seed
    return CK.flat_to_muzero_tree(ST.init_classic_params(int(input_shape[0]), rng_key_to_seed(rng_key) % (2 ** 32)))


def loss_fn_stochastic(params, batch):
    """:34-181 -> (total, (value, policy, chance, discount, reward)) on the batch's device."""
    flat = T._flat(params)
    nets = LR.ClassicMuZeroNets({k: (v.detach().cpu().numpy() if hasattr(v, "detach") else v) for k, v in flat.items()},
                                int(flat["representation/Dense_1/kernel"].shape[0]) + 6,
                                device=batch["observations"].device)
    return LR.loss_fn_stochastic(nets, batch, config["unroll_steps"])


def train_step(params, opt_state, batch):
    """:183-199 -> (new_params, new_opt_state, {total_loss, v_loss, p_loss, c_loss, d_loss, r_loss})."""
    return T.train_step(params, opt_state, batch)


def _replay(cfg, input_shape):
    return R.VectorizedReplayBufferStochastic(capacity=cfg["Buffer_Capacity"], batch_size=cfg["Buffer_batch_Size"],
                                              unroll_steps=cfg["unroll_steps"], td_steps=cfg["td_steps"],
                                              obs_shape=tuple(input_shape), action_dim=4,
                                              max_episode_length=cfg["max_episode_length"],
                                              bootstrap_value_target=cfg["Bootstrap_Value_Target"])


def _checkpoint_names(cfg, it):
    d = cfg.get("checkpoint_dir", os.path.join("MuZero_Classic_MADN", "models"))
    stem = f"TEAMstochastic_muzero_madn_{{}}_lr{cfg['learning_rate']}_g{cfg['num_games_per_iteration']}_it{it}_seed{cfg['seed']}"
    return (os.path.join(d, "params", stem.format("params") + ".params"),
            os.path.join(d, "opt_state", stem.format("opt_state") + ".opt_state"))


def test_training(config, params=None, opt_state=None, log=print):
    """:201-355 -> (params, opt_state, times_per_iteration)."""
    opt = make_optimizer(config) if opt_state is None else optimizer
    input_shape = (E.num_channels(4), E.CELLS)          # :218-239: encode_board of a 4-player reset (11, 56)
    return T.run_training(config, params, opt_state, kind="classic", play_n_games_v3=GS.play_n_games_v3,
                          make_replay=_replay, optimizer=opt, init_params=init_muzero_params,
                          input_shape=input_shape, schedule=TEMPERATURE_SCHEDULE,
                          switch_guard=lambda cfg: not cfg["Bootstrap_Value_Target"],
                          checkpoint_names=_checkpoint_names, log=log)


test_training.__test__ = False


if __name__ == "__main__":
    import time
    t0 = time.time()
    _, _, times = test_training(config=config)
    print(f"Total training time: {time.time() - t0:.1f} s; average per iteration {sum(times) / len(times):.2f} s")
