"""The det-MADN learner script's entry points (MuZero_det_MADN/train_with_reward.py), on the device engine.

Same names, arguments and meaning as the reference module:
  get_temperature(iteration, total_iterations)          :18-22
  loss_fn(params, batch)                                :24-146  (learner.loss_fn on the device)
  train_step(params, opt_state, batch)                  :148-164 -> (params, opt_state, losses)
  test_training(config, params=None, opt_state=None)    :168-309 -> (params, opt_state, times_per_iteration)
  RULES, TEMPERATURE_SCHEDULE, *_SCALING, config        :311-352
  learning_rate_schedule, optimizer                     :361-373
Differences, by design: importing this module trains nothing (the reference starts wandb and a 100-iteration
run at import; ``python -m ... train_with_reward`` does that here, without wandb); ``opt_state`` is the device
learner (training.OptState) rather than an optax pytree; checkpoints are written in flax's msgpack format
(training.save_checkpoint) instead of pickles; self-play keys are the engine's counter-RNG seeds
(nets.rng_key_to_seed) instead of threefry keys.  To switch the reference script over, replace its imports
(:13-16) and its module-level optimizer with this module's names.
"""
from __future__ import annotations

import os

from . import detmadn as E
from . import game_agent as GA
from . import learner as LR
from . import nets as N
from . import replay as R
from . import training as T

RULES = {                                   # :311-321
    'enable_teams': True,
    'enable_initial_free_pin': True,
    'enable_circular_board': False,
    'enable_friendly_fire': False,
    'enable_start_blocking': False,
    'enable_jump_in_goal_area': True,
    'enable_start_on_1': True,
    'enable_bonus_turn_on_6': True,
    'must_traverse_start': False,
}
TEMPERATURE_SCHEDULE = [2.0, 1.5, 1, 0.8, 0.6]
VALUE_SCALING = LR.VALUE_SCALING
POLICY_SCALING = LR.POLICY_SCALING
DISCOUNT_SCALING = LR.DISCOUNT_SCALING
REWARD_SCALING = LR.REWARD_SCALING
config = {                                  # :327-352
    "seed": 42,
    "learning_rate": 0.005,
    "num_games_per_iteration": 1500,
    "iterations": 100,
    "Buffer_Capacity": 20000,
    "Buffer_batch_Size": 128,
    "unroll_steps": 10,
    "td_steps": 50,
    "max_episode_length": 550,
    "MCTS_simulations": 100,
    "MCTS_max_depth": 50,
    "Bootstrap_Value_Target": False,
    "Bootstrap_Switch_Iteration": 70,
    "Temperature_Schedule": TEMPERATURE_SCHEDULE,
    "train_steps_per_iteration": 2500,
    "rules": RULES,
    "Loss scaling": {"value": VALUE_SCALING, "policy": POLICY_SCALING, "discount": DISCOUNT_SCALING,
                     "reward": REWARD_SCALING},
    # this engine's additions (the reference hard-codes them): checkpoint cadence and directory
    "checkpoint_every": 100,
    "checkpoint_dir": os.path.join("MuZero_det_MADN", "models"),
}
LR_BOUNDARIES = LR.DET_LR_BOUNDARIES        # :361-368, in iterations of train_steps_per_iteration steps


def make_optimizer(cfg: dict) -> T.Optimizer:
    """optax.chain(clip_by_global_norm(5.0), adamw(piecewise_constant_schedule, weight_decay=1e-4)) (:361-373)."""
    return T.Optimizer(LR.Learner, cfg["unroll_steps"], cfg["learning_rate"], cfg["train_steps_per_iteration"],
                       LR_BOUNDARIES)


optimizer = make_optimizer(config)


def learning_rate_schedule(step: int) -> float:
    return optimizer.schedule(step)


def get_temperature(iteration, total_iterations):
    """:18-22 (reads the module's TEMPERATURE_SCHEDULE, as the reference does)."""
    return T.get_temperature(iteration, total_iterations, TEMPERATURE_SCHEDULE)


def init_muzero_params(rng_key, input_shape) -> dict:
    """muzero_deterministic_madn.py:706-748: the Flax tree {"representation": {"params": ...}, ...} for an
    observation of ``input_shape`` = (C, 56); Flax default initialisers from a seeded NumPy stream
    (``rng_key``: int or uint32[2] key)."""
    from . import checkpoint as CK
    return CK.flat_to_muzero_tree(N.init_muzero_params(N.rng_key_to_seed(rng_key) % (2 ** 32), int(input_shape[0])))


def loss_fn(params, batch):
    """:24-146 -> (total_loss, (value_loss, policy_loss, discount_loss, reward_loss)) on the batch's device."""
    flat = T._flat(params)
    dev = batch["observations"].device
    nets = LR.MuZeroNets({k: (v.detach().cpu().numpy() if hasattr(v, "detach") else v) for k, v in flat.items()},
                         int(flat["representation/Dense_1/kernel"].shape[0]) + 6,
                         int(flat["prediction/Dense_2/kernel"].shape[1]), device=dev)
    return LR.loss_fn(nets, batch, config["unroll_steps"])


def train_step(params, opt_state, batch):
    """:148-164: one clipped AdamW step -> (new_params, new_opt_state, {total_loss, v_loss, p_loss, d_loss,
    r_loss}) (device tensors)."""
    return T.train_step(params, opt_state, batch)


def _replay(cfg, input_shape):
    return R.VectorizedReplayBuffer(capacity=cfg["Buffer_Capacity"], batch_size=cfg["Buffer_batch_Size"],
                                    unroll_steps=cfg["unroll_steps"], td_steps=cfg["td_steps"],
                                    obs_shape=tuple(input_shape), max_episode_length=cfg["max_episode_length"],
                                    bootstrap_value_target=cfg["Bootstrap_Value_Target"])


def _checkpoint_names(cfg, it):
    d = cfg.get("checkpoint_dir", os.path.join("MuZero_det_MADN", "models"))
    return (os.path.join(d, "params", f"Experiment_{cfg['seed']}_{it}.params"),
            os.path.join(d, "opt_state", f"Experiment_{cfg['seed']}_{it}.opt_state"))


def test_training(config, params=None, opt_state=None, log=print):
    """:168-309: 3 warm-up self-play calls into the device ring, then per iteration: the bootstrap switch at
    ``Bootstrap_Switch_Iteration`` (:248-252), self-play of ``num_games_per_iteration`` games with
    get_temperature, the games saved into the ring, ``train_steps_per_iteration`` train steps on sampled
    batches, a checkpoint every ``checkpoint_every`` (100) iterations (:301-307).
    -> (params, opt_state, times_per_iteration)."""
    opt = make_optimizer(config) if opt_state is None else None
    input_shape = (E.num_channels(4), E.CELLS)          # :186-205: encode_board of a 4-player reset
    # (self-play uses game_agent's own RULES, as the reference's play_n_games_v3 does)
    return T.run_training(config, params, opt_state, kind="det", play_n_games_v3=GA.play_n_games_v3,
                          make_replay=_replay,
                          optimizer=opt if opt is not None else optimizer, init_params=init_muzero_params,
                          input_shape=input_shape, schedule=TEMPERATURE_SCHEDULE,
                          switch_guard=lambda cfg: True, checkpoint_names=_checkpoint_names, log=log)


test_training.__test__ = False     # not a pytest test (the reference's name)


if __name__ == "__main__":
    import time
    t0 = time.time()
    _, _, times = test_training(config=config)
    print(f"Total training time: {time.time() - t0:.1f} s; average per iteration {sum(times) / len(times):.2f} s")
