"""The DOG learner script's entry points (MuZero_DOG/train.py), on the device engine.

The reference script cannot run as written: its ``play_batch_of_games_jitted`` (MuZero_DOG/game_agent.py:52-57),
DynamicsNetwork / PredictionNetwork (muzero_dog.py:85-99) and DOG ``encode_board`` (DOG/dog.py:1264-1272) are ``pass``,
and test_training reads ``RULES['enable_start_on_1']`` / ``['enable_bonus_turn_on_6']`` (train.py:199-200), keys its
RULES (311-322) lacks.  Here the missing pieces are the DOG slice's (muzero_dog.py, game_agent_dog.py), and the rest
keeps the reference's names, arguments and meaning:
  get_temperature(iteration, total_iterations)          :18-22
  loss_fn(params, batch)                                :24-146  (train_with_reward.py's loss on the DOG nets)
  train_step(params, opt_state, batch)                  :148-164 -> (params, opt_state, losses)
  test_training(config, params=None, opt_state=None)    :168-300 -> (params, opt_state, times_per_iteration)
  RULES, TEMPERATURE_SCHEDULE, *_SCALING, config        :311-352
  learning_rate_schedule, optimizer                     :355-373
Differences, as train_with_reward.py's mirror: importing trains nothing (no wandb session); ``opt_state`` is the device
learner (training.OptState); checkpoints in flax's msgpack format every 100 iterations (:279-286); self-play keys are
the engine's counter-RNG seeds."""
from __future__ import annotations

import os

from . import game_agent_dog as GAD
from . import learner as LR
from . import muzero_dog as MD
from . import nets as N
from . import replay as R
from . import training as T

RULES = dict(GAD.RULES)                     # :311-322
TEMPERATURE_SCHEDULE = [2.0, 1.5, 1, 0.8, 0.6]
VALUE_SCALING = LR.VALUE_SCALING            # :323-326 (4, 1, 1, 1: train_with_reward.py's)
POLICY_SCALING = LR.POLICY_SCALING
DISCOUNT_SCALING = LR.DISCOUNT_SCALING
REWARD_SCALING = LR.REWARD_SCALING
config = {                                  # :325-352
    "seed": 0,
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
    "checkpoint_every": 100,
    "checkpoint_dir": os.path.join("MuZero_DOG", "models"),
}
LR_BOUNDARIES = LR.DET_LR_BOUNDARIES        # :355-363 (30 / 60 / 85 iterations: x0.2, x0.2, x0.5)
INPUT_SHAPE = (MD.NUM_CHANNELS, 56)         # encode_board of a 4-player reset (:186-205)


class _DogOptimizer(T.Optimizer):
    def init(self, params) -> T.OptState:
        flat = {k: (v.detach().cpu().numpy() if hasattr(v, "detach") else v) for k, v in T._flat(params).items()}
        return T.OptState(LR.DogLearner(flat, unroll_steps=self.unroll_steps, graph=self.graph, lr0=self.lr0,
                                        steps_per_iteration=self.spi, boundaries=self.boundaries))


def make_optimizer(cfg: dict) -> T.Optimizer:
    """optax.chain(clip_by_global_norm(5.0), adamw(piecewise_constant_schedule, weight_decay=1e-4)) (:355-373)."""
    return _DogOptimizer(LR.DogLearner, cfg["unroll_steps"], cfg["learning_rate"], cfg["train_steps_per_iteration"],
                         LR_BOUNDARIES)


optimizer = make_optimizer(config)


def learning_rate_schedule(step: int) -> float:
    return optimizer.schedule(step)


def get_temperature(iteration, total_iterations):
    """:18-22."""
    return T.get_temperature(iteration, total_iterations, TEMPERATURE_SCHEDULE)


def init_muzero_params(rng_key, input_shape=INPUT_SHAPE) -> dict:
    """muzero_dog.py:139-181 (init_muzero_params): the Flax tree of the slice's networks; Flax default initialisers
    from a seeded NumPy stream (``rng_key``: int or uint32[2] key)."""
    from . import checkpoint as CK
    if tuple(input_shape) != INPUT_SHAPE:
        raise ValueError(f"input_shape {tuple(input_shape)} != {INPUT_SHAPE}")
    return CK.flat_to_muzero_tree(MD.init_muzero_params(N.rng_key_to_seed(rng_key) % (2 ** 32)))


def loss_fn(params, batch):
    """:24-146 -> (total_loss, (value_loss, policy_loss, discount_loss, reward_loss)) on the batch's device."""
    flat = T._flat(params)
    nets = LR.DogMuZeroNets({k: (v.detach().cpu().numpy() if hasattr(v, "detach") else v) for k, v in flat.items()},
                            device=batch["observations"].device)
    return LR.loss_fn(nets, batch, config["unroll_steps"])


def train_step(params, opt_state, batch):
    """:148-164: one clipped AdamW step -> (new_params, new_opt_state, {total_loss, v_loss, p_loss, d_loss, r_loss})."""
    return T.train_step(params, opt_state, batch)


def _replay(cfg, input_shape):
    return R.VectorizedReplayBuffer(capacity=cfg["Buffer_Capacity"], batch_size=cfg["Buffer_batch_Size"],
                                    unroll_steps=cfg["unroll_steps"], td_steps=cfg["td_steps"],
                                    obs_shape=tuple(input_shape), action_dim=MD.NUM_ACTIONS,
                                    max_episode_length=cfg["max_episode_length"],
                                    bootstrap_value_target=cfg["Bootstrap_Value_Target"])


def _checkpoint_names(cfg, it):
    d = cfg.get("checkpoint_dir", os.path.join("MuZero_DOG", "models"))
    return (os.path.join(d, "params", f"Experiment_{cfg['seed']}_{it}.params"),
            os.path.join(d, "opt_state", f"Experiment_{cfg['seed']}_{it}.opt_state"))


def test_training(config, params=None, opt_state=None, log=print):
    """:168-300: 3 warm-up self-play calls into the device ring (obs (34, 56), action_dim 806), then per iteration the
    bootstrap switch, self-play of ``num_games_per_iteration`` DOG games (game_agent_dog.play_n_games_v3), the games
    saved into the ring, ``train_steps_per_iteration`` learner steps, a checkpoint every 100 iterations."""
    opt = make_optimizer(config) if opt_state is None else None
    return T.run_training(config, params, opt_state, kind="dog", play_n_games_v3=GAD.play_n_games_v3,
                          make_replay=_replay, optimizer=opt if opt is not None else optimizer,
                          init_params=init_muzero_params, input_shape=INPUT_SHAPE, schedule=TEMPERATURE_SCHEDULE,
                          switch_guard=lambda cfg: True, checkpoint_names=_checkpoint_names, log=log)


test_training.__test__ = False     # not a pytest test (the reference's name)


if __name__ == "__main__":
    import time
    t0 = time.time()
    _, _, times = test_training(config=config)
    print(f"Total training time: {time.time() - t0:.1f} s; average per iteration {sum(times) / len(times):.2f} s")
