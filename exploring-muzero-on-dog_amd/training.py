"""The reference's functional training API on the device learner (shared by train_with_reward.py and
train_stochastic.py).

The reference trains with pure functions on pytrees (MuZero_det_MADN/train_with_reward.py:148-309,
MuZero_Classic_MADN/train_stochastic.py:183-355):

    opt_state = optimizer.init(params)
    params, opt_state, losses = train_step(params, opt_state, batch)     # jax.jit(value_and_grad + optax)

Here the parameters, Adam moments and step count live on the GPU inside a ``learner.Learner`` (graph-
captured forward + backward + muz_adamw_step).  ``OptState`` is the reference's ``opt_state``: it owns that
learner.  ``params`` handed out by ``train_step`` is the reference's Flax tree
(``{"representation": {"params": ...}, "dynamics": ..., "prediction": ...}``) whose leaves ARE the learner's
live parameter tensors, so the reference's loop -- which rebinds ``params, opt_state`` every step and passes
``params`` to ``play_n_games_v3`` once per iteration -- runs unchanged without copies.  A different tree
passed in (e.g. loaded from a checkpoint) is copied into the learner first.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from . import checkpoint as CK
from . import learner as LR


def _flat(params) -> dict:
    if isinstance(params, dict) and all(isinstance(k, str) and "/" in k for k in params):
        return params
    return CK.muzero_tree_to_flat_any(params)


class OptState:
    """The reference's ``opt_state`` (optax chain(clip_by_global_norm, adamw) state): the device learner with
    its parameters, Adam moments (mu, nu) and step count."""

    def __init__(self, learner: LR.Learner):
        self.learner = learner
        self.tree = CK.flat_to_muzero_tree(learner.nets.p)      # leaves: the live parameter tensors
        self.version = 0                                        # in-place updates of the tree so far
        from . import nets as N
        N.register_versioned_params(self.tree, lambda: self.version)

    @property
    def count(self) -> int:
        return int(self.learner.opt.count.item())

    def bind(self, params):
        """Make the learner's parameters equal ``params`` (a no-op for the tree train_step handed out)."""
        if params is self.tree:
            return
        self.version += 1
        flat = _flat(params)
        if set(flat) != set(self.learner.nets.p):
            raise ValueError("params do not match the learner's parameter names")
        with torch.no_grad():
            for k, p in self.learner.nets.p.items():
                v = flat[k]
                p.copy_(v.detach().reshape(p.shape) if isinstance(v, torch.Tensor)
                        else torch.from_numpy(np.asarray(v, np.float32).reshape(p.shape)))

    def state_dict(self) -> dict:
        """{count, mu, nu} with mu / nu as flat path-named float32 arrays (host)."""
        names = list(self.learner.nets.p)
        return {"count": self.count,
                "mu": {k: m.detach().cpu().numpy() for k, m in zip(names, self.learner.opt.mu)},
                "nu": {k: v.detach().cpu().numpy() for k, v in zip(names, self.learner.opt.nu)}}

    def load_state_dict(self, sd: dict):
        names = list(self.learner.nets.p)
        with torch.no_grad():
            for k, m, v in zip(names, self.learner.opt.mu, self.learner.opt.nu):
                m.copy_(torch.from_numpy(np.asarray(sd["mu"][k], np.float32).reshape(m.shape)))
                v.copy_(torch.from_numpy(np.asarray(sd["nu"][k], np.float32).reshape(v.shape)))
            self.learner.opt.count.fill_(float(sd["count"]))
        self.version += 1


class Optimizer:
    """``optax.chain(clip_by_global_norm(5.0), adamw(piecewise_constant_schedule(lr, boundaries), wd 1e-4))``
    with ``init(params) -> OptState`` (train_with_reward.py:361-373, train_stochastic.py:416-428)."""

    def __init__(self, learner_cls, unroll_steps: int, learning_rate: float, steps_per_iteration: int,
                 boundaries, graph: bool = True):
        self.learner_cls, self.unroll_steps = learner_cls, int(unroll_steps)
        self.lr0, self.spi, self.boundaries = float(learning_rate), int(steps_per_iteration), tuple(boundaries)
        self.graph = bool(graph)

    def init(self, params) -> OptState:
        flat = {k: (v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v, np.float32))
                for k, v in _flat(params).items()}
        C = int(flat["representation/Dense_1/kernel"].shape[0]) + 6
        kw = dict(unroll_steps=self.unroll_steps, graph=self.graph, lr0=self.lr0, steps_per_iteration=self.spi,
                  boundaries=self.boundaries)
        if self.learner_cls is LR.Learner:
            learner = LR.Learner(flat, C, int(flat["prediction/Dense_2/kernel"].shape[1]), **kw)
        else:
            learner = self.learner_cls(flat, C, **kw)
        return OptState(learner)

    def schedule(self, step: int) -> float:
        """optax.piecewise_constant_schedule(lr, {b * steps_per_iteration: s})."""
        lr = self.lr0
        for b, s in self.boundaries:
            if step >= b * self.spi:
                lr *= s
        return lr


def train_step(params, opt_state: OptState, batch: dict):
    """(params, opt_state, batch) -> (new_params, new_opt_state, losses): one clipped AdamW step on the
    MuZero loss.  The returned params / opt_state are the learner's live state (the reference rebinds both)."""
    opt_state.bind(params)
    losses = opt_state.learner.train_step(batch)
    opt_state.version += 1
    return opt_state.tree, opt_state, losses


def train_step_from(params, opt_state: OptState, replay):
    """train_step(params, opt_state, replay.sample_batch()) with the ring writing the batch straight into the
    captured step's inputs (Learner.train_step_from; same draws, same result)."""
    opt_state.bind(params)
    losses = opt_state.learner.train_step_from(replay)
    opt_state.version += 1
    return opt_state.tree, opt_state, losses


def get_temperature(iteration, total_iterations, schedule):
    """Phase-based temperature: int(iteration / total * len(schedule)), clamped (train_with_reward.py:18-22)."""
    phase = int(iteration / total_iterations * len(schedule))
    return schedule[min(phase, len(schedule) - 1)]


def save_checkpoint(params_path: str, opt_path: str, params, opt_state: OptState):
    """The reference pickles params / opt_state every 100 iterations (train_with_reward.py:301-307); here params
    go to the flax.serialization.to_bytes format (checkpoint.save_flax_msgpack, readable by the reference's
    flax.serialization.from_bytes) and opt_state to a msgpack map {count, mu, nu} of the same encoding."""
    os.makedirs(os.path.dirname(params_path) or ".", exist_ok=True)
    os.makedirs(os.path.dirname(opt_path) or ".", exist_ok=True)
    flat = {k: (v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v, np.float32))
            for k, v in _flat(params).items()}
    CK.save_flax_msgpack(params_path, CK.flat_to_muzero_tree(flat))
    sd = opt_state.state_dict()
    with open(opt_path, "wb") as f:
        f.write(CK.dumps_flax_msgpack({"count": np.asarray(sd["count"], np.int32),
                                       "mu": CK.flat_to_muzero_tree(sd["mu"]), "nu": CK.flat_to_muzero_tree(sd["nu"])}))


def load_checkpoint(params_path: str, opt_path: str | None, optimizer: Optimizer):
    """-> (params tree, opt_state) from save_checkpoint's files (opt_state fresh when opt_path is None)."""
    params = CK.load_flax_msgpack(params_path)
    st = optimizer.init(params)
    if opt_path is not None:
        with open(opt_path, "rb") as f:
            raw = CK.loads_flax_msgpack(f.read())
        st.load_state_dict({"count": int(np.asarray(raw["count"]).reshape(-1)[0]), "mu": CK.muzero_tree_to_flat(raw["mu"]),
                            "nu": CK.muzero_tree_to_flat(raw["nu"])})
    return st.tree, st


def run_training(config, params, opt_state, *, kind, play_n_games_v3, make_replay, optimizer: Optimizer,
                 init_params, input_shape, schedule, switch_guard, checkpoint_names, log=print):
    """The body of test_training (train_with_reward.py:168-309 / train_stochastic.py:201-355)."""
    seed = config["seed"]
    iterations = config["iterations"]
    num_games = config["num_games_per_iteration"]
    max_episode_length = config["max_episode_length"]
    num_simulation = config["MCTS_simulations"]
    max_depth = config["MCTS_max_depth"]
    train_steps_per_iteration = config["train_steps_per_iteration"]
    switch_to_bootstrap_iteration = config["Bootstrap_Switch_Iteration"]
    every = int(config.get("checkpoint_every", 100))

    if params is None:
        params = init_params(seed, input_shape)
    if opt_state is None:
        opt_state = optimizer.init(params)
    params = opt_state.tree if opt_state.tree is params else (opt_state.bind(params) or opt_state.tree)
    replay = make_replay(config, input_shape)

    def play(key, temp):
        # obs stay int8 (the ring's dtype): the fp32 copy the reference keeps would only be converted back
        return play_n_games_v3(params, key, input_shape, num_envs=num_games, num_simulation=num_simulation,
                               max_depth=max_depth, max_steps=max_episode_length, temp=temp, obs_dtype=torch.int8)

    log("Collecting initial games...")
    for n in range(int(config.get("game_warmup", 3))):
        replay.save_games_from_buffers(play(seed * n, get_temperature(0, iterations, schedule)))
    times_per_iteration, history = [], []
    for it in range(iterations):
        start_time = time.time()
        if it == switch_to_bootstrap_iteration and switch_guard(config):
            log("SWITCHING TO BOOTSTRAP VALUE TARGETS")
            replay.bootstrap_value_target = True
        temp = get_temperature(it, iterations, schedule)
        buffers = play(seed + it ** 3, temp)
        lengths = buffers["idx"]
        log(f"Iteration {it + 1}/{iterations}: episode lengths min={int(lengths.min())}, max={int(lengths.max())}, "
            f"mean={float(lengths.float().mean()):.1f}")
        replay.save_games_from_buffers(buffers)
        train_start = time.time()
        losses = None
        for i in range(train_steps_per_iteration):
            params, opt_state, losses = train_step_from(params, opt_state, replay)
        end_time = time.time()
        if losses is not None:
            history.append({k: float(v) for k, v in losses.items()})
            log(f"  losses {history[-1]}; play {train_start - start_time:.2f} s, train {end_time - train_start:.2f} s")
        times_per_iteration.append(end_time - start_time)
        if every > 0 and (it + 1) % every == 0:
            pp, op = checkpoint_names(config, it + 1)
            log(f"Saving checkpoint at iteration {it + 1}...")
            save_checkpoint(pp, op, params, opt_state)
    run_training.last = {"replay": replay, "history": history}
    return params, opt_state, times_per_iteration
