"""The reference-signature training entry points on the GPU (train_with_reward.py / train_stochastic.py):
test_training(config, params, opt_state) with a tiny config, train_step(params, opt_state, batch) against the
Learner it wraps, and the checkpoint round trip."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _mods():
    from exploring_muzero_on_dog_amd import learner as L
    from exploring_muzero_on_dog_amd import nets as N
    from exploring_muzero_on_dog_amd import train_stochastic as TS
    from exploring_muzero_on_dog_amd import train_with_reward as TW
    from exploring_muzero_on_dog_amd import training as T
    return L, N, TS, TW, T


def _tiny(cfg, tmp_path, **kw):
    c = copy.deepcopy(cfg)
    c.update(num_games_per_iteration=24, iterations=2, Buffer_Capacity=200, max_episode_length=160,
             MCTS_simulations=4, MCTS_max_depth=4, train_steps_per_iteration=3, Bootstrap_Switch_Iteration=1,
             checkpoint_every=1, checkpoint_dir=str(tmp_path), game_warmup=1, **kw)
    return c


def test_det_test_training_tiny(cuda, tmp_path):
    L, N, TS, TW, T = _mods()
    cfg = _tiny(TW.config, tmp_path)
    lines = []
    params, opt_state, times = TW.test_training(cfg, log=lines.append)
    assert len(times) == 2 and all(t > 0 for t in times)
    # the bootstrap switch fired once, at iteration index 1 (train_with_reward.py:248-252)
    assert sum("SWITCHING TO BOOTSTRAP" in s for s in lines) == 1
    assert T.run_training.last["replay"].bootstrap_value_target is True
    assert opt_state.count == 2 * 3
    # params is the Flax tree of the learner's live tensors; it round-trips through as_device_net
    assert set(params) == {"representation", "dynamics", "prediction"}
    net = N.as_device_net(params)
    obs = torch.from_numpy(np.random.default_rng(0).integers(0, 3, (16, 34, 56)).astype(np.float32)).cuda()
    lg, v, e = N.root_inference_fn(net, obs)
    with torch.no_grad():
        te = opt_state.learner.nets.representation(obs)
        tl, tv = opt_state.learner.nets.prediction(te)
    assert max((e - te).abs().max().item(), (lg - tl).abs().max().item(), (v - tv[:, 0]).abs().max().item()) < 2e-5
    saved = {k: v.detach().cpu().numpy().copy() for k, v in T.CK.muzero_tree_to_flat_any(params).items()}
    # a further train step changes the live tensors; as_device_net re-packs them (versioned tree) into the cached
    # DeviceNet in place (same shapes), so engines cached on it see the new weights
    params, opt_state, _ = T.train_step_from(params, opt_state, T.run_training.last["replay"])
    net2 = N.as_device_net(params)
    lg2, v2, e2 = N.root_inference_fn(net2, obs)
    with torch.no_grad():
        te2 = opt_state.learner.nets.representation(obs)
        tl2, tv2 = opt_state.learner.nets.prediction(te2)
    assert max((e2 - te2).abs().max().item(), (lg2 - tl2).abs().max().item(),
               (v2 - tv2[:, 0]).abs().max().item()) < 2e-5
    assert (lg2 - lg).abs().max().item() > 0
    # the checkpoint of the last iteration (train_with_reward.py:301-307 cadence, here every iteration) holds
    # the parameters and Adam state of that moment
    pp, op = TW._checkpoint_names(cfg, 2)
    p2, st2 = T.load_checkpoint(pp, op, TW.make_optimizer(cfg))
    assert st2.count == 2 * 3
    got = {k: v.detach().cpu().numpy() for k, v in T.CK.muzero_tree_to_flat_any(p2).items()}
    assert set(got) == set(saved) and all(np.array_equal(got[k], saved[k]) for k in saved)


def test_det_train_step_signature_matches_learner(cuda):
    """train_step(params, opt_state, batch) == Learner.train_step on the same batches; a params tree passed in
    from outside is copied into the learner first."""
    L, N, TS, TW, T = _mods()
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import replay as R
    C = 34
    params = TW.init_muzero_params(7, (C, 56))
    flat = T.CK.muzero_tree_to_flat(params)
    net = N.DeviceNet(flat, C)
    eng = GA.SelfPlayEngine(net, 16, num_players=4, max_steps=200, num_simulations=4, max_depth=4)
    ring = R.VectorizedReplayBuffer(64, 32, 10, 50, obs_shape=(C, 56), max_episode_length=200,
                                    rng=np.random.RandomState(1))
    ring.save_games_from_buffers(eng.play(seed=3))
    batches = [ring.sample_batch() for _ in range(3)]
    cfg = dict(TW.config, train_steps_per_iteration=2500)
    opt = TW.make_optimizer(cfg)
    st = opt.init(params)
    ref = L.Learner(flat, C, unroll_steps=10, graph=True)
    p = params
    for b in batches:
        p, st, losses = TW.train_step(p, st, b)
        want = ref.train_step(b)
        assert torch.equal(losses["total_loss"], want["total_loss"])
    for k in ref.nets.p:
        assert torch.equal(ref.nets.p[k], st.learner.nets.p[k]), k
    # an external tree (the initial params) resets the learner's parameters to it
    p, st, _ = TW.train_step(params, st, batches[0])
    fresh = L.Learner(flat, C, unroll_steps=10, graph=True)
    fresh.opt.count.fill_(3.0)
    for m, v, m2, v2 in zip(fresh.opt.mu, fresh.opt.nu, ref.opt.mu, ref.opt.nu):
        m.copy_(m2)
        v.copy_(v2)
    fresh.train_step(batches[0])
    for k in fresh.nets.p:
        assert torch.equal(fresh.nets.p[k], st.learner.nets.p[k]), k


def test_classic_test_training_tiny(cuda, tmp_path):
    L, N, TS, TW, T = _mods()
    cfg = _tiny(TS.config, tmp_path, Bootstrap_Value_Target=False)
    lines = []
    params, opt_state, times = TS.test_training(cfg, log=lines.append)
    assert len(times) == 2
    assert sum("SWITCHING TO BOOTSTRAP" in s for s in lines) == 1
    assert T.run_training.last["replay"].bootstrap_value_target is True
    # a run that starts on bootstrap targets never switches (train_stochastic.py:289)
    lines2 = []
    TS.test_training(_tiny(TS.config, tmp_path, Bootstrap_Value_Target=True), log=lines2.append)
    assert not any("SWITCHING" in s for s in lines2)
    from exploring_muzero_on_dog_amd import stochastic as ST
    net = ST.as_device_classic_net(params)
    obs = torch.from_numpy(np.random.default_rng(1).integers(0, 3, (8, 11, 56)).astype(np.float32)).cuda()
    lg, v, e = ST.root_inference_fn(net, obs)
    with torch.no_grad():
        te = opt_state.learner.nets.representation(obs)
        tl, tv = opt_state.learner.nets.prediction(te)
    assert max((e - te).abs().max().item(), (lg - tl).abs().max().item()) < 2e-5


def test_dog_test_training_tiny(cuda, tmp_path):
    """MuZero_DOG/train.py's test_training (train_dog.py) with a tiny config: DOG games recorded by
    game_agent_dog.play_n_games_v3 into a ring at action_dim 806, DogLearner steps, the bootstrap switch, checkpoints;
    the learner's weights reach the self-play arena (the root inference equals the torch forward)."""
    from exploring_muzero_on_dog_amd import muzero_dog as MD
    from exploring_muzero_on_dog_amd import train_dog as TD
    from exploring_muzero_on_dog_amd import training as T
    cfg = _tiny(TD.config, tmp_path)
    lines = []
    params, opt_state, times = TD.test_training(cfg, log=lines.append)
    assert len(times) == 2 and sum("SWITCHING TO BOOTSTRAP" in s for s in lines) == 1
    replay = T.run_training.last["replay"]
    assert replay.action_dim == 806 and replay.size == 3 * 24
    assert opt_state.count == 2 * 3 and all(np.isfinite(list(h.values())).all() for h in T.run_training.last["history"])
    net = MD.as_device_net(params)
    obs = replay.observations[:16, 3].float()
    lg, v, e = MD.root_inference_fn(net, obs)
    with torch.no_grad():
        te = opt_state.learner.nets.representation(obs)
        tl, tv = opt_state.learner.nets.prediction(te)
    assert max((e - te).abs().max().item(), (lg - tl).abs().max().item(), (v - tv[:, 0]).abs().max().item()) < 2e-5
    p2, o2 = T.load_checkpoint(*TD._checkpoint_names(cfg, 2), TD.optimizer)
    assert o2.count == opt_state.count
