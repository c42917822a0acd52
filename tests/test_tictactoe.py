"""TicTacToe (config (a), host code in libmuz.so) vs oracle/tictactoe.py (CPU, no GPU needed).

The product and the oracle share the counter streams and evaluate the tree in double with the same
libm calls, so everything is compared exactly: env transitions including the reference's quirks
(oldest move cleared on invalid / post-terminal steps, `done` precedence), policy logits, rollouts,
muzero_policy visit counts / weights / values / actions, and whole eval.py matches.  Results-level
check against TicTacToe/results.md: MCTS(5) beats the random bot in ~97 % of games."""
import numpy as np
import pytest

from oracle import tictactoe as OT


def _T():
    import muzpkg
    muzpkg.load()
    from exploring_muzero_on_dog_amd import tictactoe as T
    return T


def _same(dev, ora):
    return (dev.board.reshape(-1).tolist() == ora.board and dev.current_player == ora.current_player and
            dev.reward == ora.reward and dev.done == ora.done and dev.memory.tolist() == ora.memory)


def _random_walks(n_walks, length, seed):
    """States reached by uniformly random actions 0..8 (invalid and post-terminal steps included)."""
    T = _T()
    rng = np.random.default_rng(seed)
    for _ in range(n_walks):
        d, o = T.env_reset(), OT.env_reset()
        for _ in range(int(rng.integers(0, length))):
            a = int(rng.integers(0, 9))
            d, rd, dd = T.env_step(d, a)
            o, ro, do = OT.env_step(o, a)
            assert (rd, dd) == (ro, do) and _same(d, o)
        yield d, o


def test_env_step_quirks_and_policy():
    T = _T()
    n = 0
    for d, o in _random_walks(400, 14, 0):
        assert T.policy_function(d).tolist() == OT.policy_function(o)
        n += 1
    assert n == 400
    # TicTacToeV2.env_step quirks, checked on the product directly:
    e = T.env_reset()
    for a in (0, 4, 1, 8, 6, 3):        # X: 0 1 6, O: 4 8 3
        e, r, d = T.env_step(e, a)
    e, r, d = T.env_step(e, 4)          # X plays an occupied cell: refused ...
    assert (r, d) == (-1, True)
    assert e.board.reshape(-1)[0] == 0 and e.memory.tolist() == [[0, 1, 6], [4, 8, 3]]   # ... yet X's oldest piece goes
    e2, r, d = T.env_step(e, 1)         # a post-terminal step onto an occupied cell "un-finishes" the game
    assert (r, d) == (0, False) and e2.current_player == -e.current_player


def test_rollouts_match():
    T = _T()
    for i, (d, o) in enumerate(_random_walks(150, 10, 1)):
        assert T.value_function(d, 77, i) == OT.rollout(o, 77, i)


@pytest.mark.parametrize("S", [5, 25])
def test_muzero_policy_matches(S):
    T = _T()
    for i, (d, o) in enumerate(_random_walks(40, 8, 2 + S)):
        got = T.run_mcts(1000 + i, d, S, 9, 1.0, turn=i)
        a, w, v, vis = OT.muzero_policy(o, S, 9, 1.0, 1000 + i, i)
        assert got["visit_counts"].tolist() == vis
        assert got["action_weights"].tolist() == w
        assert got["value"] == v and got["action"] == a


def test_matches_and_results_md():
    T = _T()
    for g in range(12):
        p = 1 if g % 2 == 0 else -1
        assert T.match(p, 5, 3, g) == OT.match(p, 5, 3, g)
    r = T.evaluate(200, 5, seed=1)
    # TicTacToe/results.md: "MCTS (5)" vs random bot 97.10 % wins, 2.70 % losses
    assert r["win"] >= 0.9 and r["loss"] <= 0.08, r


# ---- checkpoint I/O + the reference's trained policy (TicTacToe/results.md) --------------------------
import json  # noqa: E402
import os  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF_CKPT = "/root/reference/TicTacToe/Checkpoints/TicTacToeV2_imp_net_3000ep_00001lr.params"


def _ck():
    import muzpkg
    muzpkg.load()
    from exploring_muzero_on_dog_amd import checkpoint as CK
    return CK


@pytest.mark.skipif(not os.path.exists(REF_CKPT), reason="reference checkpoint not present")
def test_flax_msgpack_roundtrip_is_byte_exact():
    CK = _ck()
    raw = open(REF_CKPT, "rb").read()
    tree = CK.load_flax_msgpack(raw)
    assert CK.dumps_flax_msgpack(tree) == raw
    fx = np.load(os.path.join(GOLDEN, "ttt_imp_net_3000ep.npz"))
    flat = CK.flatten(tree)
    assert sorted(k.replace("/", "__") for k in flat) == sorted(fx.files)
    assert all(np.array_equal(flat[k], fx[k.replace("/", "__")]) for k in flat)


def test_trained_policy_reproduces_results_md():
    """The reference's trained ImprovedTicTacToeNet (3000 episodes) against the random bot through this
    engine's TicTacToeV2: results.md reports 82.2 % wins (444 / 500 as first player, 378 / 500 as second)."""
    CK = _ck()
    T = _T()
    fx = np.load(os.path.join(GOLDEN, "ttt_imp_net_3000ep.npz"))
    net = T.PolicyNet(CK.unflatten({k.replace("__", "/"): fx[k] for k in fx.files}))
    want = json.load(open(os.path.join(GOLDEN, "ttt_imp_net_3000ep_results.json")))
    r = T.evaluate_trained(net, 2000, seed=1)
    assert abs(r["win"] - want["win"]) < 0.04, r                       # ~4.7 standard errors at n = 2000
    assert abs(r["wins_as_first"] / 1000 - 444 / 500) < 0.05, r
    assert abs(r["wins_as_second"] / 1000 - 378 / 500) < 0.06, r


def test_muzero_checkpoint_tree_roundtrip(tmp_path):
    CK = _ck()
    from oracle import nets as ON
    flat = ON.init_params(18, seed=2)
    tree = CK.flat_to_muzero_tree(flat)
    p = tmp_path / "m.params"
    CK.save_flax_msgpack(str(p), tree)
    back = CK.muzero_tree_to_flat(CK.load_flax_msgpack(str(p)))
    assert set(back) == set(flat) and all(np.array_equal(back[k], flat[k]) for k in flat)
    s = tmp_path / "m.safetensors"
    CK.save_flat(str(s), flat)
    back = CK.load_flat(str(s))
    assert all(np.array_equal(back[k], flat[k]) for k in flat)
