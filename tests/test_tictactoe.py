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
