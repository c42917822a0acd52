"""CPU checks of the DOG MuZero slice's oracle (oracle/dog_muzero.py, the LayerNorm head of oracle/nets.py,
oracle/mctx_gumbel.py's wide-action sums).  The slice is builder-defined beyond the env (parity unpinned); these
tests pin the restatement's own invariants so the GPU tests compare against a self-consistent reference."""
import numpy as np

from oracle import dog as dg
from oracle import dog_muzero as DM
from oracle import mctx_gumbel as G
from oracle import nets as ON
from tests.dog_states import RULE_SETS, random_state, reset


def test_lane_tree_sum_order():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((7, 806)).astype(np.float32)
    got = G.lane_tree_sum(x)
    # the same order written out: lane sums in slot order, then pairwise over lanes
    for b in range(7):
        lanes = []
        for l in range(32):
            s = np.float32(x[b, l])
            for a in range(l + 32, 806, 32):
                s = np.float32(s + x[b, a])
            lanes.append(s)
        while len(lanes) > 1:
            lanes = [np.float32(lanes[i] + lanes[i + 1]) for i in range(0, len(lanes), 2)]
        assert got[b] == lanes[0]
    assert np.allclose(got, x.astype(np.float64).sum(-1), rtol=1e-5, atol=1e-4)
    # small A keeps numpy's own order (the det / classic kernels restate it)
    y = rng.standard_normal((5, 24)).astype(np.float32)
    assert np.array_equal(G.row_sum(y), y.sum(-1))
    # integer-valued entries sum exactly whatever the order
    z = rng.integers(0, 5, (3, 806)).astype(np.float32)
    assert np.array_equal(G.row_sum(z), z.sum(-1))


def test_softmax_wide_sums_to_one():
    x = np.random.default_rng(1).standard_normal((4, 806)).astype(np.float32)
    p = G.softmax(x)
    assert np.allclose(p.astype(np.float64).sum(-1), 1.0, atol=1e-5)


def test_dog_encode_invariants():
    for name in ("selfplay_4p_teams", "exotic_4p"):
        kw = RULE_SETS[name]
        rng = np.random.default_rng(5)
        envs = [random_state(rng, kw, 1, g) for g in range(40)] + [reset(kw, 1, 40 + g) for g in range(8)]
        for e in envs:
            o = DM.encode_board(e)
            assert o.shape == (34, 56) and o.dtype == np.int32
            cp = e.current_player
            rolled = [(cp + r) % 4 for r in range(4)]
            # every pin on the board appears once in the player channels; home counts complete the 16 pins
            on_board = int(o[0:4].sum())
            assert on_board == int((np.asarray(e.pins) >= 0).sum())
            assert on_board + int(o[6:10, 0].sum()) == 16
            # global features are constant over the cells
            assert (o[6:] == o[6:, :1]).all()
            sub = dg.sub_player(e)
            assert np.array_equal(o[10:24, 0], np.asarray(e.hands[sub], np.int32))
            assert np.array_equal(o[24:28, 0], [int(np.asarray(e.hands[p], np.int32).sum()) for p in rolled])
            assert o[28, 0] == e.phase and o[29, 0] == e.hand_size and o[30, 0] == int(sub != cp)
            # team / opponent channels are the sums of the player channels
            if e.rules["enable_teams"]:
                assert np.array_equal(o[4], o[0] + o[2]) and np.array_equal(o[5], o[1] + o[3])
            # the current player's own pins: rolled by -10 * cp on the track
            for k in range(4):
                pos = int(e.pins[cp][k])
                if 0 <= pos < 40:
                    assert o[0, (pos - 10 * cp) % 40] == 1


def test_dog_repr_layernorm_head():
    p = DM.init_params(seed=2, randomize_affine=True)
    assert "representation/LayerNorm_7/scale" in p and p["prediction/Dense_2/kernel"].shape == (128, 806)
    assert p["dynamics/Dense_0/kernel"].shape == (806, 64) and p["representation/Dense_1/kernel"].shape == (28, 64)
    obs = np.stack([DM.encode_board(reset(RULE_SETS["selfplay_4p_teams"], 0, g)) for g in range(3)]).astype(np.float32)
    emb = ON.representation(p, obs)
    # LayerNorm head: each row is the LN of the last Dense, i.e. (x - mean) * rstd * scale + bias
    sub = ON.sub(p, "representation")
    x = emb - sub["LayerNorm_7/bias"]
    y = x / sub["LayerNorm_7/scale"]
    assert np.allclose(y.mean(-1), 0.0, atol=1e-4) and np.allclose(y.std(-1), 1.0, atol=1e-3)
    lg, v, e = DM.root_inference(p, obs)
    assert lg.shape == (3, 806) and v.shape == (3,) and np.array_equal(e, emb)
    r, d, lg2, v2, n2 = DM.recurrent_inference(p, np.array([0, 805, -1]), e)
    assert lg2.shape == (3, 806) and n2.shape == (3, 256) and (np.abs(r) <= 1).all() and (np.abs(d) <= 1).all()


def test_oracle_random_starting_player():
    """env_reset's random seat (starting_player out of range) in the three oracles: deterministic per seed / key,
    every seat reachable, the rest of the reset unchanged; without a seed / key it is refused."""
    import pytest
    from oracle import classic_madn as cm
    from oracle import detmadn as dm
    seats = [dm.start_seat(s, 4) for s in range(2000)]
    assert all(0 <= x < 4 for x in seats) and min(seats.count(k) for k in range(4)) > 400
    assert dm.start_seat(12345, 3) == dm.start_seat(12345, 3)
    e = dm.env_reset(num_players=4, starting_player=-1, seed=77, **dm.SELFPLAY_RULES)
    f = dm.env_reset(num_players=4, starting_player=dm.start_seat(77, 4), **dm.SELFPLAY_RULES)
    assert e.current_player == f.current_player and np.array_equal(e.pins, f.pins)
    assert cm.env_reset(num_players=2, starting_player=5, seed=3).current_player == dm.start_seat(3, 2)
    with pytest.raises(ValueError):
        dm.env_reset(num_players=2, starting_player=-1)
    kw = dict(RULE_SETS["selfplay_4p_teams"])
    kw.pop("num_players")
    d = dg.env_reset(4, starting_player=-1, start_key=dg.engine_start_key(5, 1), **kw)
    assert d.current_player == d.round_starter == dm.start_seat(dg.engine_start_key(5, 1), 4)
