"""Stochastic-MuZero oracle sanity on the CPU: shapes, legality, visit accounting, determinism."""
import numpy as np

from oracle import classic_madn as cm
from oracle import classic_nets as CN
from oracle import mctx_stochastic as MS


def test_oracle_stochastic_search_invariants():
    C = cm.num_channels(4)
    params = CN.init_params(C, seed=3, randomize_affine=True)
    rng = np.random.default_rng(0)
    envs = []
    for i in range(6):
        e = cm.env_reset(num_players=4, **cm.SELFPLAY_RULES)
        e = cm.throw_die(e, float(rng.random()))
        envs.append(e)
    obs = np.stack([cm.encode_board(e) for e in envs]).astype(np.float32)
    valid = np.stack([cm.valid_action(e) for e in envs])
    valid[~valid.any(1), 0] = True
    lg, v, emb = CN.root_inference(params, obs)
    dn = rng.dirichlet(np.full(4, 0.3), len(envs)).astype(np.float32)
    gm = rng.gumbel(size=(len(envs), 4)).astype(np.float32)
    S = 12
    a, w, rv, trees = MS.stochastic_muzero_policy(params, lg, v, emb, CN.decision_recurrent, CN.chance_recurrent, S,
                                                  ~valid, dn, gm, max_depth=6, temperature=1.0, seed=1, turn=2)
    a2, w2, rv2, _ = MS.stochastic_muzero_policy(params, lg, v, emb, CN.decision_recurrent, CN.chance_recurrent, S,
                                                 ~valid, dn, gm, max_depth=6, temperature=1.0, seed=1, turn=2)
    assert np.array_equal(a, a2) and np.array_equal(w, w2) and np.array_equal(rv, rv2)
    assert valid[np.arange(len(envs)), a].all()
    assert np.allclose(w.sum(1), 1.0)
    for t in trees:
        assert t.visits[0] == S + 1                       # root visited by every simulation
        assert t.c_visits[0, :4].sum() == S               # all root visits go to pin children
        assert t.is_dec[0]
        kids = t.c_index[0, :4]
        for k in kids[kids >= 0]:
            assert not t.is_dec[k]                        # pin children are chance nodes (afterstates)
    assert np.all(np.abs(rv) <= 1.0)
