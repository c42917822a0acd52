"""HIP env kernels vs the CPU oracle: golden vectors + seeded random-play transitions (GPU)."""
import numpy as np
import pytest
import torch

from oracle import detmadn as dm
from tests._detmadn_util import RULE_SETS, legal_bits_oracle, random_play_transitions
from tests.test_oracle_golden import DET_CASES

pytestmark = pytest.mark.gpu


def _E():
    from exploring_muzero_on_dog_amd import detmadn as E
    return E


def rules_of(env_or_kw):
    E = _E()
    r = env_or_kw.rules
    return E.make_rules(num_players=env_or_kw.num_players, starting_player=0,
                        **{k: v for k, v in r.items()})


def to_gpu(envs, rules):
    E = _E()
    return E.state_from_host(
        pins=np.stack([e.pins for e in envs]),
        current_player=np.array([e.current_player for e in envs]),
        rules=rules,
        action_set=np.stack([e.action_set for e in envs]),
        done=np.array([e.done for e in envs], np.uint8),
        reward=np.array([e.reward for e in envs], np.int8),
        board=np.stack([e.board for e in envs]))


def assert_same(gpu, envs, what):
    B = len(envs)
    P = envs[0].num_players
    torch.cuda.synchronize()
    pins = gpu.pins.cpu().numpy().T.reshape(B, P, 4)
    aset = gpu.action_set.cpu().numpy().T.reshape(B, P, 6)
    board = gpu.board.cpu().numpy().T
    cp = gpu.current_player.cpu().numpy()
    done = gpu.done.cpu().numpy()
    for b, e in enumerate(envs):
        ok = (np.array_equal(pins[b], e.pins) and np.array_equal(aset[b], e.action_set)
              and np.array_equal(board[b], e.board) and cp[b] == e.current_player and bool(done[b]) == e.done)
        assert ok, (what, b, pins[b].tolist(), e.pins.tolist(), aset[b].tolist(), e.action_set.tolist(),
                    int(cp[b]), e.current_player)


@pytest.mark.parametrize("case", DET_CASES, ids=[c["source"] for c in DET_CASES])
def test_golden_step_vectors(cuda, case):
    from tests.test_oracle_golden import det_env_from_case
    env = det_env_from_case(case)
    gpu = to_gpu([env], rules_of(env))
    E = _E()
    _, reward, done = E.env_step_pin_move(gpu, torch.tensor([case["pin"]]), torch.tensor([case["move"]]))
    torch.cuda.synchronize()
    pins = gpu.pins.cpu().numpy().T.reshape(2, 4)
    assert np.array_equal(pins, np.array(case["expected_valid"]))
    ref_env, ref_r, ref_d = dm.env_step(env, (case["pin"], case["move"]))
    assert int(reward.cpu()[0]) == ref_r


@pytest.mark.parametrize("rule_set,n_games,seed", [("selfplay_2p", 64, 1), ("selfplay_4p_teams", 24, 2),
                                                   ("exotic_4p", 24, 3), ("exotic_2p", 32, 4)])
def test_random_play_transitions(cuda, rule_set, n_games, seed):
    """Every transition of seeded random play (10% deliberately illegal actions) is checked:
    legal mask, encode_board, env_step / no_step, on states taken from the oracle."""
    E = _E()
    n_checked = 0
    for ply, batch in random_play_transitions(rule_set, n_games, seed):
        rules = rules_of(batch[0][1])
        envs = [e for _, e, _, _ in batch]
        gpu = to_gpu(envs, rules)
        bits = E.legal_bits(gpu).cpu().numpy()
        for b, e in enumerate(envs):
            assert int(bits[b]) & 0xFFFFFF == legal_bits_oracle(e), (rule_set, ply, b)
        obs = E.encode_board(gpu).cpu().numpy()
        obs_i8 = E.encode_board(gpu, torch.int8).cpu().numpy()
        for b, e in enumerate(envs):
            ref = dm.encode_board(e)
            assert np.array_equal(obs[b], ref), (rule_set, ply, b)
            assert np.array_equal(obs_i8[b], ref)
        steps = [(e, a) for _, e, k, a in batch if k == "step"]
        if steps:
            g = to_gpu([e for e, _ in steps], rules)
            _, rew, done = E.env_step(g, torch.tensor([a for _, a in steps], dtype=torch.int32))
            ref = [dm.env_step(e, dm.map_action(a)) for e, a in steps]
            assert_same(g, [r[0] for r in ref], f"{rule_set} step ply {ply}")
            assert rew.cpu().numpy().tolist() == [r[1] for r in ref]
            assert done.cpu().numpy().tolist() == [r[2] for r in ref]
        nos = [e for _, e, k, _ in batch if k == "nostep"]
        if nos:
            g = to_gpu(nos, rules)
            E.no_step(g)
            assert_same(g, [dm.no_step(e)[0] for e in nos], f"{rule_set} nostep ply {ply}")
        n_checked += len(batch)
    assert n_checked > 1000


def test_reset_matches_oracle(cuda):
    E = _E()
    for name, kw in RULE_SETS.items():
        gpu = E.env_reset(7, **kw)
        ref = dm.env_reset(**kw)
        assert_same(gpu, [ref] * 7, f"reset {name}")


def test_fused_next_legal(cuda):
    """muz_detmadn_step's fused next-state legal mask equals a separate valid_action launch."""
    E = _E()
    gpu = E.env_reset(4096, num_players=2, **dm.SELFPLAY_RULES)
    rng = np.random.default_rng(5)
    nl = torch.empty(4096, dtype=torch.int32, device="cuda")
    for _ in range(50):
        bits = E.legal_bits(gpu).cpu().numpy()
        act = np.array([rng.choice(np.flatnonzero([(b >> i) & 1 for i in range(24)])) if b else 0 for b in bits])
        E.env_step(gpu, torch.tensor(act, dtype=torch.int32), next_legal=nl)
        assert torch.equal(nl, E.legal_bits(gpu))
