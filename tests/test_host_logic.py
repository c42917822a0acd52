"""Host-side logic that needs no GPU: MFMA weight packing, ctypes <-> C struct layouts, search tables."""
import ctypes
import os
import subprocess
import tempfile

import numpy as np

from oracle import mctx_gumbel as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pack_dense_layout():
    """The packed B-fragment layout addresses W[k][n] exactly as csrc/nn.hpp:mfma_rows16 reads it."""
    from exploring_muzero_on_dog_amd import nets as N
    K, Nn, nw, nt = 48, 100, 4, 2
    W = np.arange(K * Nn, dtype=np.float32).reshape(K, Nn)
    p = N.pack_dense(W, nw, nt).reshape(nw, K // 16, 64, nt, 4)
    for w in range(nw):
        for kb in range(K // 16):
            for lane in range(64):
                for t in range(nt):
                    for j in range(4):
                        k = kb * 16 + 4 * (lane >> 4) + j
                        n = (w * nt + t) * 16 + (lane & 15)
                        assert p[w, kb, lane, t, j] == (W[k, n] if n < Nn else 0.0)


def test_param_shapes_match_oracle_and_reference_counts():
    """Parameter tree = Flax auto-names; totals match SURVEY App. C (1,896,352 / 535,366 / 409,753 at C=34)."""
    from exploring_muzero_on_dog_amd import nets as N
    from oracle import nets as ON
    for C in (18, 34):
        assert N.param_shapes(C) == ON.param_shapes(C)
    tot = {}
    for k, v in N.param_shapes(34).items():
        tot[k.split("/")[0]] = tot.get(k.split("/")[0], 0) + int(np.prod(v))
    assert tot == {"representation": 1896352, "dynamics": 535366, "prediction": 409753}


def test_ctypes_struct_layout_matches_header():
    from exploring_muzero_on_dog_amd import lib as L
    structs = {"muz_rules": L.MuzRules, "muz_detmadn_soa": L.MuzDetSoA, "muz_net_w": L.MuzNetW,
               "muz_repr_w": L.MuzReprW, "muz_dyn_w": L.MuzDynW, "muz_pred_w": L.MuzPredW,
               "muz_search_cfg": L.MuzSearchCfg, "muz_classic_soa": L.MuzClassicSoA, "muz_traj": L.MuzTraj,
               "muz_sp_stats": L.MuzSpStats, "muz_ring": L.MuzRing, "muz_sample": L.MuzSample,
               "muz_sdyn_w": L.MuzSdynW, "muz_classic_net_w": L.MuzClassicNetW, "muz_stoch_cfg": L.MuzStochCfg,
               "muz_traj_chance": L.MuzTrajChance, "muz_dog_soa": L.MuzDogSoA,
               "muz_ttt_state": L.MuzTttState, "muz_ttt_policy_out": L.MuzTttPolicyOut}
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"muz.h\"\nint main(){\n"
    for cname in structs:
        src += f'printf("{cname} %zu\\n", sizeof({cname}));\n'
    src += 'printf("dyn_off %zu\\n", offsetof(muz_net_w, dyn));\n'
    src += 'printf("pred_off %zu\\n", offsetof(muz_net_w, pred));\n'
    src += 'printf("seed_off %zu\\n", offsetof(muz_search_cfg, seed));\nreturn 0;}\n'
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        out = dict(line.split() for line in subprocess.run([exe], capture_output=True, text=True).stdout.split("\n")
                   if line)
    for cname, cls in structs.items():
        assert int(out[cname]) == ctypes.sizeof(cls), cname
    assert int(out["dyn_off"]) == L.MuzNetW.dyn.offset
    assert int(out["pred_off"]) == L.MuzNetW.pred.offset
    assert int(out["seed_off"]) == L.MuzSearchCfg.seed.offset


def considered_visit_closed_form(m, S, idx):
    """Python twin of csrc/search.hip:considered_visit (table-free seq-halving lookup)."""
    if m <= 1:
        return idx
    log2max = 0
    while (1 << log2max) < m:
        log2max += 1
    k, v, n = m, 0, 0
    while n < S:
        extra = max(1, S // (log2max * k))
        for _ in range(extra):
            if idx < n + k:
                return v
            n += k
            v += 1
        k = max(2, k // 2)
    return v


def test_table_free_considered_visits_equal_mctx_table():
    for S in (1, 2, 8, 25, 50, 100):
        table = G.get_table_of_considered_visits(16, S)
        for m in range(17):
            for i in range(S):
                assert considered_visit_closed_form(m, S, i) == table[m, i], (S, m, i)


def test_classic_param_shapes_match_oracle():
    from exploring_muzero_on_dog_amd import stochastic as ST
    from oracle import classic_nets as CN
    for C in (7, 11):
        assert ST.classic_param_shapes(C) == CN.param_shapes(C)
    a, b = ST.init_classic_params(11, seed=3), CN.init_params(11, seed=3)
    assert list(a) == list(b) and all(np.array_equal(a[k], b[k]) for k in a)


def test_eval_z_test():
    """compare_agents_statistically's two-proportion z-test (evaluate_agent.py:680-693)."""
    import math
    from exploring_muzero_on_dog_amd import evaluate as EV
    r = EV.z_test(600, 500, 1000)
    se = math.sqrt(0.6 * 0.4 / 1000 + 0.5 * 0.5 / 1000)
    assert abs(r["z"] - 0.1 / se) < 1e-12 and r["significant"] and 0 < r["p"] < 1e-5
    assert EV.z_test(0, 0, 100) == {"winrate1": 0.0, "winrate2": 0.0, "z": 0.0, "p": 1.0, "significant": False}
