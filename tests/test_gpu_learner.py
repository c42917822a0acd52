"""Learner on the GPU, wired to the device ring and the self-play engine (config (e) loop, small)."""
import ctypes
import numpy as np
import pytest
import torch

from oracle import nets as ON

pytestmark = pytest.mark.gpu


def _mods():
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import learner as L
    from exploring_muzero_on_dog_amd import nets as N
    from exploring_muzero_on_dog_amd import replay as R
    return E, GA, L, N, R


def test_learner_loop_and_weight_push(cuda):
    E, GA, L, N, R = _mods()
    P = 2
    C = E.num_channels(P)
    params = ON.init_params(C, seed=8)
    net = N.DeviceNet(params, C)
    eng = GA.SelfPlayEngine(net, 32, num_players=P, max_steps=60, num_simulations=4, max_depth=4)
    ring = R.VectorizedReplayBuffer(256, 16, 5, 10, obs_shape=(C, 56), max_episode_length=60,
                                    rng=np.random.RandomState(0))
    learner = L.Learner(params, C, unroll_steps=5)
    hist = L.train_loop(learner, eng, ring, iterations=2, train_steps=3, games_per_iteration=48, warmup_calls=1)
    assert len(hist) == 2 and all(np.isfinite(h["total_loss"]) for h in hist)
    # the engine now runs the learner's weights: its root inference equals the torch forward
    obs = torch.from_numpy(np.random.default_rng(1).integers(0, 3, (40, C, 56)).astype(np.float32)).cuda()
    lg, v, e = N.root_inference_fn(eng.net, obs)
    with torch.no_grad():
        te = learner.nets.representation(obs)
        tl, tv = learner.nets.prediction(te)
    assert (e - te).abs().max().item() < 2e-5
    assert (lg - tl).abs().max().item() < 2e-5 and (v - tv[:, 0]).abs().max().item() < 2e-5
    # and keeps playing
    buf = eng.play_stream(40, seed=3)
    assert int(buf["idx"].min()) > 0


def test_learner_overfits_one_batch(cuda):
    E, GA, L, N, R = _mods()
    C = E.num_channels(2)
    params = ON.init_params(C, seed=9)
    net = N.DeviceNet(params, C)
    eng = GA.SelfPlayEngine(net, 32, num_players=2, max_steps=80, num_simulations=4, max_depth=4)
    ring = R.VectorizedReplayBuffer(64, 32, 5, 10, obs_shape=(C, 56), max_episode_length=80,
                                    rng=np.random.RandomState(2))
    ring.save_games_from_buffers(eng.play(seed=1))
    batch = ring.sample_batch()
    learner = L.Learner(params, C, unroll_steps=5)
    first = float(learner.train_step(batch)["total_loss"])
    for _ in range(60):
        last = float(learner.train_step(batch)["total_loss"])
    assert last < 0.8 * first, (first, last)     # measured 4.07 -> 2.91 after 40 steps


def test_graph_captured_step_equals_eager(cuda):
    """Learner(graph=True) replays forward + backward + optimizer as one HIP graph; the parameters after a
    few steps match the eager steps on the same batches."""
    E, GA, L, N, R = _mods()
    C = E.num_channels(2)
    params = ON.init_params(C, seed=10)
    net = N.DeviceNet(params, C)
    eng = GA.SelfPlayEngine(net, 32, num_players=2, max_steps=80, num_simulations=4, max_depth=4)
    ring = R.VectorizedReplayBuffer(64, 32, 5, 10, obs_shape=(C, 56), max_episode_length=80,
                                    rng=np.random.RandomState(3))
    ring.save_games_from_buffers(eng.play(seed=2))
    batches = [ring.sample_batch() for _ in range(4)]
    eager = L.Learner(params, C, unroll_steps=5)
    graph = L.Learner(params, C, unroll_steps=5, graph=True)
    for i, b in enumerate(batches):
        le = eager.train_step(b)
        lg = graph.train_step(b)
        assert torch.equal(le["total_loss"], lg["total_loss"]), i
    # The losses are bit-identical at every step.  Round 1's drift (1.7e-5 relative in the loss) was MIOpen's
    # conv1d, whose algorithms accumulate with atomics (two EAGER runs differed; profiles/learner_determinism.py);
    # the convolutions now run as im2col GEMMs.  What remains: from the third step on, the captured and eager
    # weight-gradient GEMMs of the convolutions (reduction length 128 x 56 = 7168) round differently in the
    # last bits (Adam's first moment differs there), measured <= 2.3e-7 on the parameters after 4 steps.
    worst = max((eager.nets.p[k] - graph.nets.p[k]).abs().max().item() for k in eager.nets.p)
    print("max |parameter difference| after 4 steps:", worst)
    assert worst <= 1e-6, worst


def test_stochastic_learner_on_classic_ring(cuda):
    """train_stochastic.py's learner on batches of the stochastic device ring (graph-captured), weights
    pushed into the classic self-play arena: its root inference equals the torch forward."""
    from oracle import classic_nets as CN
    from exploring_muzero_on_dog_amd import classic as CL
    from exploring_muzero_on_dog_amd import game_agent_stochastic as GS
    from exploring_muzero_on_dog_amd import learner as L
    from exploring_muzero_on_dog_amd import replay as R
    from exploring_muzero_on_dog_amd import stochastic as S
    C = CL.num_channels(4)
    params = CN.init_params(C, seed=13)
    net = S.DeviceClassicNet(params, C)
    eng = GS.StochasticSelfPlayEngine(net, 32, max_steps=120, num_simulations=6, max_depth=5)
    ring = R.VectorizedReplayBufferStochastic(64, 32, 5, 10, obs_shape=(C, 56), max_episode_length=120,
                                              rng=np.random.RandomState(4))
    ring.save_games_from_buffers(eng.play(seed=3))
    batch = ring.sample_batch()
    lr = L.StochasticLearner(params, C, unroll_steps=5, graph=True)
    first = float(lr.train_step(batch)["total_loss"])
    for _ in range(40):
        last = float(lr.train_step(batch)["total_loss"])
    assert np.isfinite(last) and last < first, (first, last)
    lr.push_to(net)
    obs = torch.from_numpy(np.random.default_rng(2).integers(0, 3, (24, C, 56)).astype(np.float32)).cuda()
    lg, v, e = S.root_inference_fn(net, obs)
    with torch.no_grad():
        te = lr.nets.representation(obs)
        tl, tv = lr.nets.prediction(te)
    assert (e - te).abs().max().item() < 2e-5 and (lg - tl).abs().max().item() < 2e-5
    assert (v - tv[:, 0]).abs().max().item() < 2e-5
    buf = eng.play_stream(20, seed=4)
    assert int(buf["idx"].min()) > 0


def test_config_e_iteration_at_its_shape(cuda):
    """Config (e) at train_with_reward.py:311-352's shape on one GPU: 4 players in teams, 1500 games at S=100 /
    D=50 / max_len 550 streamed into a 20000 x 550 device ring, learner steps at batch 128 / unroll 10 /
    td 50 (graph-captured), weights pushed back: ring lengths equal the games' lengths, losses finite, and
    the pushed arena reproduces the torch forward within 1e-5 on the ring's own observations."""
    E, GA, L, N, R = _mods()
    P, GAMES, T, S, D = 4, 1500, 550, 100, 50
    C = E.num_channels(P)
    params = N.init_muzero_params(42, C)
    net = N.DeviceNet(params, C)
    eng = GA.SelfPlayEngine(net, GAMES, num_players=P, max_steps=T, num_simulations=S, max_depth=D)
    ring = R.VectorizedReplayBuffer(20000, 128, 10, 50, obs_shape=(C, 56), max_episode_length=T,
                                    rng=np.random.RandomState(0))
    learner = L.Learner(params, C, unroll_steps=10, graph=True)
    buf = eng.play_stream(GAMES, seed=1, temperature=1.0)
    idx = buf["idx"].clone()
    ring.save_games_from_buffers(buf)
    assert ring.size == GAMES
    assert torch.equal(ring.episode_lengths[:GAMES], idx)
    assert int(idx.min()) > 0 and int(idx.max()) <= T
    losses = [learner.train_step(ring.sample_batch()) for _ in range(6)]
    assert all(np.isfinite(float(x["total_loss"])) for x in losses)
    learner.push_to(net)
    obs = ring.observations[:64, 7].float()                      # real game observations from the ring
    lg, v, e = N.root_inference_fn(net, obs)
    act = ring.actions[:64, 7].clamp(min=0)
    r, d, rl, rv, ne = N.recurrent_inference_fn(net, act, e)
    with torch.no_grad():
        te = learner.nets.representation(obs)
        tl, tv = learner.nets.prediction(te)
        tn, trl, tdl = learner.nets.dynamics(te, act.long())
        tpl, tpv = learner.nets.prediction(tn)
    err = max((e - te).abs().max().item(), (lg - tl).abs().max().item(), (v - tv[:, 0]).abs().max().item(),
              (ne - tn).abs().max().item(), (rl - tpl).abs().max().item(), (rv - tpv[:, 0]).abs().max().item())
    from tests._parity import log
    log(f"config (e) shape: {GAMES} games 4p S={S} D={D}, {int(idx.sum())} env-steps into the 20000 x {T} ring, "
        f"6 learner steps at batch 128 / unroll 10 (losses {[round(float(x['total_loss']), 4) for x in losses]}), "
        f"pushed arena vs torch forward max |d| {err:.2e}")
    assert err <= 1e-5, err


@pytest.mark.parametrize("N,mode", [(32, 1), (64, 1), (128, 0), (256, 1), (256, 2)])
def test_fused_dense_layernorm_matches_float64_autograd(cuda, N, mode):
    """csrc/learner_ln.hip (bias + Flax LayerNorm + ReLU / residual ReLU, forward and backward) against float64
    autograd of the same expression; M = 300 rows (a partial backward block) and K = 96."""
    _, _, L, _, _ = _mods()
    g = torch.Generator().manual_seed(10 * N + mode)
    M, K = 300, 96
    x = torch.randn(M, K, generator=g, dtype=torch.float64)
    W = torch.randn(K, N, generator=g, dtype=torch.float64) * 0.2
    b, gam, bet = (torch.randn(N, generator=g, dtype=torch.float64) * s for s in (0.3, 1.0, 0.3))
    res = torch.randn(M, N, generator=g, dtype=torch.float64) if mode == 2 else None
    dout = torch.randn(M, N, generator=g, dtype=torch.float64)

    def ref(x, W, b, gam, bet, res):
        z = x @ W + b
        mean = z.mean(-1, keepdim=True)
        var = (z * z).mean(-1, keepdim=True) - mean * mean          # Flax's fast variance
        y = (z - mean) / torch.sqrt(var + 1e-6) * gam + bet
        return y if mode == 0 else (torch.relu(y) if mode == 1 else torch.relu(res + y))

    leaves = [t.clone().requires_grad_(True) for t in (x, W, b, gam, bet)] + ([res.clone().requires_grad_(True)]
                                                                               if res is not None else [])
    out_ref = ref(*leaves[:5], leaves[5] if res is not None else None)
    grads_ref = torch.autograd.grad(out_ref, leaves, dout)
    dev = [t.detach().float().cuda().requires_grad_(True) for t in leaves]
    out = L._DenseLN.apply(dev[0], dev[1], dev[2], dev[3], dev[4], dev[5] if res is not None else None, mode)
    grads = torch.autograd.grad(out, dev, dout.float().cuda())
    torch.cuda.synchronize()

    def close(a, r, what):
        a, r = a.detach().double().cpu(), r.detach()
        err = (a - r).abs().max().item() / max(1.0, r.abs().max().item())
        assert err < 2e-5, f"{what}: relative error {err:.2e}"
    close(out, out_ref, "out")
    for name, gg, gr in zip(("dx", "dW", "dbias", "dgamma", "dbeta", "dres"), grads, grads_ref):
        close(gg, gr, name)


def test_ln_film_kernels_match_float64_autograd(cuda):
    """muz_ln_film_fwd / muz_ln_film_bwd_rows (a dynamics trunk's LayerNorm_0 + FiLM in one launch each way,
    muzero_deterministic_madn.py:421-427) against float64 autograd of LN(x) * (1 + scale) + shift; M = 301 rows
    (a partial backward block)."""
    _, _, L, _, _ = _mods()
    g = torch.Generator().manual_seed(21)
    M, N = 301, 256
    x, scale, shift, dfilm = (torch.randn(M, N, generator=g, dtype=torch.float64) * s for s in (1.0, 0.3, 0.3, 1.0))
    gam, bet = (torch.randn(N, generator=g, dtype=torch.float64) * s for s in (1.0, 0.3))
    leaves = [t.clone().requires_grad_(True) for t in (x, scale, shift, gam, bet)]
    xl, sl, hl, gl, bl = leaves
    mean = xl.mean(-1, keepdim=True)
    var = (xl * xl).mean(-1, keepdim=True) - mean * mean
    y = (xl - mean) / torch.sqrt(var + 1e-6) * gl + bl
    ref = y * (1.0 + sl) + hl
    grads_ref = torch.autograd.grad(ref, leaves, dfilm)
    d = {k: v.float().cuda() for k, v in dict(x=x, s1=1.0 + scale, sh=shift, gam=gam, bet=bet, df=dfilm).items()}
    film = torch.empty(M, N, device="cuda")
    fwd = L._ln_film_fwd(d["x"], d["gam"], d["bet"], d["s1"], d["sh"], film)
    scratch = torch.empty((L._L.load().muz_ln_bwd_scratch_floats(M, N),), device="cuda")
    dscale = torch.empty(M, N, device="cuda")
    dz = L._ln_film_bwd_rows(d["df"], fwd, d["gam"], d["s1"], scratch, dscale)
    dgam, dbet, _ = L._ln_colsum(scratch, N)
    torch.cuda.synchronize()

    def close(a, r, what):
        a = a.detach().double().cpu()
        err = (a - r).abs().max().item() / max(1.0, r.abs().max().item())
        assert err < 2e-5, f"{what}: relative error {err:.2e}"
    close(film, ref.detach(), "film")
    close(fwd[0], y.detach(), "LayerNorm output")
    # bit-identical to the unfused form (LayerNorm kernel + torch.addcmul, the per-step graph's rounding): the
    # min-max extremum columns downstream depend on the last ulp
    ref_fwd = L._ln_fwd(d["x"], torch.zeros_like(d["gam"]), d["gam"], d["bet"], None, L.LN_PLAIN)
    assert all(torch.equal(a, b) for a, b in zip(fwd, ref_fwd))
    assert torch.equal(film, torch.addcmul(d["sh"], ref_fwd[0], d["s1"]))
    for name, a, r in (("dx", dz, grads_ref[0]), ("dscale", dscale, grads_ref[1]), ("dgamma", dgam, grads_ref[3]),
                       ("dbeta", dbet, grads_ref[4])):
        close(a, r, name)


def test_dense_minmax_node_matches_torch_form(cuda):
    """learner._DenseMinmax (RepresentationNetwork2's last Dense + min-max scaling: library GEMM, then bias + min-max
    in one launch each way) against the torch form (x @ W + b, amin / amax): forward bit-identical, gradients of x,
    W and b within 1e-5 relative; a row with tied extrema checks the even split."""
    _, _, L, _, _ = _mods()
    g = torch.Generator().manual_seed(31)
    M = 130
    x = torch.randn(M, 256, generator=g).cuda()
    W = (0.1 * torch.randn(256, 256, generator=g)).cuda()
    b = (0.1 * torch.randn(256, generator=g)).cuda()
    x[3] = 0.0                                   # row 3: q = b, whose extrema we tie below
    b[7] = b[9] = b.max() + 1.0
    dout = torch.randn(M, 256, generator=g).cuda()
    leaves = [t.clone().requires_grad_(True) for t in (x, W, b)]
    out = L._DenseMinmax.apply(*leaves)
    g1 = torch.autograd.grad(out, leaves, dout)
    ref_leaves = [t.clone().requires_grad_(True) for t in (x, W, b)]
    q = (ref_leaves[0] @ ref_leaves[1]).add(ref_leaves[2])
    lo, hi = torch.amin(q, -1, keepdim=True), torch.amax(q, -1, keepdim=True)
    ref = (q - lo) / (hi - lo + 1e-8)
    g2 = torch.autograd.grad(ref, ref_leaves, dout)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    for n, a, r in zip(("dx", "dW", "db"), g1, g2):
        err = (a - r).abs().max().item() / max(1e-3, r.abs().max().item())
        assert err < 1e-5, f"{n}: relative difference {err:.2e}"


@pytest.mark.parametrize("kind", ["det", "classic"])
def test_chain_boundary_launches_bit_identical(cuda, kind):
    """learner.FUSED_BOUNDARY (the min-max of application i and the LayerNorm_0 + FiLM of i + 1 as one launch each
    way: muz_minmax_film_fwd / muz_film_minmax_bwd) leaves the chain node's outputs and every gradient bit-identical
    to the separate launches; det (one weight group, heads twin) and classic (act / chance groups alternating)."""
    _, _, L, _, _ = _mods()
    g = torch.Generator().manual_seed(41)
    B, K = 96, 4
    if kind == "det":
        nets = L.MuZeroNets(ON.init_params(18, seed=4, randomize_affine=True), 18, 24, "cuda")
        names, apps, scaled, heads, T = list(L.DYN_TRUNK_PARAMS), (0,) * K, (True,) * K, True, K
    else:
        from exploring_muzero_on_dog_amd import stochastic as ST
        nets = L.ClassicMuZeroNets(ST.init_classic_params(20, seed=6), 20, "cuda")
        names = [n for k in ("act", "chance") for n in L.trunk_param_names(k)]
        apps, scaled, heads, T = (0, 1) * K, (False, True) * K, False, 2 * K
    lat0 = torch.rand(B, 256, generator=g).cuda().requires_grad_(True)
    scale = (0.3 * torch.randn(T, B, 256, generator=g)).cuda().requires_grad_(True)
    shift = (0.3 * torch.randn(T, B, 256, generator=g)).cuda().requires_grad_(True)
    w, wh = (torch.randn(T, B, 256, generator=g).cuda() for _ in range(2))
    params = [nets.p[n] for n in names]
    inputs = [lat0, scale, shift] + params
    res = []
    for fused in (True, False):
        L.FUSED_BOUNDARY, L.CHAIN_KERNEL = fused, False     # (the per-layer path: the one with boundary launches)
        try:
            o = L._TrunkChain.apply(lat0, scale, shift, 0.5, apps, scaled, heads, *params)
            out, raw = o if heads else (o, None)
            loss = (out * w).sum() + out[-1].square().sum() + ((raw * wh).sum() if heads else 0.0)
            res.append((out.detach().clone(), torch.autograd.grad(loss, inputs)))
        finally:
            L.FUSED_BOUNDARY, L.CHAIN_KERNEL = True, True
    torch.cuda.synchronize()
    assert torch.equal(res[0][0], res[1][0])
    for n, a, b in zip(["latent0", "scale", "shift"] + names, res[0][1], res[1][1]):
        assert torch.equal(a, b), n


def _chain_layer_st(chain, X, apps, lat0, outs):
    """The per-layer backward's saved tuples (_TrunkChain.forward's `st`) rebuilt from the chain kernel's forward
    buffers: (out, z, mean, rstd) per LayerNorm, out = the next weight layer's stacked input."""
    _, _, L, _, _ = _mods()
    WT, ln0, z, stats, lat, scale1, shift = chain.keep
    slot, _ = L._slots(apps, 2)
    st = []
    for i, g in enumerate(apps):
        j = slot[i]
        xin = lat0 if i == 0 else outs[i - 1]
        f = [(X[(g, L._GEMM_LAYERS[k + 1])][j], z[i, k], stats[i, k + 1, 0], stats[i, k + 1, 1]) for k in range(6)]
        f0 = (ln0[i], xin, stats[i, 0, 0], stats[i, 0, 1])
        rbs = [(X[(g, "a0")][j], f[2], f[3]), (X[(g, "a1")][j], f[4], f[5])]
        st.append((f0, X[(g, "3")][j], f[0], f[1], rbs, X[(g, "5")][j]))
    return st


@pytest.mark.parametrize("kind,B,K", [("det", 128, 10), ("det", 40, 3), ("classic", 128, 10), ("classic", 17, 2)])
def test_chain_kernel_matches_layer_path(cuda, kind, B, K):
    """csrc/learner_chain.hip (muz_trunk_chain_fwd / _bwd: every application of the unrolled chain in one launch
    each way, 16 rows per workgroup) against the per-layer launch path of the same node (library GEMMs + the row
    kernels of learner_ln.hip).  Forward: outputs within 1e-5.  Backward: both backward forms fed the SAME saved
    forward values (the chain kernel's), every gradient within 1e-5 relative to its largest entry (the GEMMs sum in
    different orders).  Fed separately because gradients are discontinuous where a ReLU input or a min-max
    extremum sits within rounding of its kink: two forwards that differ in the last bits can legitimately send a
    row's gradient down different branches (measured: 1 row of 1280 at batch 128 x 10, profiles/chain_diag.py).
    The learner's shape (batch 128, 10 unroll steps; classic: 20 alternating applications) and ragged batches
    (rows past the last 16-row tile masked)."""
    import types
    _, _, L, _, _ = _mods()
    g = torch.Generator().manual_seed(43 + B)
    if kind == "det":
        nets = L.MuZeroNets(ON.init_params(18, seed=4, randomize_affine=True), 18, 24, "cuda")
        names, apps, scaled, heads, T = list(L.DYN_TRUNK_PARAMS), (0,) * K, (True,) * K, True, K
    else:
        from exploring_muzero_on_dog_amd import stochastic as ST
        nets = L.ClassicMuZeroNets(ST.init_classic_params(20, seed=6), 20, "cuda")
        names = [n for k in ("act", "chance") for n in L.trunk_param_names(k)]
        apps, scaled, heads, T = (0, 1) * K, (False, True) * K, False, 2 * K
    lat0 = torch.rand(B, 256, generator=g).cuda()
    scale = (0.3 * torch.randn(T, B, 256, generator=g)).cuda()
    shift = (0.3 * torch.randn(T, B, 256, generator=g)).cuda()
    G = torch.randn(T, B, 256, generator=g).cuda()
    H = torch.randn(T, B, 256, generator=g).cuda() if heads else None
    P = [nets.p[n].detach() for n in names]
    with torch.no_grad():
        L.CHAIN_KERNEL = False
        try:
            ref = L._TrunkChain.apply(lat0, scale, shift, 0.5, apps, scaled, heads, *P)
        finally:
            L.CHAIN_KERNEL = True
        ref = ref[0] if heads else ref
        slot, seen = L._slots(apps, len(P) // L._NP)
        X = {(gr, n): torch.empty((max(seen[gr], 1), B, 256), device="cuda")
             for gr in range(len(seen)) for n in L._GEMM_LAYERS}
        outs, qs = torch.empty(T, B, 256, device="cuda"), torch.empty(T, B, 256, device="cuda")
        lohi, idx = torch.empty(T, B, 2, device="cuda"), torch.empty(T, B, 2, dtype=torch.int32, device="cuda")
        scale1 = 1.0 + scale
        chain = L._chain_forward(lat0, scale1, shift, apps, slot, scaled, P, X, outs, qs, lohi, idx)
        st = _chain_layer_st(chain, X, apps, lat0, outs)
        common = dict(saved_tensors=(scale1, qs, lohi), P=P, grad_scale=0.5, apps=tuple(apps), X=X)
        g_layer = L._TrunkChain.backward(types.SimpleNamespace(chain=None, st=st, boundary=True, scaled=tuple(scaled),
                                                               **common), G, H)
        g_chain = L._TrunkChain.backward(types.SimpleNamespace(chain=chain, **common), G, H)
    torch.cuda.synchronize()
    err = (outs - ref).abs().max().item()
    assert err < 1e-5, f"forward differs by {err:.2e}"
    labels = ["latent0", "scale", "shift", None, None, None, None] + names
    for n, a, b in zip(labels, g_chain, g_layer):
        if n is None:
            continue
        err = (a - b).abs().max().item() / max(1e-3, b.abs().max().item())
        assert err < 1e-5, f"{n}: relative gradient difference {err:.2e}"


@pytest.mark.parametrize("nb,M", [(6, 128), (2, 1408), (2, 37)])
def test_rbstack_kernel_matches_layer_path(cuda, nb, M):
    """csrc/learner_chain.hip's ResBlock stack (muz_rbstack_fwd / _bwd: nb ResBlocks in one launch each way; the
    representation's six at batch 128, the prediction's two at 11 x 128 rows, a ragged batch) against the per-layer
    launches (_dense_ln_fwd / _dense_ln_bwd, library GEMMs).  Forward: output within 1e-5.  Backward: the per-layer
    backward fed the stack's saved forward values (ReLU masks must agree -- see test_chain_kernel_matches_layer_path),
    dx and every parameter gradient within 1e-5 relative to its largest entry."""
    import types
    _, _, L, _, _ = _mods()
    g = torch.Generator().manual_seed(7 + M)
    P = []
    for _ in range(nb):
        for _ in range(2):
            P += [torch.randn(256, 256, generator=g) / 16, 0.1 * torch.randn(256, generator=g),
                  1 + 0.2 * torch.randn(256, generator=g), 0.1 * torch.randn(256, generator=g)]
    P = [p.cuda() for p in P]
    x = torch.relu(torch.randn(M, 256, generator=g)).cuda()
    dout = torch.randn(M, 256, generator=g).cuda()
    with torch.no_grad():
        ref, fs = x, []
        for b in range(nb):
            Wa, ba, ga, bea, Wb, bb, gb, beb = P[8 * b:8 * b + 8]
            fa = L._dense_ln_fwd(ref, Wa, ba, ga, bea, None, L.LN_RELU)
            fb = L._dense_ln_fwd(fa[0], Wb, bb, gb, beb, ref, L.LN_RESID_RELU)
            fs.append((ref, fa, fb))
            ref = fb[0]
        class _Ctx(types.SimpleNamespace):    # what the forward / backward use of autograd's ctx
            def save_for_backward(self, *t):
                self.saved_tensors = t
        ctx = _Ctx()
        out = L._ResStack.forward(ctx, x, None, *P)
        X, (WP, _, z, stats) = ctx.X, ctx.keep
        torch.cuda.synchronize()
        err = (out - ref).abs().max().item()
        assert err < 1e-5, f"forward differs by {err:.2e}"
        # the per-layer backward on the stack's saved values
        f = [((X[l + 1] if l + 1 < 2 * nb else out), z[l], stats[l, 0], stats[l, 1]) for l in range(2 * nb)]
        d, want = dout, [None] * len(P)
        for b in range(nb - 1, -1, -1):
            Wa, ba, ga, bea, Wb, bb, gb, beb = P[8 * b:8 * b + 8]
            sb = torch.empty((L._ln_scratch_floats(M, 256, 256),), device="cuda")
            sa = torch.empty_like(sb)
            dzb, dres, t = L._dense_ln_bwd(d, f[2 * b + 1], gb, L.LN_RESID_RELU, Wb, sb)
            dza, _, d = L._dense_ln_bwd(t, f[2 * b], ga, L.LN_RELU, Wa, sa, acc=dres)
            for k, (dz, s, inp) in enumerate(((dza, sa, X[2 * b]), (dzb, sb, X[2 * b + 1]))):
                dg, dbe, dbias = L._ln_colsum(s, 256)
                want[8 * b + 4 * k:8 * b + 4 * k + 4] = [inp.t() @ dz, dbias, dg, dbe]
        got = L._ResStack.backward(ctx, dout)
        torch.cuda.synchronize()
    err = (got[0] - d).abs().max().item() / max(1e-3, d.abs().max().item())
    assert err < 1e-5, f"dx: relative difference {err:.2e}"
    for i, (a, b) in enumerate(zip(got[2:], want)):
        err = (a - b).abs().max().item() / max(1e-3, b.abs().max().item())
        assert err < 1e-5, f"parameter {i}: relative gradient difference {err:.2e}"


def test_chain_kernel_host_checks(cuda):
    """muz_trunk_chain_fwd / _bwd reject what the kernels do not implement (before any launch)."""
    from exploring_muzero_on_dog_amd import lib as _L
    lib = _L.load()
    a = _L.MuzChainArgs()
    assert lib.muz_trunk_chain_fwd(ctypes.byref(a), _L.stream_ptr()) == _L.MUZ_E_INVALID     # T = 0, nulls
    a.T, a.M, a.ngroups = _L.MUZ_CHAIN_MAX_T + 1, 16, 1
    assert lib.muz_trunk_chain_fwd(ctypes.byref(a), _L.stream_ptr()) == _L.MUZ_E_INVALID
    a.T, a.ngroups = 1, 3
    assert lib.muz_trunk_chain_bwd(ctypes.byref(a), _L.stream_ptr()) == _L.MUZ_E_INVALID
    src = (ctypes.c_void_p * 1)(None)
    assert lib.muz_trunk_chain_pack(src, 1, None, None, _L.stream_ptr()) == _L.MUZ_E_INVALID
    r = _L.MuzRbstackArgs()
    assert lib.muz_rbstack_fwd(ctypes.byref(r), _L.stream_ptr()) == _L.MUZ_E_INVALID          # nb = 0, nulls
    r.nb, r.M = _L.MUZ_RBSTACK_MAX + 1, 16
    assert lib.muz_rbstack_bwd(ctypes.byref(r), _L.stream_ptr()) == _L.MUZ_E_INVALID


def test_dynamics_chain_node_matches_per_step_autograd(cuda):
    """learner._TrunkChain (the K-step latent chain as one autograd node, batched weight gradients) against the
    per-step graph of the same layers (loss_fn's CPU-style loop run on the GPU): forward within 1e-5, gradients
    of every input and parameter within 1e-5 relative (summation orders differ).  Both outputs carry a
    gradient: the scaled latent (carried on, read by Pred4) and its unscaled twin (read by the reward /
    discount heads, train_with_reward.py:49-105)."""
    _, _, L, _, _ = _mods()
    C, B, K = 18, 64, 6
    nets = L.MuZeroNets(ON.init_params(C, seed=4, randomize_affine=True), C, 24, "cuda")
    g = torch.Generator().manual_seed(3)
    lat0 = torch.rand(B, 256, generator=g).cuda().requires_grad_(True)
    scale = (0.3 * torch.randn(K, B, 256, generator=g)).cuda().requires_grad_(True)
    shift = (0.3 * torch.randn(K, B, 256, generator=g)).cuda().requires_grad_(True)
    w = torch.randn(K, B, 256, generator=g).cuda()
    wh = torch.randn(K, B, 256, generator=g).cuda()
    params = [nets.p[n] for n in L.DYN_TRUNK_PARAMS]
    inputs = [lat0, scale, shift] + params

    # the node's per-layer form (library GEMMs, like the per-step graph): both forwards round alike, so no row's
    # gradient takes a different ReLU / min-max branch (the chain kernel: test_chain_kernel_matches_layer_path)
    L.CHAIN_KERNEL = False
    try:
        out, raw = L._TrunkChain.apply(lat0, scale, shift, 0.5, (0,) * K, (True,) * K, True, *params)
        g1 = torch.autograd.grad((out * w).sum() + out[-1].square().sum() + (raw * wh).sum(), inputs)
    finally:
        L.CHAIN_KERNEL = True
    lats, raws = [lat0], []
    for k in range(K):
        nxt = nets.dynamics_trunk(lats[-1], scale[k], shift[k])
        raws.append(nxt)
        lats.append((nxt * 0.5).detach() + nxt * 0.5)
    ref = torch.stack(lats[1:])
    g2 = torch.autograd.grad((ref * w).sum() + ref[-1].square().sum() + (torch.stack(raws) * wh).sum(), inputs)
    torch.cuda.synchronize()
    # (the per-step graph's first LayerNorm is torch's two-pass one, the node's the fused Flax fast-variance one)
    assert (out - ref).abs().max().item() < 1e-5, "forward differs"
    assert torch.equal(out, raw)
    names = ["latent0", "scale", "shift"] + list(L.DYN_TRUNK_PARAMS)
    for n, a, b in zip(names, g1, g2):
        err = (a - b).abs().max().item() / max(1e-3, b.abs().max().item())
        assert err < 1e-5, f"{n}: relative gradient difference {err:.2e}"


def test_minmax_kernel_splits_tied_gradients(cuda):
    """muz_minmax_fwd / _bwd on rows with tied extrema (quantised values): the extremum gradient is split over
    the tied columns (JAX's reduce_min / reduce_max rule), against float64 amin / amax autograd; with both the
    scaled carried gradient and the unscaled head term."""
    _, _, L, _, _ = _mods()
    from exploring_muzero_on_dog_amd import lib as _L
    g = torch.Generator().manual_seed(17)
    M, Nn = 37, 256
    x = torch.round(torch.randn(M, Nn, generator=g) * 2) / 4          # few distinct values: many ties
    y = torch.zeros(M, Nn)
    bias = torch.zeros(Nn)
    G, A, Bc, H = (torch.randn(M, Nn, generator=g) for _ in range(4))
    xd = x.double().requires_grad_(True)
    lo, hi = torch.amin(xd, -1, keepdim=True), torch.amax(xd, -1, keepdim=True)
    o = (xd - lo) / (hi - lo + 1e-8)
    (want,) = torch.autograd.grad(o, xd, ((G + (A + Bc)) * 0.5 + H).double())
    dev = [t.cuda().contiguous() for t in (x, y, bias, G, A, Bc, H)]
    out, q = torch.empty(M, Nn, device="cuda"), torch.empty(M, Nn, device="cuda")
    lohi = torch.empty(M, 2, device="cuda")
    idx = torch.empty(M, 2, dtype=torch.int32, device="cuda")
    dq = torch.empty(M, Nn, device="cuda")
    lib = _L.load()
    _L.check(lib.muz_minmax_fwd(_L.ptr(dev[0]), _L.ptr(dev[1]), _L.ptr(dev[2]), M, Nn, _L.ptr(out), _L.ptr(q),
                                _L.ptr(lohi), _L.ptr(idx), _L.stream_ptr()), "fwd")
    _L.check(lib.muz_minmax_bwd(_L.ptr(dev[3]), _L.ptr(dev[4]), _L.ptr(dev[5]), _L.ptr(dev[6]), 0.5, 1, _L.ptr(q),
                                _L.ptr(lohi), M, Nn, _L.ptr(dq), _L.stream_ptr()), "bwd")
    torch.cuda.synchronize()
    assert (out.double().cpu() - o.detach()).abs().max().item() < 1e-6
    err = (dq.double().cpu() - want).abs().max().item() / want.abs().max().item()
    assert err < 1e-6, err


def test_classic_chain_node_matches_per_step_autograd(cuda):
    """The classic afterstate / state chain (act and chance trunks alternating, only the new states'
    gradient scaled) as one _TrunkChain node against loss_fn_stochastic's per-step graph on the GPU."""
    _, _, L, _, _ = _mods()
    from exploring_muzero_on_dog_amd import stochastic as ST
    C, B, K = 20, 64, 5
    params = ST.init_classic_params(C, seed=6)
    rng = np.random.default_rng(8)
    params = {k: (v + 0.1 * rng.standard_normal(v.shape).astype(np.float32)) if not k.endswith("kernel") else v
              for k, v in params.items()}
    nets = L.ClassicMuZeroNets(params, C, "cuda")
    g = torch.Generator().manual_seed(5)
    lat0 = torch.rand(B, 256, generator=g).cuda().requires_grad_(True)
    ea = torch.relu(torch.randn(K * B, 64, generator=g)).cuda().requires_grad_(True)
    ec = torch.relu(torch.randn(K * B, 64, generator=g)).cuda().requires_grad_(True)
    w = torch.randn(2 * K, B, 256, generator=g).cuda()
    names = [n for kind in ("act", "chance") for n in L.trunk_param_names(kind)]
    names += [f"dynamics/{pre}_film_{x}/{y}" for pre in ("act", "chance") for x in ("scale", "shift")
              for y in ("kernel", "bias")]
    inputs = [lat0, ea, ec] + [nets.p[n] for n in names]

    film = [torch.stack([nets._dense(f"dynamics/{pre}_film_{x}", e).reshape(K, B, -1)
                         for pre, e in (("act", ea), ("chance", ec))], 1).reshape(2 * K, B, -1) for x in ("scale", "shift")]
    L.CHAIN_KERNEL = False     # (the node's per-layer form, see test_dynamics_chain_node_matches_per_step_autograd)
    try:
        out = L._TrunkChain.apply(lat0, film[0], film[1], 0.5, (0, 1) * K, (False, True) * K, False,
                                  *(nets.p[n] for n in names[:2 * L._NP]))
        g1 = torch.autograd.grad((out * w).sum() + out[-1].square().sum(), inputs, retain_graph=True)
    finally:
        L.CHAIN_KERNEL = True
    # the per-step graph reads the same FiLM rows (row-wise GEMMs over all steps at once, as loss_fn_stochastic
    # does): a library GEMM over one step's rows may round differently from the same rows inside K steps
    # (rocBLAS picks its kernel by shape), and this test is about the chain node, not the FiLM projections
    seq, lat = [], lat0
    for k in range(K):
        after = nets._film_trunk("act", 0, lat, None, film=(film[0][2 * k], film[1][2 * k]))
        nxt = nets._film_trunk("chance", 2, after, None, film=(film[0][2 * k + 1], film[1][2 * k + 1]))
        lat = (nxt * 0.5).detach() + nxt * 0.5
        seq += [after, lat]
    ref = torch.stack(seq)
    g2 = torch.autograd.grad((ref * w).sum() + ref[-1].square().sum(), inputs)
    torch.cuda.synchronize()
    assert (out - ref).abs().max().item() < 1e-5, "forward differs"
    for n, a, b in zip(["latent0", "act_embed", "chance_embed"] + names, g1, g2):
        err = (a - b).abs().max().item() / max(1e-3, b.abs().max().item())
        assert err < 1e-5, f"{n}: relative gradient difference {err:.2e}"


def test_chain_and_stack_kernels_survive_a_second_backward(cuda):
    """_TrunkChain (CHAIN_KERNEL) and _ResStack (RESBLOCK_STACK) hand raw device pointers to their backward
    kernels; a second backward through the same graph (retain_graph) must read live buffers and give the same
    gradients, and a backward after the graph was freed must raise instead of reading freed memory."""
    _, _, L, _, _ = _mods()
    from exploring_muzero_on_dog_amd import stochastic as ST
    C, B, K = 20, 48, 4
    params = ST.init_classic_params(C, seed=9)
    nets = L.ClassicMuZeroNets(params, C, "cuda")
    g = torch.Generator().manual_seed(3)
    lat0 = torch.rand(B, 256, generator=g).cuda().requires_grad_(True)
    film = [torch.randn(2 * K, B, 256, generator=g).cuda().mul_(0.1).requires_grad_(True) for _ in range(2)]
    names = [n for kind in ("act", "chance") for n in L.trunk_param_names(kind)]
    assert L.CHAIN_KERNEL and L.RESBLOCK_STACK
    out = L._TrunkChain.apply(lat0, film[0], film[1], 0.5, (0, 1) * K, (False, True) * K, False,
                              *(nets.p[n] for n in names))
    h = nets._rbs("prediction/ResBlock_", 2, out.reshape(-1, 256))
    w = torch.randn(h.shape, generator=g).cuda()
    loss = (h * w).sum()
    inputs = [lat0, film[0], film[1]] + [nets.p[n] for n in names]
    g1 = torch.autograd.grad(loss, inputs, retain_graph=True)
    torch.cuda.synchronize()
    junk = [torch.full((1 << 22,), float("nan"), device="cuda") for _ in range(8)]   # reuse any freed block
    g2 = torch.autograd.grad(loss, inputs)
    torch.cuda.synchronize()
    del junk
    for n, a, b in zip(["latent0", "scale", "shift"] + names, g1, g2):
        assert torch.equal(a, b), n
    with pytest.raises(RuntimeError):
        torch.autograd.grad(loss, inputs)


@pytest.mark.parametrize("max_tables", [8, 0])
def test_fused_adamw_matches_foreach_form(cuda, max_tables):
    """csrc/learner_opt.hip (global-norm clip + AdamW + lr schedule in two passes over all tensors) against the
    torch._foreach form of the same step (learner.AdamW on the CPU path, here run on the GPU): 45 tensors (two
    kernel-argument tables), sizes across the 4096-element chunk edges, an empty tensor and one without a
    gradient; clipped and unclipped steps across two lr boundaries.  max_tables 8: every step through
    muz_adamw_step_table (a fresh device table per gradient-pointer set); 0: muz_adamw_step (kernel arguments)."""
    _, _, L, _, _ = _mods()
    rng = np.random.default_rng(12)
    sizes = [1, 3, 4095, 4096, 4097, 9000, 0, 256 * 256] + list(rng.integers(1, 3000, 37))
    base = [rng.standard_normal(int(n)).astype(np.float32) for n in sizes]
    p1 = [torch.from_numpy(b).cuda().requires_grad_(True) for b in base]
    p2 = [torch.from_numpy(b).cuda().requires_grad_(True) for b in base]
    kw = dict(steps_per_iteration=1, boundaries=((2, 0.2), (4, 0.5)))
    fused, ref = L.AdamW(p1, **kw), L.AdamW(p2, **kw)
    assert fused._fused is not None
    fused._fused["max_tables"] = max_tables
    ref._fused = None
    for step in range(7):
        scale = 3.0 if step in (1, 4) else 0.01                 # global norm above / below max_norm 5
        for i, (a, b) in enumerate(zip(p1, p2)):
            if i == 5:
                a.grad = b.grad = None
                continue
            g = torch.from_numpy((rng.standard_normal(a.numel()) * scale).astype(np.float32)).cuda()
            a.grad, b.grad = g.clone(), g.clone()
        n1, n2 = fused.step(), ref.step()
        torch.cuda.synchronize()
        assert abs(float(n1) - float(n2)) <= 1e-6 * float(n2), (step, float(n1), float(n2))
        for name, xs, ys in (("param", p1, p2), ("mu", fused.mu, ref.mu), ("nu", fused.nu, ref.nu)):
            for i, (a, b) in enumerate(zip(xs, ys)):
                assert torch.allclose(a, b, rtol=2e-6, atol=1e-8), (step, name, i, (a - b).abs().max().item())
    assert float(fused.count) == float(ref.count) == 7.0
    assert len(fused._fused["tables"]) == min(7, max_tables)


def test_adamw_table_survives_later_steps_in_a_graph(cuda):
    """a captured step must keep updating with the gradients it was captured with, whatever eager steps
    with other gradient pointers ran in between (each pointer set has its own never-rewritten device table).
    Sequence eager(A), capture(A), eager(B), replay(A) against the foreach form run as A, B, A."""
    _, _, L, _, _ = _mods()
    g = torch.Generator().manual_seed(3)
    init = [torch.randn(5000, generator=g), torch.randn(300, generator=g)]
    ga = [torch.randn(5000, generator=g).cuda(), torch.randn(300, generator=g).cuda()]
    gb = [torch.randn(5000, generator=g).cuda() * 50, torch.randn(300, generator=g).cuda() * 50]
    ps = [x.clone().cuda().requires_grad_(True) for x in init]
    qs = [x.clone().cuda().requires_grad_(True) for x in init]
    opt = L.AdamW(ps, steps_per_iteration=1, boundaries=())
    ref = L.AdamW(qs, steps_per_iteration=1, boundaries=())
    ref._fused = None
    for p, x in zip(ps, ga):
        p.grad = x
    opt.step()                                    # eager: writes the table of pointer set A
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            opt.step()
    torch.cuda.current_stream().wait_stream(s)
    for p, x in zip(ps, gb):
        p.grad = x
    opt.step()                                    # eager, pointer set B: its own table
    graph.replay()
    torch.cuda.synchronize()
    for grads in (ga, gb, ga):
        for q, x in zip(qs, grads):
            q.grad = x.clone()
        ref.step()
    for a, b in zip(ps, qs):
        assert torch.allclose(a, b, rtol=2e-6, atol=1e-7), float((a - b).abs().max())
    assert len(opt._fused["tables"]) == 2


@pytest.mark.parametrize("K,Cin", [(3, 6), (3, 32), (5, 64)])
def test_im2col_matches_pad_and_cat(cuda, K, Cin):
    """learner._Im2col (one kernel each way) against the pad / slice / cat form of the same 'SAME' Conv1D
    im2col matrix (MuZeroNets._conv_cols on the CPU path): forward identical, backward within float rounding."""
    _, _, L, _, _ = _mods()
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(K * 100 + Cin)
    x = torch.randn(7, 56, Cin, generator=g).cuda().requires_grad_(True)
    dc = torch.randn(7, 56, K * Cin, generator=g).cuda()
    cols = L._Im2col.apply(x, K)
    (dx,) = torch.autograd.grad(cols, x, dc)
    pl = (K - 1) // 2
    xp = F.pad(x, (0, 0, pl, K - 1 - pl))
    ref = torch.cat([xp[:, d:d + 56, :] for d in range(K)], dim=-1)
    (dref,) = torch.autograd.grad(ref, x, dc)
    assert torch.equal(cols, ref)
    assert torch.allclose(dx, dref, rtol=1e-6, atol=1e-6)


def test_train_step_from_ring_equals_sampled_batches(cuda):
    """Learner.train_step_from(ring) (the ring writes each batch into the captured graph's inputs through the
    pinned index stage) gives the same losses and parameters as train_step(ring.sample_batch()) on an
    identically seeded ring."""
    E, GA, L, N, R = _mods()
    C = E.num_channels(2)
    params = ON.init_params(C, seed=11)
    net = N.DeviceNet(params, C)
    eng = GA.SelfPlayEngine(net, 32, num_players=2, max_steps=80, num_simulations=4, max_depth=4)
    buf = eng.play(seed=5)
    rings = [R.VectorizedReplayBuffer(64, 32, 5, 10, obs_shape=(C, 56), max_episode_length=80,
                                      rng=np.random.RandomState(7)) for _ in range(2)]
    for r in rings:
        r.save_games_from_buffers(buf)
    a = L.Learner(params, C, unroll_steps=5, graph=True)
    b = L.Learner(params, C, unroll_steps=5, graph=True)
    for i in range(5):
        la = a.train_step(rings[0].sample_batch())
        lb = b.train_step_from(rings[1])
        assert torch.equal(la["total_loss"], lb["total_loss"]), i
    for k in a.nets.p:
        assert torch.equal(a.nets.p[k], b.nets.p[k]), k
