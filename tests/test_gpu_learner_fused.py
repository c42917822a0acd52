"""The learner's fused launches: grouped parameter gradients (csrc/learner_grad.hip through
learner.GradSink), one-launch Dense + LayerNorm forward / backward (csrc/learner_fused.hip) and the fused
losses (csrc/learner_loss.hip).

* muz_wgrad_grouped: X^T dZ of many problems in one launch against float64 torch -- ragged rows (not a
  multiple of 16, zero rows), K / N not multiples of 32, row strides wider than the matrix, rows over one
  2048-row segment (partials in scratch), more problems than one kernel-argument table holds (48);
* muz_colsum_grouped: LayerNorm partials (kind 0) against muz_ln_colsum and float64, and row sums (kind 1)
  against float64;
* a whole det / classic learner backward with the sink against the same backward with every gradient formed
  by its own launch (GROUPED_GRADS = False): fp32 summation-order differences only (1e-5 relative);
* the fused loss kernel (csrc/learner_loss.hip: muz_loss_heads through learner._LossHeads) against the torch
  loss ops it replaces (FUSED_LOSS = False): every loss part and the gradients of the network outputs, det and
  classic, with ragged masks, a step without any rare row, all-zero masks and K = 0;
* muz_dense_ln_fwd / muz_dense_ln_bwd against float64 autograd of the same layer (Dense -> Flax LayerNorm ->
  ReLU / residual ReLU / plain), with the transposed weight copy (muz_transpose_grouped) bit-identical to the
  plain one, and against the unfused path (library GEMM + muz_ln_fwd / muz_ln_bwd_rows):
  ragged rows, K not a multiple of 4 / 16, every width N, the accumulate input, and no input gradient."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _L():
    from exploring_muzero_on_dog_amd import lib as L
    return L


def _wgrad(problems):
    L = _L()
    arr = (L.MuzWgradProblem * len(problems))(*[L.MuzWgradProblem(*p) for p in problems])
    need = L.load().muz_wgrad_scratch_floats(arr, len(problems))
    scratch = torch.full((max(need, 1),), float("nan"), device="cuda")
    L.check(L.load().muz_wgrad_grouped(arr, len(problems), L.ptr(scratch), scratch.numel(), L.stream_ptr()),
            "muz_wgrad_grouped")
    torch.cuda.synchronize()


def _colsum(problems):
    L = _L()
    arr = (L.MuzColsumProblem * len(problems))(*[L.MuzColsumProblem(*p) for p in problems])
    L.check(L.load().muz_colsum_grouped(arr, len(problems), L.stream_ptr()), "muz_colsum_grouped")


def test_wgrad_grouped_matches_float64(cuda):
    g = torch.Generator(device="cuda").manual_seed(3)
    shapes = [(128, 256, 256), (1408, 256, 256), (7, 33, 45), (0, 64, 32), (17, 1, 1), (300, 512, 24),
              (1280, 280, 256), (16, 32, 32), (1, 300, 7), (7168, 96, 64), (513, 20, 30), (1024, 64, 64)] + \
        [(50 + 37 * i, 40 + i, 20 + 2 * i) for i in range(40)]       # > 48 problems: two argument tables
    X, D, O, probs = [], [], [], []
    for M, K, N in shapes:
        x = torch.randn((M, K + 5), generator=g, device="cuda")[:, 2:2 + K]    # row stride K + 5
        d = torch.randn((M, N + 3), generator=g, device="cuda")[:, :N]
        o = torch.full((K, N), float("nan"), device="cuda")
        X.append(x), D.append(d), O.append(o)
        probs.append((x.data_ptr(), d.data_ptr(), o.data_ptr(), M, K, N, x.stride(0), d.stride(0)))
    _wgrad(probs)
    torch.cuda.synchronize()
    for (M, K, N), x, d, o in zip(shapes, X, D, O):
        ref = x.double().t() @ d.double()
        err = float((o.double() - ref).abs().max()) / max(float(ref.abs().max()), 1.0)
        assert err < 2e-6, ((M, K, N), err)


def test_colsum_grouped_matches_ln_colsum_and_float64(cuda):
    L = _L()
    lib = L.load()
    g = torch.Generator(device="cuda").manual_seed(4)
    probs, checks = [], []
    for M, N in ((128, 256), (1408, 256), (7168, 64), (3, 128), (1280, 128)):
        nf = lib.muz_ln_bwd_scratch_floats(M, N)
        scr = torch.randn((nf,), generator=g, device="cuda")
        outs = [torch.empty((N,), device="cuda") for _ in range(3)]
        ref = [torch.empty((N,), device="cuda") for _ in range(3)]
        L.check(lib.muz_ln_colsum(L.ptr(scr), nf // (3 * N), N, *(L.ptr(r) for r in ref), L.stream_ptr()), "colsum")
        probs.append((scr.data_ptr(), *(o.data_ptr() for o in outs), 0, nf // (3 * N), N, N))
        checks.append(("ln", scr, outs, ref))
    for M, N, ld in ((1408, 24, 24), (128, 256, 260), (0, 32, 32), (5, 1, 1), (7168, 300, 301)):
        src = torch.randn((max(M, 1), ld), generator=g, device="cuda")
        out = torch.full((N,), float("nan"), device="cuda")
        probs.append((src.data_ptr(), out.data_ptr(), 0, 0, 1, M, N, ld))
        checks.append(("rows", src[:M, :N], [out], None))
    _colsum(probs)
    torch.cuda.synchronize()
    for kind, src, outs, ref in checks:
        if kind == "ln":          # against muz_ln_colsum (a different fixed order) and float64
            M, N = src.numel() // 3, outs[0].numel()
            exp = src.double().reshape(-1, 3, N).sum(0)
            for q, (o, r) in enumerate(zip(outs, ref)):
                tol = 1e-5 * max(1.0, float(src.reshape(-1, 3, N)[:, q].abs().sum(0).max()))
                assert float((o.double() - exp[q]).abs().max()) < tol
                assert float((o - r).abs().max()) < tol
        else:
            exp = src.double().sum(0)
            assert float((outs[0].double() - exp).abs().max()) < 1e-4 * max(1.0, float(src.abs().sum(0).max()))


def test_host_rejects_bad_problems(cuda):
    L = _L()
    bad = L.MuzWgradProblem(0, 0, 0, 4, 4, 4, 4, 4)          # null pointers
    assert L.load().muz_wgrad_grouped(ctypes.byref(bad), 1, None, 0, L.stream_ptr()) != 0
    big = L.MuzWgradProblem(1, 1, 1, 5000, 4, 4, 4, 4)        # several segments: needs scratch, none given
    seg = L.load().muz_wgrad_segment_rows()
    assert seg % 64 == 0 and L.load().muz_wgrad_scratch_floats(ctypes.byref(big), 1) == -(-5000 // seg) * 16
    assert L.load().muz_wgrad_grouped(ctypes.byref(big), 1, None, 0, L.stream_ptr()) != 0
    bad = L.MuzColsumProblem(0, 0, 0, 0, 3, 4, 4, 4)         # unknown kind
    assert L.load().muz_colsum_grouped(ctypes.byref(bad), 1, L.stream_ptr()) != 0


def _grads(learner_cls, params, C, batch, grouped, **kw):
    from exploring_muzero_on_dog_amd import learner as L
    old = L.GROUPED_GRADS
    L.GROUPED_GRADS = grouped
    try:
        lr = learner_cls(params, C, unroll_steps=5, **kw)
    finally:
        L.GROUPED_GRADS = old
    assert (lr.sink is not None) == grouped
    out = lr.train_step(batch)
    torch.cuda.synchronize()
    return float(out["total_loss"]), {k: p.grad.detach().clone() for k, p in lr.nets.p.items()}


def _compare(name, a, b):
    (la, ga), (lb, gb) = a, b
    assert la == lb, (name, la, lb)              # the forward does not change
    assert set(ga) == set(gb)
    for k in ga:
        err = float((ga[k] - gb[k]).norm()) / max(float(gb[k].norm()), 1e-20)
        assert err < 1e-5, (name, k, err)


def test_det_sink_gradients_equal_per_op_gradients(cuda):
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import learner as L
    from exploring_muzero_on_dog_amd import nets as N
    from exploring_muzero_on_dog_amd import replay as R
    from oracle import nets as ON
    C = E.num_channels(4)
    params = ON.init_params(C, seed=12, randomize_affine=True)
    eng = GA.SelfPlayEngine(N.DeviceNet(params, C), 32, num_players=4, max_steps=120, num_simulations=4, max_depth=4)
    ring = R.VectorizedReplayBuffer(512, 48, 5, 10, obs_shape=(C, 56), max_episode_length=120,
                                    rng=np.random.RandomState(1))
    ring.save_games_from_buffers(eng.play_stream(40, seed=1, temperature=1.0))
    batch = ring.sample_batch()
    _compare("det", _grads(L.Learner, params, C, batch, True), _grads(L.Learner, params, C, batch, False))
    # graph-captured with the sink: the replayed step equals the eager one bit for bit
    _compare("det graph", _grads(L.Learner, params, C, batch, True, graph=True),
             _grads(L.Learner, params, C, batch, True))


def test_resblock_node_gradients_bit_identical(cuda):
    """learner.RESBLOCK_NODE (a ResBlock's two fused Dense + LayerNorm layers as one autograd node whose backward adds
    the residual gradient inside the second launch, dx = dz_0 W_0^T + dres) leaves the det step's loss and every
    parameter gradient bit-identical to two _DenseLN nodes and autograd's separate add (the same kernels, and fp32
    addition commutes); grouped (GradSink) and per-parameter gradients alike."""
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import learner as L
    from exploring_muzero_on_dog_amd import nets as N
    from exploring_muzero_on_dog_amd import replay as R
    from oracle import nets as ON
    C = E.num_channels(4)
    params = ON.init_params(C, seed=14, randomize_affine=True)
    eng = GA.SelfPlayEngine(N.DeviceNet(params, C), 32, num_players=4, max_steps=120, num_simulations=4, max_depth=4)
    ring = R.VectorizedReplayBuffer(512, 48, 5, 10, obs_shape=(C, 56), max_episode_length=120,
                                    rng=np.random.RandomState(3))
    ring.save_games_from_buffers(eng.play_stream(40, seed=3, temperature=1.0))
    batch = ring.sample_batch()
    for grouped in (True, False):
        res = []
        for node in (True, False):
            L.RESBLOCK_NODE, L.RESBLOCK_STACK = node, False    # (the stack kernel would take the ResBlocks)
            try:
                res.append(_grads(L.Learner, params, C, batch, grouped))
            finally:
                L.RESBLOCK_NODE, L.RESBLOCK_STACK = True, True
        (la, ga), (lb, gb) = res
        assert la == lb
        for k in ga:
            assert torch.equal(ga[k], gb[k]), (grouped, k)


def test_classic_sink_gradients_equal_per_op_gradients(cuda):
    from exploring_muzero_on_dog_amd import classic as CL
    from exploring_muzero_on_dog_amd import game_agent_stochastic as GS
    from exploring_muzero_on_dog_amd import learner as L
    from exploring_muzero_on_dog_amd import replay as R
    from exploring_muzero_on_dog_amd import stochastic as S
    from oracle import classic_nets as CN
    C = CL.num_channels(4)
    params = CN.init_params(C, seed=13, randomize_affine=True)
    eng = GS.StochasticSelfPlayEngine(S.DeviceClassicNet(params, C), 32, max_steps=200, num_simulations=4, max_depth=4)
    ring = R.VectorizedReplayBufferStochastic(512, 48, 5, 10, obs_shape=(C, 56), max_episode_length=200,
                                              rng=np.random.RandomState(2))
    ring.save_games_from_buffers(eng.play_stream(40, seed=2))
    batch = ring.sample_batch()
    _compare("classic", _grads(L.StochasticLearner, params, C, batch, True),
             _grads(L.StochasticLearner, params, C, batch, False))


def _loss_case(classic, K, B, seed, zero_mask=False):
    g = torch.Generator(device="cuda").manual_seed(seed)
    A = 4 if classic else 24
    T = K + 1
    b = {"masks": (torch.rand((B, T), generator=g, device="cuda") > 0.2).float(),
         "target_values": torch.rand((B, T), generator=g, device="cuda") * 2 - 1,
         "policies": torch.softmax(torch.randn((B, T, A), generator=g, device="cuda"), -1),
         "rewards": torch.randint(0, 3, (B, K), generator=g, device="cuda", dtype=torch.int32),
         "discount_targets": torch.randint(0, 2, (B, K), generator=g, device="cuda", dtype=torch.int32)}
    if K:
        b["discount_targets"][:, 0] = 0          # step 0: no terminal row (n_rare clamps to 1)
    if zero_mask:
        b["masks"].zero_()
    outs = [torch.randn(((K + 1) * B, A), generator=g, device="cuda"),
            torch.tanh(torch.randn(((K + 1) * B, 1), generator=g, device="cuda"))]
    outs += [torch.randn((K * B, 2), generator=g, device="cuda"), torch.randn((K * B, 3), generator=g, device="cuda")]
    if classic:
        p = torch.softmax(torch.randn((B, K, 6), generator=g, device="cuda"), -1)
        p[:, ::2] = 1.0 / 6.0                     # uniform (not rare) rows
        b["dice_probs"] = p
        outs.append(torch.randn((K * B, 6), generator=g, device="cuda"))
    return b, [o.requires_grad_() for o in outs]


def _loss_both(classic, b, outs, K, U):
    """(parts, grads) of the loss over fixed network outputs, fused and as torch ops."""
    from exploring_muzero_on_dog_amd import learner as L
    res = []
    for fused in (True, False):
        for o in outs:
            o.grad = None
        old = L.FUSED_LOSS
        L.FUSED_LOSS = fused
        try:
            total, parts = _loss_only(L, classic, b, outs, K, U)
        finally:
            L.FUSED_LOSS = old
        total.backward()
        res.append(([float(total)] + [float(p) for p in parts],
                    [None if o.grad is None else o.grad.clone() for o in outs]))
    return res


def _loss_only(L, classic, b, outs, K, U):
    """The tail of loss_fn / loss_fn_stochastic from the network outputs on (same code paths)."""
    B = b["masks"].shape[0]
    if not classic:
        logits, v, dl, rl = outs
        if L.FUSED_LOSS:
            u = 1.0 / U
            spec = dict(batch=b, K=K, scale_value=u * L.VALUE_SCALING, scale_policy=u * L.POLICY_SCALING, norm=0,
                        terms=[(b["discount_targets"], 0, 1.0, 0.1, u * L.DISCOUNT_SCALING),
                               (b["rewards"], 0, 0.1, 1.0, u * L.REWARD_SCALING)])
            total, parts = L._LossHeads.apply(logits, v, dl if K else None, rl if K else None, None, spec)
            return total, parts[1:5]
        m = b["masks"][:, :K + 1].transpose(0, 1)
        vv = v[:, 0].reshape(K + 1, B)
        l_value = torch.mean(m * (b["target_values"][:, :K + 1].transpose(0, 1) - vv) ** 2, 1)
        logp = torch.log_softmax(logits, -1).reshape(K + 1, B, -1)
        l_policy = torch.mean(m * -(b["policies"][:, :K + 1].transpose(0, 1) * logp).sum(-1), 1)
        if K:
            l_rew = L._balanced_ce_steps(rl, b["rewards"].transpose(0, 1), m[:K], 1, 0.1, 1.0)
            l_disc = L._balanced_ce_steps(dl, b["discount_targets"].transpose(0, 1), m[:K], 1, 1.0, 0.1)
        else:
            l_rew = l_disc = torch.zeros((1,), device="cuda")
        total = ((1.0 / U) * (L.VALUE_SCALING * l_value + L.POLICY_SCALING * l_policy)).sum() + \
            (1.0 / U) * (L.DISCOUNT_SCALING * l_disc.sum() + L.REWARD_SCALING * l_rew.sum())
        return total, (l_value.sum(), l_policy.sum(), l_disc.sum(), l_rew.sum())
    logits, v, dl, rl, cl = outs
    sc = L.CLASSIC_SCALING
    if L.FUSED_LOSS:
        u = 1.0 / U
        spec = dict(batch=b, K=K, scale_value=u * sc["value"], scale_policy=u * sc["policy"], norm=1,
                    terms=[(b["dice_probs"], 0, 1.0, 0.1, u * sc["chance"]),
                           (b["discount_targets"], 0, 1.0, 0.1, u * sc["discount"]),
                           (b["rewards"], 1, 1.0, 0.1, u * sc["reward"])])
        total, parts = L._LossHeads.apply(logits, v, cl, dl, rl, spec)
        return total, parts[1:6]
    m = b["masks"][:, :K + 1].transpose(0, 1)
    vv = v[:, 0].reshape(K + 1, B)
    logp = torch.log_softmax(logits, -1).reshape(K + 1, B, -1)
    l_policy = torch.mean(m * -(b["policies"][:, :K + 1].transpose(0, 1) * logp).sum(-1), 1)
    l_value = torch.mean(m * (b["target_values"][:, :K + 1].transpose(0, 1) - vv) ** 2, 1)
    mk = m[:K]
    n_valid = mk.sum(1)
    rc, dc, tp = b["rewards"].transpose(0, 1), b["discount_targets"].transpose(0, 1), b["dice_probs"].transpose(0, 1)
    reward_ce = torch.nn.functional.cross_entropy(rl, rc.reshape(-1).long(), reduction="none").reshape(K, B)
    discount_ce = torch.nn.functional.cross_entropy(dl, dc.reshape(-1).long(), reduction="none").reshape(K, B)
    chance_ce = -(tp * torch.log_softmax(cl, -1).reshape(K, B, -1)).sum(-1)
    non_uniform = ((tp - 1.0 / 6.0) ** 2).sum(-1) > 1e-6
    l_reward = L.balanced_loss_steps(reward_ce, (rc != 1).float(), mk, n_valid)
    l_discount = L.balanced_loss_steps(discount_ce, (dc == 1).float(), mk, n_valid)
    l_chance = L.balanced_loss_steps(chance_ce, non_uniform.float(), mk, n_valid)
    total = (1.0 / U) * (sc["value"] * l_value.sum() + sc["policy"] * l_policy.sum() + sc["chance"] * l_chance.sum() +
                         sc["discount"] * l_discount.sum() + sc["reward"] * l_reward.sum())
    return total, (l_value.sum(), l_policy.sum(), l_chance.sum(), l_discount.sum(), l_reward.sum())


@pytest.mark.parametrize("classic,K,B,zero_mask", [(False, 10, 128, False), (False, 5, 100, False),
                                                   (False, 0, 64, False), (False, 3, 70, True),
                                                   (True, 10, 128, False), (True, 4, 33, False), (True, 2, 64, True),
                                                   # B > the kernel's 256 threads: a thread sums several rows
                                                   (False, 3, 384, False), (True, 3, 384, False)])
def test_fused_loss_matches_torch_ops(cuda, classic, K, B, zero_mask):
    b, outs = _loss_case(classic, K, B, seed=K * 7 + B, zero_mask=zero_mask)
    (pf, gf), (pt, gt) = _loss_both(classic, b, outs, K, U=10)
    for x, y in zip(pf, pt):
        assert abs(x - y) <= 2e-6 * max(1.0, abs(y)), (pf, pt)
    for i, (x, y) in enumerate(zip(gf, gt)):
        if x is None or y is None:      # K = 0: no head rows (fused: no gradient; torch: none either)
            assert x is None and y is None or float((x if y is None else y).abs().max()) == 0.0
            continue
        err = float((x - y).abs().max()) / max(float(y.abs().max()), 1e-12)
        assert err < 1e-5 or float((x - y).abs().max()) < 1e-9, (i, err)


def test_fused_loss_accepts_int64_labels(cuda):
    b, outs = _loss_case(False, 4, 64, seed=5)
    (pa, ga), _ = _loss_both(False, b, outs, 4, U=10)
    b64 = dict(b, rewards=b["rewards"].long(), discount_targets=b["discount_targets"].long())
    (pb, gb), _ = _loss_both(False, b64, outs, 4, U=10)
    assert pa == pb and all(torch.equal(x, y) for x, y in zip(ga, gb))


def _ln_ref(x, W, b, gam, bet, res, mode):
    y = x @ W + b
    mu = y.mean(-1, keepdim=True)
    var = (y * y).mean(-1, keepdim=True) - mu * mu           # Flax fast variance
    o = (y - mu) * torch.rsqrt(var.clamp_min(0) + 1e-6) * gam + bet
    return torch.relu(o) if mode == 1 else (torch.relu(res + o) if mode == 2 else o)


@pytest.mark.parametrize("M,K,N,mode", [(128, 256, 256, 1), (1408, 256, 256, 2), (7, 33, 64, 1), (1, 512, 256, 0),
                                        (300, 280, 128, 1), (7168, 60, 64, 1), (50, 24, 32, 2), (17, 100, 256, 2),
                                        (200, 448, 64, 1), (33, 500, 32, 0)])
def test_dense_ln_fused_matches_float64(cuda, M, K, N, mode, monkeypatch):
    from exploring_muzero_on_dog_amd import learner as L
    monkeypatch.setattr(L, "FUSED_FWD", True)      # (off in the learner by default: see learner.FUSED_FWD)
    g = torch.Generator(device="cuda").manual_seed(M + K + N)
    x = torch.randn((M, K), generator=g, device="cuda")
    W = torch.randn((K, N), generator=g, device="cuda") / K ** 0.5
    b, gam, bet = (torch.randn((N,), generator=g, device="cuda") * 0.3 for _ in range(3))
    gam = gam + 1.0
    res = torch.randn((M, N), generator=g, device="cuda") if mode == 2 else None
    out, z, mean, rstd = L._dense_ln_fwd(x, W, b, gam, bet, res, mode)
    # the transposed-weight operand (learner.WeightTranspose): the same arithmetic, bit for bit
    with L.WeightTranspose({"layer/kernel": W}) as wt:
        wt.refresh()
        assert wt.get(W) is not None
        out_t, z_t, _, _ = L._dense_ln_fwd(x, W, b, gam, bet, res, mode)
    ldt = (K + 15) // 16 * 16
    assert torch.equal(wt.get(W)[0][:, :K], W.t()) and not wt.get(W)[0][:, K:ldt].any()
    assert torch.equal(out_t, out) and torch.equal(z_t, z)
    xs = [t.double().requires_grad_() for t in (x, W, b, gam, bet)]
    rr = res.double().requires_grad_() if res is not None else None
    ref = _ln_ref(*xs, rr, mode)
    assert float((out.double() - ref).abs().max()) < 2e-5 * max(1.0, float(ref.abs().max()))
    dout = torch.randn((M, N), generator=g, device="cuda")
    acc = torch.randn((M, K), generator=g, device="cuda")
    scratch = torch.empty((L._ln_scratch_floats(M, N, K),), device="cuda")
    dz, dres, dx = L._dense_ln_bwd(dout, (out, z, mean, rstd), gam, mode, W, scratch, acc=acc)
    dg, dbe, db = L._ln_colsum(scratch, N)
    ref.backward(dout.double())
    tol = lambda r: 5e-5 * max(1.0, float(r.abs().max()))      # noqa: E731
    assert float((dx.double() - (xs[0].grad + acc.double())).abs().max()) < tol(xs[0].grad)
    assert float((db.double() - xs[2].grad).abs().max()) < tol(xs[2].grad)
    assert float((dg.double() - xs[3].grad).abs().max()) < tol(xs[3].grad)
    assert float((dbe.double() - xs[4].grad).abs().max()) < tol(xs[4].grad)
    assert float(((x.double().t() @ dz.double()) - xs[1].grad).abs().max()) < tol(xs[1].grad)
    if mode == 2:
        assert float((dres.double() - rr.grad).abs().max()) < tol(rr.grad)
    # no input gradient: the same dz / partials, dx untouched
    scratch2 = torch.empty_like(scratch)
    dz2, _, dx2 = L._dense_ln_bwd(dout, (out, z, mean, rstd), gam, mode, W, scratch2, need_dx=False)
    torch.cuda.synchronize()
    assert dx2 is None and torch.equal(dz2, dz) and torch.equal(scratch2, scratch)


@pytest.mark.parametrize("N,mode", [(256, 1), (256, 2), (64, 0)])
def test_dense_ln_fused_matches_unfused_path(cuda, N, mode, monkeypatch):
    from exploring_muzero_on_dog_amd import learner as L
    monkeypatch.setattr(L, "FUSED_FWD", True)
    g = torch.Generator(device="cuda").manual_seed(N + mode)
    M, K = 1280, 256
    x = torch.randn((M, K), generator=g, device="cuda")
    W = torch.randn((K, N), generator=g, device="cuda") / 16
    b, gam, bet = (torch.randn((N,), generator=g, device="cuda") for _ in range(3))
    res = torch.randn((M, N), generator=g, device="cuda") if mode == 2 else None
    dout = torch.randn((M, N), generator=g, device="cuda")
    outs = []
    for fused in (True, False):
        old = L.FUSED_DENSE
        L.FUSED_DENSE = fused
        try:
            f = L._dense_ln_fwd(x, W, b, gam, bet, res, mode)
            scr = torch.empty((L._ln_scratch_floats(M, N, K),), device="cuda")
            dz, dres, dx = L._dense_ln_bwd(dout, f, gam, mode, W, scr)
            outs.append((f[0], f[2], f[3], dz, dx, L._ln_colsum(scr, N)))
        finally:
            L.FUSED_DENSE = old
    (o1, m1, r1, z1, x1, c1), (o2, m2, r2, z2, x2, c2) = outs
    for a, b_ in ((o1, o2), (m1, m2), (r1, r2), (z1, z2), (x1, x2)) + tuple(zip(c1, c2)):
        assert float((a - b_).abs().max()) <= 1e-4 * max(1.0, float(b_.abs().max())), float((a - b_).abs().max())


def test_dense_ln_host_checks(cuda):
    from exploring_muzero_on_dog_amd import lib as L
    lib = L.load()
    x = torch.zeros((16, 600), device="cuda")
    W = torch.zeros((600, 256), device="cuda")
    v = torch.zeros((256,), device="cuda")
    o = torch.zeros((16, 256), device="cuda")
    m = torch.zeros((16,), device="cuda")
    # K > 1024 / width 96: unsupported, not a launch
    assert lib.muz_dense_ln_fwd(L.ptr(x), 16, 2000, L.ptr(W), None, 0, L.ptr(v), L.ptr(v), L.ptr(v), None, 256, 1, L.ptr(o),
                                L.ptr(o), L.ptr(m), L.ptr(m), L.stream_ptr()) != 0
    assert lib.muz_dense_ln_fwd(L.ptr(x), 16, 600, L.ptr(W), None, 0, L.ptr(v), L.ptr(v), L.ptr(v), None, 96, 1, L.ptr(o),
                                L.ptr(o), L.ptr(m), L.ptr(m), L.stream_ptr()) != 0
    # residual mode without a residual; a transposed copy with a too-short row
    assert lib.muz_dense_ln_fwd(L.ptr(x), 16, 500, None, L.ptr(W), 500, L.ptr(v), L.ptr(v), L.ptr(v), None, 256, 1,
                                L.ptr(o), L.ptr(o), L.ptr(m), L.ptr(m), L.stream_ptr()) != 0
    assert lib.muz_dense_ln_fwd(L.ptr(x), 16, 500, L.ptr(W), None, 0, L.ptr(v), L.ptr(v), L.ptr(v), None, 256, 2, L.ptr(o),
                                L.ptr(o), L.ptr(m), L.ptr(m), L.stream_ptr()) != 0


def test_fused_output_heads_match_library_form(cuda):
    """learner.FUSED_HEADS (_OutHeads: the policy / value / reward / discount heads as one launch each way,
    csrc/learner_heads.hip) against the same heads as library GEMMs + torch activations: the loss within 1e-6
    relative (k-order fp32 sums instead of BLAS order) and every parameter gradient within 1e-5 relative, with the
    grouped (GradSink) and the per-parameter gradient paths, eager and graph-captured."""
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import learner as L
    from exploring_muzero_on_dog_amd import nets as N
    from exploring_muzero_on_dog_amd import replay as R
    from oracle import nets as ON
    C = E.num_channels(4)
    params = ON.init_params(C, seed=14, randomize_affine=True)
    eng = GA.SelfPlayEngine(N.DeviceNet(params, C), 32, num_players=4, max_steps=120, num_simulations=4, max_depth=4)
    ring = R.VectorizedReplayBuffer(512, 48, 5, 10, obs_shape=(C, 56), max_episode_length=120,
                                    rng=np.random.RandomState(2))
    ring.save_games_from_buffers(eng.play_stream(40, seed=2, temperature=1.0))
    batch = ring.sample_batch()
    old = L.FUSED_HEADS
    try:
        for grouped, graph in ((True, False), (False, False), (True, True)):
            L.FUSED_HEADS = True
            la, ga = _grads(L.Learner, params, C, batch, grouped, graph=graph)
            L.FUSED_HEADS = False
            lb, gb = _grads(L.Learner, params, C, batch, grouped, graph=graph)
            assert abs(la - lb) <= 1e-6 * abs(lb), (grouped, graph, la, lb)
            worst = max(float((ga[k] - gb[k]).norm()) / max(float(gb[k].norm()), 1e-20) for k in ga)
            print(f"fused heads grouped={grouped} graph={graph}: loss {la:.7f} vs {lb:.7f}, worst grad rel {worst:.2e}")
            assert worst < 1e-5, (grouped, graph, worst)
    finally:
        L.FUSED_HEADS = old


@pytest.mark.parametrize("M,A", [(1280, 24), (1283, 806), (5, 24)])
def test_film_kernels_match_float64(cuda, M, A):
    """muz_film_fwd / muz_film_bwd (learner._Film: DynamicsNetwork4's one_hot -> Dense_0 -> relu -> Dense_1 | Dense_2
    for all unrolled rows) against float64 torch: the one-hot rows exact (actions outside [0, A) give the all-zero
    row), e = relu(b0 + W0[a]) bit-identical to the fp32 one-hot product, scale / shift / d e within 1e-5 relative,
    and the six parameter gradients of the autograd node against float64 autograd.  Ragged M (not a multiple of 16)
    and the DOG width A = 806."""
    from exploring_muzero_on_dog_amd import learner as L
    g = torch.Generator(device="cuda").manual_seed(M + A)
    act = torch.randint(-1, A + 1, (M,), generator=g, device="cuda")
    P = [torch.randn(s, generator=g, device="cuda") * f for s, f in
         (((A, 64), 0.3), ((64,), 0.1), ((64, 256), 0.2), ((256,), 0.1), ((64, 256), 0.2), ((256,), 0.1))]
    P = [p.requires_grad_(True) for p in P]
    oh, scale, shift = L._Film.apply(act, *P)
    P64 = [p.detach().double().requires_grad_(True) for p in P]
    ok = (act >= 0) & (act < A)
    oh64 = torch.zeros((M, A), dtype=torch.float64, device="cuda")
    oh64[ok, act[ok]] = 1.0
    e64 = torch.relu(oh64 @ P64[0] + P64[1])
    s64, t64 = e64 @ P64[2] + P64[3], e64 @ P64[4] + P64[5]
    assert torch.equal(oh, oh64.float())
    W0, b0 = P[0].detach(), P[1].detach()
    e32 = torch.relu(torch.where(ok[:, None], W0[act.clamp(0, A - 1)] + b0, b0.expand(M, 64)))
    lib, Lb = L._L.load(), L._L
    e = torch.empty((M, 64), device="cuda")
    scr = [torch.empty((M, 256), device="cuda") for _ in range(3)]
    a32 = act.to(torch.int32)
    Lb.check(lib.muz_film_fwd(Lb.ptr(a32), M, A, *(Lb.ptr(q.detach()) for q in P), None, Lb.ptr(e), Lb.ptr(scr[0]),
                              Lb.ptr(scr[1]), Lb.ptr(scr[2]), Lb.stream_ptr()), "muz_film_fwd")
    assert torch.equal(e, e32)
    assert torch.equal(scr[2], 1.0 + scr[0]) and torch.equal(scr[0], scale.detach())
    for a, b in ((scale, s64), (shift, t64)):
        assert float((a.double() - b).norm() / b.norm()) < 1e-6
    ds, dt = (torch.randn((M, 256), generator=g, device="cuda") for _ in range(2))
    torch.autograd.backward((scale, shift), (ds, dt))
    torch.autograd.backward((s64, t64), (ds.double(), dt.double()))
    for p, q in zip(P, P64):
        err = float((p.grad.double() - q.grad).norm() / max(float(q.grad.norm()), 1e-30))
        assert err < 1e-5, err


def test_fused_film_and_layernorm_match_library_form(cuda):
    """learner.FUSED_FILM_EMBED (_Film) and FUSED_LN_ONCE (_LN for PredictionNetwork4's LayerNorm_0) against the
    torch / library form of the same sub-graphs in a whole det learner step: loss within 1e-6 relative, every
    parameter gradient within 1e-5 relative, with the grouped and the per-parameter gradient paths."""
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import learner as L
    from exploring_muzero_on_dog_amd import nets as N
    from exploring_muzero_on_dog_amd import replay as R
    from oracle import nets as ON
    C = E.num_channels(4)
    params = ON.init_params(C, seed=15, randomize_affine=True)
    eng = GA.SelfPlayEngine(N.DeviceNet(params, C), 32, num_players=4, max_steps=120, num_simulations=4, max_depth=4)
    ring = R.VectorizedReplayBuffer(512, 48, 5, 10, obs_shape=(C, 56), max_episode_length=120,
                                    rng=np.random.RandomState(3))
    ring.save_games_from_buffers(eng.play_stream(40, seed=3, temperature=1.0))
    batch = ring.sample_batch()
    old = (L.FUSED_FILM_EMBED, L.FUSED_LN_ONCE)
    try:
        for grouped in (True, False):
            L.FUSED_FILM_EMBED = L.FUSED_LN_ONCE = True
            la, ga = _grads(L.Learner, params, C, batch, grouped)
            L.FUSED_FILM_EMBED = L.FUSED_LN_ONCE = False
            lb, gb = _grads(L.Learner, params, C, batch, grouped)
            assert abs(la - lb) <= 1e-6 * abs(lb), (grouped, la, lb)
            worst = max(float((ga[k] - gb[k]).norm()) / max(float(gb[k].norm()), 1e-20) for k in ga)
            print(f"fused film + ln grouped={grouped}: loss {la:.7f} vs {lb:.7f}, worst grad rel {worst:.2e}")
            assert worst < 1e-5, (grouped, worst)
    finally:
        L.FUSED_FILM_EMBED, L.FUSED_LN_ONCE = old
