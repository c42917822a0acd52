"""Learner for det-MADN MuZero: train_step of MuZero_det_MADN/train_with_reward.py in torch (autograd).

The learner sits beside the self-play hot path (SURVEY §8f "next"): it consumes batches straight from
the device replay ring (replay.VectorizedReplayBuffer.sample_batch -> device tensors, no host copy) and
hands new weights back to the self-play engine as one packed arena (``push_to``).  Reference functions
mirrored:

  repr_net / dynamics_net / pred_net   muzero_deterministic_madn.py:75-141, 391-457, 549-583 (Flax
                                       semantics: fast-variance LayerNorm eps 1e-6, 'SAME' Conv1D,
                                       one_hot of an out-of-range action = 0, min-max latent scaling)
  loss_fn                              train_with_reward.py:24-141
  train_step                           train_with_reward.py:148-162
  optimizer                            train_with_reward.py:361-372: clip_by_global_norm(5.0) ->
                                       adamw(piecewise-constant lr 0.005, x0.2 @ it 30, x0.2 @ 60,
                                       x0.5 @ 85 of 2500 steps, weight decay 1e-4), optax semantics
  test_training loop                   train_with_reward.py:167-311 (``train_loop``)

Parameters are kept under the Flax path names of nets.param_shapes, so the same dict packs into the
self-play kernels' arena (nets.DeviceNet).  Everything is fp32.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch
import torch.nn.functional as F

from . import lib as _L
from . import nets as N

EPS_LN = 1e-6
VALUE_SCALING, POLICY_SCALING, DISCOUNT_SCALING, REWARD_SCALING = 4.0, 1.0, 1.0, 1.0


LN_PLAIN, LN_RELU, LN_RESID_RELU = 0, 1, 2


class _DenseLN(torch.autograd.Function):
    """act(LayerNorm(x @ W + b)): forward = the GEMM with its bias / LayerNorm / ReLU / residual epilogue in one
    launch (csrc/learner_fused.hip), backward = the LayerNorm / ReLU backward with the input-gradient GEMM in
    one launch, the weight / LayerNorm gradients through the GradSink (or a GEMM + column sum without one).  mode LN_RELU: relu(LN(.)); LN_RESID_RELU: relu(res + LN(.)); LN_PLAIN: LN(.).
    ``owners`` = the leaf parameters (W, b, gamma, beta) for a GradSink (W may be a reshaped view of its leaf)."""

    @staticmethod
    def forward(ctx, x, W, b, gamma, beta, res, mode, owners=None):
        out, z, mean, rstd = _dense_ln_fwd(x, W, b, gamma, beta, res, mode)
        ctx.save_for_backward(x, W, gamma, out, z, mean, rstd)
        ctx.mode, ctx.owners = mode, owners
        return out

    @staticmethod
    def backward(ctx, dout):
        x, W, gamma, out, z, mean, rstd = ctx.saved_tensors
        M, Nn = out.shape
        K = x.shape[1]
        scratch = torch.empty((_ln_scratch_floats(M, Nn, K),), dtype=out.dtype, device=out.device)
        dz, dres, dx = _dense_ln_bwd(dout, (out, z, mean, rstd), gamma, ctx.mode, W, scratch,
                                     need_dx=ctx.needs_input_grad[0])
        sink = _sink()
        if sink is not None and ctx.owners is not None:
            Wp, bp, gp, bep = ctx.owners
            sink.ln_colsum(scratch, Nn, gp, bep, bp)
            sink.wgrad(x, dz, Wp)
            return dx, None, None, None, None, dres, None, None
        dgamma, dbeta, db = _ln_colsum(scratch, Nn)
        dW = x.t() @ dz if ctx.needs_input_grad[1] else None
        return dx, dW, db, dgamma, dbeta, dres, None, None


class _ResBlockLN(torch.autograd.Function):
    """relu(x + LN(Dense_1(relu(LN(Dense_0(x)))))): one ResBlock (muzero_deterministic_madn.py:12-24) as one
    autograd node.  Forward = the two Dense + LayerNorm forwards of _DenseLN; backward = their two fused
    LayerNorm-backward + input-gradient launches with the residual gradient accumulated inside the second
    (dx = dz_0 W_0^T + dres) instead of a separate autograd add.  ``owners`` = the 8 leaf parameters for a
    GradSink (Dense_0 kernel / bias, LayerNorm_0 scale / bias, then the same of the second layer)."""

    @staticmethod
    def forward(ctx, x, Wa, ba, ga, bea, Wb, bb, gb, beb, owners=None):
        fa = _dense_ln_fwd(x, Wa, ba, ga, bea, None, LN_RELU)
        fb = _dense_ln_fwd(fa[0], Wb, bb, gb, beb, x, LN_RESID_RELU)
        ctx.save_for_backward(x, Wa, ga, Wb, gb, *fa, *fb)
        ctx.owners = owners
        return fb[0]

    @staticmethod
    def backward(ctx, dout):
        x, Wa, ga, Wb, gb = ctx.saved_tensors[:5]
        fa, fb = ctx.saved_tensors[5:9], ctx.saved_tensors[9:13]
        M, Nn = fb[0].shape
        dev, dt = dout.device, dout.dtype
        sa = torch.empty((_ln_scratch_floats(M, Nn, x.shape[1]),), dtype=dt, device=dev)
        sb = torch.empty((_ln_scratch_floats(M, Nn, Nn),), dtype=dt, device=dev)
        dzb, dres, t = _dense_ln_bwd(dout, fb, gb, LN_RESID_RELU, Wb, sb)
        dza, _, dx = _dense_ln_bwd(t, fa, ga, LN_RELU, Wa, sa, acc=dres)
        sink = _sink()
        if sink is not None and ctx.owners is not None:
            o = ctx.owners
            sink.ln_colsum(sa, Nn, o[2], o[3], o[1])
            sink.wgrad(x, dza, o[0])
            sink.ln_colsum(sb, Nn, o[6], o[7], o[5])
            sink.wgrad(fa[0], dzb, o[4])
            return (dx,) + (None,) * 9
        grads = []
        for inp, dz, s in ((x, dza, sa), (fa[0], dzb, sb)):
            dg, dbe, db = _ln_colsum(s, Nn)
            grads += [inp.t() @ dz, db, dg, dbe]
        return (dx, *grads, None)


class _ResStack(torch.autograd.Function):
    """nb consecutive ResBlocks (the representation's six at the batch's rows, the prediction's two at all unroll
    steps' rows) as ONE launch each way: csrc/learner_chain.hip's muz_rbstack_fwd / _bwd, 16 rows per workgroup
    carried through every layer, the weights streamed packed (muz_trunk_chain_pack, per call).  The forward
    saves what _ResBlockLN's per-layer launches save; the parameter gradients go to the GradSink (or one GEMM /
    column sum each).  P = the 8 parameters of each block in _ResBlockLN's order; ``owners`` = the same leaves."""

    @staticmethod
    def forward(ctx, x, owners, *P):
        nb, (M, Nn) = len(P) // 8, x.shape
        L2 = 2 * nb
        dev, dt = x.device, x.dtype
        lib = _L.load()
        W = [P[8 * b + 4 * k] for b in range(nb) for k in range(2)]
        WP = _packed(W)
        if WP is None:
            WP = torch.empty((2, L2, Nn * Nn), dtype=dt, device=dev)
            src = (ctypes.c_void_p * L2)(*[w.data_ptr() for w in W])
            _L.check(lib.muz_trunk_chain_pack(src, L2, _L.ptr(WP[0]), _L.ptr(WP[1]), _L.stream_ptr()),
                     "muz_trunk_chain_pack")
        X = torch.empty((L2, M, Nn), dtype=dt, device=dev)
        out = torch.empty((M, Nn), dtype=dt, device=dev)
        z = torch.empty((L2, M, Nn), dtype=dt, device=dev)
        stats = torch.empty((L2, 2, M), dtype=dt, device=dev)
        a = _L.MuzRbstackArgs()
        a.nb, a.M = nb, M
        for l in range(L2):
            b, k = divmod(l, 2)
            a.wf[l], a.wb[l] = WP[0, l].data_ptr(), WP[1, l].data_ptr()
            a.bias[l], a.gamma[l], a.beta[l] = (P[8 * b + 4 * k + i].data_ptr() for i in (1, 2, 3))
        a.x, a.X, a.out, a.z, a.stats = x.data_ptr(), X.data_ptr(), out.data_ptr(), z.data_ptr(), stats.data_ptr()
        _L.check(lib.muz_rbstack_fwd(ctypes.byref(a), _L.stream_ptr()), "muz_rbstack_fwd")
        # the buffers the backward's pointers (ctx.args) read stay alive as long as ctx does, so a second backward
        # (retain_graph) reads valid memory; the output is held by save_for_backward (no output -> ctx cycle)
        ctx.save_for_backward(out)
        ctx.args, ctx.keep, ctx.X, ctx.P, ctx.owners = a, (WP, x, z, stats), X, P, owners
        return out

    @staticmethod
    def backward(ctx, dout):
        a, X, P = ctx.args, ctx.X, ctx.P
        L2, M, Nn = X.shape
        dev, dt = dout.device, dout.dtype
        tiles = (M + 15) // 16
        DZ = torch.empty((L2, M, Nn), dtype=dt, device=dev)
        part = torch.empty((L2, tiles * 3 * Nn), dtype=dt, device=dev)
        dx = torch.empty((M, Nn), dtype=dt, device=dev)
        dout = dout.contiguous()
        a.g, a.DZ, a.part, a.dx = dout.data_ptr(), DZ.data_ptr(), part.data_ptr(), dx.data_ptr()
        ctx.saved_tensors   # (raises if the graph was freed by an earlier backward)
        _L.check(_L.load().muz_rbstack_bwd(ctypes.byref(a), _L.stream_ptr()), "muz_rbstack_bwd")
        sink, o = _sink(), ctx.owners
        if sink is not None and o is not None:
            for l in range(L2):
                Wl, bl, gl, bel = o[4 * l:4 * l + 4]
                sink.ln_colsum(part[l], Nn, gl, bel, bl)
                sink.wgrad(X[l], DZ[l], Wl)
            return (dx, None) + (None,) * len(P)
        grads = []
        for l in range(L2):
            dg, dbe, db = _ln_colsum(part[l], Nn)
            grads += [X[l].t() @ DZ[l], db, dg, dbe]
        return (dx, None, *grads)


_ONES = {}


def _ones(M, like):
    """A cached ones vector of length M (filled on the eager warm-up step, so a captured graph reuses it)."""
    key = (M, like.device, like.dtype)
    v = _ONES.get(key)
    if v is None:
        v = _ONES[key] = torch.ones((M,), dtype=like.dtype, device=like.device)
    return v


_ZEROS = {}


def _zeros(N, like):
    """A cached zero vector of length N (muz_ln_fwd's bias operand for a plain LayerNorm; filled on the eager
    warm-up step, so a captured graph reuses it)."""
    key = (N, like.device, like.dtype)
    v = _ZEROS.get(key)
    if v is None:
        v = _ZEROS[key] = torch.zeros((N,), dtype=like.dtype, device=like.device)
    return v


class _LN(torch.autograd.Function):
    """A plain Flax LayerNorm (eps 1e-6, fast variance) as one launch each way (muz_ln_fwd / muz_ln_bwd_rows),
    its scale / bias gradients as column partials for the GradSink's grouped column sums (torch's layer_norm took
    one launch forward and three backward).  For a LayerNorm applied once per loss (PredictionNetwork4's
    LayerNorm_0 over all unrolled steps): a GradSink owns each parameter once."""

    @staticmethod
    def forward(ctx, x, gamma, beta):
        x = x.contiguous()
        fwd = _ln_fwd(x, _zeros(x.shape[1], x), gamma, beta, None, LN_PLAIN)
        ctx.save_for_backward(gamma, *fwd)
        ctx.owners = (gamma, beta) if gamma.is_leaf and beta.is_leaf else None
        return fwd[0]

    @staticmethod
    def backward(ctx, dout):
        gamma, out, z, mean, rstd = ctx.saved_tensors
        M, Nn = out.shape
        scratch = torch.empty((_L.load().muz_ln_bwd_scratch_floats(M, Nn),), dtype=out.dtype, device=out.device)
        dz, _ = _ln_bwd_rows(dout, (out, z, mean, rstd), gamma, LN_PLAIN, scratch)
        sink = _sink()
        if sink is not None and ctx.owners is not None:
            sink.ln_colsum(scratch, Nn, ctx.owners[0], ctx.owners[1])
            return dz, None, None
        dgamma, dbeta, _ = _ln_colsum(scratch, Nn)
        return dz, dgamma, dbeta


class _Dense(torch.autograd.Function):
    """x @ W + b whose bias gradient is a BLAS GEMV (dy^T @ 1) instead of torch's column-sum reduction
    (~12 us per call at the learner's 1280-1408 rows, against ~5 us); with a GradSink active both parameter
    gradients go to the grouped launches."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.owners = (W, b) if W.is_leaf and b.is_leaf else None
        return (x @ W).add_(b)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx = dy @ W.t() if ctx.needs_input_grad[0] else None
        sink = _sink()
        if sink is not None and ctx.owners is not None:
            dy2 = dy2.contiguous()
            sink.wgrad(x.reshape(-1, x.shape[-1]).contiguous(), dy2, ctx.owners[0])
            sink.colsum(dy2, ctx.owners[1])
            return dx, None, None
        dW = x.reshape(-1, x.shape[-1]).t() @ dy2 if ctx.needs_input_grad[1] else None
        db = torch.mv(dy2.t(), _ones(dy2.shape[0], dy2)) if ctx.needs_input_grad[2] else None
        return dx, dW, db


HEAD_PARAMS = ("prediction/Dense_2/kernel", "prediction/Dense_2/bias", "prediction/Dense_4/kernel",
               "prediction/Dense_4/bias", "prediction/Dense_5/kernel", "prediction/Dense_5/bias",
               "dynamics/Dense_6/kernel", "dynamics/Dense_6/bias", "dynamics/reward_head/kernel",
               "dynamics/reward_head/bias", "dynamics/Dense_7/kernel", "dynamics/Dense_7/bias",
               "dynamics/discount_head/kernel", "dynamics/discount_head/bias")


FUSED_FILM_EMBED = True   # False: the FiLM sub-graph as one-hot + library GEMMs + torch ops (A/B, test reference)
FUSED_LN_ONCE = True      # False: Pred4's LayerNorm_0 as torch layer_norm (A/B, test reference)
_FILM_PARAMS = ("Dense_0/kernel", "Dense_0/bias", "Dense_1/kernel", "Dense_1/bias", "Dense_2/kernel", "Dense_2/bias")


class _Film(torch.autograd.Function):
    """DynamicsNetwork4's action-only FiLM sub-graph for all unrolled rows as one launch each way
    (csrc/learner_film.hip, muz_film_fwd / _bwd; muzero_deterministic_madn.py:404-418): -> (one_hot [M, A],
    scale [M, 256], shift [M, 256]).  The one-hot product is a row gather (exact); the backward forms d e with one
    launch and records e^T dscale, e^T dshift, one_hot^T de and the bias column sums into the active GradSink (or
    forms them here)."""

    @staticmethod
    def forward(ctx, action, W0, b0, W1, b1, W2, b2):
        # action: the M rows as a vector, or a [B, K] int32 view with unit column stride (row k B + b = action[b, k],
        # read in place by the kernel)
        if action.dim() == 2 and action.dtype == torch.int32 and action.stride(1) == 1:
            a, (Bk, Kk), lda = action, action.shape, action.stride(0)
        else:
            a = (action.transpose(0, 1) if action.dim() == 2 else action).reshape(-1).to(torch.int32).contiguous()
            Bk, Kk, lda = a.numel(), 1, 1
        M, A = Bk * Kk, W0.shape[0]
        dev, dt = W0.device, W0.dtype
        oh = torch.empty((M, A), dtype=dt, device=dev)
        e = torch.empty((M, 64), dtype=dt, device=dev)
        scale = torch.empty((M, 256), dtype=dt, device=dev)
        shift = torch.empty((M, 256), dtype=dt, device=dev)
        P = [t.contiguous() for t in (W0, b0, W1, b1, W2, b2)]
        scale1 = torch.empty_like(scale)
        _L.check(_L.load().muz_film_fwd_strided(_L.ptr(a), Bk, Kk, lda, A, *(_L.ptr(t) for t in P), _L.ptr(oh),
                                                _L.ptr(e), _L.ptr(scale), _L.ptr(shift), _L.ptr(scale1),
                                                _L.stream_ptr()), "muz_film_fwd_strided")
        scale._muz_scale1 = scale1             # 1 + scale, bit-identical to the chain's own (fp32 add)
        ctx.save_for_backward(oh, e, P[2], P[4])
        ctx.owners = (W0, b0, W1, b1, W2, b2) if all(t.is_leaf for t in (W0, b0, W1, b1, W2, b2)) else None
        ctx.mark_non_differentiable(oh)
        ctx.set_materialize_grads(False)       # (no zero-filled gradient for the one-hot output)
        return oh, scale, shift

    @staticmethod
    def backward(ctx, doh, dscale, dshift):
        oh, e, W1, W2 = ctx.saved_tensors
        M = e.shape[0]
        dscale = torch.zeros_like(e[:, :1].expand(M, 256)) if dscale is None else dscale.reshape(M, 256).contiguous()
        dshift = torch.zeros_like(dscale) if dshift is None else dshift.reshape(M, 256).contiguous()
        de = torch.empty_like(e)
        _L.check(_L.load().muz_film_bwd(_L.ptr(dscale), _L.ptr(dshift), _L.ptr(e), _L.ptr(W1), _L.ptr(W2), M,
                                        _L.ptr(de), _L.stream_ptr()), "muz_film_bwd")
        sink = _sink()
        if sink is not None and ctx.owners is not None:
            W0, b0, W1p, b1, W2p, b2 = ctx.owners
            sink.wgrad(oh, de, W0)
            sink.colsum(de, b0)
            sink.wgrad(e, dscale, W1p)
            sink.colsum(dscale, b1)
            sink.wgrad(e, dshift, W2p)
            sink.colsum(dshift, b2)
            return (None,) * 7
        ones = _ones(M, e)
        return (None, oh.t() @ de, torch.mv(de.t(), ones), e.t() @ dscale, torch.mv(dscale.t(), ones),
                e.t() @ dshift, torch.mv(dshift.t(), ones))


class _OutHeads(torch.autograd.Function):
    """The output heads of one unrolled batch as one launch each way (csrc/learner_heads.hip, muz_heads_fwd / _bwd):
    PredictionNetwork4's policy logits (Dense_2) and value head (Dense_4 -> relu -> Dense_5 -> tanh) over the K + 1
    steps' policy / value hidden layers, DynamicsNetwork4's reward / discount heads (Dense_6 | Dense_7 -> relu ->
    reward_head | discount_head) over the K steps' [next latent, one_hot(action)] (muzero_deterministic_madn.py:
    437-455, 572-583).  As library GEMMs, bias adds and activations: ~18 launches forward, ~20 backward.  Weight /
    bias gradients: X^T dz and column sums, recorded into the active GradSink (grouped launches) or formed here.
    -> (logits [R, A], value [R, 1], reward logits [Rk, 3], discount logits [Rk, 3])."""

    @staticmethod
    def forward(ctx, pol_h, v_h, head_in, onehot, *params):
        W2, b2, W4, b4, W5, b5, W6, b6, Wr, br, W7, b7, Wd, bd = params
        R, A, Rk = pol_h.shape[0], W2.shape[1], head_in.shape[0]
        dev, dt = pol_h.device, pol_h.dtype
        pol_h, v_h, head_in, onehot = (t.contiguous() for t in (pol_h, v_h, head_in, onehot))
        emp = lambda *shape: torch.empty(shape, dtype=dt, device=dev)   # noqa: E731
        logits, value, h4 = emp(R, A), emp(R, 1), emp(R, 64)
        rl, dl, h6, h7, ri = emp(Rk, 3), emp(Rk, 3), emp(Rk, 64), emp(Rk, 64), emp(Rk, 256 + A)
        a = _L.MuzHeadsArgs()
        a.R, a.Rk, a.A = R, Rk, A
        for k, t in zip(("pol_h", "v_h", "head_in", "onehot", "W2", "b2", "W4", "b4", "W5", "b5", "W6", "b6", "Wr",
                         "br", "W7", "b7", "Wd", "bd", "logits", "value", "h4", "rl", "dl", "h6", "h7", "ri"),
                        (pol_h, v_h, head_in, onehot, *params, logits, value, h4, rl, dl, h6, h7, ri)):
            setattr(a, k, t.data_ptr())
        _L.check(_L.load().muz_heads_fwd(ctypes.byref(a), _L.stream_ptr()), "muz_heads_fwd")
        ctx.save_for_backward(pol_h, v_h, value, h4, h6, h7, ri, *params)
        ctx.owners = params if all(p.is_leaf for p in params) else None
        return logits, value, rl, dl

    @staticmethod
    def backward(ctx, g_logits, g_value, g_rl, g_dl):
        pol_h, v_h, value, h4, h6, h7, ri, *params = ctx.saved_tensors
        W2, b2, W4, b4, W5, b5, W6, b6, Wr, br, W7, b7, Wd, bd = params
        R, A, Rk = pol_h.shape[0], W2.shape[1], ri.shape[0]
        dev, dt = pol_h.device, pol_h.dtype
        emp = lambda *shape: torch.empty(shape, dtype=dt, device=dev)   # noqa: E731
        d_pol_h, d_v_h, d_head_in = emp(R, 128), emp(R, 128), emp(Rk, 256)
        dz4, dv5, dz6, dz7 = emp(R, 64), emp(R, 1), emp(Rk, 64), emp(Rk, 64)
        z = lambda t, *shape: torch.zeros(shape, dtype=dt, device=dev) if t is None else t.contiguous()  # noqa: E731
        g_logits, g_value, g_rl, g_dl = z(g_logits, R, A), z(g_value, R, 1), z(g_rl, Rk, 3), z(g_dl, Rk, 3)
        a = _L.MuzHeadsArgs()
        a.R, a.Rk, a.A = R, Rk, A
        for k, t in zip(("pol_h", "v_h", "W2", "b2", "W4", "b4", "W5", "b5", "W6", "b6", "Wr", "br", "W7", "b7", "Wd",
                         "bd", "value", "h4", "h6", "h7", "ri", "g_logits", "g_value", "g_rl", "g_dl", "d_pol_h", "d_v_h",
                         "d_head_in", "dz4", "dv5", "dz6", "dz7"),
                        (pol_h, v_h, *params, value, h4, h6, h7, ri, g_logits, g_value, g_rl, g_dl, d_pol_h, d_v_h,
                         d_head_in, dz4, dv5, dz6, dz7)):
            setattr(a, k, t.data_ptr())
        _L.check(_L.load().muz_heads_bwd(ctypes.byref(a), _L.stream_ptr()), "muz_heads_bwd")
        # weight / bias gradients: (layer input, its dz) pairs
        pairs = ((pol_h, g_logits), (v_h, dz4), (h4, dv5), (ri, dz6), (h6, g_rl), (ri, dz7), (h7, g_dl))
        sink = _sink()
        if sink is not None and ctx.owners is not None:
            for (x, dz), W, b in zip(pairs, ctx.owners[0::2], ctx.owners[1::2]):
                sink.wgrad(x, dz, W)
                sink.colsum(dz, b)
            grads = (None,) * 14
        else:
            grads = []
            for (x, dz), W in zip(pairs, params[0::2]):
                grads += [(x.t() @ dz).reshape(W.shape), dz.sum(0)]
        return (d_pol_h, d_v_h, d_head_in, None, *grads)


class _DenseMinmax(torch.autograd.Function):
    """minmax(x @ W + b) per row of 256 (RepresentationNetwork2's last layer, muzero_deterministic_madn.py:
    139-140): the library GEMM, then the bias add and the min-max scaling in one launch each way
    (muz_minmax_fwd / _bwd with no skip input; torch's add / amin / amax / sub / div and their backward were
    ~10 launches).  Same arithmetic order as the torch form; tied extrema split their gradient evenly."""

    @staticmethod
    def forward(ctx, x, W, b):
        M, Nn = x.shape[0], W.shape[1]
        y = x @ W
        out, q = torch.empty_like(y), torch.empty_like(y)
        lohi = torch.empty((M, 2), dtype=y.dtype, device=y.device)
        idx = torch.empty((M, 2), dtype=torch.int32, device=y.device)
        _L.check(_L.load().muz_minmax_fwd(None, _L.ptr(y), _L.ptr(b), M, Nn, _L.ptr(out), _L.ptr(q), _L.ptr(lohi),
                                          _L.ptr(idx), _L.stream_ptr()), "muz_minmax_fwd")
        ctx.save_for_backward(x, W, q, lohi)
        ctx.owners = (W, b) if W.is_leaf and b.is_leaf else None
        return out

    @staticmethod
    def backward(ctx, g):
        x, W, q, lohi = ctx.saved_tensors
        M, Nn = q.shape
        g = g.contiguous()
        dq = torch.empty_like(q)
        _L.check(_L.load().muz_minmax_bwd(_L.ptr(g), None, None, None, 1.0, 0, _L.ptr(q), _L.ptr(lohi), M, Nn,
                                          _L.ptr(dq), _L.stream_ptr()), "muz_minmax_bwd")
        dx = dq @ W.t() if ctx.needs_input_grad[0] else None
        sink = _sink()
        if sink is not None and ctx.owners is not None:
            sink.wgrad(x.contiguous(), dq, ctx.owners[0])
            sink.colsum(dq, ctx.owners[1])
            return dx, None, None
        dW = x.t() @ dq if ctx.needs_input_grad[1] else None
        db = torch.mv(dq.t(), _ones(M, dq)) if ctx.needs_input_grad[2] else None
        return dx, dW, db


class _Im2col(torch.autograd.Function):
    """The im2col matrix of a 'SAME' Conv1D (MuZeroNets._conv_cols) in one kernel each way
    (csrc/learner_ln.hip; torch's pad + slices + cat made ~25 kernels per convolution's backward)."""

    @staticmethod
    def forward(ctx, x, K):
        B, W, Cin = x.shape
        cols = torch.empty((B, W, K * Cin), dtype=x.dtype, device=x.device)
        # (a strided view -- the observation's first channels transposed -- is read in place)
        _L.check(_L.load().muz_im2col_fwd_strided(_L.ptr(x), B, W, Cin, K, *x.stride(), _L.ptr(cols),
                                                  _L.stream_ptr()), "muz_im2col_fwd_strided")
        ctx.K, ctx.shape = K, (B, W, Cin)
        return cols

    @staticmethod
    def backward(ctx, dcols):
        B, W, Cin = ctx.shape
        dcols = dcols.contiguous()
        dx = torch.empty((B, W, Cin), dtype=dcols.dtype, device=dcols.device)
        _L.check(_L.load().muz_im2col_bwd(_L.ptr(dcols), B, W, Cin, ctx.K, _L.ptr(dx), _L.stream_ptr()),
                 "muz_im2col_bwd")
        return dx, None


# A long-K layer on few rows (the representation's Dense_0: K = 3584, N = 256, batch 128 rows) gets one library tile
# per 32 x 32 outputs and runs its whole K serially (20 us for 0.24 GFLOP, profiles/r6q_learner_step_sequence_det.txt);
# MUZ_SPLITK_DENSE=1 runs it as a batched GEMM over K chunks of 256 whose partial planes the LayerNorm launch sums in
# chunk order (muz_ln_fwd_parts).  Off by default: deterministic (profiles/r6t_diag_splitk.log) and 10 us faster per
# step (profiles/r6r_steps.log), but its different rounding (8.9e-7 relative against the single GEMM) moved one
# classic-learner row's fp32 forward past the tests' decision margin TAU = 1e-6 (the fused and per-layer paths then
# route that row's min-max / ReLU gradient differently: 4.9e-5 on every dynamics tensor,
# test_fused_kernels_match_per_layer_path_end_to_end[classic], profiles/r6s_per_layer_sk1.log).
SPLITK_DENSE = os.environ.get("MUZ_SPLITK_DENSE", "0") == "1"


def _splitk_parts(M, K):
    if not SPLITK_DENSE or K < 1024 or M > 1024:
        return 1
    return next((S for S in (14, 16, 12, 8) if K % S == 0 and K // S >= 128), 1)


def _loss_row(vals):
    """[total, part_1, ...] as one [n] tensor: a view of the fused loss kernel's parts row when vals[1:] are its
    consecutive entries 1.. (its entry 0 holds the total), else a stack."""
    p1 = vals[1] if len(vals) > 1 else None
    if p1 is not None and all(v.dim() == 0 and v.dtype == p1.dtype for v in vals) and p1.storage_offset() >= 1 and \
            all(vals[i].untyped_storage().data_ptr() == p1.untyped_storage().data_ptr() and
                vals[i].storage_offset() == p1.storage_offset() + i - 1 for i in range(1, len(vals))):
        return p1.as_strided((len(vals),), (1,), p1.storage_offset() - 1)
    return torch.stack(vals)


def _ln_fwd(y, bias, gamma, beta, res, mode, out=None, parts=1):
    """Fused bias + LayerNorm (+ ReLU / residual ReLU) forward: -> (out, z, mean, rstd) (no autograd).
    `out`: a preallocated contiguous [M, N] destination (a row block of a stacked buffer)."""
    M, Nn = y.shape[-2:]
    out = torch.empty((M, Nn), dtype=y.dtype, device=y.device) if out is None else out
    z = torch.empty((M, Nn), dtype=y.dtype, device=y.device)
    mean = torch.empty((M,), dtype=y.dtype, device=y.device)
    rstd = torch.empty_like(mean)
    _L.check(_L.load().muz_ln_fwd_parts(_L.ptr(y), parts, _L.ptr(bias), _L.ptr(gamma), _L.ptr(beta), _L.ptr(res), M,
                                        Nn, mode, _L.ptr(out), _L.ptr(z), _L.ptr(mean), _L.ptr(rstd), _L.stream_ptr()),
             "muz_ln_fwd_parts")
    return out, z, mean, rstd


# csrc/learner_fused.hip in the learner, measured per layer at the step's shapes (HIP-graph replay,
# profiles/fused_layer_bench.py, r3): backward, LayerNorm backward + input gradient in one launch 7.4 / 8.0 us
# (M = 128 / 1408 rows) against 8.0 / 10.0 us for muz_ln_bwd_rows + library GEMM -> on; forward, GEMM + LayerNorm
# in one launch 10.0 / 10.6 us against 7.2 / 9.9 us for library GEMM + muz_ln_fwd -> off: a 16-row tile must own
# whole rows for the LayerNorm, so one CU streams the full weight matrix and carries the tile's 1024 MFMAs
# (>= 3.4 us at 32 cycles each), where the library spreads the columns over 2-4x more CUs.
FUSED_FWD = False
# ... except for the narrow layers (N <= 64: the three convolutions as GEMMs over B x 56 rows, the global-feature
# Dense_1 / Dense_2): there the whole row is 2-4 MFMA column tiles and the fused launch replaces the library GEMM +
# muz_ln_fwd pair (MUZ_FUSED_FWD_NARROW=0: the pair, for A/B timing)
FUSED_FWD_NARROW = os.environ.get("MUZ_FUSED_FWD_NARROW", "1") == "1"
FUSED_BWD = True
FUSED_DENSE = True   # False: neither (A/B timing)
RESBLOCK_NODE = True  # False: a ResBlock as two _DenseLN nodes + autograd's residual add (A/B timing)
RESBLOCK_STACK = True  # False: consecutive ResBlocks as one node each instead of one _ResStack (A/B timing)


def _fusable(K, Nn, fwd=False):
    """csrc/learner_fused.hip's shapes: K <= 512 inputs, N in {32, 64, 128, 256} outputs."""
    on = (FUSED_FWD or (FUSED_FWD_NARROW and Nn <= 64)) if fwd else FUSED_BWD
    return FUSED_DENSE and on and 0 < K <= 512 and Nn in (32, 64, 128, 256)


def _ln_scratch_floats(M, Nn, K):
    """Column-partial scratch of one layer's backward (_dense_ln_bwd)."""
    lib = _L.load()
    return lib.muz_dense_ln_bwd_scratch_floats(M, Nn) if _fusable(K, Nn) else lib.muz_ln_bwd_scratch_floats(M, Nn)


class WeightTranspose:
    """Zero-padded transposes W^T [N][K16] of every fused layer's weight, so that the forward kernel reads its
    weight operand as one 16-byte load per lane (csrc/learner_fused.hip) instead of four column loads.
    refresh() is one grouped launch (muz_transpose_grouped); the learner calls it at the start of every step
    (inside the captured graph), so the copies always equal the parameters the step reads."""

    def __init__(self, params: dict):
        self.map, probs = {}, []
        for name, p in params.items():
            if not name.endswith("/kernel") or p.dim() < 2:
                continue
            K, Nn = int(np.prod(p.shape[:-1])), int(p.shape[-1])
            if not _fusable(K, Nn, fwd=True):
                continue
            ldt = (K + 15) // 16 * 16
            wt = torch.zeros((Nn, ldt), dtype=p.dtype, device=p.device)
            self.map[p.data_ptr()] = (wt, ldt, K, Nn)
            probs.append(_L.MuzTransposeProblem(p.data_ptr(), wt.data_ptr(), K, Nn, ldt))
        self.probs = (_L.MuzTransposeProblem * max(len(probs), 1))(*probs)
        self.count = len(probs)

    def refresh(self):
        _L.check(_L.load().muz_transpose_grouped(self.probs, self.count, _L.stream_ptr()), "muz_transpose_grouped")

    def get(self, W):
        e = self.map.get(W.data_ptr())
        return e if e is not None and e[2:] == tuple(W.shape) else None

    def __enter__(self):
        global _WT
        _WT = self
        return self

    def __exit__(self, *exc):
        global _WT
        _WT = None
        return False


_WT = None      # the active WeightTranspose (set around the learner's forward)


def _dense_ln_fwd(x, W, bias, gamma, beta, res, mode, out=None):
    """act(LayerNorm(x @ W + bias)) [+ residual] -> (out, z, mean, rstd) (no autograd): one launch
    (muz_dense_ln_fwd, with the active WeightTranspose's W^T when it holds this weight) where fusable, else
    the library GEMM + muz_ln_fwd."""
    M, K = x.shape
    Nn = W.shape[1]
    if not _fusable(K, Nn, fwd=True):
        S = _splitk_parts(M, K) if x.is_contiguous() and W.is_contiguous() else 1
        if S > 1:   # [S][M][N] partial planes: x's K chunks times W's row chunks
            y = torch.bmm(x.view(M, S, K // S).transpose(0, 1), W.view(S, K // S, Nn))
            return _ln_fwd(y, bias, gamma, beta, res, mode, out=out, parts=S)
        return _ln_fwd(x @ W, bias, gamma, beta, res, mode, out=out)
    x, W = x.contiguous(), W.contiguous()
    wt = _WT.get(W) if _WT is not None else None
    out = torch.empty((M, Nn), dtype=x.dtype, device=x.device) if out is None else out
    z = torch.empty((M, Nn), dtype=x.dtype, device=x.device)
    mean = torch.empty((M,), dtype=x.dtype, device=x.device)
    rstd = torch.empty_like(mean)
    _L.check(_L.load().muz_dense_ln_fwd(_L.ptr(x), M, K, _L.ptr(W), _L.ptr(None if wt is None else wt[0]),
                                        0 if wt is None else wt[1], _L.ptr(bias), _L.ptr(gamma), _L.ptr(beta),
                                        _L.ptr(res), Nn, mode, _L.ptr(out), _L.ptr(z), _L.ptr(mean), _L.ptr(rstd),
                                        _L.stream_ptr()), "muz_dense_ln_fwd")
    return out, z, mean, rstd


def _rows_view(t, align):
    """(t, its row stride) when t is a 2-D row-major view with unit column stride whose rows the backward kernels
    can read in place (a column slice of a concatenation's gradient: no copy), else (a contiguous copy, its width).
    align: the row stride multiple (and 4 x align-byte base alignment) the kernel's row loads need."""
    if t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1] and t.stride(0) % align == 0 and \
            t.data_ptr() % (4 * align) == 0:
        return t, t.stride(0)
    t = t.contiguous()
    return t, t.shape[1]


def _dense_ln_bwd(dout, fwd, gamma, mode, W, scratch, dz=None, acc=None, dx_out=None, need_dx=True):
    """Backward of _dense_ln_fwd up to the layer input: -> (dz, dres or None, dx = dz @ W^T (+ acc) or None);
    column partials into scratch (_ln_scratch_floats).  One launch (muz_dense_ln_bwd) where fusable."""
    out = fwd[0]
    M, Nn = out.shape
    K = W.shape[0]
    if not _fusable(K, Nn):
        dz, dres = _ln_bwd_rows(dout, fwd, gamma, mode, scratch, dz)
        if not need_dx:
            return dz, dres, None
        if acc is None:
            return dz, dres, torch.mm(dz, W.t(), out=dx_out) if dx_out is not None else dz @ W.t()
        return dz, dres, torch.addmm(acc, dz, W.t(), out=dx_out) if dx_out is not None else torch.addmm(acc, dz, W.t())
    dout, ldd = _rows_view(dout, 4)
    W = W.contiguous()
    dz = torch.empty_like(out) if dz is None else dz
    dres = torch.empty_like(out) if mode == LN_RESID_RELU else None
    dx = None
    if need_dx:
        dx = torch.empty((M, K), dtype=out.dtype, device=out.device) if dx_out is None else dx_out
    _L.check(_L.load().muz_dense_ln_bwd_ld(_L.ptr(dout), ldd, *(_L.ptr(t) for t in fwd), _L.ptr(gamma), M, Nn, mode,
                                           _L.ptr(W), K, _L.ptr(acc), _L.ptr(dz), _L.ptr(dres), _L.ptr(dx),
                                           _L.ptr(scratch), _L.stream_ptr()), "muz_dense_ln_bwd_ld")
    return dz, dres, dx


def _ln_bwd_rows(dout, fwd, gamma, mode, scratch, dz=None):
    """Row half of the fused backward: -> (dz, dres or None); column partials into scratch.  `dz`: a
    preallocated contiguous destination."""
    out, z, mean, rstd = fwd
    M, Nn = out.shape
    dout, ldd = _rows_view(dout, 1)
    dz = torch.empty_like(out) if dz is None else dz
    dres = torch.empty_like(out) if mode == LN_RESID_RELU else None
    _L.check(_L.load().muz_ln_bwd_rows_ld(_L.ptr(dout), ldd, _L.ptr(out), _L.ptr(z), _L.ptr(mean), _L.ptr(rstd),
                                          _L.ptr(gamma), M, Nn, mode, _L.ptr(dz), _L.ptr(dres), _L.ptr(scratch),
                                          _L.stream_ptr()), "muz_ln_bwd_rows_ld")
    return dz, dres


def _ln_film_fwd(x, gamma, beta, scale1, shift, film):
    """LayerNorm_0 + FiLM of a dynamics trunk in one launch (muz_ln_film_fwd): film <- shift + LN(x) * scale1;
    -> (out = LN(x), z, mean, rstd) for the backward, like _ln_fwd."""
    M, Nn = x.shape
    out, z = torch.empty_like(x), torch.empty_like(x)
    mean = torch.empty((M,), dtype=x.dtype, device=x.device)
    rstd = torch.empty_like(mean)
    _L.check(_L.load().muz_ln_film_fwd(_L.ptr(x), _L.ptr(gamma), _L.ptr(beta), _L.ptr(scale1.contiguous()),
                                       _L.ptr(shift.contiguous()), M, Nn, _L.ptr(out), _L.ptr(z), _L.ptr(mean),
                                       _L.ptr(rstd), _L.ptr(film), _L.stream_ptr()), "muz_ln_film_fwd")
    return out, z, mean, rstd


def _ln_film_bwd_rows(dfilm, fwd, gamma, scale1, scratch, dscale):
    """Backward row half of _ln_film_fwd (muz_ln_film_bwd_rows): dscale <- d(film) * LN(x); -> dz of the
    LayerNorm input; column partials into scratch."""
    out, z, mean, rstd = fwd
    M, Nn = out.shape
    dz = torch.empty_like(out)
    _L.check(_L.load().muz_ln_film_bwd_rows(_L.ptr(dfilm.contiguous()), _L.ptr(out), _L.ptr(z), _L.ptr(mean),
                                            _L.ptr(rstd), _L.ptr(gamma), _L.ptr(scale1.contiguous()), M, Nn, _L.ptr(dz),
                                            _L.ptr(dscale), _L.ptr(scratch), _L.stream_ptr()), "muz_ln_film_bwd_rows")
    return dz


def _ln_colsum(scratch, Nn):
    """-> (dgamma, dbeta, dbias) from the column partials of any number of row-half calls."""
    dg, db_, dbias = (torch.empty((Nn,), dtype=scratch.dtype, device=scratch.device) for _ in range(3))
    _L.check(_L.load().muz_ln_colsum(_L.ptr(scratch), scratch.numel() // (3 * Nn), Nn, _L.ptr(dg), _L.ptr(db_),
                                     _L.ptr(dbias), _L.stream_ptr()), "muz_ln_colsum")
    return dg, db_, dbias


class GradSink:
    """The weight / bias / LayerNorm parameter gradients of one backward as TWO grouped launches
    (csrc/learner_grad.hip: muz_wgrad_grouped, muz_colsum_grouped) instead of one library GEMM / column sum
    each (~130 launches per det step).  While a sink is active (``with sink:`` around ``loss.backward()``) the
    dense / LayerNorm autograd nodes record (X, dZ) pairs and column-sum partials here and return no gradient for
    those parameters; ``flush()`` computes them into per-parameter buffers (allocated once, stable pointers: a
    captured HIP graph replays into them) and points each parameter's ``.grad`` at its buffer.  A parameter is
    owned by exactly one node (recorded twice -> error).  Recorded tensors are kept alive until the flush."""

    def __init__(self):
        self.buf, self.wg, self.cs, self.keep, self.owned = {}, [], [], [], set()
        self.scratch = {}       # segment partials of the long weight-gradient reductions, one buffer per launch
        self.side = None        # the stream the grouped launches run on (ASYNC_GRADS), joined at flush()
        self.nlaunch = 0        # grouped launches issued in this backward (their scratch buffers' keys)

    def __enter__(self):
        global _SINK
        _SINK = self
        return self

    def __exit__(self, *exc):
        global _SINK
        _SINK = None
        return False

    def _grad(self, p):
        if id(p) in self.owned:
            raise RuntimeError("GradSink: a parameter's gradient was recorded twice")
        self.owned.add(id(p))
        g = self.buf.get(id(p))
        if g is None:
            g = self.buf[id(p)] = (p, torch.empty_like(p, memory_format=torch.contiguous_format))
        return g[1]

    def wgrad(self, x2d, dz2d, p):
        """grad(p) = x2d^T @ dz2d (p viewed as [K, N])."""
        M, K = x2d.shape
        N = dz2d.shape[1]
        g = self._grad(p)
        if g.numel() != K * N or x2d.stride(1) != 1 or dz2d.stride(1) != 1 or dz2d.shape[0] != M:
            raise ValueError("GradSink.wgrad: shapes / layouts do not match the parameter")
        self.keep += [x2d, dz2d]
        self.wg.append((x2d.data_ptr(), dz2d.data_ptr(), g.data_ptr(), M, K, N, x2d.stride(0), dz2d.stride(0)))

    def ln_colsum(self, scratch, N, gamma=None, beta=None, bias=None):
        """dgamma / dbeta / dbias from muz_ln_bwd_rows partials (any subset of the three)."""
        outs = [0 if q is None else self._grad(q).data_ptr() for q in (gamma, beta, bias)]
        self.keep.append(scratch)
        self.cs.append((scratch.data_ptr(), *outs, 0, scratch.numel() // (3 * N), N, N))

    def colsum(self, dz2d, p):
        """grad(p) = column sums of dz2d (a bias)."""
        g = self._grad(p)
        if dz2d.stride(1) != 1 or g.numel() != dz2d.shape[1]:
            raise ValueError("GradSink.colsum: layout")
        self.keep.append(dz2d)
        self.cs.append((dz2d.data_ptr(), g.data_ptr(), 0, 0, 1, dz2d.shape[0], dz2d.shape[1], dz2d.stride(0)))

    def _launch(self):
        """The grouped launches of everything recorded since the last one (on the side stream when ASYNC_GRADS)."""
        if not self.wg and not self.cs:
            return
        lib, cur = _L.load(), torch.cuda.current_stream()
        if ASYNC_GRADS:
            if self.side is None:
                self.side = torch.cuda.Stream(device=cur.device)
            self.side.wait_stream(cur)    # the recorded inputs are complete on the backward's stream
            stream = self.side
        else:
            stream = cur
        st = _L.stream_ptr(stream)
        if self.wg:
            arr = (_L.MuzWgradProblem * len(self.wg))(*[_L.MuzWgradProblem(*w) for w in self.wg])
            need = lib.muz_wgrad_scratch_floats(arr, len(self.wg))
            sc = self.scratch.get(self.nlaunch)
            if sc is None or sc.numel() < need:    # kept: a captured graph replays into it
                with torch.cuda.stream(stream):
                    sc = self.scratch[self.nlaunch] = torch.empty((max(need, 1),), dtype=torch.float32,
                                                                  device=self.keep[0].device)
            _L.check(lib.muz_wgrad_grouped(arr, len(self.wg), _L.ptr(sc), sc.numel(), st), "muz_wgrad_grouped")
        if self.cs:
            arr = (_L.MuzColsumProblem * len(self.cs))(*[_L.MuzColsumProblem(*c) for c in self.cs])
            _L.check(lib.muz_colsum_grouped(arr, len(self.cs), st), "muz_colsum_grouped")
        self.wg, self.cs = [], []
        self.nlaunch += 1

    def flush_early(self):
        """Called by a backward node before / after a long launch of its own (the trunk chain on 8 CUs): the
        gradients recorded so far are formed on the side stream meanwhile.  No-op unless ASYNC_GRADS."""
        if ASYNC_GRADS:
            self._launch()

    def flush(self):
        self._launch()
        if self.side is not None and ASYNC_GRADS:
            # the recorded tensors (self.keep) stay referenced until here, after the join
            torch.cuda.current_stream().wait_stream(self.side)
        self.nlaunch = 0
        for p, g in self.buf.values():
            if id(p) in self.owned:
                if p.grad is not None and p.grad is not g:
                    # the parameter also reached autograd through a plain torch op: keep that term
                    g.add_(p.grad)
                p.grad = g
        self.wg, self.cs, self.keep, self.owned = [], [], [], set()


class _transposed:
    """with _transposed(wt): refresh the W^T copies, then run the forward with them (no-op for None)."""

    def __init__(self, wt):
        self.wt = wt

    def __enter__(self):
        if self.wt is not None:
            self.wt.refresh()
            self.wt.__enter__()

    def __exit__(self, *exc):
        if self.wt is not None:
            self.wt.__exit__()
        return False


_UNIT = {}


def _unit_grad(like):
    """A cached scalar 1 (filled on the eager warm-up step): the learner's root gradient, so _LossHeads can hand its
    saved output gradients on without a scaling launch and autograd fills no ones tensor."""
    key = (like.device, like.dtype)
    v = _UNIT.get(key)
    if v is None:
        v = _UNIT[key] = torch.ones((), dtype=like.dtype, device=like.device)
    return v


def _backward(loss, sink):
    """loss.backward() with the parameter gradients formed by `sink`'s grouped launches (None: by autograd)."""
    if sink is None:
        loss.backward(_unit_grad(loss))
        return
    with sink:
        loss.backward(_unit_grad(loss))
    sink.flush()


FUSED_LOSS = True      # False: the losses as torch ops (A/B timing, and the fused kernel's test reference)
FUSED_HEADS = True     # False: the output heads as library GEMMs + torch activations (A/B timing, test reference)
GROUPED_GRADS = True   # False: every weight / bias / LayerNorm gradient as its own launch (A/B timing)
# MUZ_ASYNC_GRADS=1: the grouped gradient launches on a side stream, the ones recorded before / during the trunk
# chain's backward overlapping it and the representation's backward.  Off: measured slower (1.607 -> 1.741 ms per det
# step, profiles/r5y_async_grads.log -- k_chain_bwd 429 -> 475 us beside the gradient launches on its CUs)
ASYNC_GRADS = os.environ.get("MUZ_ASYNC_GRADS", "0") == "1"
_SINK = None     # the active GradSink (module-global: autograd runs GPU backward nodes on its own thread)


def _sink():
    return _SINK


_RB_PARAMS = ("Dense_0/kernel", "Dense_0/bias", "LayerNorm_0/scale", "LayerNorm_0/bias",
              "Dense_1/kernel", "Dense_1/bias", "LayerNorm_1/scale", "LayerNorm_1/bias")


def trunk_param_names(kind: str = "det") -> list:
    """The 28 parameters of one FiLM trunk, in _TrunkChain's order: input LayerNorm, two Dense + LayerNorm
    layers, two ResBlocks, the projection.  kind "det": DynamicsNetwork4 (muzero_deterministic_madn.py:
    391-457); "act" / "chance": the afterstate / chance trunks of StochasticDynamicsNetwork4
    (muzero_classic_madn.py:329-408; ResBlocks 0-1 / 2-3)."""
    d = "dynamics"
    if kind == "det":
        head = ["LayerNorm_0/scale", "LayerNorm_0/bias", "Dense_3/kernel", "Dense_3/bias", "LayerNorm_1/scale",
                "LayerNorm_1/bias", "Dense_4/kernel", "Dense_4/bias", "LayerNorm_2/scale", "LayerNorm_2/bias"]
        rbs, tail = (0, 1), ["Dense_5/kernel", "Dense_5/bias"]
    elif kind in ("act", "chance"):
        head = [f"{kind}_{n}" for n in ("input_ln/scale", "input_ln/bias", "dense1/kernel", "dense1/bias",
                                        "ln1/scale", "ln1/bias", "dense2/kernel", "dense2/bias", "ln2/scale",
                                        "ln2/bias")]
        rbs, tail = ((0, 1) if kind == "act" else (2, 3)), [f"{kind}_proj/kernel", f"{kind}_proj/bias"]
    else:
        raise ValueError(f"unknown trunk kind {kind!r}")
    return [f"{d}/{n}" for n in head] + [f"{d}/ResBlock_{r}/{n}" for r in rbs for n in _RB_PARAMS] + \
        [f"{d}/{n}" for n in tail]


DYN_TRUNK_PARAMS = tuple(trunk_param_names("det"))


# ---- one packing launch per step for every persistent GEMM kernel's weights ----------------------------------------
# _ResStack (representation, prediction) and the trunk chain each repacked their weights into MFMA operand order with
# a launch of their own (3 per step).  prepack() packs all of them with ONE muz_trunk_chain_pack at the top of the
# loss; each forward finds its slice by the weights' data pointers (a forward whose weights were not pre-packed packs
# them itself, as before).  The buffer is kept by the caller (a captured graph replays into it).
_PACKED = {}


def prepack(weight_lists, keep):
    """Pack the lists of [256, 256] weights (each one consumer's, in its layer order) with one launch; ``keep``:
    a dict owned by the caller that holds the buffer across graph replays."""
    _PACKED.clear()
    ws = [w for lst in weight_lists for w in lst]
    if not ws or not all(w.is_cuda and w.dtype == torch.float32 and tuple(w.shape) == (256, 256) for w in ws):
        return
    n = len(ws)
    WP = keep.get("WP")
    if WP is None or WP.shape[1] != n:
        WP = keep["WP"] = torch.empty((2, n, 256 * 256), dtype=torch.float32, device=ws[0].device)
    src = (ctypes.c_void_p * n)(*[w.data_ptr() for w in ws])
    _L.check(_L.load().muz_trunk_chain_pack(src, n, _L.ptr(WP[0]), _L.ptr(WP[1]), _L.stream_ptr()),
             "muz_trunk_chain_pack")
    o = 0
    for lst in weight_lists:
        _PACKED[tuple(w.data_ptr() for w in lst)] = WP[:, o:o + len(lst)]
        o += len(lst)


def _packed(ws):
    """The pre-packed [2, len(ws), 65536] slice of these weights (prepack), or None."""
    return _PACKED.get(tuple(w.data_ptr() for w in ws))


def _rbstack_weights(p, name, nb):
    return [p[f"{name}{b}/Dense_{k}/kernel"] for b in range(nb) for k in range(2)]


def _cat0(ts):
    """torch.cat(ts, 0), without the copy when ts is one tensor already (the chain's stacked latents)."""
    return ts[0] if len(ts) == 1 else torch.cat(ts, 0)


def _prepack_nets(nets):
    """prepack() of the det / DOG loss's three packed consumers: the representation's six ResBlocks, the dynamics trunk
    chain, the prediction's two ResBlocks (whichever the parameter set has; the lists _PACKED serves are cleared again
    once the loss's forward is built)."""
    p = nets.p
    if not (RESBLOCK_STACK and CHAIN and p[DYN_TRUNK_PARAMS[_CHAIN_W[0]]].is_cuda):
        return
    lists = []
    for name, nb in (("representation/ResBlock_", 6), ("prediction/ResBlock_", 2)):
        if all(f"{name}{b}/Dense_{k}/kernel" in p for b in range(nb) for k in range(2)) and f"{name}{nb}/Dense_0/kernel" not in p:
            lists.append(_rbstack_weights(p, name, nb))
    if all(n in p for n in DYN_TRUNK_PARAMS):
        lists.append([p[DYN_TRUNK_PARAMS[k]] for k in _CHAIN_W])
    keep = nets.__dict__.setdefault("_packkeep", {})
    prepack(lists, keep)
CHAIN = True                     # False: the losses build the per-step autograd graph instead (A/B timing)
STACK_LATENTS = True             # the det loss takes the chain's output as the stacked latents (False: torch.cat, A/B)
FUSED_FILM = True                # False: a trunk's LayerNorm_0 + FiLM as LayerNorm + addcmul (A/B, diagnosis)
FUSED_BOUNDARY = True            # False: min-max of application i and LayerNorm_0 + FiLM of i + 1 as separate launches
_NP = len(DYN_TRUNK_PARAMS)      # 28 per trunk


_GEMM_LAYERS = ("3", "4", "a0", "b0", "a1", "b1", "5")   # the trunk's weight layers, named by their input


# weight layer (named by its input) -> indices of (kernel, bias, LN scale, LN bias) in trunk_param_names order
_TRUNK_LAYER_PARAMS = (("3", (2, 3, 4, 5)), ("4", (6, 7, 8, 9)), ("a0", (10, 11, 12, 13)), ("b0", (14, 15, 16, 17)),
                       ("a1", (18, 19, 20, 21)), ("b1", (22, 23, 24, 25)))


def _slots(apps, ngroups):
    """-> (slot, seen): application i's index among its group's applications, and each group's count."""
    slot, seen = [], [0] * ngroups
    for g in apps:
        slot.append(seen[g])
        seen[g] += 1
    return slot, seen


class _TrunkChain(torch.autograd.Function):
    """The sequential FiLM-trunk applications of an unrolled loss as ONE autograd node.  Application i maps
    x_i -> x_{i+1} = minmax(x_i + proj(trunk(LN(x_i) * (1 + scale_i) + shift_i))) with trunk group apps[i]'s
    weights; the gradient reaching x_{i+1} is scaled by grad_scale where scaled[i].  det loss_fn: one group,
    apps = (0,) * K, all scaled (train_with_reward.py:98-107); classic loss_fn_stochastic: groups (act, chance),
    apps = (0, 1) * K, only the chance outputs (the new states) scaled (train_stochastic.py:95-121).
    heads=True adds a second output with the same values whose gradient is NOT scaled: the det reward /
    discount heads read the next latent inside dynamics_net, before the scaling (train_with_reward.py:49-105).

    Forward = the fused kernels of csrc/learner_ln.hip + library GEMMs; the hand-written backward walks the
    applications in reverse and, because a group's weights are shared by all its applications, forms each
    weight gradient with ONE GEMM and each LayerNorm / bias gradient with ONE column sum per group (per-step
    autograd made K GEMMs, K column sums and K - 1 accumulation adds per parameter).  min / max split their
    gradient evenly over tied columns (JAX's reduce_min / reduce_max rule).  Inputs: x_0 [B, 256], FiLM scale / shift [T, B, 256],
    the groups' parameters concatenated, each in trunk_param_names order.  Output: x_1..x_T as [T, B, 256]
    (and its unscaled-gradient twin when heads)."""

    @staticmethod
    def forward(ctx, latent0, scale, shift, grad_scale, apps, scaled, heads, *P):
        T, B, Nn = scale.shape
        if len(apps) != T or len(scaled) != T or len(P) != _NP * (max(apps) + 1):
            raise ValueError("apps / scaled / parameters do not match the FiLM rows")
        dev, dt = latent0.device, latent0.dtype
        # heads == 2 (the det loss): the first output is the stack [latent0, x_1 .. x_T] the prediction reads whole
        # (no torch.cat of the latents, no unbind / stack in the backward), the twin written by the chain kernel
        # itself (no clone), the stack's block-0 gradient added to d latent0 inside the backward kernel
        stack = heads == 2
        full = torch.empty((T + 1, B, Nn), dtype=dt, device=dev) if stack else None
        outs = full[1:] if stack else torch.empty((T, B, Nn), dtype=dt, device=dev)
        qs = torch.empty((T, B, Nn), dtype=dt, device=dev)                  # min-max inputs and their extrema
        lohi = torch.empty((T, B, 2), dtype=dt, device=dev)
        idx = torch.empty((T, B, 2), dtype=torch.int32, device=dev)
        src = scale if scale._base is None else scale._base     # (_Film's output, or the view the loss passes)
        scale1 = getattr(src, "_muz_scale1", None)
        if scale1 is None or scale1.numel() != scale.numel() or src.data_ptr() != scale.data_ptr():
            scale1 = 1.0 + scale
        else:
            scale1 = scale1.view(scale.shape)
        lib = _L.load()
        st = []
        slot, seen = _slots(apps, len(P) // _NP)
        # every weight layer's inputs of all applications of a group, stacked [apps, B, N]: each layer writes
        # its output straight into the next layer's block, so the backward's weight gradient is one GEMM
        # over the stack without concatenating anything
        X = {(g, n): torch.empty((max(seen[g], 1), B, Nn), dtype=dt, device=dev)
             for g in range(len(seen)) for n in _GEMM_LAYERS}
        lat = latent0.contiguous()
        ctx.chain = None
        ctx.stack = stack
        if _chain_usable(T, B, Nn, len(seen)):
            twin = torch.empty_like(outs) if stack else None
            ctx.chain = _chain_forward(lat, scale1, shift.contiguous(), apps, slot, scaled, P, X, outs, qs, lohi, idx,
                                       twin=twin, stack0=full[0] if stack else None)
            ctx.X, ctx.P, ctx.grad_scale, ctx.apps = X, P, float(grad_scale), tuple(apps)
            # outs (a view of full when stacked): read by the backward kernel (a.out); the output itself is saved
            ctx.save_for_backward(scale1, qs, lohi, full if stack else outs)
            if stack:
                return full, twin
            return (outs, outs.clone()) if heads else outs
        f0_next = None    # LayerNorm_0 + FiLM of the next application, formed by the boundary launch
        for i in range(T):
            g, j = apps[i], slot[i]
            Q = P[_NP * g:_NP * (g + 1)]
            g0, be0, W3, b3, g1, be1, W4, b4, g2, be2 = Q[:10]
            x0 = X[(g, "3")][j]
            if f0_next is not None:
                f0 = f0_next
            elif FUSED_FILM:    # LayerNorm_0 + FiLM, one launch
                f0 = _ln_film_fwd(lat, g0, be0, scale1[i], shift[i], x0)
            else:
                f0 = _ln_fwd(lat, torch.zeros_like(g0), g0, be0, None, LN_PLAIN)
                torch.addcmul(shift[i], f0[0], scale1[i], out=x0)
            f3 = _dense_ln_fwd(x0, W3, b3, g1, be1, None, LN_RELU, out=X[(g, "4")][j])
            f4 = _dense_ln_fwd(f3[0], W4, b4, g2, be2, None, LN_RELU, out=X[(g, "a0")][j])
            x, rbs = f4[0], []
            for r in range(2):
                Wa, ba, ga, bea, Wb, bb, gb, beb = Q[10 + 8 * r:18 + 8 * r]
                fa = _dense_ln_fwd(x, Wa, ba, ga, bea, None, LN_RELU, out=X[(g, f"b{r}")][j])
                fb = _dense_ln_fwd(fa[0], Wb, bb, gb, beb, x, LN_RESID_RELU, out=X[(g, "a1" if r == 0 else "5")][j])
                rbs.append((x, fa, fb))
                x = fb[0]
            y5 = x @ Q[26]
            if FUSED_BOUNDARY and FUSED_FILM and i + 1 < T:   # min-max of i + LayerNorm_0 / FiLM of i + 1
                gn, jn = apps[i + 1], slot[i + 1]
                Qn = P[_NP * gn:_NP * (gn + 1)]
                f0_next = (torch.empty_like(lat), torch.empty_like(lat), torch.empty((B,), dtype=dt, device=dev),
                           torch.empty((B,), dtype=dt, device=dev))
                _L.check(lib.muz_minmax_film_fwd(
                    _L.ptr(lat), _L.ptr(y5), _L.ptr(Q[27]), B, Nn, _L.ptr(outs[i]), _L.ptr(qs[i]), _L.ptr(lohi[i]),
                    _L.ptr(idx[i]), _L.ptr(Qn[0]), _L.ptr(Qn[1]), _L.ptr(scale1[i + 1]), _L.ptr(shift[i + 1].contiguous()),
                    *(_L.ptr(t) for t in f0_next), _L.ptr(X[(gn, "3")][jn]), _L.stream_ptr()), "muz_minmax_film_fwd")
            else:
                f0_next = None
                _L.check(lib.muz_minmax_fwd(_L.ptr(lat), _L.ptr(y5), _L.ptr(Q[27]), B, Nn, _L.ptr(outs[i]),
                                            _L.ptr(qs[i]), _L.ptr(lohi[i]), _L.ptr(idx[i]), _L.stream_ptr()),
                         "muz_minmax_fwd")
            st.append((f0, x0, f3, f4, rbs, x))
            lat = outs[i]
        ctx.st, ctx.X, ctx.P, ctx.grad_scale = st, X, P, float(grad_scale)
        ctx.boundary = FUSED_BOUNDARY and FUSED_FILM
        ctx.apps, ctx.scaled = tuple(apps), tuple(scaled)
        ctx.save_for_backward(scale1, qs, lohi)
        if stack:
            full[0].copy_(latent0)
            return full, outs.clone()
        return (outs, outs.clone()) if heads else outs

    @staticmethod
    def backward(ctx, G, H=None):
        scale1, qs, lohi = ctx.saved_tensors[:3]
        T, B, Nn = scale1.shape
        G0 = None
        if getattr(ctx, "stack", False):   # G: the stack's gradient [T + 1, B, N]; block 0 belongs to latent0
            G = G.contiguous()
            G0, G = G[0], G[1:]
        G = G.contiguous()
        H = None if H is None else H.contiguous()
        if ctx.chain is not None:
            sink = _sink()
            if sink is not None:     # the heads' / prediction stack's gradients run beside the chain kernel
                sink.flush_early()
            dlat, dscale, dshift, DZ, scr = _chain_backward(ctx.chain, G, H, ctx.grad_scale, ctx.apps, ctx.P, B, Nn,
                                                            G0=G0)
            grads = _trunk_param_grads(ctx.X, DZ, scr, ctx.P, _slots(ctx.apps, len(ctx.P) // _NP)[1], Nn)
            if sink is not None:     # the chain's own beside the representation's backward
                sink.flush_early()
            return (dlat, dscale, dshift, None, None, None, None, *grads)
        P, st, s, apps = ctx.P, ctx.st, ctx.grad_scale, ctx.apps
        dev, dt = G.device, G.dtype
        lib = _L.load()
        nf = {n: lib.muz_ln_bwd_scratch_floats(B, Nn) if n == "0" else _ln_scratch_floats(B, Nn, Nn)
              for n in ("0", "3", "4", "a0", "b0", "a1", "b1")}
        ngroups = len(P) // _NP
        slot, seen = _slots(apps, ngroups)       # application i's row in its group's stacked buffers
        layers = ("0", "3", "4", "a0", "b0", "a1", "b1")
        scr = {(g, n): torch.empty((max(seen[g], 1), nf[n]), dtype=dt, device=dev) for g in range(ngroups) for n in layers}
        # output gradients of the weight layers, stacked like the forward's inputs (ctx.X)
        DZ = {(g, n): torch.empty((max(seen[g], 1), B, Nn), dtype=dt, device=dev)
              for g in range(ngroups) for n in _GEMM_LAYERS}
        dscale, dshift = torch.empty_like(scale1), torch.empty_like(scale1)
        ca = cb = None                            # the carried gradient of x_{i+1}: ca + cb
        for i in range(T - 1, -1, -1):
            g, j = apps[i], slot[i]
            Q = P[_NP * g:_NP * (g + 1)]
            f0, x0, f3, f4, rbs, x5 = st[i]
            dq = DZ[(g, "5")][j]
            if not (ctx.boundary and i + 1 < T):   # (else formed by application i + 1's boundary launch)
                _L.check(lib.muz_minmax_bwd(_L.ptr(G[i]), _L.ptr(ca), _L.ptr(cb), _L.ptr(None if H is None else H[i]),
                                            s, int(ctx.scaled[i]), _L.ptr(qs[i]), _L.ptr(lohi[i]), B, Nn, _L.ptr(dq),
                                            _L.stream_ptr()), "muz_minmax_bwd")
            dx = dq @ Q[26].t()
            for r in (1, 0):
                xin, fa, fb = rbs[r]
                Wa, ga, Wb, gb = Q[10 + 8 * r], Q[12 + 8 * r], Q[14 + 8 * r], Q[16 + 8 * r]
                _, dres, t = _dense_ln_bwd(dx, fb, gb, LN_RESID_RELU, Wb, scr[(g, f"b{r}")][j], DZ[(g, f"b{r}")][j])
                # dres + dza Wa^T, the residual accumulated inside the same launch
                _, _, dx = _dense_ln_bwd(t, fa, ga, LN_RELU, Wa, scr[(g, f"a{r}")][j], DZ[(g, f"a{r}")][j], acc=dres)
            _, _, t = _dense_ln_bwd(dx, f4, Q[8], LN_RELU, Q[6], scr[(g, "4")][j], DZ[(g, "4")][j])
            _, _, dx0 = _dense_ln_bwd(t, f3, Q[4], LN_RELU, Q[2], scr[(g, "3")][j], DZ[(g, "3")][j], dx_out=dshift[i])
            if ctx.boundary and i >= 1:   # LayerNorm_0 / FiLM backward of i + min-max backward of i - 1
                gp, jp = apps[i - 1], slot[i - 1]
                _L.check(lib.muz_film_minmax_bwd(
                    _L.ptr(dx0.contiguous()), *(_L.ptr(t) for t in f0), _L.ptr(Q[0]), _L.ptr(scale1[i]), B, Nn,
                    _L.ptr(dscale[i]), _L.ptr(scr[(g, "0")][j]), _L.ptr(G[i - 1]), _L.ptr(dq),
                    _L.ptr(None if H is None else H[i - 1]), s, int(ctx.scaled[i - 1]), _L.ptr(qs[i - 1]),
                    _L.ptr(lohi[i - 1]), _L.ptr(DZ[(gp, "5")][jp]), _L.stream_ptr()), "muz_film_minmax_bwd")
                ca = cb = None
                continue
            if FUSED_FILM:
                dz0 = _ln_film_bwd_rows(dx0, f0, Q[0], scale1[i], scr[(g, "0")][j], dscale[i])
            else:
                torch.mul(dx0, f0[0], out=dscale[i])
                dz0, _ = _ln_bwd_rows(dx0 * scale1[i], f0, Q[0], LN_PLAIN, scr[(g, "0")][j])
            ca, cb = dz0, dq
        grads = _trunk_param_grads(ctx.X, DZ, scr, P, seen, Nn)
        dlat = ca + cb
        return (dlat if G0 is None else dlat + G0, dscale, dshift, None, None, None, None, *grads)


def _trunk_param_grads(X, DZ, scr, P, seen, Nn):
    """The chain's parameter gradients from the stacked layer inputs X, output gradients DZ and LayerNorm
    column partials scr (keys (group, layer input name)): one weight-gradient GEMM and one column sum per
    parameter over all of a group's applications -- recorded into the active GradSink, or formed here."""
    ngroups = len(P) // _NP
    grads = [None] * len(P)
    sink = _sink()
    for g in range(ngroups):
        if not seen[g]:
            grads[_NP * g:_NP * (g + 1)] = [torch.zeros_like(p) for p in P[_NP * g:_NP * (g + 1)]]
            continue
        o = _NP * g
        if sink is not None:       # the same gradients, formed by the sink's grouped launches after backward
            Q = P[o:o + _NP]
            sink.ln_colsum(scr[(g, "0")], Nn, Q[0], Q[1])
            for n, (iw, ib, ig, ibe) in _TRUNK_LAYER_PARAMS:
                Xs, Ds = (t[(g, n)][:seen[g]].reshape(-1, Nn) for t in (X, DZ))
                sink.wgrad(Xs, Ds, Q[iw])
                sink.ln_colsum(scr[(g, n)], Nn, Q[ig], Q[ibe], Q[ib])
            Xs, Ds = (t[(g, "5")][:seen[g]].reshape(-1, Nn) for t in (X, DZ))
            sink.wgrad(Xs, Ds, Q[26])
            sink.colsum(Ds, Q[27])
            continue
        grads[o], grads[o + 1], _ = _ln_colsum(scr[(g, "0")], Nn)
        for n, (iw, ib, ig, ibe) in _TRUNK_LAYER_PARAMS:
            Xs, Ds = (t[(g, n)][:seen[g]].reshape(-1, Nn) for t in (X, DZ))
            grads[o + iw] = Xs.t() @ Ds
            grads[o + ig], grads[o + ibe], grads[o + ib] = _ln_colsum(scr[(g, n)], Nn)
        Xs, Ds = (t[(g, "5")][:seen[g]].reshape(-1, Nn) for t in (X, DZ))
        grads[o + 26], grads[o + 27] = Xs.t() @ Ds, torch.mv(Ds.t(), _ones(Ds.shape[0], Ds))
    return grads


# csrc/learner_chain.hip: the whole chain as one launch each way (muz_trunk_chain_fwd / _bwd)
CHAIN_KERNEL = True              # False: the per-layer launch train below (A/B timing; the kernels' test reference)
_CHAIN_W = (2, 6, 10, 14, 18, 22, 26)          # trunk_param_names index of each weight layer's kernel (bias + 1,
                                               # LayerNorm scale / bias + 2 / + 3)
_CHAIN_PARTS = ("0",) + _GEMM_LAYERS[:6]       # the kernels' part[] order: LayerNorm_0, then the 6 Dense + LN layers


def _chain_usable(T, B, Nn, ngroups):
    return CHAIN_KERNEL and Nn == 256 and 1 <= T <= _L.MUZ_CHAIN_MAX_T and 1 <= ngroups <= 2 and B > 0


class _Chain:
    """What _chain_forward hands to _chain_backward: the filled muz_chain_args and the buffers it points at."""

    def __init__(self, args, keep):
        self.args, self.keep = args, keep


def _chain_forward(lat, scale1, shift, apps, slot, scaled, P, X, outs, qs, lohi, idx, twin=None, stack0=None):
    """muz_trunk_chain_fwd over all applications: writes outs / qs / lohi / idx and the stacks X like the
    per-layer path, plus the LayerNorm outputs / pre-LayerNorm values / statistics its backward reads."""
    T, B, Nn = scale1.shape
    ngroups = len(P) // _NP
    dev, dt = lat.device, lat.dtype
    lib = _L.load()
    # both GEMM directions stream the weights as packed MFMA operands, repacked here every call (one launch)
    WP = _packed([P[_NP * g + k] for g in range(ngroups) for k in _CHAIN_W])
    if WP is not None:
        WP = WP.view(2, ngroups, 7, Nn * Nn)
    else:
        WP = torch.empty((2, ngroups, 7, Nn * Nn), dtype=dt, device=dev)
        src = (ctypes.c_void_p * (7 * ngroups))(*[P[_NP * g + k].data_ptr() for g in range(ngroups) for k in _CHAIN_W])
        _L.check(lib.muz_trunk_chain_pack(src, 7 * ngroups, _L.ptr(WP[0]), _L.ptr(WP[1]), _L.stream_ptr()),
                 "muz_trunk_chain_pack")
    ln0 = torch.empty((T, B, Nn), dtype=dt, device=dev)
    z = torch.empty((T, 6, B, Nn), dtype=dt, device=dev)
    stats = torch.empty((T, 7, 2, B), dtype=dt, device=dev)
    a = _L.MuzChainArgs()
    a.T, a.M, a.ngroups = T, B, ngroups
    for i in range(T):
        a.app[i], a.slot[i], a.scaled[i] = apps[i], slot[i], int(scaled[i])
    for g in range(ngroups):
        Q = P[_NP * g:_NP * (g + 1)]
        grp = a.group[g]
        grp.ln0_gamma, grp.ln0_beta = Q[0].data_ptr(), Q[1].data_ptr()
        for l, k in enumerate(_CHAIN_W):
            grp.wf[l], grp.wb[l], grp.bias[l] = WP[0, g, l].data_ptr(), WP[1, g, l].data_ptr(), Q[k + 1].data_ptr()
            grp.X[l] = X[(g, _GEMM_LAYERS[l])].data_ptr()
            if l < 6:
                grp.gamma[l], grp.beta[l] = Q[k + 2].data_ptr(), Q[k + 3].data_ptr()
    a.latent0, a.scale1, a.shift = lat.data_ptr(), scale1.data_ptr(), shift.data_ptr()
    a.out, a.q, a.lohi, a.idx = outs.data_ptr(), qs.data_ptr(), lohi.data_ptr(), idx.data_ptr()
    a.out_twin = 0 if twin is None else twin.data_ptr()
    a.stack0 = 0 if stack0 is None else stack0.data_ptr()
    a.ln0_out, a.z, a.stats = ln0.data_ptr(), z.data_ptr(), stats.data_ptr()
    _L.check(lib.muz_trunk_chain_fwd(ctypes.byref(a), _L.stream_ptr()), "muz_trunk_chain_fwd")
    # kept as long as the autograd node (a second backward, retain_graph, reads them again); outs is the node's output
    # and is held by its save_for_backward instead (an output stored on ctx would make an output -> ctx cycle)
    return _Chain(a, (WP, ln0, z, stats, lat, scale1, shift))


def _chain_backward(chain, G, H, grad_scale, apps, P, B, Nn, G0=None):
    """muz_trunk_chain_bwd: -> (d latent0, d scale, d shift, DZ stacks, LayerNorm partials) for
    _trunk_param_grads.  G0: the stacked form's block-0 gradient, added to d latent0 inside the kernel."""
    ngroups = len(P) // _NP
    seen = _slots(apps, ngroups)[1]
    T = len(apps)
    dev, dt = G.device, G.dtype
    tiles = (B + 15) // 16
    DZ = {(g, n): torch.empty((max(seen[g], 1), B, Nn), dtype=dt, device=dev)
          for g in range(ngroups) for n in _GEMM_LAYERS}
    scr = {(g, n): torch.empty((max(seen[g], 1), tiles * 3 * Nn), dtype=dt, device=dev)
           for g in range(ngroups) for n in _CHAIN_PARTS}
    dscale = torch.empty((T, B, Nn), dtype=dt, device=dev)
    dshift = torch.empty_like(dscale)
    dlat = torch.empty((B, Nn), dtype=dt, device=dev)
    a = chain.args
    for g in range(ngroups):
        grp = a.group[g]
        for l in range(7):
            grp.DZ[l] = DZ[(g, _GEMM_LAYERS[l])].data_ptr()
            grp.part[l] = scr[(g, _CHAIN_PARTS[l])].data_ptr()
    a.g, a.h = G.data_ptr(), (0 if H is None else H.data_ptr())
    a.g0 = 0 if G0 is None else G0.data_ptr()
    a.grad_scale = grad_scale
    a.dscale, a.dshift, a.dlatent0 = dscale.data_ptr(), dshift.data_ptr(), dlat.data_ptr()
    _L.check(_L.load().muz_trunk_chain_bwd(ctypes.byref(a), _L.stream_ptr()), "muz_trunk_chain_bwd")
    return dlat, dscale, dshift, DZ, scr


class MuZeroNets:
    """Flax-named fp32 parameters of (RepresentationNetwork2, DynamicsNetwork4, PredictionNetwork4)."""

    def __init__(self, params: dict, obs_channels: int, num_actions: int = 24, device="cuda",
                 dtype=torch.float32, shapes: dict | None = None):
        self.C, self.A = int(obs_channels), int(num_actions)
        shapes = N.param_shapes(self.C, self.A) if shapes is None else shapes
        if set(shapes) != set(params):
            raise ValueError("parameter names differ from nets.param_shapes")
        self.p = {k: torch.tensor(np.asarray(params[k]).reshape(shapes[k]), dtype=dtype, device=device,
                                  requires_grad=True) for k in shapes}

    def parameters(self):
        return list(self.p.values())

    def numpy(self) -> dict:
        return {k: v.detach().float().cpu().numpy() for k, v in self.p.items()}

    # ---- layers (oracle/nets.py restates the same Flax semantics) ----------------------------------
    def _dense(self, name, x):
        # (not addmm: torch routes a GEMM with a bias epilogue to hipBLASLt whatever the preferred BLAS, and
        # hipBLASLt's macro-tiles make these small GEMMs ~33 us each; see prefer_rocblas)
        if x.is_cuda:
            return _Dense.apply(x, self.p[f"{name}/kernel"], self.p[f"{name}/bias"])
        return x @ self.p[f"{name}/kernel"] + self.p[f"{name}/bias"]

    def _ln(self, name, x):
        # Flax computes the variance as E[x^2] - E[x]^2 (fast variance); the fused two-pass kernel agrees to
        # ~1e-7 relative on these activations (tests/test_learner.py holds the forward to 1e-5)
        return F.layer_norm(x, (x.shape[-1],), self.p[f"{name}/scale"], self.p[f"{name}/bias"], EPS_LN)

    def _ln_once(self, name, x):
        """_ln for a LayerNorm applied once per loss: one launch each way (_LN) on the GPU."""
        g, b = self.p[f"{name}/scale"], self.p[f"{name}/bias"]
        if FUSED_LN_ONCE and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.shape[1] in (32, 64, 128, 256):
            return _LN.apply(x, g, b)
        return self._ln(name, x)

    def _dense_ln(self, dense, ln, x, mode=LN_RELU, res=None, W=None):
        """act(LayerNorm(Dense(x))) (mode: LN_RELU, LN_RESID_RELU = relu(res + .), LN_PLAIN).  On the GPU the
        fused epilogue of csrc/learner_ln.hip; on the CPU (the host tests) the same layers as torch ops."""
        W = self.p[f"{dense}/kernel"] if W is None else W
        if x.is_cuda:
            lead, Nn = x.shape[:-1], W.shape[-1]
            r = None if res is None else res.reshape(-1, Nn).contiguous()
            own = (self.p[f"{dense}/kernel"], self.p[f"{dense}/bias"], self.p[f"{ln}/scale"], self.p[f"{ln}/bias"])
            out = _DenseLN.apply(x.reshape(-1, x.shape[-1]).contiguous(), W, *own[1:], r, mode, own)
            return out.reshape(*lead, Nn)
        y = self._ln(ln, x @ W + self.p[f"{dense}/bias"])
        return F.relu(y) if mode == LN_RELU else (F.relu(res + y) if mode == LN_RESID_RELU else y)

    def _conv_cols(self, name, x):
        """Flax Conv 'SAME', stride 1, NWC input [B, W, Cin]: the im2col matrix [B, W, K * Cin] and the kernel
        (K, Cin, Cout) as the [K * Cin, Cout] matrix, so the conv is one GEMM.  MIOpen's conv1d picks
        algorithms that accumulate with atomics (run-to-run different losses and gradients, measured:
        profiles/learner_determinism.py); the GEMM form is deterministic, so eager and graph-captured steps
        are bit-identical."""
        k = self.p[f"{name}/kernel"]
        K, Cin, Cout = k.shape
        if x.is_cuda:
            return _Im2col.apply(x, K), k.reshape(K * Cin, Cout)
        pl = (K - 1) // 2
        W = x.shape[1]
        xp = F.pad(x, (0, 0, pl, K - 1 - pl))
        return torch.cat([xp[:, d:d + W, :] for d in range(K)], dim=-1), k.reshape(K * Cin, Cout)

    def _rbs(self, name, nb, x):
        """ResBlocks name0 .. name{nb-1} in sequence: one _ResStack node on the GPU (RESBLOCK_STACK)."""
        if x.is_cuda and RESBLOCK_STACK and x.shape[-1] == 256 and 1 <= nb <= _L.MUZ_RBSTACK_MAX:
            own = tuple(self.p[f"{name}{b}/{n}"] for b in range(nb) for n in _RB_PARAMS)
            out = _ResStack.apply(x.reshape(-1, x.shape[-1]).contiguous(), own, *own)
            return out.reshape(x.shape)
        for b in range(nb):
            x = self._rb(f"{name}{b}", x)
        return x

    def _rb(self, name, x):
        if x.is_cuda and RESBLOCK_NODE:
            own = tuple(self.p[f"{name}/{n}"] for n in ("Dense_0/kernel", "Dense_0/bias", "LayerNorm_0/scale",
                                                        "LayerNorm_0/bias", "Dense_1/kernel", "Dense_1/bias",
                                                        "LayerNorm_1/scale", "LayerNorm_1/bias"))
            out = _ResBlockLN.apply(x.reshape(-1, x.shape[-1]).contiguous(), *own, own)
            return out.reshape(x.shape)
        y = self._dense_ln(f"{name}/Dense_0", f"{name}/LayerNorm_0", x, LN_RELU)
        return self._dense_ln(f"{name}/Dense_1", f"{name}/LayerNorm_1", y, LN_RESID_RELU, res=x)

    @staticmethod
    def _minmax(x):
        # amin / amax: the gradient of a tied extremum is split evenly, as jnp.min / jnp.max do
        lo = torch.amin(x, -1, keepdim=True)
        hi = torch.amax(x, -1, keepdim=True)
        return (x - lo) / (hi - lo + 1e-8)

    # ---- networks ------------------------------------------------------------------------------------
    def representation(self, obs):
        """RepresentationNetwork2: the trunk, then Dense_4 and the min-max scaling (muzero_deterministic_madn.py:
        139-140)."""
        r = "representation"
        h = self.representation_trunk(obs)
        if h.is_cuda and h.shape[-1] == 256 and self.p[f"{r}/Dense_4/kernel"].shape[1] == 256:
            return _DenseMinmax.apply(h.contiguous(), self.p[f"{r}/Dense_4/kernel"], self.p[f"{r}/Dense_4/bias"])
        return self._minmax(self._dense(f"{r}/Dense_4", h))

    def representation_trunk(self, obs):
        """RepresentationNetwork2 up to its last Dense: convolutions, global features, Dense_3 and 6 ResBlocks."""
        r = "representation"
        sp = obs[:, :6, :].transpose(1, 2)
        g = obs[:, 6:, 0]
        for i in range(3):
            cols, k = self._conv_cols(f"{r}/Conv_{i}", sp)
            sp = self._dense_ln(f"{r}/Conv_{i}", f"{r}/LayerNorm_{i}", cols, LN_RELU, W=k)
        flat = self._dense_ln(f"{r}/Dense_0", f"{r}/LayerNorm_3", sp.reshape(sp.shape[0], -1))
        g = self._dense_ln(f"{r}/Dense_1", f"{r}/LayerNorm_4", g)
        g = self._dense_ln(f"{r}/Dense_2", f"{r}/LayerNorm_5", g)
        h = self._dense_ln(f"{r}/Dense_3", f"{r}/LayerNorm_6", torch.cat([flat, g], -1))
        return self._rbs(f"{r}/ResBlock_", 6, h)

    def dynamics_film(self, action):
        """The action-only FiLM sub-graph of DynamicsNetwork4 (one_hot -> Dense_0 -> Dense_1 | Dense_2); it
        does not depend on the latent, so the learner evaluates it for all unroll steps in one batch."""
        d = "dynamics"
        W0 = self.p[f"{d}/Dense_0/kernel"]
        if FUSED_FILM_EMBED and W0.is_cuda and W0.dtype == torch.float32 and W0.shape[1] == 64 and \
                self.p[f"{d}/Dense_1/kernel"].shape == (64, 256):
            return _Film.apply(action, *(self.p[f"{d}/{n}"] for n in _FILM_PARAMS))
        if action.dim() == 2:       # a [B, K] batch view: rows step-major
            action = action.transpose(0, 1).reshape(-1)
        oh = (action.long()[:, None] == torch.arange(self.A, device=action.device)[None, :]).to(
            self.p[f"{d}/Dense_0/bias"].dtype)
        e = F.relu(self._dense(f"{d}/Dense_0", oh))
        return oh, self._dense(f"{d}/Dense_1", e), self._dense(f"{d}/Dense_2", e)

    def dynamics_trunk(self, latent, scale, shift):
        """latent -> next latent (the sequential part of the unroll)."""
        d = "dynamics"
        x = self._ln(f"{d}/LayerNorm_0", latent) * (1.0 + scale) + shift
        x = self._dense_ln(f"{d}/Dense_3", f"{d}/LayerNorm_1", x)
        x = self._dense_ln(f"{d}/Dense_4", f"{d}/LayerNorm_2", x)
        for b in range(2):
            x = self._rb(f"{d}/ResBlock_{b}", x)
        return self._minmax(latent + self._dense(f"{d}/Dense_5", x))

    def dynamics_heads(self, nxt, oh):
        """Reward / discount logits of (next latent, one_hot(action)); row-wise, so batchable over steps."""
        d = "dynamics"
        ri = torch.cat([nxt, oh], -1)
        rl = self._dense(f"{d}/reward_head", F.relu(self._dense(f"{d}/Dense_6", ri)))
        dl = self._dense(f"{d}/discount_head", F.relu(self._dense(f"{d}/Dense_7", ri)))
        return rl, dl

    def dynamics(self, latent, action):
        oh, scale, shift = self.dynamics_film(action)
        nxt = self.dynamics_trunk(latent, scale, shift)
        rl, dl = self.dynamics_heads(nxt, oh)
        return nxt, rl, dl

    def prediction_hidden(self, latent):
        """PredictionNetwork4 up to its heads: (policy hidden after LayerNorm_2, value hidden after LayerNorm_3)."""
        p = "prediction"
        x = self._ln_once(f"{p}/LayerNorm_0", latent)
        x = self._rbs(f"{p}/ResBlock_", 2, x)
        pol = self._dense_ln(f"{p}/Dense_0", f"{p}/LayerNorm_1", x)
        pol = self._dense_ln(f"{p}/Dense_1", f"{p}/LayerNorm_2", pol)
        return pol, self._dense_ln(f"{p}/Dense_3", f"{p}/LayerNorm_3", x)

    def prediction(self, latent):
        p = "prediction"
        x = self._ln_once(f"{p}/LayerNorm_0", latent)
        x = self._rbs(f"{p}/ResBlock_", 2, x)
        pol = self._dense_ln(f"{p}/Dense_0", f"{p}/LayerNorm_1", x)
        pol = self._dense_ln(f"{p}/Dense_1", f"{p}/LayerNorm_2", pol)
        logits = self._dense(f"{p}/Dense_2", pol)
        v = self._dense_ln(f"{p}/Dense_3", f"{p}/LayerNorm_3", x)
        v = F.relu(self._dense(f"{p}/Dense_4", v))
        return logits, torch.tanh(self._dense(f"{p}/Dense_5", v))


def loss_fn(nets: MuZeroNets, batch: dict, unroll_steps: int = 10, grad_scale: float = 0.5):
    """train_with_reward.py:24-141 -> (total_loss, (value_loss, policy_loss, discount_loss, reward_loss)).
    grad_scale: the gradient share carried through the unrolled latent (0.5 in the reference, line 106;
    the forward value does not depend on it)."""
    obs = batch["observations"].to(nets.p["prediction/Dense_5/bias"].dtype)
    _prepack_nets(nets)
    latent = nets.representation(obs)
    B, K = batch["actions"].shape
    dev = obs.device
    # Only the latent chain is sequential: the action FiLM rows, Pred4 on every step's latent and the
    # reward / discount heads are row-wise, so each runs once over all K (+1) steps stacked along the batch
    # (same per-row arithmetic as the step-by-step loop of the reference; far fewer kernel launches).
    oh, scale, shift = nets.dynamics_film(batch["actions"][:, :K])     # (rows step-major: k B + b)
    latents = [latent]
    # The reward / discount heads read the next latent inside dynamics_net (muzero_deterministic_madn.py:
    # 437-455), BEFORE the loss scales the gradient of the latent it carries on (line 105): the heads take
    # the unscaled outputs.
    if K and latent.is_cuda and CHAIN:     # the whole latent chain as one autograd node (fused kernels, batched weight grads)
        chain, raw = _TrunkChain.apply(latent, scale.reshape(K, B, -1), shift.reshape(K, B, -1), grad_scale,
                                       (0,) * K, (True,) * K, 2 if STACK_LATENTS else True,
                                       *(nets.p[n] for n in DYN_TRUNK_PARAMS))
        if STACK_LATENTS:            # chain = [latent, x_1 .. x_K] already stacked
            latents = [chain.reshape((K + 1) * B, -1)]
        else:
            latents += list(chain.unbind(0))
        head_in = raw.reshape(K * B, -1)
    else:
        raws = []
        for k in range(K):
            nxt = nets.dynamics_trunk(latents[-1], scale[k * B:(k + 1) * B], shift[k * B:(k + 1) * B])
            raws.append(nxt)
            latents.append((nxt * (1.0 - grad_scale)).detach() + nxt * grad_scale)   # gradient scaling (fwd identity)
        head_in = torch.cat(raws, 0) if K else None
    if K and obs.is_cuda and FUSED_HEADS and nets.A <= 32:
        pol_h, v_h = nets.prediction_hidden(_cat0(latents))
        logits_all, v_all, rl_all, dl_all = _OutHeads.apply(pol_h, v_h, head_in, oh,
                                                             *(nets.p[n] for n in HEAD_PARAMS))
    else:
        logits_all, v_all = nets.prediction(_cat0(latents))
        rl_all, dl_all = nets.dynamics_heads(head_in, oh) if K else (None, None)
    if obs.is_cuda and FUSED_LOSS:
        u = 1.0 / unroll_steps
        spec = dict(batch=batch, K=K, scale_value=u * VALUE_SCALING, scale_policy=u * POLICY_SCALING, norm=0,
                    terms=[(batch["discount_targets"], 0, 1.0, 0.1, u * DISCOUNT_SCALING),     # terminal 1.0, other 0.1
                           (batch["rewards"], 0, 0.1, 1.0, u * REWARD_SCALING)])               # neutral 0.1, win/lose 1.0
        total, parts = _LossHeads.apply(logits_all, v_all, dl_all, rl_all, None, spec)
        _PACKED.clear()
        return total, (parts[1], parts[2], parts[3], parts[4])
    _PACKED.clear()
    # The per-step losses, all K (+1) steps at once ([K+1, B] views; row k = unroll step k).
    disc_t, rew_t = batch["discount_targets"].int(), batch["rewards"].int()
    m = batch["masks"][:, :K + 1].transpose(0, 1).to(obs.dtype)
    v = v_all[:, 0].reshape(K + 1, B)
    l_value = torch.mean(m * (batch["target_values"][:, :K + 1].transpose(0, 1).to(obs.dtype) - v) ** 2, 1)
    logp = F.log_softmax(logits_all, -1).reshape(K + 1, B, -1)
    l_policy = torch.mean(m * -(batch["policies"][:, :K + 1].transpose(0, 1).to(obs.dtype) * logp).sum(-1), 1)
    zero = torch.zeros((), dtype=obs.dtype, device=dev)
    if K:
        l_rew = _balanced_ce_steps(rl_all, rew_t[:, :K].transpose(0, 1), m[:K], 1, 0.1, 1.0)    # neutral 0.1, win/lose 1.0
        l_disc = _balanced_ce_steps(dl_all, disc_t[:, :K].transpose(0, 1), m[:K], 1, 1.0, 0.1)  # terminal 1.0, other 0.1
    else:
        l_rew = l_disc = zero[None]
    total = ((1.0 / unroll_steps) * (VALUE_SCALING * l_value + POLICY_SCALING * l_policy)).sum() + \
        (1.0 / unroll_steps) * (DISCOUNT_SCALING * l_disc.sum() + REWARD_SCALING * l_rew.sum())
    return total, (l_value.sum(), l_policy.sum(), l_disc.sum(), l_rew.sum())


_TICKETS = {}


def _loss_ticket(dev):
    """The loss kernel's last-workgroup counter: zero between launches (the kernel resets it), one per device, kept
    alive so a captured graph replays with the same one.  Launches sharing it must not overlap: the learner's are
    ordered on one stream (its eager warm-up step completes before the capture).  Made on the first (eager) step --
    keyed by stream, the capture stream's own counter was a zero-fill launch inside every replayed step."""
    key = str(dev)
    t = _TICKETS.get(key)
    if t is None:
        t = _TICKETS[key] = torch.zeros((1,), dtype=torch.int32, device=dev)
    return t


class _LossHeads(torch.autograd.Function):
    """All losses of one unrolled batch and their gradients w.r.t. the network outputs as ONE launch
    (csrc/learner_loss.hip: muz_loss_heads; ~120 torch launches forward + backward before).  Forward computes
    the gradients too; backward scales them by the incoming gradient of the total (one foreach launch).
    spec: K, batch, scale_value, scale_policy, norm and terms = [(labels | probs, rare_not_one, w_rare, w_common,
    scale)] matching the logits tensors t0..t2.  -> (total, parts [6] = total, value, policy, term 0..2)."""

    @staticmethod
    def forward(ctx, logits, value, t0, t1, t2, spec):
        b, K = spec["batch"], spec["K"]
        B, A = b["masks"].shape[0], logits.shape[-1]
        dev, dt = logits.device, logits.dtype
        logits, value = logits.contiguous(), value.contiguous()
        a = _L.MuzLossArgs()
        a.K, a.B, a.A, a.T = K, B, A, b["masks"].shape[1]
        masks, tv, pol = (b[k].to(dt).contiguous() for k in ("masks", "target_values", "policies"))
        if tv.shape[1] != a.T or pol.shape[1] != a.T or pol.shape[2] != A or logits.shape[0] != (K + 1) * B:
            raise ValueError("_LossHeads: batch / output shapes disagree")
        dlogits, dvalue = torch.empty_like(logits), torch.empty_like(value)
        a.masks, a.target_values, a.policies = masks.data_ptr(), tv.data_ptr(), pol.data_ptr()
        a.value, a.logits, a.dvalue, a.dlogits = value.data_ptr(), logits.data_ptr(), dvalue.data_ptr(), dlogits.data_ptr()
        a.scale_value, a.scale_policy, a.norm = spec["scale_value"], spec["scale_policy"], spec["norm"]
        keep, dts = [masks, tv, pol, logits, value], []
        terms = [t for t in (t0, t1, t2) if t is not None]
        a.nterms = len(terms)
        for j, (t, (tgt, rare_not_one, w_rare, w_common, scale)) in enumerate(zip(terms, spec["terms"])):
            t = t.contiguous()
            # class labels as int32 [B, K] (reference-style batches may carry them as int64 / float);
            # distributions as float [B, K, ncls]
            tgt = (tgt.to(dt) if tgt.dim() == 3 else tgt.to(torch.int32)).contiguous()
            d = torch.empty_like(t)
            keep += [t, tgt]
            dts.append(d)
            q = a.term[j]
            q.logits, q.dlogits, q.ncls, q.ld = t.data_ptr(), d.data_ptr(), t.shape[-1], tgt.shape[1]
            if tgt.dtype == torch.int32:
                q.labels = tgt.data_ptr()
            else:
                q.probs = tgt.data_ptr()
                if tgt.shape[2] != t.shape[-1]:
                    raise ValueError("_LossHeads: target width")
            if t.shape[0] != K * B or tgt.shape[0] != B:
                raise ValueError("_LossHeads: term shapes")
            q.rare_not_one, q.w_rare, q.w_common, q.scale = int(rare_not_one), w_rare, w_common, scale
        parts = torch.empty((6,), dtype=dt, device=dev)
        total = torch.empty((), dtype=dt, device=dev)
        partials = torch.empty((5 * (K + 1),), dtype=dt, device=dev)
        a.parts, a.total, a.partials, a.ticket = parts.data_ptr(), total.data_ptr(), partials.data_ptr(), \
            _loss_ticket(dev).data_ptr()
        _L.check(_L.load().muz_loss_heads(ctypes.byref(a), _L.stream_ptr()), "muz_loss_heads")
        ctx.d = (dlogits, dvalue, *dts)
        ctx.present = tuple(t is not None for t in (t0, t1, t2))
        ctx.mark_non_differentiable(parts)
        ctx.set_materialize_grads(False)       # (no zero-filled gradient for `parts`)
        return total, parts

    @staticmethod
    def backward(ctx, g_total, g_parts):
        if g_total is None:
            return (None,) * 6
        if g_total.data_ptr() == _unit_grad(g_total).data_ptr():
            # the learner's own backward (_backward: loss.backward(_unit_grad)): the saved gradients are the answer
            it = iter(ctx.d[2:])
            return (ctx.d[0], ctx.d[1], *(next(it) if p else None for p in ctx.present), None)
        # out of place: the saved output gradients stay intact for a second backward (retain_graph, gradcheck)
        d = torch._foreach_mul(list(ctx.d), g_total)
        it = iter(d[2:])
        return (d[0], d[1], *(next(it) if p else None for p in ctx.present), None)


def _balanced_ce_steps(logits, labels, mask, special, w_special, w_other):
    """Per-class balanced cross-entropy (train_with_reward.py:54-86) of every unroll step at once:
    logits [K*B, n] (step-major), labels / mask [K, B] -> [K]."""
    Kk, B = labels.shape
    ce = F.cross_entropy(logits, labels.reshape(-1).long(), reduction="none").reshape(Kk, B)
    is_s = labels == special
    n_s = torch.clamp((mask * is_s).sum(1), min=1.0)
    n_o = torch.clamp((mask * ~is_s).sum(1), min=1.0)
    return (w_special * (mask * torch.where(is_s, ce, torch.zeros_like(ce))).sum(1) / n_s +
            w_other * (mask * torch.where(~is_s, ce, torch.zeros_like(ce))).sum(1) / n_o)


def lr_schedule(step: int, lr0: float = 0.005, steps_per_iteration: int = 2500) -> float:
    """optax.piecewise_constant_schedule (train_with_reward.py:361-368)."""
    lr = lr0
    for boundary, scale in ((30, 0.2), (60, 0.2), (85, 0.5)):
        if step >= boundary * steps_per_iteration:
            lr *= scale
    return lr


DET_LR_BOUNDARIES = ((30, 0.2), (60, 0.2), (85, 0.5))          # train_with_reward.py:361-368
CLASSIC_LR_BOUNDARIES = ((40, 0.1), (85, 0.2), (105, 0.5))     # train_stochastic.py:415-422


def _lr_from_count(count: torch.Tensor, lr0=0.005, steps_per_iteration=2500,
                   boundaries=DET_LR_BOUNDARIES) -> torch.Tensor:
    """lr_schedule on a device step counter (no host sync: capturable in a HIP graph)."""
    lr = torch.full_like(count, lr0)
    for boundary, scale in boundaries:
        lr = torch.where(count >= boundary * steps_per_iteration, lr * scale, lr)
    return lr


class AdamW:
    """optax.chain(clip_by_global_norm(5.0), adamw(schedule, b1 0.9, b2 0.999, eps 1e-8, weight_decay 1e-4)).

    Multi-tensor (torch._foreach_*) updates with every scalar (step count, learning rate, bias corrections,
    clip factor) kept on the device, so a whole train step can be captured in one HIP graph."""

    def __init__(self, params: list, max_norm=5.0, b1=0.9, b2=0.999, eps=1e-8, wd=1e-4, lr0=0.005,
                 steps_per_iteration=2500, boundaries=DET_LR_BOUNDARIES):
        self.params = params
        self.mu = [torch.zeros_like(p) for p in params]
        self.nu = [torch.zeros_like(p) for p in params]
        dev, dt = params[0].device, params[0].dtype
        self.count = torch.zeros((), dtype=torch.float64, device=dev)
        self.max_norm, self.b1, self.b2, self.eps, self.wd = max_norm, b1, b2, eps, wd
        self.lr0, self.spi, self.boundaries = lr0, steps_per_iteration, boundaries
        self.dt = dt

        self._fused = None
        if dev.type == "cuda":
            import ctypes
            n = len(params)
            if dt != torch.float32 or any(not p.is_contiguous() for p in params) or len(boundaries) > 4:
                raise ValueError("AdamW on the GPU takes contiguous float32 parameters and <= 4 lr boundaries")
            numel = (ctypes.c_int64 * n)(*[p.numel() for p in params])
            nbytes = _L.load().muz_adamw_scratch_bytes(n, numel)
            self._fused = dict(
                n=n, numel=numel, scratch=torch.empty((nbytes,), dtype=torch.uint8, device=dev),
                gnorm=torch.zeros((), dtype=torch.float32, device=dev),
                p=(ctypes.c_void_p * n)(*[q.data_ptr() for q in params]),
                m=(ctypes.c_void_p * n)(*[q.data_ptr() for q in self.mu]),
                v=(ctypes.c_void_p * n)(*[q.data_ptr() for q in self.nu]),
                bounds=(ctypes.c_double * max(1, 2 * len(boundaries)))(*[float(x) for b in boundaries for x in b]),
                gtype=ctypes.c_void_p * n, tables={}, max_tables=8)

    @torch.no_grad()
    def step(self):
        if self._fused is not None:
            # csrc/learner_opt.hip: norm + clip + AdamW over all tensors in two passes (the foreach form
            # below is the same arithmetic; it stays for the CPU host tests)
            f = self._fused
            grads = f["gtype"](*[q.grad.data_ptr() if q.grad is not None else None for q in self.params])
            if any(q.grad is not None and (q.grad.dtype != torch.float32 or not q.grad.is_contiguous())
                   for q in self.params):
                raise ValueError("AdamW on the GPU takes contiguous float32 gradients")
            lib = _L.load()
            # one device tensor table per gradient-pointer set, written once (eagerly) and never rewritten: a
            # graph that captured a step keeps reading exactly the table it was captured with
            key = tuple(grads[i] or 0 for i in range(f["n"]))
            table = f["tables"].get(key)
            if table is None and len(f["tables"]) < f["max_tables"] and not torch.cuda.is_current_stream_capturing():
                table = torch.empty((lib.muz_adamw_table_bytes(f["n"]),), dtype=torch.uint8,
                                    device=self.params[0].device)
                _L.check(lib.muz_adamw_table_write(_L.ptr(table), f["p"], grads, f["m"], f["v"], f["numel"], f["n"],
                                                   _L.stream_ptr()), "muz_adamw_table_write")
                f["tables"][key] = table
            hyper = (_L.ptr(self.count), _L.ptr(f["scratch"]), _L.ptr(f["gnorm"]), self.max_norm, self.b1, self.b2,
                     self.eps, self.wd, self.lr0, float(self.spi), f["bounds"], len(self.boundaries), _L.stream_ptr())
            if table is not None:
                _L.check(lib.muz_adamw_step_table(_L.ptr(table), f["numel"], f["n"], *hyper), "muz_adamw_step_table")
            else:   # first seen under capture, or too many pointer sets: the tensors go in the kernel arguments
                _L.check(lib.muz_adamw_step(f["p"], grads, f["m"], f["v"], f["numel"], f["n"], *hyper),
                         "muz_adamw_step")
            return f["gnorm"]
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self.params]
        # per-tensor norms in one multi-tensor kernel (a sum(g * g) per tensor was ~200 launches per step)
        g_norm = torch.sqrt(torch.stack(torch._foreach_norm(grads)).square().sum())
        trigger = g_norm < self.max_norm
        denom = torch.where(trigger, torch.ones_like(g_norm), g_norm)
        mult = torch.where(trigger, torch.ones_like(g_norm), torch.full_like(g_norm, self.max_norm))
        g = torch._foreach_div(grads, denom)                # clip_by_global_norm: g / ||g|| * max_norm
        torch._foreach_mul_(g, mult)
        lr = _lr_from_count(self.count, self.lr0, self.spi, self.boundaries).to(self.dt)
        self.count.add_(1.0)
        c1 = (1.0 - torch.pow(torch.full_like(self.count, self.b1), self.count)).to(self.dt)
        c2 = (1.0 - torch.pow(torch.full_like(self.count, self.b2), self.count)).to(self.dt)
        torch._foreach_mul_(self.mu, self.b1)
        torch._foreach_add_(self.mu, g, alpha=1.0 - self.b1)
        gg = torch._foreach_mul(g, g)
        torch._foreach_mul_(self.nu, self.b2)
        torch._foreach_add_(self.nu, gg, alpha=1.0 - self.b2)
        mh = torch._foreach_div(self.mu, c1)
        vh = torch._foreach_div(self.nu, c2)
        torch._foreach_sqrt_(vh)
        torch._foreach_add_(vh, self.eps)
        u = torch._foreach_div(mh, vh)
        torch._foreach_add_(u, self.params, alpha=self.wd)
        torch._foreach_mul_(u, lr)
        torch._foreach_sub_(self.params, u)
        return g_norm


def prefer_rocblas():
    """The learner's GEMMs are small (M = 128 or 1408 rows, N and K <= 512).  hipBLASLt (torch's default on
    ROCm) runs them on 256x256 / 256x128 macro-tiles at ~33 us each; rocBLAS picks tiles that fit and the
    graph-captured det step drops from 17.4 to 12.4 ms on MI355X (8.4 ms with the losses vectorised and no
    addmm; profiles/r2_learner_profile.log).
    Process-wide torch setting; the self-play path does not use torch GEMMs."""
    if torch.cuda.is_available():
        torch.backends.cuda.preferred_blas_library("cublas")   # = rocBLAS on ROCm


class Learner:
    """train_step (train_with_reward.py:148-162) on batches sampled from the device ring.

    ``graph=True`` captures forward + backward + optimizer of one step into a HIP graph on the first call
    (static batch buffers; later steps copy the batch in and replay): the step is hundreds of small
    kernels at batch 128, so replaying them as one graph removes the launch overhead."""

    KEYS = ("observations", "actions", "rewards", "policies", "masks", "target_values", "discount_targets")

    def __init__(self, params: dict, obs_channels: int, num_actions: int = 24, unroll_steps: int = 10,
                 device="cuda", graph: bool = False, **opt):
        prefer_rocblas()
        self.nets = MuZeroNets(params, obs_channels, num_actions, device)
        self.opt = AdamW(self.nets.parameters(), **opt)
        self.unroll_steps = int(unroll_steps)
        self.graph = bool(graph)
        self._g = None
        self.sink = GradSink() if GROUPED_GRADS and torch.device(device).type == "cuda" else None
        self.wt = WeightTranspose(self.nets.p) if FUSED_DENSE and FUSED_FWD and torch.device(device).type == "cuda" \
            else None

    def _step(self, batch):
        with _transposed(self.wt):
            loss, (v, pl, d, r) = loss_fn(self.nets, batch, self.unroll_steps)
        _backward(loss, self.sink)
        self.opt.step()
        return {"total_loss": loss.detach(), "v_loss": v.detach(), "p_loss": pl.detach(), "d_loss": d.detach(),
                "r_loss": r.detach()}

    def _device_net(self, net):
        return N.DeviceNet(self.nets.numpy(), net.C, net.A, device=net.buffer.device)

    def train_step(self, batch: dict) -> dict:
        if not self.graph:
            for p in self.nets.parameters():
                p.grad = None
            return self._step(batch)
        if self._g is None:
            self._static = {k: batch[k].clone() for k in self.KEYS}
            # capture-time allocations come from a private pool; warm up the kernels on a side stream first
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                state = ([p.detach().clone() for p in self.nets.parameters()], [m.clone() for m in self.opt.mu],
                         [v.clone() for v in self.opt.nu], self.opt.count.clone())
                for p in self.nets.parameters():
                    p.grad = None
                self._step(self._static)
                with torch.no_grad():                  # undo the warm-up update
                    for p, s in zip(self.nets.parameters(), state[0]):
                        p.copy_(s)
                    for m, s in zip(self.opt.mu, state[1]):
                        m.copy_(s)
                    for v, s in zip(self.opt.nu, state[2]):
                        v.copy_(s)
                    self.opt.count.copy_(state[3])
            torch.cuda.current_stream().wait_stream(side)
            for p in self.nets.parameters():
                p.grad = None
            self._g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g):
                self._out = self._step(self._static)
                # the losses packed into one buffer inside the graph, so a replay hands them out with one copy: the
                # fused loss kernel's own [total, parts...] row when the outputs are its consecutive entries
                # (muz_loss_args: parts[0] = total), else one stack launch
                self._packed = _loss_row(list(self._out.values()))
        for k in self.KEYS:
            self._static[k].copy_(batch[k])
        self._g.replay()
        return self._outputs()

    def _outputs(self, losses: bool = True):
        if not losses:
            return None
        return self._outputs_copy()

    def _outputs_copy(self) -> dict:
        """The captured losses are overwritten by the next replay: one copy of the packed buffer, handed out as
        per-key views so a caller may keep them."""
        c = self._packed.clone()
        return {k: c[i] for i, k in enumerate(self._out)}

    def train_step_from(self, ring, losses: bool = True):
        """train_step on the next batch of a device ring (``ring.sample_batch()``).  Once the step is captured,
        the ring writes the batch straight into the graph's static inputs (no per-key copy).  losses=False: a
        captured step hands out nothing (no copy of the loss row; a loop that does not log every step)."""
        if self.graph and self._g is not None:
            ep, t = ring.draw_indices()
            if not getattr(self, "_static_full", False):    # the batch fields the step does not read
                B, K = len(ep), ring.unroll_steps + 1
                fresh = ring._new_batch(B, K, ring.obs_shape[0], ring.action_dim, dict(device=ring.device))
                for k, v in fresh.items():
                    self._static.setdefault(k, v)
                self._static_full = True
            ring.sample_at(ep, t, out=self._static)
            self._g.replay()
            return self._outputs(losses)
        return self.train_step(ring.sample_batch())

    def push_to(self, net: "N.DeviceNet"):
        """Pack the current parameters into the self-play engine's arena (same layout) in place."""
        fresh = self._device_net(net)
        net.buffer.copy_(fresh.buffer)
        net.prepare()


# ---- classic MADN: Stochastic MuZero (MuZero_Classic_MADN/train_stochastic.py) -------------------------
CLASSIC_SCALING = dict(value=4.0, policy=2.0, chance=0.5, discount=1.0, reward=1.0)   # train_stochastic.py:374-378


class ClassicMuZeroNets(MuZeroNets):
    """Repr2 / Pred4 (A = 4) + StochasticDynamicsNetwork4 (muzero_classic_madn.py:314-408)."""

    def __init__(self, params: dict, obs_channels: int, device="cuda", dtype=torch.float32):
        from .stochastic import classic_param_shapes
        super().__init__(params, obs_channels, 4, device, dtype, shapes=classic_param_shapes(obs_channels))
        self.NC = 6

    def _film_trunk(self, pre, rb0, x_in, e, film=None):
        """film: precomputed (scale, shift) rows of this step (e unused) -- loss_fn_stochastic evaluates the FiLM
        projections for all steps at once."""
        d = "dynamics"
        ln = self._ln(f"{d}/{pre}_input_ln", x_in)
        if film is None:
            film = (self._dense(f"{d}/{pre}_film_scale", e), self._dense(f"{d}/{pre}_film_shift", e))
        x = ln * (1.0 + film[0]) + film[1]
        x = self._dense_ln(f"{d}/{pre}_dense1", f"{d}/{pre}_ln1", x)
        x = self._dense_ln(f"{d}/{pre}_dense2", f"{d}/{pre}_ln2", x)
        for r in range(rb0, rb0 + 2):
            x = self._rb(f"{d}/ResBlock_{r}", x)
        return self._minmax(x_in + self._dense(f"{d}/{pre}_proj", x))

    def _one_hot(self, a, n, like):
        return (a.long()[:, None] == torch.arange(n, device=like.device)[None, :]).to(like.dtype)

    def action_embed(self, action):
        oh = self._one_hot(action, self.A, self.p["dynamics/act_embed/bias"])
        return oh, F.relu(self._dense("dynamics/act_embed", oh))

    def chance_embed(self, chance):
        return F.relu(self._dense("dynamics/chance_embed", self._one_hot(chance, self.NC, self.p["dynamics/chance_embed/bias"])))

    def action_heads(self, latent, after, oh):
        """(reward, chance, discount) logits of action_dynamics; row-wise, batchable over unroll steps."""
        d = "dynamics"
        rl = self._dense(f"{d}/reward_head", F.relu(self._dense(f"{d}/reward_dense", torch.cat([after, oh], -1))))
        dl = self._dense(f"{d}/discount_head", self._dense_ln(f"{d}/discount_dense", f"{d}/discount_ln", latent))
        cl = self._dense(f"{d}/chance_head", after)
        return rl, cl, dl

    def action_dynamics(self, latent, action):
        """-> (afterstate, reward_logits, chance_logits, discount_logits) (329-371)."""
        oh, e = self.action_embed(action)
        after = self._film_trunk("act", 0, latent, e)
        rl, cl, dl = self.action_heads(latent, after, oh)
        return after, rl, cl, dl

    def chance_dynamics(self, afterstate, chance):
        """-> next state (373-408)."""
        return self._film_trunk("chance", 2, afterstate, self.chance_embed(chance))


def loss_fn_stochastic(nets: ClassicMuZeroNets, batch: dict, unroll_steps: int = 10, grad_scale: float = 0.5):
    """train_stochastic.py:34-180 -> (total, (value, policy, chance, discount, reward) losses)."""
    _PACKED.clear()   # (its consumers pack their own weights)
    dt = nets.p["prediction/Dense_5/bias"].dtype
    obs = batch["observations"].to(dt)
    latent = nets.representation(obs)
    B, K = batch["actions"].shape
    dev = obs.device
    acts = batch["actions"]
    dice = torch.cat([batch["dice_outcomes"][:, 1:].long(), torch.zeros((B, 1), dtype=torch.long, device=dev)], 1)
    sc = CLASSIC_SCALING
    # Only the afterstate / state chain is sequential; the embeddings, Pred4 and the action heads run once
    # over all steps stacked along the batch (same per-row arithmetic, far fewer launches).
    oh_all, ea_all = nets.action_embed(acts[:, :K].transpose(0, 1).reshape(-1))
    ec_all = nets.chance_embed(dice[:, :K].transpose(0, 1).reshape(-1))
    latents, afters = [latent], []
    if K and latent.is_cuda and CHAIN:     # the afterstate / state chain as one autograd node (as loss_fn's latent chain)
        d = "dynamics"
        film = [torch.stack([nets._dense(f"{d}/{pre}_film_{w}", e).reshape(K, B, -1) for pre, e in
                             (("act", ea_all), ("chance", ec_all))], 1).reshape(2 * K, B, -1)
                for w in ("scale", "shift")]                       # rows interleaved: act_0, chance_0, act_1, ...
        chain = _TrunkChain.apply(latent, film[0], film[1], grad_scale, (0, 1) * K, (False, True) * K, False,
                                  *(nets.p[n] for kind in ("act", "chance") for n in trunk_param_names(kind)))
        afters = list(chain[0::2].unbind(0))
        latents += list(chain[1::2].unbind(0))
    for k in range(len(afters), K):
        after = nets._film_trunk("act", 0, latents[-1], ea_all[k * B:(k + 1) * B])
        afters.append(after)
        nxt = nets._film_trunk("chance", 2, after, ec_all[k * B:(k + 1) * B])
        latents.append((nxt * (1.0 - grad_scale)).detach() + nxt * grad_scale)
    logits_all, v_all = nets.prediction(torch.cat(latents, 0))
    if K:
        rl_all, cl_all, dl_all = nets.action_heads(torch.cat(latents[:K], 0), torch.cat(afters, 0), oh_all)
    if obs.is_cuda and FUSED_LOSS and K:
        u = 1.0 / unroll_steps
        spec = dict(batch=batch, K=K, scale_value=u * sc["value"], scale_policy=u * sc["policy"], norm=1,
                    terms=[(batch["dice_probs"], 0, 1.0, 0.1, u * sc["chance"]),
                           (batch["discount_targets"], 0, 1.0, 0.1, u * sc["discount"]),      # rare: terminal
                           (batch["rewards"], 1, 1.0, 0.1, u * sc["reward"])])                 # rare: won / lost
        total, parts = _LossHeads.apply(logits_all, v_all, cl_all, dl_all, rl_all, spec)
        return total, (parts[1], parts[2], parts[3], parts[4], parts[5])
    # all K (+1) steps at once, as in loss_fn
    probs, disc_t, rew_t = batch["dice_probs"].to(dt), batch["discount_targets"].int(), batch["rewards"].int()
    m = batch["masks"][:, :K + 1].transpose(0, 1).to(dt)
    v = v_all[:, 0].reshape(K + 1, B)
    logp = F.log_softmax(logits_all, -1).reshape(K + 1, B, -1)
    l_policy = torch.mean(m * -(batch["policies"][:, :K + 1].transpose(0, 1).to(dt) * logp).sum(-1), 1)
    l_value = torch.mean(m * (batch["target_values"][:, :K + 1].transpose(0, 1).to(dt) - v) ** 2, 1)
    zero = torch.zeros((1,), dtype=dt, device=dev)
    if K:
        mk = m[:K]
        n_valid = mk.sum(1)
        rc, dc = rew_t[:, :K].transpose(0, 1), disc_t[:, :K].transpose(0, 1)
        tp = probs[:, :K].transpose(0, 1)                                          # [K, B, 6]
        reward_ce = F.cross_entropy(rl_all, rc.reshape(-1).long(), reduction="none").reshape(K, B)
        discount_ce = F.cross_entropy(dl_all, dc.reshape(-1).long(), reduction="none").reshape(K, B)
        chance_ce = -(tp * F.log_softmax(cl_all, -1).reshape(K, B, -1)).sum(-1)
        non_uniform = ((tp - 1.0 / 6.0) ** 2).sum(-1) > 1e-6
        l_reward = balanced_loss_steps(reward_ce, (rc != 1).to(dt), mk, n_valid)
        l_discount = balanced_loss_steps(discount_ce, (dc == 1).to(dt), mk, n_valid)
        l_chance = balanced_loss_steps(chance_ce, non_uniform.to(dt), mk, n_valid)
    else:
        l_chance = l_discount = l_reward = zero
    total = (1.0 / unroll_steps) * (sc["value"] * l_value.sum() + sc["policy"] * l_policy.sum() +
                                    sc["chance"] * l_chance.sum() + sc["discount"] * l_discount.sum() +
                                    sc["reward"] * l_reward.sum())
    return total, (l_value.sum(), l_policy.sum(), l_chance.sum(), l_discount.sum(), l_reward.sum())


def balanced_loss_steps(ce, is_rare, mask, n_valid, w_rare=1.0, w_common=0.1):
    """train_stochastic.py:25-32 for every unroll step at once ([K, B] -> [K]; n_common counts against the
    clamped n_rare, as the reference does)."""
    masked_rare = mask * is_rare
    n_rare = torch.clamp(masked_rare.sum(1), min=1.0)
    n_common = torch.clamp(n_valid - n_rare, min=1.0)
    return w_rare * (masked_rare * ce).sum(1) / n_rare + w_common * ((mask - masked_rare) * ce).sum(1) / n_common


class StochasticLearner(Learner):
    """train_step of train_stochastic.py:183-193 (clip 5.0 -> adamw, lr 0.005 x0.1 @ it 40, x0.2 @ 85,
    x0.5 @ 105 of 2500 steps) on batches of replay.VectorizedReplayBufferStochastic."""

    KEYS = Learner.KEYS + ("dice_outcomes", "dice_probs")

    def __init__(self, params: dict, obs_channels: int, unroll_steps: int = 10, device="cuda", graph: bool = False,
                 **opt):
        opt.setdefault("boundaries", CLASSIC_LR_BOUNDARIES)
        prefer_rocblas()
        self.nets = ClassicMuZeroNets(params, obs_channels, device)
        self.opt = AdamW(self.nets.parameters(), **opt)
        self.unroll_steps = int(unroll_steps)
        self.graph = bool(graph)
        self._g = None
        self.sink = GradSink() if GROUPED_GRADS and torch.device(device).type == "cuda" else None
        self.wt = WeightTranspose(self.nets.p) if FUSED_DENSE and FUSED_FWD and torch.device(device).type == "cuda" \
            else None

    def _step(self, batch):
        with _transposed(self.wt):
            loss, (v, pl, c, d, r) = loss_fn_stochastic(self.nets, batch, self.unroll_steps)
        _backward(loss, self.sink)
        self.opt.step()
        return {"total_loss": loss.detach(), "v_loss": v.detach(), "p_loss": pl.detach(), "c_loss": c.detach(),
                "d_loss": d.detach(), "r_loss": r.detach()}

    def _device_net(self, net):
        from .stochastic import DeviceClassicNet
        return DeviceClassicNet(self.nets.numpy(), net.C, device=net.buffer.device)


# ---- DOG: MuZero_DOG/train.py (its loss_fn / train_step, 24-164, are train_with_reward.py's) ------------------------
class DogMuZeroNets(MuZeroNets):
    """The DOG MuZero slice's networks (muzero_dog.py): MuZero_DOG/muzero_dog.py:25-83's RepresentationNetwork (the det
    trunk with LayerNorm_7 after its last Dense instead of the min-max scaling, lines 80-81) and DynamicsNetwork4 /
    PredictionNetwork4 at A = 806 (the slice's definition; muzero_dog.py:85-99 are `pass`), on 34 x 56 observations.
    The 806-wide one-hot inputs (Dynamics Dense_0, Dense_6 / Dense_7's action rows) stay matrix products, as the
    reference computes them (66 MFLOP per step at batch 128 x 10, against ~10 GFLOP for the whole step)."""

    def __init__(self, params: dict, device="cuda", dtype=torch.float32):
        from . import muzero_dog as MD
        super().__init__(params, MD.NUM_CHANNELS, MD.NUM_ACTIONS, device, dtype, shapes=MD.param_shapes())

    def representation(self, obs):
        r = "representation"
        return self._dense_ln(f"{r}/Dense_4", f"{r}/LayerNorm_7", self.representation_trunk(obs), LN_PLAIN)


class DogLearner(Learner):
    """train_step of MuZero_DOG/train.py:148-164 (= train_with_reward.py's: clip 5.0 -> adamw, lr 0.005 x0.2 @ it 30,
    x0.2 @ 60, x0.5 @ 85 of 2500 steps, wd 1e-4; train.py:355-373) on the DOG nets, batches from a device ring at
    action_dim 806, obs (34, 56)."""

    def __init__(self, params: dict, unroll_steps: int = 10, device="cuda", graph: bool = False, **opt):
        prefer_rocblas()
        self.nets = DogMuZeroNets(params, device)
        self.opt = AdamW(self.nets.parameters(), **opt)
        self.unroll_steps = int(unroll_steps)
        self.graph = bool(graph)
        self._g = None
        self.sink = GradSink() if GROUPED_GRADS and torch.device(device).type == "cuda" else None
        self.wt = WeightTranspose(self.nets.p) if FUSED_DENSE and FUSED_FWD and torch.device(device).type == "cuda" \
            else None

    def _device_net(self, net):
        from .muzero_dog import DeviceDogNet
        return DeviceDogNet(self.nets.numpy(), device=net.buffer.device)


def train_loop(learner: Learner, engine, ring, iterations: int, train_steps: int, games_per_iteration: int,
               temperature_schedule=(2.0, 1.5, 1.0, 0.8, 0.6), seed: int = 42, warmup_calls: int = 3):
    """test_training (train_with_reward.py:167-311) with the device engine: streamed self-play into the
    ring, train_steps sampled batches per iteration, new weights pushed to the engine each iteration."""
    def temp(it):
        ph = min(int(it / max(iterations, 1) * len(temperature_schedule)), len(temperature_schedule) - 1)
        return temperature_schedule[ph]

    for n in range(warmup_calls):
        ring.save_games_from_buffers(engine.play_stream(games_per_iteration, seed * n, temp(0)))
    history = []
    for it in range(iterations):
        ring.save_games_from_buffers(engine.play_stream(games_per_iteration, seed + it ** 3, temp(it)))
        for _ in range(train_steps):
            losses = learner.train_step_from(ring)
        learner.push_to(engine.net)
        history.append({k: float(v) for k, v in losses.items()})
    return history
