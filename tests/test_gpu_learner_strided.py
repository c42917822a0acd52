"""The round-6 learner launch forms, each against the form it replaces, bit for bit:

* muz_ln_bwd_rows_ld / muz_dense_ln_bwd_ld (the gradient read as a column slice of a wider one, e.g. a
  concatenation's gradient) against muz_ln_bwd_rows / muz_dense_ln_bwd on a contiguous copy of the slice;
* muz_ln_fwd_parts (a long-K layer's partial planes summed in plane order before the LayerNorm) against
  muz_ln_fwd of the planes added one by one in that order;
* muz_wgrad_grouped's segment partials (k_seg_sum) against float64, for problems of several segments."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _L():
    from exploring_muzero_on_dog_amd import lib as L
    return L


def _fwd_saved(M, N, g):
    """a LayerNorm forward's saved values (out, z, mean, rstd) of mode RELU for random rows"""
    L = _L()
    y = torch.randn(M, N, generator=g).cuda()
    bias, gamma, beta = (0.2 * torch.randn(N, generator=g)).cuda(), (1 + 0.2 * torch.randn(N, generator=g)).cuda(), \
        (0.2 * torch.randn(N, generator=g)).cuda()
    out, z = torch.empty(M, N, device="cuda"), torch.empty(M, N, device="cuda")
    mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    L.check(L.load().muz_ln_fwd(L.ptr(y), L.ptr(bias), L.ptr(gamma), L.ptr(beta), None, M, N, 1, L.ptr(out), L.ptr(z),
                                L.ptr(mean), L.ptr(rstd), L.stream_ptr()), "muz_ln_fwd")
    return (out, z, mean, rstd), gamma


@pytest.mark.parametrize("M,N,col0,width", [(128, 64, 256, 320), (128, 256, 0, 320), (37, 32, 32, 96)])
def test_ln_bwd_rows_ld_equals_contiguous(cuda, M, N, col0, width):
    L = _L()
    g = torch.Generator().manual_seed(M + N)
    fwd, gamma = _fwd_saved(M, N, g)
    wide = torch.randn(M, width, generator=g).cuda()
    dout = wide[:, col0:col0 + N]
    nf = L.load().muz_ln_bwd_scratch_floats(M, N)
    res = []
    for strided in (True, False):
        d = dout if strided else dout.contiguous()
        dz = torch.empty(M, N, device="cuda")
        scratch = torch.full((nf,), float("nan"), device="cuda")
        fn = L.load().muz_ln_bwd_rows_ld
        L.check(fn(L.ptr(d), d.stride(0), *(L.ptr(t) for t in fwd), L.ptr(gamma), M, N, 1, L.ptr(dz), None,
                   L.ptr(scratch), L.stream_ptr()), "muz_ln_bwd_rows_ld")
        torch.cuda.synchronize()
        res.append((dz, scratch))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    # and the plain entry point is the same launch with the row stride N
    dz = torch.empty(M, N, device="cuda")
    scratch = torch.full((nf,), float("nan"), device="cuda")
    c = dout.contiguous()
    L.check(L.load().muz_ln_bwd_rows(L.ptr(c), *(L.ptr(t) for t in fwd), L.ptr(gamma), M, N, 1, L.ptr(dz), None,
                                     L.ptr(scratch), L.stream_ptr()), "muz_ln_bwd_rows")
    torch.cuda.synchronize()
    assert torch.equal(dz, res[0][0]) and torch.equal(scratch, res[0][1])


@pytest.mark.parametrize("M,N,K,col0,width", [(128, 64, 28, 256, 320), (100, 32, 64, 0, 96)])
def test_dense_ln_bwd_ld_equals_contiguous(cuda, M, N, K, col0, width):
    L = _L()
    g = torch.Generator().manual_seed(7 * M + N)
    fwd, gamma = _fwd_saved(M, N, g)
    W = (0.1 * torch.randn(K, N, generator=g)).cuda()
    wide = torch.randn(M, width, generator=g).cuda()
    dout = wide[:, col0:col0 + N]
    nf = L.load().muz_dense_ln_bwd_scratch_floats(M, N)
    res = []
    for strided in (True, False):
        d = dout if strided else dout.contiguous()
        dz, dx = torch.empty(M, N, device="cuda"), torch.empty(M, K, device="cuda")
        scratch = torch.full((nf,), float("nan"), device="cuda")
        L.check(L.load().muz_dense_ln_bwd_ld(L.ptr(d), d.stride(0), *(L.ptr(t) for t in fwd), L.ptr(gamma), M, N, 1,
                                             L.ptr(W), K, None, L.ptr(dz), None, L.ptr(dx), L.ptr(scratch),
                                             L.stream_ptr()), "muz_dense_ln_bwd_ld")
        torch.cuda.synchronize()
        res.append((dz, dx, scratch))
    for a, b in zip(*res):
        assert torch.equal(a, b)
    # a row stride that is not a multiple of 4 is refused (the kernel reads 16-byte rows)
    assert L.load().muz_dense_ln_bwd_ld(L.ptr(dout), N + 1, *(L.ptr(t) for t in fwd), L.ptr(gamma), M, N, 1, L.ptr(W),
                                        K, None, L.ptr(dz), None, L.ptr(dx), L.ptr(scratch), L.stream_ptr()) != 0


@pytest.mark.parametrize("S,M,N", [(14, 128, 256), (3, 50, 64), (17, 9, 32)])
def test_ln_fwd_parts_equals_planes_added_in_order(cuda, S, M, N):
    L = _L()
    g = torch.Generator().manual_seed(S * M + N)
    planes = torch.randn(S, M, N, generator=g).cuda()
    bias, gamma, beta = (0.2 * torch.randn(N, generator=g)).cuda(), (1 + 0.2 * torch.randn(N, generator=g)).cuda(), \
        (0.2 * torch.randn(N, generator=g)).cuda()
    y = planes[0].clone()
    for q in range(1, S):
        y = y + planes[q]           # one rounding per plane, in plane order
    outs = []
    for parts, src in ((S, planes), (1, y)):
        o, z = torch.empty(M, N, device="cuda"), torch.empty(M, N, device="cuda")
        mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
        L.check(L.load().muz_ln_fwd_parts(L.ptr(src), parts, L.ptr(bias), L.ptr(gamma), L.ptr(beta), None, M, N, 1,
                                          L.ptr(o), L.ptr(z), L.ptr(mean), L.ptr(rstd), L.stream_ptr()),
                "muz_ln_fwd_parts")
        torch.cuda.synchronize()
        outs.append((o, z, mean, rstd))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_wgrad_segment_sums(cuda):
    """problems of 1, several and many segments (k_seg_sum adds each output's partials in segment order) against
    float64, with row strides wider than the matrices"""
    L = _L()
    seg = L.load().muz_wgrad_segment_rows()
    g = torch.Generator().manual_seed(11)
    shapes = [(seg, 64, 32), (3 * seg + 17, 256, 256), (7168, 320, 64), (1280, 256, 256), (5, 18, 32)]
    probs, ref, outs, keep = [], [], [], []
    for M, K, N in shapes:
        X = torch.randn(M, K + 3, generator=g).cuda()[:, :K]
        D = torch.randn(M, N + 5, generator=g).cuda()[:, :N]
        o = torch.full((K, N), float("nan"), device="cuda")
        keep += [X, D]
        outs.append(o)
        ref.append(X.double().t() @ D.double())
        probs.append((X.data_ptr(), D.data_ptr(), o.data_ptr(), M, K, N, X.stride(0), D.stride(0)))
    arr = (L.MuzWgradProblem * len(probs))(*[L.MuzWgradProblem(*p) for p in probs])
    need = L.load().muz_wgrad_scratch_floats(arr, len(probs))
    assert need > 0
    scratch = torch.full((need,), float("nan"), device="cuda")
    L.check(L.load().muz_wgrad_grouped(arr, len(probs), L.ptr(scratch), need, L.stream_ptr()), "muz_wgrad_grouped")
    torch.cuda.synchronize()
    for (M, K, N), o, r in zip(shapes, outs, ref):
        err = float((o.double() - r).abs().max()) / max(1.0, float(r.abs().max()))
        assert err < 1e-5, (M, K, N, err)
