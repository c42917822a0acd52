import sys, torch
sys.path.insert(0, ".")
import muzpkg
muzpkg.load()
from exploring_muzero_on_dog_amd import learner as L
g = torch.Generator().manual_seed(1)
M, N = 640, 256
x = torch.rand(M, N, generator=g).cuda()
gam = (1 + 0.1 * torch.randn(N, generator=g)).cuda(); bet = (0.1 * torch.randn(N, generator=g)).cuda()
s1 = (1 + 0.3 * torch.randn(M, N, generator=g)).cuda(); sh = (0.3 * torch.randn(M, N, generator=g)).cuda()
a = L._ln_fwd(x, torch.zeros_like(gam), gam, bet, None, L.LN_PLAIN)
film_ref = torch.addcmul(sh, a[0], s1)
film_mul_add = a[0] * s1 + sh
film = torch.empty_like(x)
b = L._ln_film_fwd(x, gam, bet, s1, sh, film)
torch.cuda.synchronize()
for n, u, v in zip(("out", "z", "mean", "rstd"), a, b):
    print(n, torch.equal(u, v), (u - v).abs().max().item())
print("film vs addcmul", torch.equal(film, film_ref), (film - film_ref).abs().max().item())
print("film vs mul+add", torch.equal(film, film_mul_add), (film - film_mul_add).abs().max().item())
print("addcmul vs mul+add", torch.equal(film_ref, film_mul_add))
