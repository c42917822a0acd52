"""Env-round kernel time with and without the observation phase (muz_detmadn_random_round_variant), per variant
and batch: HIP-event time per launch on the launch stream, after a pre-roll so games are mid-play."""
import sys
import torch

sys.path.insert(0, ".")
import muzpkg  # noqa: E402

muzpkg.load()
from exploring_muzero_on_dog_amd import detmadn as E  # noqa: E402
from oracle import detmadn as dm  # noqa: E402

rules = dict(num_players=2, **dm.SELFPLAY_RULES)
for B in (65536, 1 << 20):
    for variant in (1, 3, 4):
        for with_obs in (True, False):
            env = E.env_reset(B, **rules)
            legal = E.legal_bits(env)
            obs = torch.empty((B, 18, 56), dtype=torch.int8, device="cuda") if with_obs else None
            for t in range(100):
                E.random_round(env, legal, 5, t, obs=obs, variant=variant)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for t in range(100, 200):
                E.random_round(env, legal, 5, t, obs=obs, variant=variant)
            b.record()
            torch.cuda.synchronize()
            print(f"B={B:8d} variant={variant} obs={int(with_obs)}: {a.elapsed_time(b) / 100 * 1000:8.1f} us/launch",
                  flush=True)
