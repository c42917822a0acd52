"""Dump the learner-oracle tests' classic / det batches (and their init seeds) to gpurun_out/r5_batch_{classic,det}.npz,
so the float64 oracle's near-threshold analysis (profiles/r5_flip_sites.py) can run on the CPU."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "profiles"))
import r5_classic_grad_diag as D  # noqa: E402

os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
for kind, setup in (("classic", D.classic_setup), ("det", D.det_setup)):
    params, C, batch, _ = setup()
    np.savez(os.path.join(ROOT, "gpurun_out", f"r5_batch_{kind}.npz"),
             **{k: v.detach().cpu().numpy() for k, v in batch.items()})
    print(kind, {k: tuple(v.shape) for k, v in batch.items()})
