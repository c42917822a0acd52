"""Round-5 diagnosis, step 4 (CPU): the learner's near-threshold decisions in the float64 oracle.

Runs oracle/learner_grad.py's float64 loss on a dumped test batch (profiles/r5_dump_batches.py) and records every
ReLU input and every min-max extremum: the elements closest to a ReLU's kink (|x| smallest) and the min-max rows
whose two largest (smallest) entries are closest (gap / (hi - lo)).  A forward difference of ~3e-7 (the fp32
kernels against each other) flips any decision closer than that, and each flip moves the gradient by a fixed
quantum (profiles/r5c_sensitivity.log).  Test infrastructure (imports oracle/).

usage: python profiles/r5_flip_sites.py classic|det [batch.npz]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import learner_grad as OG  # noqa: E402

def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "classic"
    path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", f"r5_batch_{kind}.npz")
    b = dict(np.load(path))
    if kind == "classic":
        from oracle import classic_nets as CN
        params = CN.init_params(11, seed=32, randomize_affine=True)
    else:
        from oracle import nets as ON
        params = ON.init_params(34, seed=31, randomize_affine=True)
    rows, sites = OG.decision_margins(params, b, unroll_steps=10, classic=kind == "classic")
    print(f"{kind}: closest decisions of the float64 forward (distance, kind, call #, batch row, column):")
    for it in sites[:16]:
        print(f"  {it[0]:.3e}  {it[1]:6s} call {it[2]:4d} row {it[3]:3d} col {it[4]}")
    for thr in (1e-7, 3e-7, 1e-6, 3e-6, 1e-5):
        print(f"batch rows with a decision within {thr:.0e}: {np.flatnonzero(rows < thr).tolist()}")


if __name__ == "__main__":
    main()
