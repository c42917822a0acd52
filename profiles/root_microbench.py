"""Microbenchmark of root_inference_fn (k_repr_conv + k_root_dense) at B games (HIP events).

    python profiles/root_microbench.py [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import muzpkg  # noqa: E402

muzpkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exploring_muzero_on_dog_amd import nets as N  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
C = 18
net = N.DeviceNet(N.init_muzero_params(0, C), C)
obs = torch.from_numpy(np.random.default_rng(0).integers(0, 2, (B, C, 56)).astype(np.float32)).cuda()
for _ in range(3):
    N.root_inference_fn(net, obs)
torch.cuda.synchronize()
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 20
st.record()
for _ in range(reps):
    N.root_inference_fn(net, obs)
en.record()
torch.cuda.synchronize()
print(f"{os.path.basename(os.environ.get('MUZ_LIB', 'libmuz.so'))}: root_inference B={B}: {st.elapsed_time(en) / reps * 1000:.1f} us")
