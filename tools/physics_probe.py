"""Time phc_physics_step (N3) at a given env count: average launch duration over K launches on the
current stream, env-steps/s and env-substeps/s.  Usage: python tools/physics_probe.py [num_envs] [K]."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import phc_amd_path  # noqa: E402

phc_amd_path.register()
from puffer_phc_amd import _native  # noqa: E402
from puffer_phc_amd.physics import ArticulatedPhysics, BodyModel, PhysicsConfig, rest_state  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = "cuda:0"
bm = BodyModel(device=dev)
phys = ArticulatedPhysics(PhysicsConfig(self_collision=os.environ.get("PHC_SELF_COL", "1") == "1"), model=bm)
rb_t, dof_t = rest_state(bm, n, 0.0, device=dev)
rb_t[:, 0, 0] += torch.arange(n, device=dev, dtype=torch.float32) * 2.0
rng = np.random.default_rng(0)
f_t = torch.zeros((n, 69), device=dev)
tgt = torch.tensor(rng.normal(0, 0.1, (n, 69)), dtype=torch.float32, device=dev)
env_c = _native.physics_env_struct(rb_t, dof_t, f_t)
for _ in range(5):
    _native.physics_step(env_c, tgt, bm.table, phys.params)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
t0 = time.perf_counter()
for _ in range(K):
    _native.physics_step(env_c, tgt, bm.table, phys.params)
e.record()
torch.cuda.synchronize()
wall = time.perf_counter() - t0
ms = s.elapsed_time(e) / K
sub = phys.config.control_freq_inv * phys.config.substeps
print(f"envs {n}  {ms * 1e3:.1f} us/launch  {n / ms * 1e3 / 1e6:.2f} M env-steps/s  "
      f"{n * sub / ms * 1e3 / 1e6:.1f} M env-substeps/s  (wall {wall / K * 1e6:.1f} us)  "
      f"finite={bool(torch.isfinite(rb_t).all())} root_z_mean={rb_t[:, 0, 2].mean().item():.4f}")
