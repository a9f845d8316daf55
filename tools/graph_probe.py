"""Which parts of the rollout step can be captured in a hipGraph (debug aid)."""
import sys
import traceback

import numpy as np
import torch

sys.path.insert(0, ".")
import phc_amd_path  # noqa: E402

phc_amd_path.register()
from puffer_phc_amd.envs.humanoid_phc import Box  # noqa: E402
from puffer_phc_amd.policies import PHCPolicy, Policy  # noqa: E402

torch.set_float32_matmul_precision("high")


class _Env:
    single_observation_space = Box(np.full(934, -np.inf), np.full(934, np.inf))
    single_action_space = Box(-np.ones(69), np.ones(69))
    amp_observation_space = None


dev = "cuda:0"
pol = Policy(PHCPolicy(_Env())).to(dev)
obs = torch.randn((4096, 934), device=dev)


def try_capture(name, fn, mode="global"):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, capture_error_mode=mode):
            fn()
        g.replay()
        torch.cuda.synchronize()
        print(f"{name:40s} [{mode}] OK", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{name:40s} [{mode}] FAIL {type(e).__name__}: {str(e).splitlines()[0]}", flush=True)
        traceback.print_exc(limit=3)
        torch.cuda.synchronize()


with torch.no_grad():
    try_capture("randn", lambda: torch.randn(16, device=dev))
    try_capture("normal", lambda: torch.normal(torch.zeros(16, device=dev), torch.ones(16, device=dev)))
    try_capture("rms_normalize", lambda: pol.policy.obs_norm(obs))
    try_capture("mm xf32", lambda: torch.mm(obs, obs.t()[:, :512].contiguous()))
    try_capture("encode_observations", lambda: pol.policy.encode_observations(obs))
    try_capture("policy forward", lambda: pol(obs))
    try_capture("policy forward thread_local", lambda: pol(obs), mode="thread_local")
    try_capture("policy forward relaxed", lambda: pol(obs), mode="relaxed")
