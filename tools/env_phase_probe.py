"""Where one fused env step's time goes, per wave (measurement build, csrc/phc_measure.h: lane 0 of every wave
stamps the 100 MHz constant clock at the phase boundaries of k_env_replay; phc_env_phase_copy reads them).

usage: tools/build_variants.sh phases "-DPHC_MEASURE_ENV_PHASES=1"
       PHC_HIP_LIB=.../libphc_hip_phases.so python tools/env_phase_probe.py [envs ...]
Prints, per env count, the launch span and the median / p90 of each phase's duration over the waves, and
when the waves start relative to the first one (waves that start late queued behind earlier ones).
"""
import ctypes
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["scalars", "frame rows", "replay+reward", "obs row", "copy out", "stats"]


def main():
    import torch

    import phc_amd_path

    phc_amd_path.register()
    import bench
    from puffer_phc_amd import _native as N

    lib = N.lib()
    lib.phc_env_phase_copy.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    for envs in [int(x) for x in sys.argv[1:]] or [4096, 32768]:
        a = types.SimpleNamespace(envs=envs, min_len=60, max_len=300, physics="replay", amp=False)
        env, _, _ = bench.build_env(a, 0)
        act = torch.rand((envs, 69), device="cuda") * 2 - 1
        for _ in range(10):
            env.step(act)
        torch.cuda.synchronize()
        waves = envs // 2
        res = []
        for rep in range(5):
            env.step(act)
            torch.cuda.synchronize()
            buf = np.zeros(waves * 8, dtype=np.uint64)
            assert lib.phc_env_phase_copy(buf.ctypes.data, waves) == 0
            res.append(buf.reshape(waves, 8)[:, :7].astype(np.int64))
        for r in res[-1:]:
            t0 = r[:, 0].min()
            span = (r[:, 6].max() - t0) / 100.0  # 100 MHz ticks -> us
            d = np.diff(r, axis=1) / 100.0
            start = (r[:, 0] - t0) / 100.0
            print(f"envs {envs}: span {span:.2f} us over {waves} waves; wave start offset median {np.median(start):.2f} "
                  f"p90 {np.percentile(start, 90):.2f} max {start.max():.2f} us; wave life median "
                  f"{np.median((r[:, 6] - r[:, 0]) / 100.0):.2f} us")
            life = (r[:, 6] - r[:, 0]) / 100.0
            end = (r[:, 6] - t0) / 100.0
            print(f"   wave life p90 {np.percentile(life, 90):.2f} p99 {np.percentile(life, 99):.2f} max {life.max():.2f} us; "
                  f"wave end median {np.median(end):.2f} p90 {np.percentile(end, 90):.2f} p99 {np.percentile(end, 99):.2f} "
                  f"max {end.max():.2f} us")
            for k, name in enumerate(NAMES):
                print(f"   {name:14s} median {np.median(d[:, k]):6.2f}  p90 {np.percentile(d[:, k], 90):6.2f} us")


if __name__ == "__main__":
    main()
