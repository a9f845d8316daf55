"""The HBM clip pool (motion_lib.ClipPool) against the per-clip loop it replaces (the reference's
load_motion_with_skeleton crop + heading draws, motion_lib.py:766-800): the same clips, crops,
counts, fps and heading draws, bit for bit, from the same python / numpy generator states.  Runs
on the CPU (the pool lives on whatever device the library names); the C3-scale resample on the
GPU is tests/test_gpu_resample.py."""

import random
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from puffer_phc_amd import motion_lib as ML


def _clips(n, seed=0, lo=5, hi=40, f32=False):
    rng = np.random.default_rng(seed)
    out = {}
    for i in range(n):
        t = int(rng.integers(lo, hi))
        q = rng.normal(size=(t, 24, 4))
        q /= np.linalg.norm(q, axis=-1, keepdims=True)
        dt = np.float32 if f32 and i % 2 else np.float64
        out[f"clip_{i:04d}"] = {"pose_quat_global": q.astype(dt),
                                "root_trans_offset": torch.from_numpy(rng.normal(size=(t, 3))),
                                "pose_aa": rng.normal(size=(t, 24, 3)).astype(dt), "fps": 30 if i % 3 else 60}
    return out


def _lib(clips, max_length, deterministic, im_eval=False):
    lib = ML.MotionLibBase.__new__(ML.MotionLibBase)
    lib.m_cfg = SimpleNamespace(max_length=max_length, is_deterministic=deterministic, im_eval=im_eval)
    lib._device = "cpu"
    lib.load_data(clips)
    return lib


@pytest.mark.parametrize("max_length,deterministic", [(-1, False), (20, False), (20, True), (5, False)])
def test_pool_gather_matches_per_clip_loop(monkeypatch, max_length, deterministic):
    clips = _clips(37, f32=True)
    ids = np.random.default_rng(1).integers(0, 37, size=64)
    out = []
    for pool in (False, True):
        monkeypatch.setattr(ML, "MOTION_POOL", pool)
        random.seed(11)
        np.random.seed(12)
        lib = _lib(clips, max_length, deterministic)
        out.append(lib._gather_clips(ids))
        out[-1] = out[-1] + (random.random(), np.random.random())  # the generators end in the same state
    (q0, t0, a0, c0, f0, h0, r0, n0), (q1, t1, a1, c1, f1, h1, r1, n1) = out
    assert c0 == c1 and f0 == f1 and h0 == h1 and r0 == r1 and n0 == n1
    for x, y in ((q0, q1), (t0, t1), (a0, a1)):
        assert x.dtype == y.dtype == torch.float64 and torch.equal(x, y)
    if max_length != -1:
        assert max(c1) <= max_length


def test_pool_is_built_once_and_reused(monkeypatch):
    monkeypatch.setattr(ML, "MOTION_POOL", True)
    clips = _clips(9)
    lib = _lib(clips, -1, True)
    lib._gather_clips(np.array([0, 3]))
    pool = lib._pool
    q, _, _, c, _, _ = lib._gather_clips(np.array([8, 8, 1]))
    assert lib._pool is pool and q.shape[0] == sum(c)
    np.testing.assert_array_equal(q[: c[0]].numpy(), clips["clip_0008"]["pose_quat_global"])


def test_pool_chunked_upload(monkeypatch):
    """Clips staged over several host chunks land at their offsets."""
    monkeypatch.setattr(ML.ClipPool, "CHUNK_FRAMES", 50)
    clips = _clips(20, lo=10, hi=45)
    pool = ML.ClipPool(list(clips.values()), "cpu")
    for i, c in enumerate(clips.values()):
        s, n = pool.starts[i], pool.lens[i]
        np.testing.assert_array_equal(pool.quat[s:s + n].numpy(), c["pose_quat_global"])
        np.testing.assert_array_equal(pool.trans[s:s + n].numpy(), c["root_trans_offset"].numpy())
        np.testing.assert_array_equal(pool.aa[s:s + n].numpy(), c["pose_aa"].reshape(n, -1))


def test_pool_falls_back_to_the_loop_when_it_does_not_fit(monkeypatch):
    """the pool is built only when it fits the free-memory budget; else the per-clip loop
    (same values) and no pool."""
    clips = _clips(9)
    ids = np.array([0, 3, 8, 8])
    monkeypatch.setattr(ML, "MOTION_POOL", True)
    monkeypatch.setattr(ML, "POOL_MAX_FREE_FRACTION", 0.0)
    lib = _lib(clips, -1, True)
    out = lib._gather_clips(ids)
    assert lib._pool is False
    monkeypatch.setattr(ML, "MOTION_POOL", False)
    ref = _lib(clips, -1, True)._gather_clips(ids)
    for x, y in zip(out[:3], ref[:3]):
        assert torch.equal(x, y)
    frames = sum(c["root_trans_offset"].shape[0] for c in clips.values())
    assert ML.ClipPool.footprint(list(clips.values())) == 8 * frames * (24 * 4 + 3 + 72)
