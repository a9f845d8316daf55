"""HIP kernels vs the reference's golden vectors and the CPU oracle (needs an MI355X).

Tolerances (BASELINE north_star): float32 obs / reward / motion state within atol 1e-5,
rtol 1e-5; frame indices, reset / terminate flags and counters bit-exact (ties of a reset
distance within 1e-6 of its threshold are excluded from the bit-exact flag comparison).
"""

import numpy as np
import pytest
import torch

from oracle import phc_oracle as O

pytestmark = pytest.mark.gpu

ATOL = 1e-5
RTOL = 1e-5
DEV = "cuda:0"


def close(a, b, atol=ATOL, rtol=RTOL):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    np.testing.assert_allclose(a.astype(np.float64), np.asarray(b, np.float64), atol=atol, rtol=rtol)


@pytest.fixture(scope="module")
def N():
    from puffer_phc_amd import _native

    _native.lib()
    return _native


def _t(x, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(DEV)


class DevLib:
    """Device copy of a packed motion library (tensors kept alive for the C struct)."""

    def __init__(self, N, gts, grs, lrs, gvs, gavs, dvs, lengths, dts, nframes, starts):
        self.frames = _t(np.concatenate([gts, grs, gvs, gavs], -1).astype(np.float32))
        self.lrs = _t(lrs.astype(np.float32))
        self.dvs = _t(dvs.astype(np.float32))
        self.len = _t(lengths.astype(np.float32))
        self.dt = _t(dts.astype(np.float32))
        self.nf = _t(nframes.astype(np.int64))
        self.ls = _t(starts.astype(np.int64))
        self.c = N.motion_lib_struct(self.frames, self.lrs, self.dvs, self.len, self.dt, self.nf, self.ls)


@pytest.fixture(scope="module")
def golden_lib(golden, N):
    m = golden("motion_lib")
    return DevLib(N, m["gts"], m["grs"], m["lrs"], m["gvs"], m["gavs"], m["dvs"], m["motion_lengths"],
                  m["motion_dt"], m["motion_num_frames"], m["length_starts"])


@pytest.fixture(scope="module")
def oracle_lib(golden):
    m = golden("motion_lib")
    return O.MotionLib(m["gts"], m["grs"], m["lrs"], m["gvs"], m["gavs"], m["dvs"], m["motion_num_frames"],
                       m["motion_fps"])


def test_motion_state_vs_reference(golden, golden_lib, N):
    g = golden("motion_state")
    body, dof_pos, dof_vel = N.motion_state(golden_lib.c, _t(g["motion_ids"]), _t(g["motion_times"]),
                                            _t(g["offset"]))
    torch.cuda.synchronize()
    b = body.cpu().numpy()
    np.testing.assert_array_equal(b[..., 0:3], g["rg_pos"])  # exact IEEE lerp + offset
    close(b[..., 3:7], g["rb_rot"])
    close(b[..., 7:10], g["body_vel"])
    close(b[..., 10:13], g["body_ang_vel"])
    close(dof_pos, g["dof_pos"])
    close(dof_vel, g["dof_vel"])


def _env_buffers(N, n, rb, dof_vel, dof_force, mids, progress, start, start_off, goff, with_book=True):
    bufs = dict(
        rigid_body_state=_t(rb.astype(np.float32)),
        root_state=torch.zeros((n, 13), dtype=torch.float32, device=DEV),
        dof_state=_t(np.stack([np.zeros_like(dof_vel), dof_vel], -1).astype(np.float32)),
        dof_force=_t(dof_force.astype(np.float32)),
        progress=_t(progress.astype(np.int16)),
        motion_ids=_t(mids.astype(np.int64)),
        start_times=_t(start.astype(np.float32)),
        start_offset=_t(start_off.astype(np.float32)),
        global_offset=_t(goff.astype(np.float32)),
        obs=torch.full((n, 934), np.nan, dtype=torch.float32, device=DEV),
        rew=torch.zeros(n, dtype=torch.float32, device=DEV),
        reward_raw=torch.zeros((n, 5), dtype=torch.float32, device=DEV),
        reset=torch.zeros(n, dtype=torch.bool, device=DEV),
        terminate=torch.zeros(n, dtype=torch.bool, device=DEV),
    )
    if with_book:
        bufs.update(
            terminals=torch.zeros(n, dtype=torch.bool, device=DEV),
            truncations=torch.zeros(n, dtype=torch.bool, device=DEV),
            masks=torch.ones(n, dtype=torch.bool, device=DEV),
            episode_return=torch.rand(n, device=DEV),
            episode_length=torch.randint(0, 50, (n,), dtype=torch.int32, device=DEV),
            stats=torch.zeros((N.lib().phc_stats_blocks(n), N.STATS_SLOTS), dtype=torch.float64, device=DEV),
        )
    c = N.env_struct(n, **bufs)
    return bufs, c


def _params(N, reset_ids, term_dist, use_mean):
    from types import SimpleNamespace

    rw = SimpleNamespace(**O.REWARD)
    return N.step_params_struct(float(O.DT), rw, 0.0005, True, True, use_mean, reset_ids, term_dist)


@pytest.mark.parametrize("mode", ["train", "eval"])
def test_env_step_vs_reference(golden, golden_lib, N, mode):
    g = golden("env_step")
    n = len(g["motion_ids"])
    bufs, c = _env_buffers(N, n, g["rb_state"], g["dof_vel"], g["dof_force"], g["motion_ids"],
                           g["progress"].astype(np.int32) - 1, g["start"], g["start_offset"], g["global_offset"])
    ret0 = bufs["episode_return"].clone()
    len0 = bufs["episode_length"].clone()
    if mode == "train":
        p = _params(N, g["reset_body_ids"], g["term_dist"], False)
    else:
        p = _params(N, g["eval_reset_body_ids"], g["eval_term_dist"], True)
    N.env_step(c, golden_lib.c, p)
    torch.cuda.synchronize()
    pre = mode + "_"
    close(bufs["obs"], g[pre + "obs"])
    close(bufs["rew"], g[pre + "rew"])
    close(bufs["reward_raw"], g[pre + "reward_raw"])
    np.testing.assert_array_equal(bufs["progress"].cpu().numpy(), g["progress"])
    ties = np.any(np.abs(g[pre + "reset_dist"] - (0.25 if mode == "train" else 0.5)) < 1e-6, -1)
    reset = bufs["reset"].cpu().numpy()
    term = bufs["terminate"].cpu().numpy()
    np.testing.assert_array_equal(reset[~ties], g[pre + "reset"][~ties])
    np.testing.assert_array_equal(term[~ties], g[pre + "terminate"][~ties])
    # PHCPufferEnv bookkeeping (clean_pufferl/env.py:103-140)
    np.testing.assert_array_equal(bufs["terminals"].cpu().numpy(), term)
    np.testing.assert_array_equal(bufs["truncations"].cpu().numpy(), reset & ~term)
    np.testing.assert_array_equal(bufs["masks"].cpu().numpy(), ~(reset & ~term))
    rew = bufs["rew"].cpu().numpy()
    exp_ret = np.where(reset, 0.0, ret0.cpu().numpy()) + rew
    exp_len = np.where(reset, 0, len0.cpu().numpy()) + 1
    np.testing.assert_allclose(bufs["episode_return"].cpu().numpy(), exp_ret, rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(bufs["episode_length"].cpu().numpy(), exp_len)
    st = bufs["stats"].sum(0).cpu().numpy()
    np.testing.assert_allclose(st[0:5], g[pre + "reward_raw"].astype(np.float64).sum(0), rtol=1e-5, atol=1e-4)
    assert st[7] == reset.sum() and st[8] == (reset & ~term).sum() and st[9] == term.sum()
    np.testing.assert_allclose(st[5], ret0.cpu().numpy()[reset].astype(np.float64).sum(), rtol=1e-6)
    assert st[6] == len0.cpu().numpy()[reset].sum()


def test_reset_envs_vs_reference(golden, golden_lib, N):
    g = golden("reset")
    n = len(g["motion_ids"])
    z3 = np.zeros((n, 3), np.float32)
    rb = np.zeros((n, 24, 13), np.float32)
    bufs, c = _env_buffers(N, n, rb, np.zeros((n, 69)), np.zeros((n, 69)), g["motion_ids"],
                           np.full(n, 17), np.full(n, 5.0), np.full(n, 0.3), g["global_offset_old"], False)
    bufs["reset"].fill_(True)
    bufs["terminate"].fill_(True)
    p = _params(N, np.arange(24), np.full(24, 0.25), False)
    N.reset_envs(c, golden_lib.c, p, mask=None, phase=_t(g["phase"]))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(bufs["start_times"].cpu().numpy(), g["motion_times"])
    rbs = bufs["rigid_body_state"].cpu().numpy()
    np.testing.assert_array_equal(rbs[..., 0:3], g["ref_rg_pos"])
    close(rbs[..., 3:7], g["ref_rb_rot"])
    close(rbs[..., 7:10], g["ref_body_vel"])
    close(rbs[..., 10:13], g["ref_body_ang_vel"])
    np.testing.assert_array_equal(bufs["root_state"].cpu().numpy(), rbs[:, 0])
    ds = bufs["dof_state"].cpu().numpy()
    close(ds[..., 0], g["ref_dof_pos"])
    close(ds[..., 1], g["ref_dof_vel"])
    close(bufs["obs"], g["obs"])
    assert (bufs["progress"] == 0).all() and not bufs["reset"].any() and not bufs["terminate"].any()
    assert (bufs["global_offset"] == 0).all() and (bufs["start_offset"] == 0).all()


def test_reset_envs_mask_only_touches_masked(golden, golden_lib, N):
    g = golden("reset")
    n = len(g["motion_ids"])
    rb = np.random.default_rng(0).normal(size=(n, 24, 13)).astype(np.float32)
    bufs, c = _env_buffers(N, n, rb, np.zeros((n, 69)), np.zeros((n, 69)), g["motion_ids"], np.full(n, 17),
                           np.full(n, 5.0), np.full(n, 0.3), g["global_offset_old"], False)
    mask = torch.zeros(n, dtype=torch.bool, device=DEV)
    mask[::3] = True
    before = {k: v.clone() for k, v in bufs.items()}
    N.reset_envs(c, golden_lib.c, _params(N, np.arange(24), np.full(24, 0.25), False), mask=mask,
                 phase=_t(g["phase"]))
    torch.cuda.synchronize()
    keep = ~mask
    for k in ("rigid_body_state", "progress", "start_times", "global_offset", "dof_state"):
        assert torch.equal(bufs[k][keep], before[k][keep]), k
    assert (bufs["progress"][mask] == 0).all()
    np.testing.assert_array_equal(bufs["start_times"][mask].cpu().numpy(), g["motion_times"][::3])


def test_env_step_auto_reset_equals_step_then_reset(golden, golden_lib, N):
    """The fused in-launch reset must equal env_step followed by phc_reset_envs, bit for bit."""
    g = golden("env_step")
    n = len(g["motion_ids"])
    outs = []
    for auto in (True, False):
        bufs, _ = _env_buffers(N, n, g["rb_state"], g["dof_vel"], g["dof_force"], g["motion_ids"],
                               g["progress"].astype(np.int32) - 1, g["start"], g["start_offset"],
                               g["global_offset"])
        bufs["episode_return"].zero_()
        bufs["episode_length"].zero_()
        bufs["rng_counter"] = torch.arange(n, dtype=torch.int32, device=DEV) * 3
        c = N.env_struct(n, **bufs)
        from types import SimpleNamespace

        p = N.step_params_struct(float(O.DT), SimpleNamespace(**O.REWARD), 0.0005, True, True, False,
                                 np.arange(24), np.full(24, 0.25), auto_reset=auto, seed=1234)
        N.env_step(c, golden_lib.c, p)
        if not auto:
            N.reset_envs(c, golden_lib.c, p, mask=None, phase=None, seed=1234)
        torch.cuda.synchronize()
        outs.append({k: v.clone() for k, v in bufs.items()})
    a, b = outs
    assert g["train_reset"].any()
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert not a["reset"].any()
    np.testing.assert_array_equal(a["terminals"].cpu().numpy(), g["train_terminate"])


def test_fk_vs_reference(golden, N):
    s, m = golden("skeleton"), golden("motion_lib")
    order = m["sample_idxes"]
    q = np.concatenate([m[f"in_quat_{i}"] for i in order])
    tr = np.concatenate([m[f"in_trans_{i}"] for i in order])
    counts = m["motion_num_frames"]
    starts = m["length_starts"]
    frames, lrs, dvs = N.fk_motions(_t(q), _t(tr), _t(starts), _t(counts), _t(np.full(len(counts), 30.0, np.float32)),
                                    _t(s["parent_indices"]), _t(s["local_translation"]),
                                    _t(O.gaussian_weights()))
    torch.cuda.synchronize()
    fr = frames.cpu().numpy()
    close(fr[..., 0:3], m["gts"], atol=2e-5)
    np.testing.assert_array_equal(fr[..., 3:7], m["grs"])
    close(fr[..., 7:10], m["gvs"], atol=2e-5)
    close(fr[..., 10:13], m["gavs"], atol=2e-5)
    close(lrs, m["lrs"])
    close(dvs, m["dvs"], atol=2e-5)


def test_gae_vs_reference(golden, N):
    g = golden("gae")
    for sfx in ("", "2"):
        adv = N.compute_gae(_t(g["dones" + sfx]), _t(g["values" + sfx]), _t(g["rewards" + sfx]),
                            float(g["gamma" + sfx]), float(g["lam" + sfx]))
        torch.cuda.synchronize()
        close(adv, g["adv" + sfx], atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("n", [1, 2, 17, 4097, 131072])
def test_gae_sizes_vs_oracle(N, n):
    rng = np.random.default_rng(n)
    d = (rng.random(n) < 0.02).astype(np.float32)
    v = rng.normal(size=n).astype(np.float32)
    r = rng.random(n).astype(np.float32)
    ref = O.compute_gae(d, v, r, 0.98, 0.2) if n <= 4097 else None
    adv = N.compute_gae(_t(d), _t(v), _t(r), 0.98, 0.2).cpu().numpy()
    if ref is not None:
        np.testing.assert_allclose(adv, ref, atol=1e-5, rtol=1e-5)
    else:
        # size-independent property: the recurrence holds element by element
        nnt = 1 - d[1:]
        lhs = adv[:-1]
        rhs = (r[1:] + np.float32(0.98) * v[1:] * nnt - v[:-1]) + np.float32(0.98 * 0.2) * nnt * adv[1:]
        np.testing.assert_allclose(lhs, rhs, atol=2e-5, rtol=1e-5)
        assert adv[-1] == 0


def test_rms_vs_reference(golden, N):
    g = golden("rms")
    F = g["x1"].shape[1]
    mean = torch.zeros((1, F), device=DEV)
    var = torch.ones((1, F), device=DEV)
    count = torch.ones(1, device=DEV)
    N.rms_update(_t(g["x1"]), mean, var, count)
    torch.cuda.synchronize()
    close(mean, g["mean1"])
    close(var, g["var1"])
    assert count.item() == g["count1"][0]
    N.rms_update(_t(g["x2"]), mean, var, count)
    close(mean, g["mean2"])
    close(var, g["var2"])
    y = N.rms_normalize(_t(g["xq"]), mean, var)
    close(y, g["y"], atol=2e-5)


def test_actions_to_pd_vs_oracle(N):
    rng = np.random.default_rng(3)
    a = (rng.normal(size=(1000, 69)) * 2).astype(np.float32)
    off, scale = O.pd_action_scale()
    frozen = np.zeros(69, np.uint8)
    frozen[O.FROZEN_DOFS] = 1
    pd = torch.empty((1000, 69), device=DEV)
    N.actions_to_pd(_t(a), pd, _t(off), _t(scale), _t(frozen))
    np.testing.assert_array_equal(pd.cpu().numpy(), O.actions_to_pd(a))
    # EnvConfig.clip_actions = False: no clip (clean_pufferl/env.py:91)
    N.actions_to_pd(_t(a), pd, _t(off), _t(scale), _t(frozen), clip=False)
    np.testing.assert_array_equal(pd.cpu().numpy(), O.actions_to_pd(a, clip=False))
    assert np.abs(pd.cpu().numpy()).max() > np.pi * 1.5


@pytest.mark.parametrize("physics", ["replay", "articulated"])
def test_env_honours_clip_actions(physics):
    """cfg.clip_actions reaches every folded action -> PD map (the fused replay launch and the
    articulated physics launch): with it off the PD targets are offset + scale * a unclipped."""
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    for clip in (True, False):
        q, t, c, fps = synthetic_clips(4, 20, 60, seed=1, device=DEV)
        env = PHCPufferEnv(EnvConfig(num_envs=8, seed=1, clip_actions=clip, physics=physics),
                           motion_data=PackedMotions.from_global_rotations(q, t, c, fps))
        env.reset()
        act = torch.randn((8, 69), device=DEV, generator=torch.Generator(device=DEV).manual_seed(2)) * 3
        env.step(act)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(env.env.pd_target.cpu().numpy(), O.actions_to_pd(act.cpu().numpy(), clip=clip))


def test_bad_arguments_raise(N, golden_lib):
    with pytest.raises(ValueError):
        N.motion_state(golden_lib.c, torch.zeros(4, dtype=torch.int32, device=DEV), torch.zeros(4, device=DEV))
    with pytest.raises(ValueError):
        N.motion_state(golden_lib.c, torch.zeros(4, dtype=torch.int64), torch.zeros(4))
    body, _, _ = N.motion_state(golden_lib.c, torch.zeros(0, dtype=torch.int64, device=DEV),
                                torch.zeros(0, device=DEV))
    assert body.shape == (0, 24, 13)
