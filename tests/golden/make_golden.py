"""Generate the golden fixtures that pin the CPU oracle and the HIP path.

Runs ONLY in the build container, where the reference is mounted read-only at
/root/reference.  It imports the reference's own modules (torch_utils, envs/common,
poselib_skeleton, motion_lib, policies, c_gae.pyx) and records inputs + outputs as
small .npz files under tests/golden/.  Nothing from the reference is copied; the
fixtures are data (inputs and the reference's outputs on them).

Stubs used (test tooling, never shipped): `smpl_sim.smpllib.smpl_parser.SMPL_Parser`
(only used by the SMPL height fix, which needs license-gated model files),
`tyro.conf.{Suppress,Fixed}` (identity generics) and `pufferlib.pytorch.layer_init`
(for the state-dict key list only).

The reference's sample clip (sample_data/cmu_mocap_05_06.pkl) is a joblib pickle; this
round's rules forbid unpickling files shipped inside the reference, so the motion
fixtures use synthetic clips of the same schema (24 joints, 30 fps, f64 global quats,
f64 root translation) written by this script.

Usage:  python tests/golden/make_golden.py
"""

import os
import sys
import types
import tempfile
from types import SimpleNamespace

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# ---------------------------------------------------------------- stubs ----
def _install_stubs():
    smpl_sim = types.ModuleType("smpl_sim")
    smpllib = types.ModuleType("smpl_sim.smpllib")
    parser = types.ModuleType("smpl_sim.smpllib.smpl_parser")

    class SMPL_Parser:  # noqa: N801 - stub for an un-vendored dependency
        def __init__(self, *a, **k):  # constructed by MotionLibSMPL, never used (mesh_parsers=None)
            pass

    parser.SMPL_Parser = SMPL_Parser
    sys.modules["smpl_sim"] = smpl_sim
    sys.modules["smpl_sim.smpllib"] = smpllib
    sys.modules["smpl_sim.smpllib.smpl_parser"] = parser

    tyro = types.ModuleType("tyro")
    conf = types.ModuleType("tyro.conf")

    class _Ident:
        def __class_getitem__(cls, item):
            return item

    conf.Suppress = _Ident
    conf.Fixed = _Ident
    tyro.conf = conf
    sys.modules["tyro"] = tyro
    sys.modules["tyro.conf"] = conf

    puffer = types.ModuleType("pufferlib")
    ppt = types.ModuleType("pufferlib.pytorch")
    pmodels = types.ModuleType("pufferlib.models")

    def layer_init(layer, std=np.sqrt(2), bias_const=0.0):
        torch.nn.init.orthogonal_(layer.weight, std)
        torch.nn.init.constant_(layer.bias, bias_const)
        return layer

    class LSTMWrapper(torch.nn.Module):
        def __init__(self, *a, **k):
            super().__init__()

    ppt.layer_init = layer_init
    pmodels.LSTMWrapper = LSTMWrapper
    puffer.pytorch = ppt
    puffer.models = pmodels
    sys.modules["pufferlib"] = puffer
    sys.modules["pufferlib.pytorch"] = ppt
    sys.modules["pufferlib.models"] = pmodels


_install_stubs()
sys.path.insert(0, REF)

from puffer_phc import torch_utils as tu  # noqa: E402
from puffer_phc.envs import common  # noqa: E402
from puffer_phc.poselib_skeleton import SkeletonTree  # noqa: E402
from puffer_phc import motion_lib as ml  # noqa: E402
from puffer_phc.body_sets import BODY_NAMES, DOF_NAMES, REMOVE_NAMES, KEY_BODIES, EVAL_BODIES  # noqa: E402
from puffer_phc.config import RewardConfig  # noqa: E402
from dataclasses import asdict  # noqa: E402

torch.set_num_threads(1)
DT = 2 * (1.0 / 60.0)  # IsaacGymBase.dt (puffer_phc/envs/isaacgym_env.py:41)


# ------------------------------------------------------ synthetic motion ----
def _rand_unit_quat(rng, n):
    q = rng.normal(size=(n, 4))
    return q / np.linalg.norm(q, axis=-1, keepdims=True)


def _slerp_np(q0, q1, t):
    d = np.sum(q0 * q1, -1, keepdims=True)
    q1 = np.where(d < 0, -q1, q1)
    d = np.abs(d)
    th = np.arccos(np.clip(d, -1, 1))
    s = np.sin(th)
    a = np.where(s < 1e-6, 1 - t, np.sin((1 - t) * th) / np.where(s < 1e-6, 1, s))
    b = np.where(s < 1e-6, t, np.sin(t * th) / np.where(s < 1e-6, 1, s))
    q = a * q0 + b * q1
    return q / np.linalg.norm(q, axis=-1, keepdims=True)


def synth_motion(rng, num_frames, num_joints=24, key_every=15):
    """Smooth synthetic clip: global rotations slerped between random keyframes that stay
    near an upright pose, root translation = smoothed random walk at ~0.9 m height."""
    nkeys = num_frames // key_every + 2
    base = np.tile(np.array([0.0, 0.0, 0.0, 1.0]), (num_joints, 1))
    keys = []
    for _ in range(nkeys):
        pert = rng.normal(scale=0.35, size=(num_joints, 4))
        k = base + pert
        k /= np.linalg.norm(k, axis=-1, keepdims=True)
        keys.append(k)
    keys = np.stack(keys)
    quats = np.zeros((num_frames, num_joints, 4))
    for f in range(num_frames):
        k0, r = divmod(f, key_every)
        quats[f] = _slerp_np(keys[k0], keys[k0 + 1], r / key_every)
    # random sign flips (the loader must handle q and -q)
    flip = rng.random((num_frames, num_joints, 1)) < 0.1
    quats = np.where(flip, -quats, quats)
    steps = rng.normal(scale=0.02, size=(num_frames, 3))
    steps[:, 2] *= 0.2
    trans = np.cumsum(steps, 0)
    trans[:, 2] += 0.9
    pose_aa = rng.normal(scale=0.3, size=(num_frames, num_joints * 3))
    return {
        "root_trans_offset": torch.from_numpy(trans),
        "pose_aa": pose_aa,
        "pose_quat_global": quats,
        "beta": np.zeros(16),
        "gender": "neutral",
        "fps": 30,
    }


# ------------------------------------------------------------ fixtures ----
def gen_skeleton():
    sk = SkeletonTree.from_mjcf(os.path.join(REF, "puffer_phc/assets/smpl_humanoid.xml"))
    out = dict(
        node_names=np.array(sk.node_names),
        parent_indices=sk.parent_indices.numpy().astype(np.int64),
        local_translation=sk.local_translation.numpy().astype(np.float32),
    )
    np.savez_compressed(os.path.join(OUT, "skeleton.npz"), **out)
    return sk


def gen_motion_lib(sk, lengths=(47, 61, 90, 150, 5, 2), num_envs=8, seed=0):
    rng = np.random.default_rng(seed)
    import joblib

    motions = {f"synth_{i:02d}": synth_motion(rng, n) for i, n in enumerate(lengths)}
    tmp = tempfile.mkdtemp()
    path = os.path.join(tmp, "synth_motions.pkl")
    joblib.dump(motions, path)  # our own file

    cfg = SimpleNamespace(
        motion_file=path,
        device="cpu",
        fix_height=ml.FixHeightMode.no_fix,
        min_length=-1,
        max_length=300,
        im_eval=False,
        num_thread=1,
        smpl_type="smpl",
        step_dt=DT,
        is_deterministic=True,
    )
    lib = ml.MotionLibSMPL(cfg)
    lib.mesh_parsers = None
    lib.load_motions(
        skeleton_trees=[sk] * num_envs,
        gender_betas=torch.zeros(num_envs, 17),
        limb_weights=torch.zeros(num_envs, 10),
        random_sample=False,
        start_idx=0,
    )
    inp = {}
    for i, (k, m) in enumerate(motions.items()):
        inp[f"in_quat_{i}"] = m["pose_quat_global"]
        inp[f"in_trans_{i}"] = m["root_trans_offset"].numpy()
    out = dict(
        num_input_motions=np.int64(len(lengths)),
        sample_idxes=lib._curr_motion_ids.numpy().astype(np.int64),
        gts=lib.gts.numpy(),
        grs=lib.grs.numpy(),
        lrs=lib.lrs.numpy(),
        grvs=lib.grvs.numpy(),
        gravs=lib.gravs.numpy(),
        gavs=lib.gavs.numpy(),
        gvs=lib.gvs.numpy(),
        dvs=lib.dvs.numpy(),
        length_starts=lib.length_starts.numpy().astype(np.int64),
        motion_lengths=lib._motion_lengths.numpy(),
        motion_num_frames=lib._motion_num_frames.numpy().astype(np.int64),
        motion_dt=lib._motion_dt.numpy(),
        motion_fps=lib._motion_fps.numpy(),
        **inp,
    )
    np.savez_compressed(os.path.join(OUT, "motion_lib.npz"), **out)
    return lib


def _motion_state_np(res):
    keys = ["root_pos", "root_rot", "dof_pos", "root_vel", "root_ang_vel", "dof_vel",
            "rg_pos", "rb_rot", "body_vel", "body_ang_vel"]
    return {k: res[k].numpy().astype(np.float32) for k in keys}


def gen_motion_state(lib, seed=1):
    rng = np.random.default_rng(seed)
    n = 96
    M = lib._num_motions
    ids = rng.integers(0, M, size=n).astype(np.int64)
    lens = lib._motion_lengths.numpy()[ids]
    nf = lib._motion_num_frames.numpy()[ids]
    t = (rng.random(n) * 1.2 - 0.1) * lens
    # exact frame boundaries, t<0, t>len, t==len, tiny motions
    t[:12] = np.floor(rng.random(12) * nf[:12]) / 30.0
    t[12:16] = -rng.random(4)
    t[16:20] = lens[16:20] + rng.random(4)
    t[20:24] = lens[20:24]
    t = t.astype(np.float32)
    offset = (rng.normal(size=(n, 3)) * 0.5).astype(np.float32)
    offset[: n // 2] = 0
    res = lib.get_motion_state(torch.from_numpy(ids), torch.from_numpy(t), torch.from_numpy(offset))
    out = dict(motion_ids=ids, motion_times=t, offset=offset, **_motion_state_np(res))
    # _calc_frame_blend indices (bit-exact targets)
    f0, f1, blend = lib._calc_frame_blend(
        torch.from_numpy(t), lib._motion_lengths[ids], lib._motion_num_frames[ids], lib._motion_dt[ids]
    )
    out.update(frame_idx0=f0.numpy().astype(np.int64), frame_idx1=f1.numpy().astype(np.int64),
               blend=blend.numpy().astype(np.float32))
    np.savez_compressed(os.path.join(OUT, "motion_state.npz"), **out)


def _compose_step(lib, motion_ids, progress, start, start_off, goffset, rb_state, dof_vel, dof_force,
                  term_dist, reset_body_ids, use_mean, enable_et=True):
    """HumanoidPHC.step post-physics composition (humanoid_phc.py:136-146, 1228-1333, 935-1112).
    `progress` is the value AFTER `progress_buf += 1`."""
    rwd = asdict(RewardConfig())
    prog = torch.from_numpy(progress)
    body = torch.from_numpy(rb_state)
    body_pos, body_rot, body_vel, body_ang_vel = body[..., 0:3], body[..., 3:7], body[..., 7:10], body[..., 10:13]
    mids = torch.from_numpy(motion_ids)
    st = torch.from_numpy(start)
    so = torch.from_numpy(start_off)
    go = torch.from_numpy(goffset)

    # reward (time t)
    t = prog * DT + st + so
    res = lib.get_motion_state(mids, t, go)
    rew, rraw = common.compute_imitation_reward(
        body_pos[:, 0], body_rot[:, 0], body_pos, body_rot, body_vel, body_ang_vel,
        res["rg_pos"], res["rb_rot"], res["body_vel"], res["body_ang_vel"], rwd)
    power = torch.abs(torch.multiply(torch.from_numpy(dof_force), torch.from_numpy(dof_vel))).sum(dim=-1)
    power_reward = -0.0005 * power
    power_reward[prog <= 3] = 0
    rew = rew + power_reward
    reward_raw = torch.cat([rraw, power_reward[:, None]], -1)

    # reset (time t)
    pass_time = t >= lib._motion_lengths[mids]
    rb_ids = torch.from_numpy(reset_body_ids)
    reset_buf = torch.zeros(len(mids), dtype=torch.bool)
    reset, term = common.compute_humanoid_im_reset(
        reset_buf, prog, torch.zeros(len(mids), 24, 3), torch.zeros(4, dtype=torch.long),
        body_pos[:, rb_ids].clone(), res["rg_pos"][:, rb_ids].clone(), pass_time, enable_et,
        torch.from_numpy(term_dist)[rb_ids], use_mean)

    # obs (time t + dt)
    t1 = (prog + 1) * DT + st + so
    res1 = lib.get_motion_state(mids, t1, go)
    self_obs = common.compute_humanoid_observations_smpl_max(
        body_pos, body_rot, body_vel, body_ang_vel, None, None, True, True, True, False, False)
    task_obs = common.compute_imitation_observations_v6(
        body_pos[:, 0], body_rot[:, 0], body_pos, body_rot, body_vel, body_ang_vel,
        res1["rg_pos"], res1["rb_rot"], res1["body_vel"], res1["body_ang_vel"], 1, True)
    obs = torch.cat([self_obs, task_obs], -1)
    # the per-body distances behind the reset decision (for margin-aware comparisons)
    dist = torch.norm(body_pos[:, rb_ids] - res["rg_pos"][:, rb_ids], dim=-1)
    return dict(rew=rew.numpy(), reward_raw=reward_raw.numpy(), reset=reset.numpy(),
                terminate=term.numpy(), obs=obs.numpy(), time=t.numpy(), time_next=t1.numpy(),
                reset_dist=dist.numpy())


def _noisy_states(rng, lib, mids, t_eval, go, pos_sigma=0.02):
    res = lib.get_motion_state(torch.from_numpy(mids), torch.from_numpy(t_eval), torch.from_numpy(go))
    n = len(mids)
    pos = res["rg_pos"].numpy() + rng.normal(scale=pos_sigma, size=(n, 24, 3))
    rot = res["rb_rot"].numpy() + rng.normal(scale=0.05, size=(n, 24, 4))
    rot /= np.linalg.norm(rot, axis=-1, keepdims=True)
    vel = res["body_vel"].numpy() + rng.normal(scale=0.3, size=(n, 24, 3))
    avel = res["body_ang_vel"].numpy() + rng.normal(scale=0.5, size=(n, 24, 3))
    return np.concatenate([pos, rot, vel, avel], -1).astype(np.float32)


def gen_step(lib, seed=2, n=64):
    rng = np.random.default_rng(seed)
    M = lib._num_motions
    mids = rng.integers(0, M, size=n).astype(np.int64)
    nf = lib._motion_num_frames.numpy()[mids]
    lens = lib._motion_lengths.numpy()[mids]
    # start times snapped to 1/30 like sample_time_interval
    start = (np.floor(rng.random(n) * lens / np.float32(1 / 30)) * np.float32(1 / 30)).astype(np.float32)
    room = np.maximum(1, np.floor((lens - start) * 30)).astype(np.int64)
    progress = (rng.random(n) * room).astype(np.int16)
    progress[:10] = np.arange(10) % 5  # progress in {0..4}
    progress[10:14] = np.ceil((lens[10:14] - start[10:14]) * 30).astype(np.int16)  # pass_time edge
    start_off = np.zeros(n, np.float32)
    start_off[20:24] = rng.random(4).astype(np.float32) * 0.1
    go = np.zeros((n, 3), np.float32)
    go[24:32, :2] = rng.normal(size=(8, 2)).astype(np.float32)
    t_eval = (progress.astype(np.float32) * np.float32(DT) + start + start_off).astype(np.float32)
    rb = _noisy_states(rng, lib, mids, t_eval, go)
    # rows far beyond / just below the 0.25 threshold on one body
    rb[40:44, 5, 0] += 0.6
    rb[44:48, :, 2] += 0.1
    rb[48:52, 17, 1] += 0.3
    dof_vel = rng.normal(size=(n, 69)).astype(np.float32)
    dof_force = rng.normal(size=(n, 69)).astype(np.float32) * 50
    term_train = np.full(24, 0.25, np.float32)
    all_ids = np.arange(24, dtype=np.int64)
    out = dict(motion_ids=mids, progress=progress, start=start, start_offset=start_off,
               global_offset=go, rb_state=rb, dof_vel=dof_vel, dof_force=dof_force,
               term_dist=term_train, reset_body_ids=all_ids)
    r = _compose_step(lib, mids, progress, start, start_off, go, rb, dof_vel, dof_force,
                      term_train, all_ids, False)
    out.update({f"train_{k}": v for k, v in r.items()})
    eval_ids = np.array([BODY_NAMES.index(b) for b in EVAL_BODIES], dtype=np.int64)
    term_eval = np.full(24, 0.5, np.float32)
    r = _compose_step(lib, mids, progress, start, start_off, go, rb, dof_vel, dof_force,
                      term_eval, eval_ids, True)
    out.update({f"eval_{k}": v for k, v in r.items()})
    out["eval_reset_body_ids"] = eval_ids
    out["eval_term_dist"] = term_eval
    np.savez_compressed(os.path.join(OUT, "env_step.npz"), **out)


def gen_reset(lib, seed=3, n=32):
    """Reset path for a subset: sample_time_interval (motion_lib.py:526-535) with a fixed
    phase, get_motion_state with the OLD global offset (humanoid_phc.py:843-873), then obs of
    the subset at progress 0 with offset 0 (humanoid_phc.py:1061-1065)."""
    rng = np.random.default_rng(seed)
    M = lib._num_motions
    mids = rng.integers(0, M, size=n).astype(np.int64)
    phase = rng.random(n).astype(np.float32)
    phase[:3] = [0.0, 0.9999999, 0.5]
    go_old = (rng.normal(size=(n, 3)) * 0.3).astype(np.float32)
    orig_rand = torch.rand
    torch.rand = lambda *a, **k: torch.from_numpy(phase.copy())
    try:
        mt = lib.sample_time_interval(torch.from_numpy(mids))
    finally:
        torch.rand = orig_rand
    res = lib.get_motion_state(torch.from_numpy(mids), mt, torch.from_numpy(go_old))
    st = _motion_state_np(res)
    rb = np.concatenate([st["rg_pos"], st["rb_rot"], st["body_vel"], st["body_ang_vel"]], -1)
    progress = np.zeros(n, np.int16)
    zero_off = np.zeros((n, 3), np.float32)
    # obs recomputed for the subset: reward/reset are not, only obs (humanoid_phc.py:663-674)
    body = torch.from_numpy(rb)
    bp, br, bv, bav = body[..., 0:3], body[..., 3:7], body[..., 7:10], body[..., 10:13]
    t1 = (torch.from_numpy(progress) + 1) * DT + mt + torch.zeros(n)
    res1 = lib.get_motion_state(torch.from_numpy(mids), t1, torch.from_numpy(zero_off))
    self_obs = common.compute_humanoid_observations_smpl_max(bp, br, bv, bav, None, None, True, True, True, False, False)
    task_obs = common.compute_imitation_observations_v6(
        bp[:, 0], br[:, 0], bp, br, bv, bav, res1["rg_pos"], res1["rb_rot"], res1["body_vel"],
        res1["body_ang_vel"], 1, True)
    obs = torch.cat([self_obs, task_obs], -1).numpy()
    np.savez_compressed(os.path.join(OUT, "reset.npz"), motion_ids=mids, phase=phase,
                        global_offset_old=go_old, motion_times=mt.numpy().astype(np.float32),
                        obs=obs, **{f"ref_{k}": v for k, v in st.items()})


def gen_amp(lib, seed=4, n=16):
    rng = np.random.default_rng(seed)
    mids = rng.integers(0, lib._num_motions, size=n).astype(np.int64)
    t = (rng.random(n) * lib._motion_lengths.numpy()[mids]).astype(np.float32)
    res = lib.get_motion_state(torch.from_numpy(mids), torch.from_numpy(t))
    key_ids = torch.tensor([BODY_NAMES.index(b) for b in KEY_BODIES])
    disc = []
    for idx, name in enumerate(DOF_NAMES):
        if name not in REMOVE_NAMES:
            disc.append(np.arange(idx * 3, (idx + 1) * 3))
    dof_subset = torch.from_numpy(np.concatenate(disc))
    amp = common.build_amp_observations_smpl(
        res["root_pos"], res["root_rot"], res["root_vel"], res["root_ang_vel"], res["dof_pos"],
        res["dof_vel"], res["rg_pos"][:, key_ids], torch.zeros(n, 11), torch.zeros(n, 10),
        dof_subset, True, True, True, False, False, True)
    np.savez_compressed(os.path.join(OUT, "amp_obs.npz"), motion_ids=mids, motion_times=t,
                        dof_subset=dof_subset.numpy().astype(np.int64), key_body_ids=key_ids.numpy(),
                        amp_obs=amp.numpy(), **{f"ref_{k}": v for k, v in _motion_state_np(res).items()})


def gen_gae(seed=5, B=4096):
    import pyximport

    pyximport.install(setup_args={"include_dirs": np.get_include()}, build_dir=tempfile.mkdtemp())
    sys.path.insert(0, os.path.join(REF, "puffer_phc"))
    from c_gae import compute_gae

    rng = np.random.default_rng(seed)
    dones = (rng.random(B) < 0.01).astype(np.float32)
    values = rng.normal(size=B).astype(np.float32)
    rewards = rng.random(B).astype(np.float32)
    adv = compute_gae(dones, values, rewards, 0.98, 0.2)
    # a second case with episodes breaking on long runs of dones and large values
    dones2 = (rng.random(B) < 0.2).astype(np.float32)
    values2 = (rng.normal(size=B) * 30).astype(np.float32)
    rewards2 = (rng.normal(size=B) * 2).astype(np.float32)
    adv2 = compute_gae(dones2, values2, rewards2, 0.99, 0.95)
    np.savez_compressed(os.path.join(OUT, "gae.npz"), dones=dones, values=values, rewards=rewards,
                        gamma=np.float32(0.98), lam=np.float32(0.2), adv=adv,
                        dones2=dones2, values2=values2, rewards2=rewards2, gamma2=np.float32(0.99),
                        lam2=np.float32(0.95), adv2=adv2)


def gen_rms(seed=6):
    from puffer_phc.policies.running_norm import RunningNorm

    rng = np.random.default_rng(seed)
    F = 934
    x1 = (rng.normal(size=(128, F)) * 3 + 1).astype(np.float32)
    x2 = (rng.normal(size=(96, F)) * 0.5 - 2).astype(np.float32)
    xq = (rng.normal(size=(16, F)) * 20).astype(np.float32)
    rn = RunningNorm(F)
    rn.update(torch.from_numpy(x1))
    m1, v1, c1 = rn.running_mean.numpy().copy(), rn.running_var.numpy().copy(), rn.count.numpy().copy()
    rn.update(torch.from_numpy(x2))
    y = rn(torch.from_numpy(xq)).detach().numpy()
    np.savez_compressed(os.path.join(OUT, "rms.npz"), x1=x1, x2=x2, xq=xq, mean1=m1, var1=v1, count1=c1,
                        mean2=rn.running_mean.numpy(), var2=rn.running_var.numpy(), count2=rn.count.numpy(), y=y)


def gen_state_dict():
    from puffer_phc.policies.phc_policy import PHCPolicy

    class Box:
        def __init__(self, n, high=1.0):
            self.shape = (n,)
            self.high = np.full(n, high, np.float32)

    rows = []
    for amp in (False, True):
        env = SimpleNamespace(single_observation_space=Box(934, np.inf), single_action_space=Box(69),
                              amp_observation_space=Box(1960, np.inf) if amp else None)
        pol = PHCPolicy(env, hidden_size=512, layer_sizes=(2048, 1536, 1024, 1024, 512))
        wrapped = torch.nn.Module()
        wrapped.policy = pol  # pufferlib.cleanrl.Policy stores the module as .policy
        for k, v in wrapped.state_dict().items():
            rows.append(f"{int(amp)}\t{k}\t{'x'.join(map(str, v.shape))}\t{str(v.dtype)}")
        n_train = sum(p.numel() for p in pol.parameters() if p.requires_grad)
        rows.append(f"{int(amp)}\t#trainable\t{n_train}\t-")
    with open(os.path.join(OUT, "state_dict_keys.tsv"), "w") as f:
        f.write("\n".join(rows) + "\n")


def lstm_fill(module):
    """Deterministic weights for the LSTM-policy fixture (the test applies the same rule to the
    port): parameter / buffer i of state_dict() order from torch.Generator seed 1000 + i."""
    with torch.no_grad():
        for i, (k, v) in enumerate(module.state_dict().items()):
            g = torch.Generator().manual_seed(1000 + i)
            x = torch.randn(v.shape, generator=g, dtype=torch.float64)
            if k.endswith("running_var"):
                x = x.abs() + 0.5
            elif k.endswith("count"):
                x = torch.full(v.shape, 10.0, dtype=torch.float64)
            elif k.endswith("sigma"):
                x = x * 0.1 - 1.0
            else:
                x = x * (0.5 / max(1, v.shape[-1]) ** 0.5)
            v.copy_(x.to(v.dtype))


def gen_lstm(seed=7, rows=8):
    """N4: LSTMCriticPolicy / LSTMActorPolicy (puffer_phc/policies/lstm_policy.py:25-148) on fixed
    weights (lstm_fill) and inputs: state-dict keys / shapes, encode_observations, decode_actions
    (Normal mean / std, value, mean bound loss in training mode).  pufferlib.models.LSTMWrapper is
    stubbed (the Recurrent wrapper itself stays unpinned)."""
    from puffer_phc.policies.lstm_policy import LSTMActorPolicy, LSTMCriticPolicy

    class Box:
        def __init__(self, n, high=1.0):
            self.shape = (n,)
            self.high = np.full(n, high, np.float32)

    rng = np.random.default_rng(seed)
    obs = (rng.normal(size=(rows, 934)) * 2).astype(np.float32)
    hid = rng.normal(size=(rows, 512)).astype(np.float32)
    out, keys = {"obs": obs, "hidden_in": hid}, []
    env = SimpleNamespace(single_observation_space=Box(934, np.inf), single_action_space=Box(69),
                          amp_observation_space=None)
    for name, cls in (("critic", LSTMCriticPolicy), ("actor", LSTMActorPolicy)):
        pol = cls(env, hidden_size=512)
        for k, v in pol.state_dict().items():
            keys.append(f"{name}\t{k}\t{'x'.join(map(str, v.shape))}\t{str(v.dtype)}")
        keys.append(f"{name}\t#trainable\t{sum(p.numel() for p in pol.parameters() if p.requires_grad)}\t-")
        lstm_fill(pol)
        with torch.no_grad():
            for training in (False, True):
                pol.train(training)
                h, _ = pol.encode_observations(torch.from_numpy(obs))
                probs, value = pol.decode_actions(torch.from_numpy(hid))
                tag = f"{name}_{'train' if training else 'eval'}"
                out[f"{tag}_encoded"] = h.numpy()
                out[f"{tag}_mu"] = probs.mean.numpy()
                out[f"{tag}_std"] = probs.stddev.numpy()
                out[f"{tag}_value"] = value.numpy()
                if training:
                    out[f"{tag}_bound"] = np.float32(pol.mean_bound_loss)
    np.savez_compressed(os.path.join(OUT, "lstm_policy.npz"), **out)
    with open(os.path.join(OUT, "lstm_state_dict_keys.tsv"), "w") as f:
        f.write("\n".join(keys) + "\n")


if __name__ == "__main__" and len(sys.argv) > 1:  # only the named generators, e.g. `make_golden.py lstm`
    for name in sys.argv[1:]:
        globals()[f"gen_{name}"]()
elif __name__ == "__main__":
    sk = gen_skeleton()
    lib = gen_motion_lib(sk)
    gen_motion_state(lib)
    gen_step(lib)
    gen_reset(lib)
    gen_amp(lib)
    gen_gae()
    gen_rms()
    gen_state_dict()
    gen_lstm()
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))
