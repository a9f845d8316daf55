"""Motion library: MotionLibSMPL drop-in (puffer_phc/motion_lib.py:180-825) on the HIP path.

Load path (R3-R5): the selected clips are cropped, optionally heading-randomised, packed back
to back and uploaded once as float64; forward kinematics, linear/angular velocities and dof
velocities run on the GPU (`phc_fk_motions`), producing the packed library:

    frames [F, 24, 13] = gts(3) grs(4) gvs(3) gavs(3)   one 1248-byte record per frame
    local_rot [F, 24, 4], dof_vel [F, 23, 3], motion scalars [M]

so a per-step reference lookup gathers whole 1248-byte frame rows.  Per-step queries
(get_motion_state, R6+R7) go through `phc_motion_state`; the fused env step reads the same
packed rows directly.
"""

import glob
import os
import os.path as osp
import random
from enum import Enum

import numpy as np
import torch

from . import _native
from .skeleton import SkeletonTree


class MotionlibMode(Enum):
    file = 1
    directory = 2


class FixHeightMode(Enum):
    no_fix = 0
    full_fix = 1
    ankle_fix = 2


def gaussian_weights(sigma=2.0, truncate=4.0):
    """Kernel of scipy.ndimage.gaussian_filter1d (order 0), float64, as scipy builds it."""
    radius = int(truncate * float(sigma) + 0.5)
    x = np.arange(-radius, radius + 1)
    phi = np.exp((-0.5 / (sigma * sigma) * x) * x, dtype=np.float64)
    phi /= phi.sum()
    return phi


def _quat_mul_t(a, b):
    """Hamilton product (xyzw) on torch tensors (heading randomisation only)."""
    x1, y1, z1, w1 = a.unbind(-1)
    x2, y2, z2, w2 = b.unbind(-1)
    return torch.stack([w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                        w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                        w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2,
                        w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2], -1)


class PackedMotions:
    """Device-resident packed motion library + its C-ABI descriptor."""

    def __init__(self, frames, local_rot, dof_vel, num_frames, fps):
        self.frames = frames
        self.local_rot = local_rot
        self.dof_vel = dof_vel
        self.num_frames = num_frames
        self.fps = fps
        fps64 = fps.double()
        self.motion_dt = (1.0 / fps64).float()
        self.motion_len = (1.0 / fps64 * (num_frames - 1).double()).float()
        ls = num_frames.roll(1)
        ls[0] = 0
        self.length_starts = ls.cumsum(0)
        self.c = _native.motion_lib_struct(frames, local_rot, dof_vel, self.motion_len, self.motion_dt, num_frames,
                                           self.length_starts)

    @classmethod
    def from_global_rotations(cls, quat_global, root_trans, counts, fps, skeleton=None):
        """FK + velocities on device.  quat_global f64 [F,24,4], root_trans f64 [F,3] (device),
        counts int64 [M] (device), fps float32 [M] (device)."""
        sk = skeleton or SkeletonTree.smpl()
        dev = quat_global.device
        counts = counts.to(dev, torch.int64).contiguous()
        starts = counts.roll(1)
        starts[0] = 0
        starts = starts.cumsum(0)
        frames, lrs, dvs = _native.fk_motions(
            quat_global.contiguous(), root_trans.contiguous(), starts.contiguous(), counts,
            fps.to(dev, torch.float32).contiguous(), sk.parent_indices.to(dev).contiguous(),
            sk.local_translation.to(dev).contiguous(),
            torch.from_numpy(gaussian_weights()).to(dev))
        return cls(frames, lrs, dvs, counts, fps.to(dev, torch.float32))

    # reference tensor names, as views of the packed records
    @property
    def gts(self):
        return self.frames[..., 0:3]

    @property
    def grs(self):
        return self.frames[..., 3:7]

    @property
    def gvs(self):
        return self.frames[..., 7:10]

    @property
    def gavs(self):
        return self.frames[..., 10:13]


class ClipPool:
    """Every clip of an in-memory (file-mode) library resident in HBM back to back, as float64 the way
    load_motions uploads them: quat [P, 24, 4], trans [P, 3], aa [P, A]; per-clip first frame, length
    and fps on the host.  Built once, on the first load; each (re)load then gathers the selected clips'
    cropped frames with one device index gather instead of the reference's per-clip host loop
    (load_motion_with_skeleton, motion_lib.py:766-800: crop, convert and heading-rotate each clip,
    fanned out over num_thread processes at motion_lib.py:334-368), which at C3 scale (4,096 clips
    per resample out of 11,313) is the reload's cost."""

    CHUNK_FRAMES = 1 << 18  # host staging per upload (about 200 MB of float64 rows)

    @staticmethod
    def footprint(clips):
        """Device bytes the pool of `clips` takes: float64 quat [24, 4] + trans [3] + aa [A] per frame."""
        frames = sum(int(c["root_trans_offset"].shape[0]) for c in clips)
        j = int(np.asarray(clips[0]["pose_quat_global"]).shape[1])
        n0 = int(clips[0]["root_trans_offset"].shape[0])
        a = int(np.asarray(clips[0]["pose_aa"]).reshape(n0, -1).shape[1])
        return 8 * frames * (4 * j + 3 + a)

    def __init__(self, clips, device):
        n = len(clips)
        self.lens = np.fromiter((c["root_trans_offset"].shape[0] for c in clips), np.int64, n)
        self.starts = np.concatenate([[0], np.cumsum(self.lens)[:-1]]).astype(np.int64)
        self.fps = np.fromiter((float(c.get("fps", 30)) for c in clips), np.float64, n)
        total = int(self.lens.sum())
        j = int(np.asarray(clips[0]["pose_quat_global"]).shape[1])
        a = int(np.asarray(clips[0]["pose_aa"]).reshape(self.lens[0], -1).shape[1])
        self.quat = torch.empty((total, j, 4), dtype=torch.float64, device=device)
        self.trans = torch.empty((total, 3), dtype=torch.float64, device=device)
        self.aa = torch.empty((total, a), dtype=torch.float64, device=device)
        # host staging in chunks of whole clips, one upload per chunk
        i = 0
        while i < n:
            k = i
            while k < n and (k == i or self.starts[k] + self.lens[k] - self.starts[i] <= self.CHUNK_FRAMES):
                k += 1
            f0, f1 = int(self.starts[i]), int(self.starts[k - 1] + self.lens[k - 1])
            hq = np.empty((f1 - f0, j, 4))
            ht = np.empty((f1 - f0, 3))
            ha = np.empty((f1 - f0, a))
            for c in range(i, k):
                s, e = int(self.starts[c]) - f0, int(self.starts[c] + self.lens[c]) - f0
                clip = clips[c]
                rt = clip["root_trans_offset"]
                hq[s:e] = np.asarray(clip["pose_quat_global"], np.float64)
                ht[s:e] = np.asarray(rt.numpy() if isinstance(rt, torch.Tensor) else rt, np.float64)
                ha[s:e] = np.asarray(clip["pose_aa"], np.float64).reshape(e - s, -1)
            self.quat[f0:f1].copy_(torch.from_numpy(hq))
            self.trans[f0:f1].copy_(torch.from_numpy(ht))
            self.aa[f0:f1].copy_(torch.from_numpy(ha))
            i = k

    def gather(self, ids, crop_start, counts):
        """The frames [crop_start, crop_start + count) of clips `ids` (numpy), back to back."""
        dev = self.quat.device
        n = len(ids)
        cnt = torch.from_numpy(np.asarray(counts, np.int64)).to(dev)
        total = int(np.asarray(counts).sum())
        src0 = torch.from_numpy(self.starts[ids] + crop_start).to(dev)
        dst0 = cnt.cumsum(0) - cnt
        seg = torch.repeat_interleave(torch.arange(n, device=dev), cnt, output_size=total)
        idx = torch.arange(total, device=dev) - dst0[seg] + src0[seg]
        return self.quat[idx], self.trans[idx], self.aa[idx]


# PHC_MOTION_POOL=0: the per-clip host loop for in-memory libraries too (the directory mode, whose
# clips load from disk one by one, always takes it)
MOTION_POOL = os.environ.get("PHC_MOTION_POOL", "1") != "0"
# the pool is built only when it takes at most this share of the device memory free at the first load
# (else the per-clip loop): float64 rows, 8 * (24 * 4 + 3 + A) bytes per frame (~1.4 KB for A = 72); the
# 11,313-clip AMASS library (~40 M frames) would be ~55 GB, well inside 288 GB, which an 8-rank node pays
# once per rank
POOL_MAX_FREE_FRACTION = float(os.environ.get("PHC_MOTION_POOL_MAX_FREE_FRACTION", "0.5"))


class MotionLibBase:
    def __init__(self, motion_lib_cfg):
        self.m_cfg = motion_lib_cfg
        self._sim_fps = 1 / getattr(self.m_cfg, "step_dt", 1 / 30)
        self._device = self.m_cfg.device
        self.mesh_parsers = None
        self.packed = None
        self.load_data(self.m_cfg.motion_file, min_length=self.m_cfg.min_length, im_eval=self.m_cfg.im_eval)
        self.setup_constants(fix_height=self.m_cfg.fix_height, num_thread=getattr(self.m_cfg, "num_thread", 1))

    # ------------------------------------------------------------ data --
    def load_data(self, motion_file, min_length=-1, im_eval=False):
        """motion_lib.py:192-231.  `motion_file` may also be an in-memory dict {key: clip}."""
        if isinstance(motion_file, dict):
            self.mode = MotionlibMode.file
            self._motion_data_load = motion_file
        elif osp.isfile(motion_file):
            import joblib  # user motion files are joblib pickles (scripts/convert_amass_data.py)

            self.mode = MotionlibMode.file
            self._motion_data_load = joblib.load(motion_file)
        else:
            self.mode = MotionlibMode.directory
            self._motion_data_load = glob.glob(osp.join(motion_file, "*.pkl"))
            assert len(self._motion_data_load) > 0
        if self.mode == MotionlibMode.file:
            items = list(self._motion_data_load.items())
            if min_length != -1:
                items = [(k, v) for k, v in items if len(v["pose_quat_global"]) >= min_length]
            elif im_eval:
                items = sorted(items, key=lambda e: len(e[1]["pose_quat_global"]), reverse=True)
            self._motion_data_list = [v for _, v in items]
            self._motion_data_keys = np.array([k for k, _ in items])
        else:
            self._motion_data_list = list(self._motion_data_load)
            self._motion_data_keys = np.array(self._motion_data_load)
        self._num_unique_motions = len(self._motion_data_list)

    def setup_constants(self, fix_height=FixHeightMode.full_fix, num_thread=1):
        self.fix_height = fix_height
        self.num_thread = max(num_thread, 1)
        self._curr_motion_ids = None
        n = self._num_unique_motions
        self._termination_history = torch.zeros(n, device=self._device)
        self._success_rate = torch.zeros(n, device=self._device)
        self._sampling_history = torch.zeros(n, device=self._device)
        self._sampling_prob = torch.ones(n, device=self._device) / n
        self._sampling_batch_prob = None

    def _clip(self, idx):
        c = self._motion_data_list[idx]
        if not isinstance(c, dict):
            import joblib

            key = osp.basename(c).split(".")[0]
            c = joblib.load(c)[key]
        return c

    # ----------------------------------------------------------- load ---
    def _gather_clips(self, ids):
        """The selected clips cropped to max_length (a random window unless deterministic, the
        reference's random.randint per long clip, motion_lib.py:776-781) with their heading draws
        (np.random per clip, motion_lib.py:790-793): (quat f64 [F, J, 4], trans f64 [F, 3], aa f64
        [F, A] on the device, counts, fps, heading).  The draws come from the same generators in the
        same order as the reference's loop: python `random` for the crops, then numpy for headings."""
        max_length = self.m_cfg.max_length
        randomize = not (self.m_cfg.is_deterministic or self.m_cfg.im_eval)
        dev = self._device
        pool = None
        if MOTION_POOL and self.mode == MotionlibMode.file and isinstance(self._motion_data_list[0], dict):
            pool = getattr(self, "_pool", None)
            if pool is None:  # first load: build it when it fits (else False: the per-clip loop from now on)
                need = ClipPool.footprint(self._motion_data_list)
                if str(dev).startswith("cuda"):
                    free = torch.cuda.mem_get_info(dev)[0]
                else:  # a host-memory pool (tests)
                    import psutil

                    free = psutil.virtual_memory().available
                pool = self._pool = ClipPool(self._motion_data_list, dev) if need <= POOL_MAX_FREE_FRACTION * free \
                    else False
        if pool:
            lens = pool.lens[ids]
            start = np.zeros(len(ids), np.int64)
            counts = lens.copy()
            if max_length != -1:
                long = lens >= max_length
                counts[long] = max_length
                if not self.m_cfg.is_deterministic:
                    for j in np.flatnonzero(long):
                        start[j] = random.randint(0, int(lens[j]) - max_length)
            heading = np.pi * (2 * np.random.random(len(ids)) - 1.0) if randomize else np.zeros(len(ids))
            q, t, aa = pool.gather(ids, start, counts)
            return q, t, aa, counts.tolist(), pool.fps[ids].tolist(), heading.tolist()
        quats, trans, counts, fps, aas, heading = [], [], [], [], [], []
        for idx in ids.tolist():
            clip = self._clip(idx)
            seq_len = clip["root_trans_offset"].shape[0]
            if max_length == -1 or seq_len < max_length:
                start, end = 0, seq_len
            else:
                start = 0 if self.m_cfg.is_deterministic else random.randint(0, seq_len - max_length)
                end = start + max_length
            rt = clip["root_trans_offset"]
            rt = rt.numpy() if isinstance(rt, torch.Tensor) else np.asarray(rt)
            quats.append(np.asarray(clip["pose_quat_global"][start:end], np.float64))
            trans.append(np.asarray(rt[start:end], np.float64))
            aas.append(np.asarray(clip["pose_aa"][start:end], np.float64).reshape(end - start, -1))
            counts.append(end - start)
            fps.append(float(clip.get("fps", 30)))
            heading.append(np.pi * (2 * np.random.random() - 1.0) if randomize else 0.0)
        q = torch.from_numpy(np.concatenate(quats)).to(dev)
        t = torch.from_numpy(np.concatenate(trans)).to(dev)
        aa = torch.from_numpy(np.concatenate(aas)).to(dev)
        return q, t, aa, counts, fps, heading

    def _load_motions(self, skeleton_trees, gender_betas, limb_weights, random_sample=True, start_idx=0, max_len=-1,
                      sample_idxes=None):
        """motion_lib.py:257-429 with FK on the GPU."""
        num_motion_to_load = len(skeleton_trees)
        self.num_joints = len(skeleton_trees[0])
        if sample_idxes is None or len(sample_idxes) != num_motion_to_load:
            if not self.m_cfg.is_deterministic and random_sample:
                sample_idxes = torch.multinomial(self._sampling_prob, num_samples=num_motion_to_load,
                                                 replacement=True).to(self._device)
            else:
                sample_idxes = torch.remainder(torch.arange(num_motion_to_load) + start_idx,
                                               self._num_unique_motions).to(self._device)
        sample_idxes = torch.as_tensor(sample_idxes, device=self._device).long()
        self._curr_motion_ids = sample_idxes
        self.curr_motion_keys = self._motion_data_keys[sample_idxes.cpu().numpy()]
        self._sampling_batch_prob = self._sampling_prob[sample_idxes] / self._sampling_prob[sample_idxes].sum()

        q, t, aa, counts, fps, heading = self._gather_clips(sample_idxes.cpu().numpy())
        dev = self._device
        cnt = torch.tensor(counts, dtype=torch.int64, device=dev)
        hd = torch.tensor(heading, dtype=torch.float64, device=dev)
        if bool((hd != 0).any()):
            # heading randomisation (motion_lib.py:790-800): q <- h * q, trans <- R(h) trans
            th = torch.repeat_interleave(hd, cnt)
            h = torch.zeros((th.shape[0], 4), dtype=torch.float64, device=dev)
            h[:, 2] = torch.sin(th / 2)
            h[:, 3] = torch.cos(th / 2)
            q = _quat_mul_t(h[:, None, :].expand_as(q), q).contiguous()
            c, s = torch.cos(th), torch.sin(th)
            t = torch.stack([c * t[:, 0] - s * t[:, 1], s * t[:, 0] + c * t[:, 1], t[:, 2]], -1).contiguous()
        self.packed = PackedMotions.from_global_rotations(q, t, cnt, torch.tensor(fps, device=dev),
                                                          skeleton_trees[0])
        p = self.packed
        self._motion_lengths = p.motion_len
        self._motion_fps = torch.tensor(fps, dtype=torch.float32, device=dev)
        self._motion_dt = p.motion_dt
        self._motion_num_frames = p.num_frames
        self.length_starts = p.length_starts
        self._motion_aa = aa.float()
        self._motion_bodies = torch.as_tensor(np.asarray(gender_betas), dtype=torch.float32, device=dev)
        self._motion_limb_weights = torch.as_tensor(np.asarray(limb_weights), dtype=torch.float32, device=dev)
        self._num_motions = num_motion_to_load
        self.motion_ids = torch.arange(num_motion_to_load, dtype=torch.long, device=dev)
        self.num_bodies = self.num_joints
        return p

    @classmethod
    def from_packed(cls, packed, device, step_dt=1 / 30):
        """A library over an already-packed set of clips (synthetic data built on device)."""
        from types import SimpleNamespace

        self = cls.__new__(cls)
        self.m_cfg = SimpleNamespace(motion_file=None, device=device, fix_height=FixHeightMode.no_fix, min_length=-1,
                                     max_length=-1, im_eval=False, num_thread=1, smpl_type="smpl", step_dt=step_dt,
                                     is_deterministic=True)
        self._sim_fps = 1 / step_dt
        self._device = device
        self.mesh_parsers = None
        M = packed.num_frames.shape[0]
        self.mode = MotionlibMode.file
        self._motion_data_list = [None] * M
        self._motion_data_keys = np.array([f"packed_{i:05d}" for i in range(M)])
        self._num_unique_motions = M
        self.setup_constants(fix_height=FixHeightMode.no_fix)
        self.load_packed(packed)
        return self

    def load_motions(self, *args, **kwargs):  # noqa: F811 - packed libraries have no clip source
        if self.packed is not None and self._motion_data_list and self._motion_data_list[0] is None:
            return self.packed
        return self._load_motions(*args, **kwargs)

    def load_packed(self, packed, sample_idxes=None):
        """Install an already-packed library (e.g. synthetic, built on device)."""
        self.packed = packed
        M = packed.num_frames.shape[0]
        dev = packed.frames.device
        self._curr_motion_ids = sample_idxes if sample_idxes is not None else torch.arange(M, device=dev)
        self._motion_lengths = packed.motion_len
        self._motion_dt = packed.motion_dt
        self._motion_fps = packed.fps
        self._motion_num_frames = packed.num_frames
        self.length_starts = packed.length_starts
        self._motion_aa = torch.zeros((packed.frames.shape[0], 72), device=dev)
        self._motion_bodies = torch.zeros((M, 17), device=dev)
        self._motion_limb_weights = torch.zeros((M, 10), device=dev)
        self._num_motions = M
        self.num_joints = self.num_bodies = 24
        self.motion_ids = torch.arange(M, dtype=torch.long, device=dev)

    # reference attribute names
    gts = property(lambda self: self.packed.gts)
    grs = property(lambda self: self.packed.grs)
    lrs = property(lambda self: self.packed.local_rot)
    gvs = property(lambda self: self.packed.gvs)
    gavs = property(lambda self: self.packed.gavs)
    dvs = property(lambda self: self.packed.dof_vel)
    grvs = property(lambda self: self.packed.gvs[:, 0])
    gravs = property(lambda self: self.packed.gavs[:, 0])

    def num_motions(self):
        return self._num_motions

    def get_total_length(self):
        return float(self._motion_lengths.sum())

    # ---------------------------------------------------- sampling --
    def update_hard_sampling_weight(self, failed_keys):
        """motion_lib.py:454-470."""
        if len(failed_keys) > 0:
            keys = self._motion_data_keys.tolist()
            idx = [keys.index(k) for k in failed_keys]
            self._sampling_prob[:] = 0
            self._sampling_prob[idx] = 1 / len(idx)
        else:
            self._sampling_prob = torch.ones(self._num_unique_motions, device=self._device) / self._num_unique_motions

    def update_soft_sampling_weight(self, failed_keys):
        """motion_lib.py:472-492."""
        if len(failed_keys) > 0:
            keys = self._motion_data_keys.tolist()
            idx = [keys.index(k) for k in failed_keys]
            self._termination_history[idx] += 1
            self.update_sampling_prob(self._termination_history)
        else:
            self._sampling_prob = torch.ones(self._num_unique_motions, device=self._device) / self._num_unique_motions

    def update_sampling_prob(self, termination_history):
        """motion_lib.py:494-500."""
        if len(termination_history) == len(self._termination_history) and termination_history.sum() > 0:
            self._sampling_prob[:] = termination_history / termination_history.sum()
            self._termination_history = termination_history
            return True
        return False

    def sample_motions(self, n):
        return torch.multinomial(self._sampling_batch_prob, num_samples=n, replacement=True).to(self._device)

    def sample_time(self, motion_ids, truncate_time=None):
        phase = torch.rand(motion_ids.shape, device=self._device)
        motion_len = self._motion_lengths[motion_ids]
        if truncate_time is not None:
            assert truncate_time >= 0.0
            motion_len = motion_len - truncate_time
        return phase * motion_len

    def sample_time_interval(self, motion_ids, truncate_time=None):
        """motion_lib.py:526-535."""
        phase = torch.rand(motion_ids.shape, device=self._device)
        motion_len = self._motion_lengths[motion_ids]
        if truncate_time is not None:
            assert truncate_time >= 0.0
            motion_len = motion_len - truncate_time
        curr_fps = 1 / 30
        return ((phase * motion_len) / curr_fps).long() * curr_fps

    def get_motion_length(self, motion_ids=None):
        return self._motion_lengths if motion_ids is None else self._motion_lengths[motion_ids]

    def get_motion_num_steps(self, motion_ids=None):
        nf = self._motion_num_frames if motion_ids is None else self._motion_num_frames[motion_ids]
        fps = self._motion_fps if motion_ids is None else self._motion_fps[motion_ids]
        return (nf * self._sim_fps / fps).ceil().int()

    # ------------------------------------------------------ queries --
    def _calc_frame_blend(self, time, length, num_frames, dt):
        """motion_lib.py:655-665 (host-facing helper; the kernels inline the same arithmetic)."""
        time = time.clone()
        phase = torch.clip(time / length, 0.0, 1.0)
        time[time < 0] = 0
        f0 = (phase * (num_frames - 1)).long()
        f1 = torch.min(f0 + 1, num_frames - 1)
        blend = torch.clip((time - f0 * dt) / dt, 0.0, 1.0)
        return f0, f1, blend

    def get_motion_state(self, motion_ids, motion_times, offset=None):
        """motion_lib.py:549-626 via phc_motion_state."""
        ids = motion_ids.to(self._device, torch.int64).contiguous()
        times = motion_times.to(self._device, torch.float32).contiguous()
        off = None if offset is None else offset.to(self._device, torch.float32).contiguous()
        body, dof_pos, dof_vel = _native.motion_state(self.packed.c, ids, times, off)
        rg_pos, rb_rot = body[..., 0:3], body[..., 3:7]
        body_vel, body_ang_vel = body[..., 7:10], body[..., 10:13]
        f0 = self._calc_frame_blend(times, self._motion_lengths[ids], self._motion_num_frames[ids],
                                    self._motion_dt[ids])[0]
        return {
            "root_pos": rg_pos[:, 0].clone(),
            "root_rot": rb_rot[:, 0].clone(),
            "dof_pos": dof_pos,
            "root_vel": body_vel[:, 0].clone(),
            "root_ang_vel": body_ang_vel[:, 0].clone(),
            "dof_vel": dof_vel,
            "motion_aa": self._motion_aa[f0 + self.length_starts[ids]],
            "rg_pos": rg_pos,
            "rb_rot": rb_rot,
            "body_vel": body_vel,
            "body_ang_vel": body_ang_vel,
            "motion_bodies": self._motion_bodies[ids],
            "motion_limb_weights": self._motion_limb_weights[ids],
        }

    def get_root_pos_smpl(self, motion_ids, motion_times):
        """motion_lib.py:628-653."""
        return {"root_pos": self.get_motion_state(motion_ids, motion_times)["root_pos"]}


class MotionLibSMPL(MotionLibBase):
    """SMPL motion library.  The SMPL height fix (motion_lib.py:697-742) needs license-gated
    SMPL model files; like the reference without `smpl/` models, mesh_parsers stays None."""

    @staticmethod
    def fix_trans_height(pose_aa, trans, curr_gender_betas, mesh_parsers, fix_height_mode):
        if fix_height_mode == FixHeightMode.no_fix or mesh_parsers is None:
            return trans, 0
        raise NotImplementedError("SMPL height fix needs the SMPL body model (not shipped)")
