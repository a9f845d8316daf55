"""Synthetic motion clips generated on device (the AMASS library is not available offline).

BASELINE configs C2/C3: 24-joint clips of U{min_len..max_len} frames at 30 fps.  Global joint
rotations are slerped between random keyframes (every 15 frames) that stay within a moderate
cone around the upright pose; the root translation is a smoothed random walk at ~0.9 m.  The
output is the schema the loader's FK consumes: float64 global quaternions [F,24,4] and root
translations [F,3], plus per-clip frame counts.
"""

import torch


def _slerp64(q0, q1, t):
    d = (q0 * q1).sum(-1, keepdim=True)
    q1 = torch.where(d < 0, -q1, q1)
    d = d.abs().clamp(max=1.0)
    th = torch.acos(d)
    s = torch.sin(th)
    small = s < 1e-6
    ss = torch.where(small, torch.ones_like(s), s)
    a = torch.where(small, 1 - t, torch.sin((1 - t) * th) / ss)
    b = torch.where(small, t, torch.sin(t * th) / ss)
    q = a * q0 + b * q1
    return q / q.norm(dim=-1, keepdim=True)


def synthetic_clips(num_motions, min_len=60, max_len=300, seed=0, device="cuda", key_every=15, joints=24):
    """Returns (quat_global f64 [F,J,4], root_trans f64 [F,3], counts int64 [M], fps f32 [M])."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    counts = torch.randint(min_len, max_len + 1, (num_motions,), generator=g)
    nkeys = counts // key_every + 2
    kstart = torch.cumsum(nkeys, 0) - nkeys
    K = int(nkeys.sum())
    keys = torch.zeros((K, joints, 4), dtype=torch.float64)
    keys[..., 3] = 1.0
    keys += torch.randn((K, joints, 4), generator=g, dtype=torch.float64) * 0.35
    keys /= keys.norm(dim=-1, keepdim=True)
    F = int(counts.sum())
    mot = torch.repeat_interleave(torch.arange(num_motions), counts)
    fstart = torch.cumsum(counts, 0) - counts
    t_local = torch.arange(F) - fstart[mot]
    k0 = kstart[mot] + t_local // key_every
    frac = ((t_local % key_every).double() / key_every)[:, None, None]
    keys = keys.to(device)
    q = _slerp64(keys[k0.to(device)], keys[(k0 + 1).to(device)], frac.to(device))
    steps = torch.randn((F, 3), generator=g, dtype=torch.float64) * 0.02
    steps[:, 2] *= 0.2
    cs = torch.cumsum(steps, 0)
    base = torch.cat([torch.zeros((1, 3), dtype=torch.float64), cs])[fstart][mot]
    trans = cs - base
    trans[:, 2] += 0.9
    fps = torch.full((num_motions,), 30.0)
    return q.contiguous(), trans.to(device).contiguous(), counts.to(device), fps.to(device)


def standing_clips(num_motions, frames=300, height=0.94, sway=0.0, seed=0, device="cuda", key_every=30, joints=24):
    """Clips of the humanoid standing in the upright zero pose (every global rotation the identity)
    with its root `height` above the ground — the physics body model's rest height is 0.937 m
    (physics.BodyModel.rest_root_height) — optionally swaying: keyframes every `key_every` frames
    drawn within a `sway`-radian cone around the upright pose, the root fixed.  The articulated
    physics' balance task (profiles/r03_train_articulated_standing.log).  Same outputs as
    synthetic_clips."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    counts = torch.full((num_motions,), int(frames), dtype=torch.int64)
    nkeys = frames // key_every + 2
    keys = torch.zeros((num_motions, nkeys, joints, 4), dtype=torch.float64)
    keys[..., 3] = 1.0
    if sway > 0:
        keys[..., :3] += torch.randn((num_motions, nkeys, joints, 3), generator=g, dtype=torch.float64) * (0.5 * sway)
        keys /= keys.norm(dim=-1, keepdim=True)
    t = torch.arange(frames)
    k0 = t // key_every
    frac = ((t % key_every).double() / key_every)[None, :, None, None]
    q = _slerp64(keys[:, k0], keys[:, k0 + 1], frac).reshape(-1, joints, 4)
    trans = torch.zeros((num_motions * frames, 3), dtype=torch.float64)
    trans[:, 2] = height
    fps = torch.full((num_motions,), 30.0)
    return q.to(device).contiguous(), trans.to(device).contiguous(), counts.to(device), fps.to(device)
