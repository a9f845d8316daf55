"""N3: the articulated-body physics step on the HIP path (phc_physics_step), a drop-in for the
reference's `gym.simulate(sim)` x control_freq_inv (puffer_phc/envs/humanoid_phc.py:129-134).

`BodyModel` packs the SMPL humanoid's physical model (assets/smpl_body_model.json, extracted from the
reference's assets/smpl_humanoid.xml by tools/make_body_model.py) into the device table the kernel
reads; `ArticulatedPhysics` is the physics object `HumanoidPHC` steps after writing its PD targets,
in place of the replay stand-in (`HumanoidPHC(cfg, physics=ArticulatedPhysics(cfg))`).  The
simulator's settings follow the reference where it states them (sim_dt 1/60 and control_freq_inv 2,
envs/isaacgym_env.py:6-42; PD gains x kp_scale / kd_scale, humanoid_phc.py:274-281; ground friction
1, :255-262; angular damping and velocity cap, :212-213; self-collision filters, :370-381); the
contact model and the substep count are this solver's own (PhysX's TGS solver is a
closed binary) and documented in DESIGN.md §8.
"""

import json
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _native

MODEL_JSON = os.path.join(os.path.dirname(__file__), "assets", "smpl_body_model.json")
MAX_POINTS = 8


@dataclass
class PhysicsConfig:
    sim_dt: float = 1.0 / 60.0
    control_freq_inv: int = 2
    substeps: int = 8
    kp_scale: float = 1.0
    kd_scale: float = 1.0
    contact_stiffness: float = 5.0e4
    contact_damping: float = 1.0e3
    friction: float = 1.0
    friction_damping: float = 1.0e3
    gravity: float = -9.81
    # AssetOptions of the humanoid asset (puffer_phc/envs/humanoid_phc.py:212-213): per-link angular
    # damping (a torque -d Ic w) and the cap on every joint's / the root's angular velocity (rad/s)
    angular_damping: float = 0.01
    max_angular_velocity: float = 100.0
    # RobotConfig.has_self_collision (puffer_phc/config.py:43, humanoid_phc.py:338 and :370-381):
    # penalty contact between the body pairs the shape filters leave colliding
    self_collision: bool = True


# Shape collision filters of the capsule humanoid (has_mesh False, puffer_phc/envs/
# humanoid_phc.py:374): two shapes whose filter words share a bit never collide
SELF_COLLISION_FILTER = (0, 0, 7, 16, 12, 0, 56, 2, 33, 128, 0, 192, 0, 64, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)


def collision_segment(shape):
    """The geom as a capsule for self-collision: (p0, p1, radius) in body coordinates.  A sphere is
    a zero-length segment, a capsule itself, a box the segment along its longest half-axis shortened
    by the radius, the radius the smallest of the other two half-extents (inside the box)."""
    if shape["type"] == "sphere":
        c = list(shape["center"])
        return c, c, shape["radius"]
    if shape["type"] == "capsule":
        return list(shape["p0"]), list(shape["p1"]), shape["radius"]
    if shape["type"] == "box":
        c, h = np.asarray(shape["center"], dtype=np.float64), np.asarray(shape["half"], dtype=np.float64)
        k = int(np.argmax(h))
        r = float(min(h[(k + 1) % 3], h[(k + 2) % 3]))
        d = np.zeros(3)
        d[k] = max(h[k] - r, 0.0)
        return list(c - d), list(c + d), r
    raise ValueError(f"unsupported geom type {shape['type']!r}")


def self_collision_masks(parents, filters=SELF_COLLISION_FILTER):
    """Per body the bit set of the bodies it collides with: filter words disjoint, not the same
    body, not joined by a joint (PhysX never collides a link with its parent)."""
    n = len(parents)
    masks = [0] * n
    for i in range(n):
        for j in range(n):
            if i == j or parents[i] == j or parents[j] == i or (filters[i] & filters[j]):
                continue
            masks[i] |= 1 << j
    return masks


def contact_points(shape):
    """Contact points (x, y, z, radius) of one geom in body coordinates: a sphere's centre, a
    capsule's two end-sphere centres, a box's 8 corners (radius 0)."""
    if shape["type"] == "sphere":
        return [list(shape["center"]) + [shape["radius"]]]
    if shape["type"] == "capsule":
        return [list(shape["p0"]) + [shape["radius"]], list(shape["p1"]) + [shape["radius"]]]
    if shape["type"] == "box":
        c, h = np.asarray(shape["center"]), np.asarray(shape["half"])
        return [list(c + h * np.array([sx, sy, sz])) + [0.0] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]
    raise ValueError(f"unsupported geom type {shape['type']!r}")


class BodyModel:
    """The [24, 80] float32 body table of phc_physics.hip (row layout documented there)."""

    def __init__(self, path=MODEL_JSON, device="cuda"):
        with open(path) as f:
            d = json.load(f)
        bodies = d["bodies"]
        n = len(bodies)
        if n != _native.NUM_BODIES:
            raise ValueError(f"body model has {n} bodies, the kernels are built for {_native.NUM_BODIES}")
        level = [0] * n
        children = [[] for _ in range(n)]
        for i, b in enumerate(bodies):
            p = b["parent"]
            if i == 0:
                if p != -1:
                    raise ValueError("body 0 must be the root")
                continue
            if not 0 <= p < i:
                raise ValueError(f"body {i}: parent {p} must precede it")
            level[i] = level[p] + 1
            children[p].append(i)
        if max(len(c) for c in children) > 3:
            raise ValueError("at most 3 children per body")
        self.depth = max(level)
        if not 1 <= self.depth <= 15:
            raise ValueError(f"tree depth {self.depth} outside 1..15")
        t = np.zeros((n, _native.BODY_MODEL_STRIDE), dtype=np.float32)
        for i, b in enumerate(bodies):
            I = np.asarray(b["inertia"])
            pts = contact_points(b["shape"])
            if len(pts) > MAX_POINTS:
                raise ValueError(f"body {i}: more than {MAX_POINTS} contact points")
            t[i, 0] = max(b["parent"], 0)
            t[i, 1] = level[i]
            t[i, 2] = len(children[i])
            t[i, 3:3 + len(children[i])] = children[i]
            t[i, 6:9] = b["offset"]
            t[i, 9] = b["mass"]
            t[i, 10:13] = b["com"]
            t[i, 13:19] = [I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]]
            t[i, 19:22] = b["kp"]
            t[i, 22:25] = b["kd"]
            t[i, 25:28] = b["armature"]
            t[i, 28] = len(pts)
            t[i, 32:32 + 4 * len(pts)] = np.asarray(pts, dtype=np.float32).reshape(-1)
            s0, s1, rad = collision_segment(b["shape"])
            t[i, 64:67], t[i, 67:70], t[i, 70] = s0, s1, rad
        self.masks = self_collision_masks([b["parent"] for b in bodies])
        t[:, 71] = self.masks  # < 2^24: exact in float32
        self.names = [b["name"] for b in bodies]
        self.total_mass = float(sum(b["mass"] for b in bodies))
        # zero pose (every joint rotation the identity): body origins are the summed offsets, and
        # the root height that puts the lowest contact point on the ground
        origin = np.zeros((n, 3))
        for i in range(1, n):
            origin[i] = origin[bodies[i]["parent"]] + np.asarray(bodies[i]["offset"])
        low = min(origin[i][2] + p[2] - p[3] for i in range(n) for p in
                  (t[i, 32:32 + 4 * int(t[i, 28])].reshape(-1, 4).astype(np.float64)))
        self.rest_root_height = float(-low)
        self.host = t
        self.table = torch.from_numpy(t).to(device)


def rest_state(model, num_envs, clearance=0.0, device="cuda"):
    """Env buffers of `num_envs` humanoids standing in the zero pose at rest, the lowest contact
    point `clearance` above the ground: (rigid_body_state [N,24,13] with the root record set — the
    physics step reads only that record and dof_state — and dof_state [N,69,2])."""
    rb = torch.zeros((num_envs, _native.NUM_BODIES, 13), device=device)
    rb[:, :, 6] = 1.0
    rb[:, 0, 2] = model.rest_root_height + clearance
    dof = torch.zeros((num_envs, _native.NUM_DOF, 2), device=device)
    return rb, dof


class ArticulatedPhysics:
    """Physics object for HumanoidPHC: one phc_physics_step launch per env step (control_freq_inv
    sim steps of `substeps` substeps) on the env's rigid-body / dof buffers and PD targets."""

    def __init__(self, config=None, kp_scale=None, kd_scale=None, model=None, device="cuda"):
        self.config = config or PhysicsConfig()
        if kp_scale is not None:
            self.config.kp_scale = kp_scale
        if kd_scale is not None:
            self.config.kd_scale = kd_scale
        self.model = model or BodyModel(device=device)
        self.params = self._params()
        self.timer = None  # bench: a _native.KernelTimer timing every launch

    def _params(self):
        c = self.config
        return _native.PhysicsParamsC(float(c.sim_dt), int(c.control_freq_inv), int(c.substeps), int(self.model.depth),
                                      float(c.kp_scale), float(c.kd_scale), float(c.contact_stiffness),
                                      float(c.contact_damping), float(c.friction), float(c.friction_damping),
                                      float(c.gravity), float(c.angular_damping), float(c.max_angular_velocity),
                                      int(bool(c.self_collision)))

    def step(self, env):
        """One step from env.pd_target (written by the caller)."""
        _native.physics_step(env._env_c, env.pd_target, self.model.table, self.params, timer=self.timer)

    def step_actions(self, env, pd):
        """One step with the action -> PD-target map (R13) folded into the physics launch."""
        _native.physics_step_actions(env._env_c, pd, self.model.table, self.params, timer=self.timer)
