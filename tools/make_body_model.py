"""Extract the SMPL humanoid's physical model from the reference MJCF asset into
puffer-phc_amd/assets/smpl_body_model.json (data: per body its parent, joint offset, single
geom, mass properties computed from the geom and density, and its three hinge joints' PD gains /
armature).  Run in the build container (reads /root/reference/puffer_phc/assets/smpl_humanoid.xml;
the JSON is what the package and the GPU box use).

Mass properties follow MuJoCo's geom conventions: sphere, box (half sizes), capsule (a cylinder of
the `fromto` segment plus two hemispherical caps), uniform density."""
import json
import math
import sys
import xml.etree.ElementTree as ET

import numpy as np

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/puffer_phc/assets/smpl_humanoid.xml"
OUT = sys.argv[2] if len(sys.argv) > 2 else "puffer-phc_amd/assets/smpl_body_model.json"


def vec(s):
    return [float(x) for x in s.split()]


def geom_mass(g):
    t = g.get("type", "capsule")
    rho = float(g.get("density", "1000"))
    if t == "sphere":
        r = vec(g.get("size"))[0]
        m = rho * 4.0 / 3.0 * math.pi * r ** 3
        com = np.array(vec(g.get("pos", "0 0 0")))
        inertia = np.eye(3) * (0.4 * m * r * r)
        shape = {"type": "sphere", "radius": r, "center": com.tolist()}
    elif t == "box":
        a, b, c = vec(g.get("size"))
        m = rho * 8.0 * a * b * c
        com = np.array(vec(g.get("pos", "0 0 0")))
        inertia = np.diag([m * (b * b + c * c) / 3.0, m * (a * a + c * c) / 3.0, m * (a * a + b * b) / 3.0])
        q = vec(g.get("quat", "1 0 0 0"))
        assert abs(q[0] - 1.0) < 1e-6, "rotated boxes are not used by this asset"
        shape = {"type": "box", "half": [a, b, c], "center": com.tolist()}
    else:  # capsule from `fromto`
        r = vec(g.get("size"))[0]
        ft = np.array(vec(g.get("fromto")))
        p0, p1 = ft[:3], ft[3:]
        L = float(np.linalg.norm(p1 - p0))
        mc = rho * math.pi * r * r * L
        mh = rho * 2.0 / 3.0 * math.pi * r ** 3  # one hemisphere
        m = mc + 2 * mh
        com = 0.5 * (p0 + p1)
        i_ax = 0.5 * mc * r * r + 2 * (0.4 * mh * r * r)
        i_perp = mc * (3 * r * r + L * L) / 12.0 + 2 * (mh * 83.0 / 320.0 * r * r + mh * (L / 2 + 3.0 * r / 8.0) ** 2)
        u = (p1 - p0) / L if L > 0 else np.array([0.0, 0.0, 1.0])
        inertia = i_perp * np.eye(3) + (i_ax - i_perp) * np.outer(u, u)
        shape = {"type": "capsule", "radius": r, "p0": p0.tolist(), "p1": p1.tolist()}
    return m, com, inertia, shape


def main():
    root = ET.parse(SRC).getroot()
    world = root.find("worldbody")
    bodies = []

    def walk(el, parent):
        idx = len(bodies)
        g = el.find("geom")
        m, com, inertia, shape = geom_mass(g)
        joints = el.findall("joint")
        kp = [float(j.get("stiffness")) for j in joints]
        kd = [float(j.get("damping")) for j in joints]
        arm = [float(j.get("armature")) for j in joints]
        axes = [vec(j.get("axis")) for j in joints]
        if joints:
            assert axes == [[1, 0, 0], [0, 1, 0], [0, 0, 1]], el.get("name")
        bodies.append({"name": el.get("name"), "parent": parent, "offset": vec(el.get("pos")), "mass": m,
                       "com": com.tolist(), "inertia": inertia.tolist(), "shape": shape,
                       "kp": kp or [0.0, 0.0, 0.0], "kd": kd or [0.0, 0.0, 0.0], "armature": arm or [0.0, 0.0, 0.0]})
        for ch in el.findall("body"):
            walk(ch, idx)

    walk(world.find("body"), -1)
    model = {"source": "derived from puffer_phc/assets/smpl_humanoid.xml by tools/make_body_model.py",
             "gravity": [0.0, 0.0, -9.81], "sim_dt": 1.0 / 60.0, "control_freq_inv": 2,
             "bodies": bodies, "total_mass": sum(b["mass"] for b in bodies)}
    with open(OUT, "w") as f:
        json.dump(model, f, indent=1)
    print(f"{len(bodies)} bodies, total mass {model['total_mass']:.2f} kg -> {OUT}")


if __name__ == "__main__":
    main()
