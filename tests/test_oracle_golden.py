"""Pin the CPU oracle (oracle/phc_oracle.py) to the reference's own outputs.

Tolerances: float32 results within atol=1e-5, rtol=1e-5 (BASELINE north_star: obs/reward
within 1e-5); frame indices, reset and terminate flags bit-exact except where a reset
distance lies within 1e-6 of its threshold (ties are flagged, not compared).
"""

import os

import numpy as np
import pytest

from oracle import phc_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ATOL = 1e-5
RTOL = 1e-5


def close(a, b, atol=ATOL, rtol=RTOL):
    np.testing.assert_allclose(np.asarray(a, np.float64), np.asarray(b, np.float64), atol=atol, rtol=rtol)


@pytest.fixture(scope="module")
def lib(golden):
    m = golden("motion_lib")
    return O.MotionLib(m["gts"], m["grs"], m["lrs"], m["gvs"], m["gavs"], m["dvs"],
                       m["motion_num_frames"], m["motion_fps"])


def test_skeleton_matches_fixture(golden):
    s = golden("skeleton")
    assert list(s["node_names"]) == list(O.BODY_NAMES)
    assert s["parent_indices"].tolist() == [-1, 0, 1, 2, 3, 0, 5, 6, 7, 0, 9, 10, 11, 12, 11, 14, 15, 16, 17,
                                            11, 19, 20, 21, 22]


def test_motion_lib_scalars(golden, lib):
    m = golden("motion_lib")
    np.testing.assert_array_equal(lib.length_starts, m["length_starts"])
    np.testing.assert_array_equal(lib.motion_lengths, m["motion_lengths"])
    np.testing.assert_array_equal(lib.motion_dt, m["motion_dt"])


def test_fk_and_velocities(golden):
    s, m = golden("skeleton"), golden("motion_lib")
    order = m["sample_idxes"]
    starts = m["length_starts"]
    for k, mi in enumerate(order):
        q = m[f"in_quat_{mi}"]
        tr = m[f"in_trans_{mi}"]
        out = O.fk_motion(s["parent_indices"], s["local_translation"], q, tr, fps=30)
        sl = slice(starts[k], starts[k] + len(q))
        for key in ("gts", "grs", "lrs", "gvs", "gavs", "dvs"):
            close(out[key], m[key][sl], atol=2e-5)
        np.testing.assert_array_equal(out["grs"], m["grs"][sl])


def test_frame_blend_bit_exact(golden, lib):
    g = golden("motion_state")
    ids = g["motion_ids"]
    f0, f1, blend = O.calc_frame_blend(g["motion_times"], lib.motion_lengths[ids], lib.num_frames[ids],
                                       lib.motion_dt[ids])
    np.testing.assert_array_equal(f0, g["frame_idx0"])
    np.testing.assert_array_equal(f1, g["frame_idx1"])
    np.testing.assert_array_equal(blend, g["blend"])


def test_motion_state(golden, lib):
    g = golden("motion_state")
    st = O.motion_state(lib, g["motion_ids"], g["motion_times"], g["offset"])
    for k in ("root_pos", "root_rot", "dof_pos", "root_vel", "root_ang_vel", "dof_vel", "rg_pos", "rb_rot",
              "body_vel", "body_ang_vel"):
        close(st[k], g[k])
    np.testing.assert_array_equal(st["rg_pos"], g["rg_pos"])  # lerp + offset: exact IEEE ops


def _check_step(out, g, prefix):
    close(out["rew"], g[prefix + "rew"])
    close(out["reward_raw"], g[prefix + "reward_raw"])
    close(out["obs"], g[prefix + "obs"])
    np.testing.assert_array_equal(out["time"], g[prefix + "time"])
    np.testing.assert_array_equal(out["time_next"], g[prefix + "time_next"])
    # bit-exact flags, margin-aware at exact ties
    ties = np.any(np.abs(g[prefix + "reset_dist"] - 0.25) < 1e-6, -1)
    np.testing.assert_array_equal(out["reset"][~ties], g[prefix + "reset"][~ties])
    np.testing.assert_array_equal(out["terminate"][~ties], g[prefix + "terminate"][~ties])


def test_env_step_train(golden, lib):
    g = golden("env_step")
    out = O.env_step(lib, g["motion_ids"], g["progress"], g["start"], g["start_offset"], g["global_offset"],
                     g["rb_state"], g["dof_vel"], g["dof_force"], g["term_dist"], g["reset_body_ids"], False)
    _check_step(out, g, "train_")
    assert out["reset"].any() and out["terminate"].any() and not out["reset"].all()


def test_env_step_eval(golden, lib):
    g = golden("env_step")
    out = O.env_step(lib, g["motion_ids"], g["progress"], g["start"], g["start_offset"], g["global_offset"],
                     g["rb_state"], g["dof_vel"], g["dof_force"], g["eval_term_dist"], g["eval_reset_body_ids"],
                     True)
    _check_step(out, g, "eval_")


def test_reset_subset(golden, lib):
    g = golden("reset")
    out = O.reset_subset(lib, g["motion_ids"], g["phase"], g["global_offset_old"])
    np.testing.assert_array_equal(out["motion_times"], g["motion_times"])
    for k in ("rg_pos", "rb_rot", "body_vel", "body_ang_vel", "dof_pos", "dof_vel", "root_pos", "root_rot"):
        close(out["ref"][k], g["ref_" + k])
    close(out["obs"], g["obs"])


def test_amp_obs(golden, lib):
    g = golden("amp_obs")
    st = O.motion_state(lib, g["motion_ids"], g["motion_times"])
    np.testing.assert_array_equal(O.dof_subset(), g["dof_subset"])
    kb = st["rg_pos"][:, g["key_body_ids"]]
    out = O.amp_obs(st["root_pos"], st["root_rot"], st["root_vel"], st["root_ang_vel"], st["dof_pos"],
                    st["dof_vel"], kb)
    close(out, g["amp_obs"])


def test_gae(golden):
    g = golden("gae")
    np.testing.assert_array_equal(O.compute_gae(g["dones"], g["values"], g["rewards"], g["gamma"], g["lam"]), g["adv"])
    np.testing.assert_array_equal(O.compute_gae(g["dones2"], g["values2"], g["rewards2"], g["gamma2"], g["lam2"]),
                                  g["adv2"])


def test_gae_c_restatement(golden):
    """oracle/gae.c (the CPU baseline's GAE) == the reference's Cython output, bit for bit."""
    import subprocess

    from oracle import c_oracle

    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    g = golden("gae")
    for k in ("", "2"):
        out = c_oracle.compute_gae(g["dones" + k], g["values" + k], g["rewards" + k], g["gamma" + k], g["lam" + k])
        np.testing.assert_array_equal(out, g["adv" + k])


def test_rms(golden):
    g = golden("rms")
    F = g["x1"].shape[1]
    m, v, c = np.zeros((1, F), np.float32), np.ones((1, F), np.float32), np.ones(1, np.float32)
    m, v, c = O.rms_update(m, v, c, g["x1"])
    close(m, g["mean1"])
    close(v, g["var1"])
    np.testing.assert_array_equal(c, g["count1"])
    m, v, c = O.rms_update(m, v, c, g["x2"])
    close(m, g["mean2"])
    close(v, g["var2"])
    close(O.rms_normalize(g["xq"], m, v), g["y"], atol=2e-5)
