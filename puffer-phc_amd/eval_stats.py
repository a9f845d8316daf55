"""Evaluation over the whole motion set (reference: scripts/train.py:75-257
EvalStats and :392-429 rollout).

The env is switched to eval mode (HumanoidPHC.toggle_eval_mode: sequential motion batches,
termination distance 0.5, mean-distance termination, every reset at motion time 0), the policy
acts deterministically, and after every step the per-env bookkeeping below decides when the
current batch of motions has been played out (or terminated); then the next batch is loaded
(forward_motion_samples).  Success rate = 1 - fraction of motions that terminated before their
last frame; per-motion MPJPE & co come from `metrics.compute_metrics_lite` over the recorded
body positions.  The per-step positions are copied to the host as the reference does (the eval
path is outside the training hot loop).
"""

import numpy as np
import torch

from .metrics import compute_metrics_lite


class EvalStats:
    def __init__(self, vec_env, failed_save_path=None, progress=True):
        self.task_env = vec_env.env
        self.num_envs = self.task_env.cfg.num_envs
        dev = self.task_env.device
        self.failed_save_path = failed_save_path
        self.num_unique_motions = self.task_env.toggle_eval_mode()
        self.terminate_state = torch.zeros(self.num_envs, dtype=torch.bool, device=dev)
        self.played_steps_buf = torch.zeros(self.num_envs, dtype=torch.int16, device=dev)
        self.terminate_memory, self.motion_length, self.played_steps = [], [], []
        self.mpjpe, self.mpjpe_all = [], []
        self.gt_pos, self.gt_pos_all = [], []
        self.pred_pos, self.pred_pos_all = [], []
        self.curr_steps = 0
        self.success_rate = 0.0
        self.failed_keys = []
        self.results = None
        self.results_by_motion = None
        self.pbar = None
        if progress:
            from tqdm import tqdm

            self.pbar = tqdm(range(max(self.num_unique_motions // self.num_envs, 1)))

    def _batch_horizon(self, motion_num_steps):
        """Step count at which the current batch is complete (scripts/train.py:118-137)."""
        alive = ~self.terminate_state
        if not bool(alive.any()):
            return int(motion_num_steps.max())
        last_id = self.num_unique_motions - 1
        curr_ids = self.task_env.current_motion_ids
        at_last = curr_ids == last_id
        if bool(at_last.any()):
            # more envs than remaining motions: envs past the last motion id are not counted
            bound = int(at_last.nonzero()[0]) + 1
            if bool(alive[:bound].any()):
                horizon = int(motion_num_steps[:bound][alive[:bound]].max())
            else:
                horizon = self.curr_steps - 1
                self.terminate_state[bound:] = True
        else:
            horizon = int(motion_num_steps[alive].max())
        if self.curr_steps >= horizon:
            horizon = self.curr_steps + 1
        return horizon

    def post_step_eval(self):
        """Book-keeping after one env step.  Returns (all motions evaluated, moved to next batch)."""
        env = self.task_env
        motion_num_steps = env.get_motion_steps()
        info = env.extras
        # a termination on or after the last frame is not a failure (curr_steps lags the sim by one)
        terminated = torch.logical_and(self.curr_steps < motion_num_steps, info["terminate"])
        torch.logical_or(terminated, self.terminate_state, out=self.terminate_state)
        playing = torch.logical_and(~self.terminate_state, self.curr_steps < motion_num_steps)
        self.played_steps_buf += playing.to(self.played_steps_buf.dtype)
        horizon = self._batch_horizon(motion_num_steps)

        self.mpjpe.append(info["mpjpe"])
        self.gt_pos.append(info["body_pos_gt"])
        self.pred_pos.append(info["body_pos"])
        self.curr_steps += 1

        next_batch = False
        if self.curr_steps >= horizon or int(self.terminate_state.sum()) == self.num_envs:
            self.curr_steps = 0
            self.terminate_memory.append(self.terminate_state.cpu().numpy())
            steps = env.get_motion_steps().cpu().numpy()
            self.motion_length.append(steps)
            self.played_steps.append(self.played_steps_buf.cpu().numpy())
            self.success_rate = 1 - np.concatenate(self.terminate_memory)[: self.num_unique_motions].mean()

            mpjpe = torch.stack(self.mpjpe)
            self.mpjpe_all.append([mpjpe[: (n - 1), i].mean() for i, n in enumerate(steps)])
            pred = np.stack(self.pred_pos)
            gt = np.stack(self.gt_pos)
            self.pred_pos_all += [pred[: (n - 1), i] for i, n in enumerate(steps)]
            self.gt_pos_all += [gt[: (n - 1), i] for i, n in enumerate(steps)]

            if env.motion_sample_start_idx + self.num_envs >= self.num_unique_motions:
                return self.get_final_stats(), next_batch
            next_batch = True
            env.forward_motion_samples()
            self.terminate_state[:] = False
            self.played_steps_buf[:] = 0
            if self.pbar is not None:
                self.pbar.update(1)
            self.mpjpe, self.gt_pos, self.pred_pos = [], [], []
        if self.pbar is not None:
            mp = np.mean([float(x) for b in self.mpjpe_all for x in b]) * 1000 if self.mpjpe_all else 0.0
            self.pbar.set_description(f"Terminated: {int(self.terminate_state.sum())} | max frames: {horizon} | "
                                      f"Succ rate: {self.success_rate:.3f} | Mpjpe: {mp:.3f}")
        return False, next_batch

    def get_final_stats(self):
        if self.pbar is not None:
            self.pbar.clear()
        n = self.num_unique_motions
        terminated = np.concatenate(self.terminate_memory)[:n]
        succ = np.flatnonzero(~terminated).tolist()
        pred_all, gt_all = self.pred_pos_all[:n], self.gt_pos_all[:n]
        self.failed_keys = self.task_env.motion_data_keys[terminated]
        m_all = compute_metrics_lite(pred_all, gt_all)
        m_succ = compute_metrics_lite([pred_all[i] for i in succ], [gt_all[i] for i in succ])
        all_p = {k: float(np.mean(v)) for k, v in m_all.items()}
        succ_p = {k: float(np.mean(v)) for k, v in m_succ.items()} if succ else dict(all_p)
        self.results = {
            "eval/success_rate": float(self.success_rate),
            "eval/mpjpe_all": all_p["mpjpe_g"],
            "eval/mpjpe_succ": succ_p["mpjpe_g"],
            "eval/accel_dist": succ_p["accel_dist"],
            "eval/vel_dist": succ_p["vel_dist"],
            "eval/mpjpel_all": all_p["mpjpe_l"],
            "eval/mpjpel_succ": succ_p["mpjpe_l"],
            "eval/mpjpe_pa": succ_p["mpjpe_pa"],
        }
        self.results_by_motion = {
            "motion_keys": self.task_env.motion_data_keys.tolist(),
            "motion_length": np.concatenate(self.motion_length)[:n],
            "played_steps": np.concatenate(self.played_steps)[:n],
            "success": ~terminated,
        }
        return True

    def update_env_and_close(self):
        """Back to training mode; the termination history feeds the PMCP sampling weights."""
        history = self.task_env.untoggle_eval_mode(self.failed_keys)
        if self.failed_save_path:
            import joblib

            joblib.dump({"failed_keys": self.failed_keys, "termination_history": history}, self.failed_save_path)
        return self.results


def eval_rollout(vec_env, policy, eval_stats, max_steps=None):
    """scripts/train.py:392-429 rollout with EvalStats: deterministic actions until every motion
    of the eval set has been played.  Returns the number of env steps taken."""
    pol = policy.policy if hasattr(policy, "policy") else policy
    pol.set_deterministic_action(True)
    obs, _ = vec_env.reset()
    steps = 0
    try:
        while max_steps is None or steps < max_steps:
            with torch.no_grad():
                action, _, _, _ = policy(obs)
            obs, _, _, _, _ = vec_env.step(action)
            steps += 1
            done, _ = eval_stats.post_step_eval()
            if done:
                break
    finally:
        pol.set_deterministic_action(False)
    return steps
