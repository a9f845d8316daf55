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

Data parallel: the motion set is sharded over the ranks (batch b of num_envs
motions is played by rank b % world), each rank keeps per-motion rows (terminated, lengths, metric
sums), one all-reduce merges them, so every rank derives the same failed keys and PMCP sampling
weights, which rank 0 then broadcasts (motion_lib.py:454-500).
"""

import numpy as np
import torch

from . import distributed as D
from .metrics import compute_metrics_lite

METRICS = ("mpjpe_g", "mpjpe_l", "mpjpe_pa", "accel_dist", "vel_dist")
# per-motion columns of the shard merge: evaluated, terminated, motion length, played steps, then
# (sum over frames, frame count) of every metric
COLS = 4 + 2 * len(METRICS)


def merge_eval_shards(rows, reduce_sum=None):
    """Merge the per-motion rows [n, COLS] of every rank's eval shard (disjoint motion sets, zero
    rows elsewhere) by one all-reduce (eval is sharded over data-parallel
    ranks; every rank then holds the whole-set result)."""
    reduce_sum = D.allreduce_sum_ if reduce_sum is None else reduce_sum
    out = reduce_sum(rows.clone())
    if bool((out[:, 0] > 1.5).any()):
        raise RuntimeError("eval shards overlap: a motion was evaluated on more than one rank")
    return out


def summarize_eval(rows):
    """Reference results (scripts/train.py:187-236) from merged per-motion rows."""
    r = rows.double().cpu().numpy()
    if not np.all(r[:, 0] == 1):
        raise RuntimeError(f"{int((r[:, 0] != 1).sum())} motions were not evaluated")
    terminated = r[:, 1] > 0.5
    succ = ~terminated

    def mean(sel, k):
        s, c = r[sel, 4 + 2 * k].sum(), r[sel, 5 + 2 * k].sum()
        return float(s / c) if c > 0 else float("nan")

    all_p = {m: mean(slice(None), k) for k, m in enumerate(METRICS)}
    succ_p = {m: mean(succ, k) for k, m in enumerate(METRICS)} if succ.any() else dict(all_p)
    results = {
        "eval/success_rate": float(1 - terminated.mean()),
        "eval/mpjpe_all": all_p["mpjpe_g"],
        "eval/mpjpe_succ": succ_p["mpjpe_g"],
        "eval/accel_dist": succ_p["accel_dist"],
        "eval/vel_dist": succ_p["vel_dist"],
        "eval/mpjpel_all": all_p["mpjpe_l"],
        "eval/mpjpel_succ": succ_p["mpjpe_l"],
        "eval/mpjpe_pa": succ_p["mpjpe_pa"],
    }
    return results, terminated, r[:, 2].astype(np.int64), r[:, 3].astype(np.int64)


def sync_sampling_state(motion_lib, src=0):
    """After untoggle_eval_mode every rank updated its sampling weights from the same merged
    failed keys; broadcast rank src's _sampling_prob / _termination_history anyway so the replicas
    cannot drift (reference motion_lib.py:454-500 has one process)."""
    if not D.is_dist():
        return
    import torch.distributed as dist

    for name in ("_sampling_prob", "_termination_history"):
        t = getattr(motion_lib, name).contiguous()
        dist.broadcast(t, src)
        setattr(motion_lib, name, t)


class EvalStats:
    def __init__(self, vec_env, failed_save_path=None, progress=True, shard=None):
        """shard = (rank, world): this rank evaluates motion batches rank, rank + world, ... of
        num_envs motions each (default: the data-parallel rank / world size; (0, 1) is the
        reference's sequential pass over every motion)."""
        self.task_env = vec_env.env
        self.num_envs = self.task_env.cfg.num_envs
        dev = self.task_env.device
        self.failed_save_path = failed_save_path
        self.rank, self.world = shard if shard is not None else (D.rank(), D.world_size())
        self.num_unique_motions = self.task_env.toggle_eval_mode(shard=(self.rank, self.world))
        # more ranks than motion batches: this rank has nothing to play, it only joins the merge
        self.idle = self.task_env.motion_sample_start_idx >= self.num_unique_motions
        self.terminate_state = torch.zeros(self.num_envs, dtype=torch.bool, device=dev)
        self.played_steps_buf = torch.zeros(self.num_envs, dtype=torch.int16, device=dev)
        self.terminate_memory, self.motion_length, self.played_steps = [], [], []
        self.batch_ids = []  # motion ids of every finished batch (this rank's shard, in order)
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

            self.pbar = tqdm(range(max(self.num_unique_motions // (self.num_envs * self.world), 1)))

    def _valid(self):
        """Envs of the current batch that play a motion of the set (the batch may wrap around
        past the last motion; those envs are not counted, scripts/train.py:119-130)."""
        return min(self.num_envs, self.num_unique_motions - self.task_env.motion_sample_start_idx)

    def _batch_horizon(self, motion_num_steps):
        """Step count at which the current batch is complete (scripts/train.py:118-137)."""
        alive = ~self.terminate_state
        if not bool(alive.any()):
            return int(motion_num_steps.max())
        bound = self._valid()
        if bound < self.num_envs:
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
        if self.idle:
            return self.get_final_stats(), False
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
            start, bound = env.motion_sample_start_idx, self._valid()
            self.batch_ids.append(np.arange(start, start + bound))
            self.terminate_memory.append(self.terminate_state.cpu().numpy()[:bound])
            steps = env.get_motion_steps().cpu().numpy()[:bound]
            self.motion_length.append(steps)
            self.played_steps.append(self.played_steps_buf.cpu().numpy()[:bound])
            self.success_rate = 1 - np.concatenate(self.terminate_memory).mean()

            mpjpe = torch.stack(self.mpjpe)
            self.mpjpe_all.append([mpjpe[: (n - 1), i].mean() for i, n in enumerate(steps)])
            pred = np.stack(self.pred_pos)
            gt = np.stack(self.gt_pos)
            self.pred_pos_all += [pred[: (n - 1), i] for i, n in enumerate(steps)]
            self.gt_pos_all += [gt[: (n - 1), i] for i, n in enumerate(steps)]

            if start + self.world * self.num_envs >= self.num_unique_motions:
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

    def local_rows(self):
        """[n, COLS] float64 per-motion rows of this rank's shard (zero rows for other motions)."""
        rows = torch.zeros((self.num_unique_motions, COLS), dtype=torch.float64)
        if not self.batch_ids:
            return rows
        ids = np.concatenate(self.batch_ids)
        m = compute_metrics_lite(self.pred_pos_all, self.gt_pos_all, concatenate=False)
        loc = np.zeros((len(ids), COLS))
        loc[:, 0] = 1.0
        loc[:, 1] = np.concatenate(self.terminate_memory)
        loc[:, 2] = np.concatenate(self.motion_length)
        loc[:, 3] = np.concatenate(self.played_steps)
        for k, name in enumerate(METRICS):
            loc[:, 4 + 2 * k] = [float(np.sum(v)) for v in m[name]]
            loc[:, 5 + 2 * k] = [float(len(v)) for v in m[name]]
        rows[torch.from_numpy(ids)] = torch.from_numpy(loc)
        return rows

    def get_final_stats(self, reduce_sum=None):
        if self.pbar is not None:
            self.pbar.clear()
        rows = self.local_rows()
        if self.world > 1 or reduce_sum is not None:
            dev = self.task_env.device if D.is_dist() else "cpu"
            rows = merge_eval_shards(rows.to(dev), reduce_sum).cpu()
        self.results, terminated, lengths, played = summarize_eval(rows)
        self.success_rate = self.results["eval/success_rate"]
        self.failed_keys = self.task_env.motion_data_keys[terminated]
        self.results_by_motion = {
            "motion_keys": self.task_env.motion_data_keys.tolist(),
            "motion_length": lengths,
            "played_steps": played,
            "success": ~terminated,
        }
        return True

    def update_env_and_close(self):
        """Back to training mode; the termination history feeds the PMCP sampling weights, the
        same merged failure set on every rank (then rank 0's weights broadcast)."""
        history = self.task_env.untoggle_eval_mode(self.failed_keys)
        if self.world > 1:
            sync_sampling_state(self.task_env._motion_lib)
            history = self.task_env._motion_lib._termination_history.clone()
        if self.failed_save_path and D.rank() == 0:
            import joblib

            joblib.dump({"failed_keys": self.failed_keys, "termination_history": history}, self.failed_save_path)
        return self.results


def eval_rollout(vec_env, policy, eval_stats, max_steps=None):
    """scripts/train.py:392-429 rollout with EvalStats: deterministic actions until every motion
    of this rank's eval shard has been played (an idle rank only joins the final merge).
    Returns the number of env steps taken."""
    pol = policy.policy if hasattr(policy, "policy") else policy
    if eval_stats.idle:
        eval_stats.get_final_stats()
        return 0
    pol.set_deterministic_action(True)
    obs, _ = vec_env.reset()
    steps = 0
    recurrent = hasattr(policy, "lstm")
    state = None
    try:
        while max_steps is None or steps < max_steps:
            with torch.no_grad():
                if recurrent:  # the LSTM state carried per env, zeroed on reset (train.py:398-415)
                    action, _, _, _, state = policy(obs, state)
                else:
                    action, _, _, _ = policy(obs)
            obs, _, done, trunc, _ = vec_env.step(action)
            steps += 1
            if recurrent:
                reset = torch.logical_or(done.bool(), trunc.bool())
                if bool(reset.any()):
                    state[0][:, reset] = 0
                    state[1][:, reset] = 0
            done, next_batch = eval_stats.post_step_eval()
            if done:
                break
            if recurrent and next_batch and state is not None:
                state[0].zero_()
                state[1].zero_()
    finally:
        pol.set_deterministic_action(False)
    return steps
