"""Training entry point, drop-in for the reference's scripts/train.py (modes train | play | eval).

    python scripts/train.py --env.motion-file data/motion/amass_train.pkl --train.total-timesteps 1e9
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 scripts/train.py ...   # one rank per GPU

`--env.motion-file synthetic:<num_motions>` builds a synthetic SMPL library on the device
(no dataset needed).  Checkpoints keep the reference layout (experiments/<exp_id>/model_*.pt).
"""

import math
import os
import sys
import uuid
from dataclasses import dataclass, field
from typing import Optional

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import phc_amd_path  # noqa: E402

phc_amd_path.register()

from puffer_phc_amd import clean_pufferl, cli  # noqa: E402
from puffer_phc_amd import distributed as D  # noqa: E402
from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv  # noqa: E402
from puffer_phc_amd.config import EnvConfig, PolicyConfig, RNNConfig, TrainConfig  # noqa: E402
from puffer_phc_amd.eval_stats import EvalStats, eval_rollout  # noqa: E402
from puffer_phc_amd.policies import PHCPolicy, Policy  # noqa: E402


@dataclass
class AppConfig:
    policy_name: str = "PHCPolicy"
    rnn_name: Optional[str] = None
    mode: str = "train"
    checkpoint_path: Optional[str] = None
    track: bool = False
    wandb_project: str = "pufferlib"
    run_name: Optional[str] = None
    skip_resample: bool = False
    final_eval: bool = False
    env: EnvConfig = field(default_factory=EnvConfig)
    policy: PolicyConfig = field(default_factory=PolicyConfig)
    rnn: RNNConfig = field(default_factory=RNNConfig)
    train: TrainConfig = field(default_factory=TrainConfig)

    def __post_init__(self):
        self.exp_id = self.env.name + "-" + str(uuid.uuid4())[:8]


def make_motion_data(env_cfg):
    mf = env_cfg.motion_file
    if isinstance(mf, str) and mf.startswith("synthetic:"):
        from puffer_phc_amd.motion_lib import PackedMotions
        from puffer_phc_amd.synthetic import synthetic_clips

        q, t, c, fps = synthetic_clips(env_cfg.num_envs, seed=env_cfg.seed, device=env_cfg.device)
        return PackedMotions.from_global_rotations(q, t, c, fps)
    if isinstance(mf, str) and mf.startswith("standing:"):  # standing:<num_motions>[:<sway radians>]
        from puffer_phc_amd.motion_lib import PackedMotions
        from puffer_phc_amd.synthetic import standing_clips

        parts = mf.split(":")
        sway = float(parts[2]) if len(parts) > 2 else 0.0
        q, t, c, fps = standing_clips(int(parts[1]), sway=sway, seed=env_cfg.seed, device=env_cfg.device)
        return PackedMotions.from_global_rotations(q, t, c, fps)
    return None


def make_policy(env, args):
    """scripts/train.py:259-272: PHCPolicy (the fused MFMA path) or an LSTM policy, optionally under
    the Recurrent wrapper (`--policy-name LSTMCriticPolicy --rnn-name Recurrent`)."""
    from puffer_phc_amd import policies

    if args.policy_name == "PHCPolicy":
        inner = PHCPolicy(env, hidden_size=args.policy.hidden_size, layer_sizes=args.policy.layer_sizes)
    elif args.policy_name in ("LSTMCriticPolicy", "LSTMActorPolicy"):
        inner = getattr(policies, args.policy_name)(env, hidden_size=args.policy.hidden_size)
    else:
        raise ValueError(f"unknown policy {args.policy_name!r} (PHCPolicy | LSTMCriticPolicy | LSTMActorPolicy)")
    if args.rnn_name:
        if args.rnn_name != "Recurrent":
            raise ValueError(f"unknown rnn {args.rnn_name!r} (Recurrent)")
        rnn = policies.Recurrent(env, inner, input_size=args.rnn.input_size, hidden_size=args.rnn.hidden_size)
        return policies.RecurrentPolicy(rnn).to(args.train.device)
    return Policy(inner).to(args.train.device)


def train(args, vec_env, policy):
    cfg = args.train
    components, state, utilization = clean_pufferl.create(args.exp_id, cfg, args.env, vec_env, policy)
    data_dir = os.path.join(cfg.data_dir, args.exp_id)
    os.makedirs(data_dir, exist_ok=True)
    results = {}
    while state.global_step < cfg.total_timesteps:
        if not args.skip_resample and state.epoch > 0 and state.epoch % cfg.motion_resample_interval == 0:
            if state.epoch % cfg.checkpoint_interval == 0:  # scripts/train.py:318-327
                eval_stats = EvalStats(vec_env, failed_save_path=os.path.join(data_dir, f"failed_{state.epoch:06d}.pkl"),
                                       progress=D.rank() == 0)
                eval_rollout(vec_env, policy, eval_stats)
                eval_stats.update_env_and_close()
            vec_env.env.resample_motions()
            vec_env.reset()
            exp = components.experience
            if exp.lstm_h is not None:  # reset the envs and the LSTM hidden states (train.py:329-333)
                exp.lstm_h.zero_()
                exp.lstm_c.zero_()
        _, env_infos = clean_pufferl.evaluate(components, state)
        rms = getattr(components.policy.policy, "update_obs_rms", None)
        if rms:
            rms(components.experience.obs)
        if state.use_amp_obs:
            components.policy.policy.update_amp_obs_rms(components.experience.amp_obs)
        losses = clean_pufferl.train(components, state, utilization)
        if cfg.lr_decay_rate > 0:  # scripts/train.py:352-356
            decay = max(math.exp(-cfg.lr_decay_rate * state.epoch), cfg.lr_decay_floor)
            components.optimizer.param_groups[0]["lr"] = cfg.learning_rate * decay
        if D.rank() == 0:
            ep = {k: sum(float(x) for x in v) / len(v) for k, v in env_infos.items() if len(v)}
            print(f"epoch {state.epoch} step {state.global_step} SPS {state.profile.SPS:.0f} "
                  f"pg {losses.policy_loss:.4f} v {losses.value_loss:.4f} kl {losses.approx_kl:.5f} "
                  f"ep_len {ep.get('episode_length', float('nan')):.1f} ep_ret {ep.get('episode_return', float('nan')):.3f} "
                  f"rew_pos {ep.get('rew_body_pos', float('nan')):.4f}", flush=True)
    if args.final_eval:
        eval_stats = EvalStats(vec_env, progress=D.rank() == 0)
        eval_rollout(vec_env, policy, eval_stats)
        results.update(eval_stats.update_env_and_close())
    clean_pufferl.close(components, state, utilization)
    return results


def evaluate_policy(vec_env, policy, out_prefix="eval"):
    """--mode eval (scripts/train.py:468-482): success rate / MPJPE over every motion, written as
    a JSON summary and a per-motion TSV."""
    import json
    from datetime import datetime

    eval_stats = EvalStats(vec_env)
    eval_rollout(vec_env, policy, eval_stats)
    stamp = datetime.now().strftime("%m%d_%H%M")
    with open(f"{out_prefix}_summary_{stamp}.json", "w") as f:
        json.dump(eval_stats.results, f, indent=4)
    rbm = eval_stats.results_by_motion
    with open(f"results_by_motion_{stamp}.tsv", "w") as f:
        f.write("\t".join(rbm) + "\n")
        for row in zip(*rbm.values()):
            f.write("\t".join(str(x) for x in row) + "\n")
    eval_stats.update_env_and_close()
    return eval_stats.results


def rollout(vec_env, policy, steps=1000):
    policy.policy.set_deterministic_action(True)
    obs, _ = vec_env.reset()
    state = None
    for _ in range(steps):
        with torch.no_grad():
            if hasattr(policy, "lstm"):
                action, _, _, _, state = policy(obs, state)
            else:
                action, _, _, _ = policy(obs)
        obs, _, done, trunc, info = vec_env.step(action)
        if state is not None:
            reset = torch.logical_or(done.bool(), trunc.bool())
            state[0][:, reset] = 0
            state[1][:, reset] = 0
        if info:
            print(info[0])
    policy.policy.set_deterministic_action(False)


def main(argv=None):
    args = cli.parse(AppConfig(), argv)
    rank, world = D.init_from_env()
    if world > 1:
        args.env.device_id = args.train.device_id = int(os.environ.get("LOCAL_RANK", 0))
        args.env.seed = args.env.seed + rank
    if args.mode == "play":
        args.env.num_envs = 16
    vec_env = PHCPufferEnv(args.env, motion_data=make_motion_data(args.env))
    policy = make_policy(vec_env, args)
    if args.checkpoint_path:
        ckpt = torch.load(args.checkpoint_path, map_location=args.train.device, weights_only=True)
        policy.load_state_dict(ckpt["state_dict"])
    if args.mode == "train":
        train(args, vec_env, policy)
    elif args.mode == "play":
        vec_env.env.set_termination_distances(10)
        rollout(vec_env, policy)
    elif args.mode == "eval":
        print(evaluate_policy(vec_env, policy))
    else:
        raise ValueError(f"unknown mode {args.mode!r} (train | play | eval)")


if __name__ == "__main__":
    main()
