"""The AMP replay buffer's refresh in Experience.flatten_batch (reference clean_pufferl/structs.py:165-176:
rows replaced with probability amp_obs_update_prob, then a random permutation of the replay rows per
minibatch) from the counter-based draw (round 6: capture-safe, the same numbers graphed or eager).  CPU:
the first call copies the buffer, later calls replace exactly the rows whose draw falls below p with a
select, the replay index is a permutation, and the draws depend only on the device iteration counter."""
import numpy as np
import torch

from puffer_phc_amd.clean_pufferl import structs as S


def _exp(p=0.25, batch=512, mb=128):
    e = S.Experience(batch, 8, mb, (4,), device="cpu", use_amp_obs=True, amp_obs_size=6, amp_obs_update_prob=p)
    e.env_ids[:] = torch.arange(batch) % 16
    return e


def _mix64_ref(z):
    m = (1 << 64) - 1
    z &= m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def test_mix64_matches_splitmix_finaliser():
    zs = [0, 1, 123456789123, 2**62 + 7, 2**63 + 5]
    got = S._mix64(torch.tensor([z - 2**64 if z >= 2**63 else z for z in zs], dtype=torch.int64)).tolist()
    want = [_mix64_ref(z) for z in zs]
    assert [g & ((1 << 64) - 1) for g in got] == want


def test_replay_refresh_replaces_the_drawn_rows_and_permutes():
    e = _exp()
    e.sort_training_data()
    e.amp_obs.copy_(torch.arange(512 * 6, dtype=torch.float32).reshape(512, 6))
    e.flatten_batch()
    assert torch.equal(e.amp_obs_replay, e.amp_obs)  # first call: the whole buffer
    old = e.amp_obs_replay.clone()
    e.amp_obs.add_(10_000.0)
    e.flatten_batch()
    it = e._amp_iter.clone()  # an int64 tensor: the product wraps as on the device
    idx = torch.arange(512, dtype=torch.int64)
    u = S._lsr(S._mix64(idx + it * S._GOLD), 40).float() * (1.0 / 16777216.0)
    upd = u < 0.25
    assert 0 < int(upd.sum()) < 512
    assert torch.equal(e.amp_obs_replay[upd], e.amp_obs[upd]) and torch.equal(e.amp_obs_replay[~upd], old[~upd])
    rep = e.b_amp_rep_idx.reshape(-1)
    assert e.b_amp_rep_idx.shape == (4, 128) and torch.equal(torch.sort(rep).values, idx)


def test_replay_draws_follow_the_counter_only():
    a, b = _exp(), _exp()
    for e in (a, b):
        e.sort_training_data()
        e.flatten_batch()
        e.flatten_batch()
    assert torch.equal(a.b_amp_rep_idx, b.b_amp_rep_idx)
    a.flatten_batch()
    assert not torch.equal(a.b_amp_rep_idx, b.b_amp_rep_idx)  # the next iteration draws anew
    fr = np.mean([float((S._lsr(S._mix64(torch.arange(4096) + torch.tensor(k) * S._GOLD), 40).float() / 16777216.0 < 0.01)
                        .float().mean()) for k in range(1, 9)])
    assert 0.005 < fr < 0.015  # rows replaced at the configured rate
