"""PendingLossComponents (clean_pufferl/structs.py): train()'s loss row arrives by a non-blocking copy;
the first read of ANY attribute — dunder access such as vars(), __dict__, dataclasses.asdict,
copy included — waits on the copy's event and fills every LossComponents field
(clean_pufferl/core.py:367-374, the reference's LossComponents, puffer_phc/clean_pufferl/structs.py)."""

import copy
import dataclasses

import numpy as np
import torch

from puffer_phc_amd.clean_pufferl.core import _fill_losses
from puffer_phc_amd.clean_pufferl.structs import LossComponents, PendingLossComponents

FIELDS = [f.name for f in dataclasses.fields(LossComponents)]


class _Event:
    def __init__(self):
        self.waits = 0

    def synchronize(self):
        self.waits += 1


def _row():
    return torch.arange(14, dtype=torch.float64) + 0.5


def _expected():
    ref = LossComponents()
    _fill_losses(ref, _row().numpy())
    return dataclasses.asdict(ref)


def test_attribute_read_fills_once():
    ev = _Event()
    p = PendingLossComponents(_row(), ev, _fill_losses)
    assert p.policy_loss == 0.5 and ev.waits == 1
    assert p.value_loss == 1.5 and ev.waits == 1
    assert p.explained_variance == 13.5


def test_dunder_access_fills():
    for read in (vars, lambda x: x.__dict__, dataclasses.asdict, copy.copy, copy.deepcopy):
        ev = _Event()
        p = PendingLossComponents(_row(), ev, _fill_losses)
        out = read(p)
        assert ev.waits == 1
        got = out if isinstance(out, dict) else {k: getattr(out, k) for k in FIELDS}
        exp = _expected()
        for k in FIELDS:
            np.testing.assert_equal(got[k], exp[k], err_msg=k)


def test_explained_variance_nan_when_var_y_zero():
    row = _row()
    row[12] = 0
    p = PendingLossComponents(row, _Event(), _fill_losses)
    assert np.isnan(p.explained_variance)


def test_pinned_ring_resolves_a_slot_before_reuse(monkeypatch):
    """train()'s loss-row buffers are reused round-robin (clean_pufferl/core.py _PinnedRing): a slot
    whose PendingLossComponents was never read is resolved, with its own values, before it is
    overwritten."""
    from puffer_phc_amd.clean_pufferl import core

    real_empty = torch.empty
    monkeypatch.setattr(torch, "empty", lambda *a, pin_memory=False, **k: real_empty(*a, **k))
    ring = core._PinnedRing(n=2)
    owners = []
    for i in range(3):
        row = _row() + 100.0 * i
        slot = ring.take(row, None)
        if i < 2:
            assert len(ring.slots[(tuple(row.shape), row.dtype)]) == i + 1
        else:  # the first slot again: its unread owner resolved first
            assert slot is ring.slots[(tuple(row.shape), row.dtype)][0]
            assert object.__getattribute__(owners[0], "__dict__").get("_pending") is None
        slot[0].copy_(row)
        p = PendingLossComponents(slot[0], _Event(), _fill_losses)
        slot[1] = p
        owners.append(p)
    assert owners[0].policy_loss == 0.5  # the values it held before the buffer was reused
    assert owners[2].policy_loss == 200.5
