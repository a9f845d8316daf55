"""R18 Experience.store on the device (phc_compact_rows via _native.RowCompactor) against a numpy
restatement of clean_pufferl/structs.py:113-131: the mask-true rows of a step are appended at the
buffer's cursor in row order, clamped to the remaining capacity; bool flags become 0.0 / 1.0.
Covers the flat-word copy kernel (rows of <= 2048 words: the rollout's shape) and the per-field
copy loop (a wider row), every field kind, all-true / random / empty masks and the capacity clamp."""
import numpy as np
import pytest
import torch

from puffer_phc_amd import _native as N

pytestmark = pytest.mark.gpu
dev = "cuda:0"


def _fields(n, cap, obs_w, g):
    obs = torch.randn((n, obs_w), device=dev, generator=g)
    act = torch.randn((n, 69), device=dev, generator=g)
    val = torch.randn(n, device=dev, generator=g)
    ids = torch.randint(0, 1 << 40, (n,), device=dev, generator=g)
    done = torch.rand(n, device=dev, generator=g) < 0.3
    trunc = torch.rand(n, device=dev, generator=g) < 0.1
    srcs = [obs, act, val, ids, done, trunc]
    dsts = [torch.full((cap, obs_w), -7.0, device=dev), torch.full((cap, 69), -7.0, device=dev),
            torch.full((cap,), -7.0, device=dev), torch.full((cap,), -7, dtype=torch.int64, device=dev),
            torch.full((cap,), -7.0, device=dev), torch.full((cap,), -7.0, device=dev)]
    return srcs, dsts


def _expect(srcs, dsts_np, masks, cap):
    ptr = 0
    for s_list, m in zip(srcs, masks):
        idx = np.nonzero(m)[0] if m is not None else np.arange(s_list[0].shape[0])
        take = idx[: max(0, cap - ptr)]
        for s, d in zip(s_list, dsts_np):
            v = s[take]
            d[ptr:ptr + len(take)] = v.astype(d.dtype) if v.dtype == np.bool_ else v
        ptr += len(take)
    return ptr


@pytest.mark.parametrize("obs_w", [934, 2100])  # 1,010 words: flat kernel; 2,176 words: per-field loop
@pytest.mark.parametrize("mask_kind", ["none", "random", "empty"])
def test_row_store_matches_restatement(obs_w, mask_kind):
    n, cap, steps = 1000, 2600, 3  # the third step overruns the capacity
    g = torch.Generator(device=dev).manual_seed(obs_w + len(mask_kind))
    srcs0, dsts = _fields(n, cap, obs_w, g)
    rc = N.RowCompactor(list(zip(srcs0, dsts)), n, cap, dev)
    exp_d = [d.cpu().numpy().copy() for d in dsts]
    all_src, masks = [], []
    for s in range(steps):
        for t in srcs0:  # fresh source values per step
            if t.dtype == torch.bool:
                t.copy_(torch.rand(n, device=dev, generator=g) < 0.5)
            elif t.dtype == torch.int64:
                t.copy_(torch.randint(0, 1 << 40, (n,), device=dev, generator=g))
            else:
                t.copy_(torch.randn(t.shape, device=dev, generator=g))
        if mask_kind == "none":
            m = None
        elif mask_kind == "empty":
            m = torch.zeros(n, dtype=torch.bool, device=dev)
        else:
            m = torch.rand(n, device=dev, generator=g) < 0.7
        rc(m)
        all_src.append([t.cpu().numpy().copy() for t in srcs0])
        masks.append(None if m is None else m.cpu().numpy())
    torch.cuda.synchronize()
    ptr = _expect(all_src, exp_d, masks, cap)
    assert int(rc.cursor.item()) == ptr
    for d, e in zip(dsts, exp_d):
        np.testing.assert_array_equal(d.cpu().numpy(), e)
    n_valid, taken = rc.counts[2:4].tolist()
    assert taken == ptr
    assert n_valid == sum(n if m is None else int(m.sum()) for m in masks)
