"""Keys of the GEMM-operand weight caches (twin trunks, discriminator).

The MFMA GEMMs read f16 / bf16 copies of the fp32 parameters (twin_mlp.mfma_operands,
disc_mlp.disc_operands), refreshed when a parameter changes.  torch bumps a tensor's version
counter on in-place ops, but FlatAdam (optim.py) updates the flat parameter buffer through a raw
pointer (phc_opt_step) and broadcast_params writes through `.data`: neither is seen by the version
counters.  Every such writer advances this process-wide generation instead, and every cache key
carries it, so a cache is never read across an optimizer step.

A cache may also register its refresh plan (register_plan): FlatAdam's fused step then writes the
copies itself from the updated values (phc_opt_step_operands) and marks the cache fresh again, so no
separate refresh launch re-reads the parameters after every optimizer step.  An owner registers
`plan_jobs` [(src param, dst, dst_t)], `fresh_dtype` / `fresh_params` (what its key is computed
from) and keeps its current key in `key`.
"""

import weakref

_GENERATION = 0
_OWNERS = {}
_OWNERS_VERSION = 0


def generation():
    return _GENERATION


def bump():
    """Invalidate every operand cache (called after any parameter write torch cannot see)."""
    global _GENERATION
    _GENERATION += 1


def cache_key(dtype, params):
    """(dtype, generation, (version, data pointer) per parameter)."""
    return (dtype, _GENERATION) + tuple((p._version, p.data_ptr()) for p in params)


def layout_key(dtype, params):
    """What a refresh plan depends on: the dtype and where every parameter lives."""
    return (dtype,) + tuple(p.data_ptr() for p in params)


def register_plan(owner):
    """(Re-)register an operand cache whose plan_jobs changed (a new layout or dtype)."""
    global _OWNERS_VERSION
    _OWNERS[id(owner)] = weakref.ref(owner)
    _OWNERS_VERSION += 1


def plan_owners():
    """The live registered caches."""
    out = []
    for k, ref in list(_OWNERS.items()):
        o = ref()
        if o is None:
            del _OWNERS[k]
        else:
            out.append(o)
    return out


def plans_version():
    return _OWNERS_VERSION


def is_fresh(owner):
    return owner.key is not None and owner.key == cache_key(owner.fresh_dtype, owner.fresh_params)


def mark_fresh(owner):
    """After a writer rewrote every copy of owner's plan from the current parameter values."""
    owner.key = cache_key(owner.fresh_dtype, owner.fresh_params)
