"""Keys of the GEMM-operand weight caches (twin trunks, discriminator).

The MFMA GEMMs read f16 / bf16 copies of the fp32 parameters (twin_mlp.mfma_operands,
disc_mlp.disc_operands), refreshed when a parameter changes.  torch bumps a tensor's version
counter on in-place ops, but FlatAdam (optim.py) updates the flat parameter buffer through a raw
pointer (phc_opt_step) and broadcast_params writes through `.data`: neither is seen by the version
counters.  Every such writer advances this process-wide generation instead, and every cache key
carries it, so a cache is never read across an optimizer step.
"""

_GENERATION = 0


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
