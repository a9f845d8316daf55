from .phc_policy import PHCPolicy
from .discriminator_policy import DiscriminatorPolicy
from .running_norm import RunningNorm
from .pufferl_policy import Policy, sample_logits

__all__ = ["PHCPolicy", "DiscriminatorPolicy", "RunningNorm", "Policy", "sample_logits"]
