from .phc_policy import PHCPolicy
from .discriminator_policy import DiscriminatorPolicy
from .running_norm import RunningNorm
from .pufferl_policy import Policy, sample_logits
from .lstm_policy import LSTMActorPolicy, LSTMCriticPolicy, LSTMWrapper, Recurrent, RecurrentPolicy

__all__ = ["PHCPolicy", "DiscriminatorPolicy", "RunningNorm", "Policy", "sample_logits", "LSTMCriticPolicy",
           "LSTMActorPolicy", "LSTMWrapper", "Recurrent", "RecurrentPolicy"]
