from enum import Enum


class StateInit(Enum):
    """puffer_phc/envs/state_init.py:4-8."""

    Default = 0
    Start = 1
    Random = 2
    Hybrid = 3
