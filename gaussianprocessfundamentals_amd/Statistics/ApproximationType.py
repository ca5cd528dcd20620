"""Global approximation kinds (gpbasics/Statistics/ApproximationType.py:4-12).

The reference writes each member with a trailing comma, so every value is a 1-tuple; the values are
kept as such so that ``.value`` compares equal across the two packages."""
from enum import Enum


class GlobalApproximations(Enum):
    Nystroem = (0,)
    SKC = (1,)
    SKI = (2,)
    SOD_Grid = (3,)           # subset of data on a grid
    SOD_Random = (4,)         # random subset of data
    SOD_SmoothedGrid = (5,)
