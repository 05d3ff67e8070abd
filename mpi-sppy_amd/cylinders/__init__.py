"""Hub-and-spoke cylinders (mpisppy/cylinders/): PHHub, the spoke class
hierarchy, the Lagrangian outer-bound spoke and the xhat-xbar inner-bound
spoke, over node-local shared-memory windows (spwindow.py)."""
from .spoke import (ConvergerSpokeType, Spoke, InnerBoundSpoke, OuterBoundSpoke, OuterBoundWSpoke,  # noqa: F401
                    InnerBoundNonantSpoke, OuterBoundNonantSpoke)
from .hub import Hub, PHHub  # noqa: F401
from .lagrangian_bounder import LagrangianOuterBound  # noqa: F401
from .xhatxbar_bounder import XhatXbarInnerBound  # noqa: F401
