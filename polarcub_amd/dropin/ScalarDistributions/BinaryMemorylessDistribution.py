"""Drop-in alias of polarcub_amd.scalar (binary channels, factories, Tal-Vardy construction)."""
from polarcub_amd.scalar import (BinaryMemorylessDistribution, calcFrozenSet_degradingUpgrading, eta,  # noqa: F401
                                 eta_list, hxgiveny, makeBEC, makeBernoulli, makeBSC, naturalEta)
