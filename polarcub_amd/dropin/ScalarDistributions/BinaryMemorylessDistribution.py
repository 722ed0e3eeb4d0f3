"""Drop-in alias of polarcub_amd.scalar (binary channels, factories, Tal-Vardy construction)."""
from polarcub_amd.scalar import (BinaryMemorylessDistribution, _calcKey_degrade, _calcKey_upgrade,  # noqa: F401
                                 _listIndexingHelper, calcFrozenSet_degradingUpgrading, eta, eta_list, hxgiveny,
                                 makeBEC, makeBernoulli, makeBSC, naturalEta, upgradedLeftRightProbs, use_fast)
