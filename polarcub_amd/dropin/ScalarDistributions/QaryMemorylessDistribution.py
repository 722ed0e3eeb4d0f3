"""Drop-in alias of polarcub_amd.scalar_qary (q-ary channels, factories and the q-ary construction)."""
from polarcub_amd.scalar_qary import (Binning, QaryMemorylessDistribution, calcFrozenSet_degradingUpgrading,  # noqa: F401
                                      calcTVAndPe_degradingUpgrading, degrade_cost_lower_bound,
                                      degrade_dynamic_upper_bound, eta_list, lcrCenter, lcrLeft, lcrRight, makeAWGN,
                                      makeInputDistribution, makeQEC, makeQSC, makeQuantizedUniform,
                                      recursivlyBuildQuantizedUniform, upgrade_cost_lower_bound,
                                      upgrade_dynamic_upper_bound)
