"""Drop-in alias of polarcub_amd.scalar_qary (q-ary channels and factories)."""
from polarcub_amd.scalar_qary import QaryMemorylessDistribution, eta_list, makeQEC, makeQSC  # noqa: F401
