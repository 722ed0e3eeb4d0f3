"""Drop-in alias of polarcub_amd.vectors.QaryMemorylessVectorDistribution."""
from polarcub_amd.vectors import QaryMemorylessVectorDistribution  # noqa: F401
