"""Drop-in alias of polarcub_amd.vectors.BinaryMemorylessVectorDistribution."""
from polarcub_amd.vectors import BinaryMemorylessVectorDistribution  # noqa: F401
