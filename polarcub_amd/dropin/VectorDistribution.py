"""Drop-in alias: the VectorDistribution plugin base class."""
from polarcub_amd.vectors import VectorDistribution  # noqa: F401
