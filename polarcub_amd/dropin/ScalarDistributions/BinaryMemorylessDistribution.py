"""Drop-in alias of polarcub_amd.scalar (binary channels and factories)."""
from polarcub_amd.scalar import BinaryMemorylessDistribution, eta, hxgiveny, makeBEC, makeBSC  # noqa: F401
