"""Drop-in alias of the guard-band functions in polarcub_amd.deletion (the reference's Guardbands module)."""
from polarcub_amd.deletion import addDeletionGuardBands, removeDeletionGuardBands, trimZerosAtEdges  # noqa: F401
