"""Drop-in alias of the trellis plugin in polarcub_amd.deletion (VectorDistributions/BinaryTrellis.py)."""
from polarcub_amd.deletion import (BinaryTrellis, Edge, Vertex, buildTrellis_uniformInput_deletion,  # noqa: F401
                                   deletionChannelSimulation)
