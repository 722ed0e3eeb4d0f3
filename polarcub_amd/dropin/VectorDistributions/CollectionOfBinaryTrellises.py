"""Drop-in alias of the trellis collection in polarcub_amd.deletion
(VectorDistributions/CollectionOfBinaryTrellises.py)."""
from polarcub_amd.deletion import (CollectionOfBinaryTrellises,  # noqa: F401
                                   buildCollectionOfBinaryTrellises_uniformInput_deletion)
