"""Drop-in alias of polarcub_amd.coding (the reference's BinaryPolarEncoderDecoder module)."""
from polarcub_amd.coding import (BinaryPolarEncoderDecoder, encodeDecodeSimulation,  # noqa: F401
                                 frozenSetFromTVAndPe, genieEncodeDecodeSimulation, polarTransformOfBits,
                                 uIndexType)
