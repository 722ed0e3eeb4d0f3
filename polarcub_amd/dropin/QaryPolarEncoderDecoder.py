"""Drop-in alias of polarcub_amd.coding_qary (the reference's QaryPolarEncoderDecoder module, SC part)."""
from polarcub_amd.coding_qary import (QaryPolarEncoderDecoder, encodeDecodeSimulation,  # noqa: F401
                                      frozenSetFromTVAndPe, polarTransformOfQudits, uIndexType)
