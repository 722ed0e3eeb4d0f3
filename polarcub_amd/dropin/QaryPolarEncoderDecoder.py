"""Drop-in alias of polarcub_amd.coding_qary (the reference's QaryPolarEncoderDecoder module)."""
from polarcub_amd.coding_qary import (ProbResult, QaryPolarEncoderDecoder, calcNormalizationVector,  # noqa: F401
                                      encodeDecodeSimulation, encodeListDecodeSimulation, frozenSetFromTVAndPe,
                                      genieEncodeDecodeSimulation, hamming, irSimulation,
                                      normalize, normalizeDistList, polarTransformOfQudits, uIndexType)
