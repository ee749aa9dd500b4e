"""genomealignmenttools_amd -- MI355X-native chain scoring / netting engine.

Drop-in for the hot path of hillerlab/GenomeAlignmentTools (scoreChain,
chainNet -rescore, chainCleaner suspect rescoring): hand-written HIP kernels
for gfx950 behind the C ABI in include/gachain.h (libgachain.so), C host tools
with the reference's command-line surface in bin/, and this thin Python
mirror for tests and benchmarks.
"""
from ._lib import BIN_DIR, LIB_PATH, GacError  # noqa: F401

__all__ = ["BIN_DIR", "LIB_PATH", "GacError"]
