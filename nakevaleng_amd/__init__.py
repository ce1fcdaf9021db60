"""nakevaleng_amd -- MI355X-native Merkle step of nakevaleng's SSTable build.

Drop-in for the reference's ds/merkletree hot path (leaf hash + tree build +
Serialize image), with hand-written gfx950 HIP kernels behind the C-ABI in
include/nkv_merkle.h.  See DESIGN.md.
"""
__version__ = "0.1.0"
