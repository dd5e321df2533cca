"""narwhal_amd -- MI355X-native (gfx950) signature-and-digest hot path of Narwhal.

Drop-in for the reference's `crypto` crate verify/digest path: Ed25519
`verify_strict` / `verify_batch` and SHA-512 batch digests as hand-written HIP kernels behind
the C ABI in include/nwc.h (libnwc.so).  `narwhal_amd.crypto` mirrors the crate's API.
"""
__version__ = "0.1.0"
