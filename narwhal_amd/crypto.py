"""Host-side mirror of the reference's `crypto` crate (/root/reference/crypto/src/lib.rs),
backed by the MI355X kernels in libnwc.so.

Same names, argument meaning and error behaviour as the Rust API, so that parity tests read
like crypto/src/tests/crypto_tests.rs:
  Digest            lib.rs:20-57     32-byte digest, Debug/Display = base64
  Hash              lib.rs:59-62     `digest()`; `Hash for &[u8]` = SHA-512[..32] (tests :8-12)
  PublicKey         lib.rs:64-118    32 bytes, serde as base64
  SecretKey         lib.rs:120-161   64 bytes (seed || public), zeroised on drop
  generate_keypair  lib.rs:167-175
  Signature         lib.rs:177-219   new / verify / verify_batch, Default = 64 zero bytes
  CryptoError       lib.rs:18        opaque verification failure (Rust `Err`)
Device/runtime failures raise `DeviceError` -- never `CryptoError`.
Verification, hashing and signing all run on the GPU; there is no CPU path here.
"""
from __future__ import annotations

import base64
import ctypes
import os
from typing import Iterable, Optional, Sequence, Tuple

from . import _lib
from ._lib import DeviceError

__all__ = ["CryptoError", "DeviceError", "Digest", "Hash", "PublicKey", "SecretKey", "Signature",
           "generate_keypair", "generate_production_keypair", "digest_bytes", "digest_many"]


class CryptoError(Exception):
    """`pub type CryptoError = ed25519::Error` -- an opaque verification failure."""


class Digest:
    __slots__ = ("_b",)

    def __init__(self, b: bytes = bytes(32)):
        b = bytes(b)
        if len(b) != 32:
            raise ValueError("Digest must be 32 bytes")
        self._b = b

    @classmethod
    def try_from(cls, item: bytes) -> "Digest":
        return cls(item)

    def to_vec(self) -> bytes:
        return self._b

    def size(self) -> int:
        return 32

    def __bytes__(self) -> bytes:
        return self._b

    def __eq__(self, o) -> bool:
        return isinstance(o, Digest) and o._b == self._b

    def __lt__(self, o) -> bool:
        return self._b < o._b

    def __hash__(self) -> int:
        return hash(self._b)

    def __repr__(self) -> str:  # Debug = base64 (lib.rs:34-38)
        return base64.b64encode(self._b).decode()

    def __str__(self) -> str:  # Display = first 16 base64 chars (lib.rs:40-44)
        return base64.b64encode(self._b).decode()[:16]


class Hash:
    """`pub trait Hash { fn digest(&self) -> Digest; }`"""

    def digest(self) -> Digest:  # pragma: no cover - interface
        raise NotImplementedError


def digest_bytes(data: bytes) -> Digest:
    """`impl Hash for &[u8]`: Digest(Sha512::digest(data)[..32]) -- on the GPU."""
    lib = _lib.load()
    out = ctypes.create_string_buffer(32)
    data = bytes(data)
    _lib.check(lib.nwc_digest32(_lib.buf(data) if data else None, len(data), out))
    return Digest(out.raw)


def digest_many(messages: Sequence[bytes]) -> list:
    """Batched worker digests (worker/src/processor.rs:38) for many serialized batches."""
    lib = _lib.load()
    offs = [0]
    for m in messages:
        offs.append(offs[-1] + len(m))
    data = b"".join(messages)
    offsets = (ctypes.c_uint64 * len(offs))(*offs)
    out = ctypes.create_string_buffer(32 * len(messages))
    _lib.check(lib.nwc_sha512_trunc32_many(_lib.buf(data) if data else None, offsets, len(messages), out))
    raw = out.raw
    return [Digest(raw[32 * i:32 * i + 32]) for i in range(len(messages))]


class PublicKey:
    __slots__ = ("_b",)

    def __init__(self, b: bytes = bytes(32)):
        b = bytes(b)
        if len(b) != 32:
            raise ValueError("PublicKey must be 32 bytes")
        self._b = b

    def encode_base64(self) -> str:
        return base64.b64encode(self._b).decode()

    @classmethod
    def decode_base64(cls, s: str) -> "PublicKey":
        raw = base64.b64decode(s, validate=True)
        if len(raw) < 32:
            raise ValueError("InvalidLength")
        return cls(raw[:32])

    def __bytes__(self) -> bytes:
        return self._b

    def __eq__(self, o) -> bool:
        return isinstance(o, PublicKey) and o._b == self._b

    def __lt__(self, o) -> bool:
        return self._b < o._b

    def __hash__(self) -> int:
        return hash(self._b)

    def __repr__(self) -> str:
        return self.encode_base64()

    def __str__(self) -> str:
        return self.encode_base64()[:16]


class SecretKey:
    """64 bytes = dalek Keypair::to_bytes() = seed || public key."""
    __slots__ = ("_b",)

    def __init__(self, b: bytes):
        b = bytearray(b)
        if len(b) != 64:
            raise ValueError("SecretKey must be 64 bytes")
        self._b = b

    def encode_base64(self) -> str:
        return base64.b64encode(bytes(self._b)).decode()

    @classmethod
    def decode_base64(cls, s: str) -> "SecretKey":
        raw = base64.b64decode(s, validate=True)
        if len(raw) < 64:
            raise ValueError("InvalidLength")
        return cls(raw[:64])

    def seed(self) -> bytes:
        return bytes(self._b[:32])

    def __eq__(self, o) -> bool:
        return isinstance(o, SecretKey) and bytes(o._b) == bytes(self._b)

    def __del__(self):
        for i in range(len(self._b)):
            self._b[i] = 0


def _keygen_sign(seeds: bytes, msgs: bytes, n: int) -> Tuple[bytes, bytes]:
    """RFC 8032 keygen + sign of n (seed, 32-byte msg) pairs on the GPU (k_keygen_sign)."""
    from . import device
    return device.keygen_sign_host(seeds, msgs, n)


def generate_keypair(rng) -> Tuple[PublicKey, SecretKey]:
    """`generate_keypair(csprng)`: 32 seed bytes from rng (dalek Keypair::generate)."""
    if hasattr(rng, "fill_bytes"):
        seed = rng.fill_bytes(32)
    elif hasattr(rng, "randbytes"):
        seed = rng.randbytes(32)
    else:
        seed = bytes(rng(32))
    pk, _ = _keygen_sign(seed, bytes(32), 1)
    return PublicKey(pk), SecretKey(seed + pk)


def generate_production_keypair() -> Tuple[PublicKey, SecretKey]:
    return generate_keypair(os.urandom)


class Signature:
    """`Signature { part1: R (32 B), part2: s (32 B) }`; Default = 64 zero bytes."""
    __slots__ = ("part1", "part2")

    def __init__(self, part1: bytes = bytes(32), part2: bytes = bytes(32)):
        if len(part1) != 32 or len(part2) != 32:
            raise ValueError("Unexpected signature length")
        self.part1 = bytes(part1)
        self.part2 = bytes(part2)

    @classmethod
    def default(cls) -> "Signature":
        return cls()

    @classmethod
    def from_bytes(cls, b: bytes) -> "Signature":
        return cls(b[:32], b[32:64])

    @classmethod
    def new(cls, digest: Digest, secret: SecretKey) -> "Signature":
        """`Signature::new(digest, secret)` = dalek sign over the 32 digest bytes (GPU)."""
        _, sig = _keygen_sign(secret.seed(), digest.to_vec(), 1)
        return cls.from_bytes(sig)

    def flatten(self) -> bytes:
        return self.part1 + self.part2

    def verify(self, digest: Digest, public_key: PublicKey) -> None:
        """`Signature::verify` -> dalek verify_strict. Raises CryptoError on an invalid signature."""
        lib = _lib.load()
        rc = _lib.check(lib.nwc_verify_strict(_lib.buf(digest.to_vec()), _lib.buf(bytes(public_key)),
                                              _lib.buf(self.flatten())))
        if rc != _lib.NWC_OK:
            raise CryptoError("signature verification failed")

    @staticmethod
    def verify_batch(digest: Digest, votes: Iterable[Tuple[PublicKey, "Signature"]],
                     bad: Optional[list] = None) -> None:
        """`Signature::verify_batch(digest, votes)`. Raises CryptoError if any vote fails.
        If `bad` is a list, it receives the indices of the failing votes (bisection result)."""
        votes = list(votes)
        lib = _lib.load()
        n = len(votes)
        pks = b"".join(bytes(p) for p, _ in votes)
        sigs = b"".join(s.flatten() for _, s in votes)
        bitmap = ctypes.create_string_buffer((n + 7) // 8 or 1)
        rc = _lib.check(lib.nwc_verify_batch(_lib.buf(digest.to_vec()), _lib.buf(pks) if n else None,
                                             _lib.buf(sigs) if n else None, n, bitmap))
        if bad is not None:
            raw = bitmap.raw
            bad.extend(i for i in range(n) if (raw[i >> 3] >> (i & 7)) & 1)
        if rc != _lib.NWC_OK:
            raise CryptoError("batch verification failed")

    def __eq__(self, o) -> bool:
        return isinstance(o, Signature) and o.flatten() == self.flatten()

    def __repr__(self) -> str:
        return "Signature { part1: %s, part2: %s }" % (list(self.part1), list(self.part2))
