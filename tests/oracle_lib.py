"""ctypes access to the CPU restatement (oracle/build/libnwc_oracle.so) -- the checker.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "libnwc_oracle.so")


class Oracle:
    def __init__(self, lib):
        self.lib = lib
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        lib.orc_verify_strict.argtypes = [vp, vp, vp]
        lib.orc_leaf.argtypes = [vp, vp, vp]
        lib.orc_vote_class.argtypes = [vp, vp, vp]
        lib.orc_verify_batch.argtypes = [vp, vp, vp, sz, vp]
        lib.orc_sha512.argtypes = [vp, sz, vp]
        lib.orc_public_key.argtypes = [vp, vp]
        lib.orc_sign.argtypes = [vp, vp, sz, vp]
        for f in ("orc_verify_strict_many", "orc_leaf_many", "orc_vote_class_many"):
            getattr(lib, f).argtypes = [vp, vp, vp, sz, vp, ctypes.c_int]
        lib.orc_verify_batch_many.argtypes = [vp, vp, vp, vp, sz, vp, vp, ctypes.c_int]
        lib.orc_verify_batch_straus.argtypes = [vp, vp, vp, sz, ctypes.c_uint64]
        lib.orc_verify_batch_straus_many.argtypes = [vp, vp, vp, vp, sz, vp, ctypes.c_int]
        lib.orc_digest32_many_mt.argtypes = [vp, vp, sz, vp, ctypes.c_int]
        lib.orc_keygen_sign_many.argtypes = [vp, vp, sz, sz, vp, vp, ctypes.c_int]
        lib.orc_batch_z_many.argtypes = [vp, vp, vp, vp, vp, sz, vp, ctypes.c_int]

    @staticmethod
    def _p(a):
        if isinstance(a, np.ndarray):
            return a.ctypes.data_as(ctypes.c_void_p)
        if a is None:
            return None
        return ctypes.cast(ctypes.c_char_p(bytes(a)), ctypes.c_void_p)

    def verify_strict(self, m, pk, sig) -> bool:
        return bool(self.lib.orc_verify_strict(self._p(m), self._p(pk), self._p(sig)))

    def leaf(self, m, pk, sig) -> bool:
        return bool(self.lib.orc_leaf(self._p(m), self._p(pk), self._p(sig)))

    def sha512(self, data: bytes) -> bytes:
        out = ctypes.create_string_buffer(64)
        self.lib.orc_sha512(self._p(data) if data else None, len(data), out)
        return out.raw

    def public_key(self, seed: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.lib.orc_public_key(self._p(seed), out)
        return out.raw

    def sign(self, seed: bytes, msg: bytes) -> bytes:
        out = ctypes.create_string_buffer(64)
        self.lib.orc_sign(self._p(seed), self._p(msg), len(msg), out)
        return out.raw

    def strict_many(self, msgs: np.ndarray, pks: np.ndarray, sigs: np.ndarray, threads: int = 8) -> np.ndarray:
        n = pks.shape[0]
        out = np.zeros(n, dtype=np.uint8)
        self.lib.orc_verify_strict_many(self._p(msgs), self._p(pks), self._p(sigs), n, self._p(out), threads)
        return out.astype(bool)

    def leaf_many(self, msgs: np.ndarray, pks: np.ndarray, sigs: np.ndarray, threads: int = 8) -> np.ndarray:
        n = pks.shape[0]
        out = np.zeros(n, dtype=np.uint8)
        self.lib.orc_leaf_many(self._p(msgs), self._p(pks), self._p(sigs), n, self._p(out), threads)
        return out.astype(bool)

    def vote_class_many(self, msgs: np.ndarray, pks: np.ndarray, sigs: np.ndarray, threads: int = 8) -> np.ndarray:
        """orc_vote_class per triple: -1 parse/decode failure, 0 ok, 1 randomized, 2 err."""
        n = len(msgs)
        out = np.empty(n, np.uint8)
        self.lib.orc_vote_class_many(self._p(msgs), self._p(pks), self._p(sigs), n, self._p(out), threads)
        return out.astype(np.int8) - 1

    def batch_many(self, digests: np.ndarray, offsets: np.ndarray, pks: np.ndarray, sigs: np.ndarray,
                   threads: int = 8):
        m = offsets.shape[0] - 1
        cert = np.zeros(m, dtype=np.uint8)
        bad = np.zeros(int(offsets[-1]), dtype=np.uint8)
        self.lib.orc_verify_batch_many(self._p(digests), self._p(offsets.astype(np.uint32)), self._p(pks),
                                       self._p(sigs), m, self._p(cert), self._p(bad), threads)
        return cert.astype(bool), bad.astype(bool)

    def batch_straus_many(self, digests: np.ndarray, offsets: np.ndarray, pks: np.ndarray, sigs: np.ndarray,
                          threads: int = 8) -> np.ndarray:
        """dalek 1.0.1 verify_batch algorithm (random z_i, Straus MSM) per certificate."""
        m = len(offsets) - 1
        out = np.zeros(m, dtype=np.uint8)
        offs = np.ascontiguousarray(offsets, dtype=np.uint32)
        self.lib.orc_verify_batch_straus_many(self._p(digests), self._p(offs), self._p(pks), self._p(sigs), m,
                                              self._p(out), threads)
        return out.astype(bool)

    def batch_z_many(self, digests: np.ndarray, offsets: np.ndarray, pks: np.ndarray, sigs: np.ndarray,
                     zs: np.ndarray, z8: bool) -> np.ndarray:
        """dalek's batch equation per certificate for given z_i (zs: 16 bytes per vote), term by term
        (orc_batch_eq_z) or in E[8] = Z/8 as the GPU resolves it (orc_batch_z8)."""
        m = offsets.shape[0] - 1
        out = np.zeros(m, dtype=np.uint8)
        self.lib.orc_batch_z_many(self._p(digests), self._p(offsets.astype(np.uint32)), self._p(pks), self._p(sigs),
                                  self._p(zs), m, self._p(out), 1 if z8 else 0)
        return out.astype(bool)

    def keygen_sign_many(self, seeds: np.ndarray, msgs: np.ndarray, threads: int = 8):
        n = seeds.shape[0]
        pks = np.zeros((n, 32), dtype=np.uint8)
        sigs = np.zeros((n, 64), dtype=np.uint8)
        self.lib.orc_keygen_sign_many(self._p(seeds), self._p(msgs), msgs.shape[1], n, self._p(pks), self._p(sigs),
                                      threads)
        return pks, sigs

    def digest_many(self, data: np.ndarray, offsets: np.ndarray, threads: int = 8) -> np.ndarray:
        n = offsets.shape[0] - 1
        out = np.zeros((n, 32), dtype=np.uint8)
        self.lib.orc_digest32_many_mt(self._p(data), self._p(offsets.astype(np.uint64)), n, self._p(out), threads)
        return out


OSSL_SO = os.path.join(ROOT, "oracle", "build", "libnwc_ossl.so")


def openssl_verify_many(msgs: np.ndarray, pks: np.ndarray, sigs: np.ndarray, threads: int = 8) -> np.ndarray:
    """OpenSSL EVP Ed25519 verification per triple (oracle/openssl_ed25519.c): bench.py's
    third-party CPU point -- NOT dalek semantics (accepts what verify_strict rejects)."""
    if not os.path.exists(OSSL_SO):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = ctypes.CDLL(OSSL_SO)
    vp = ctypes.c_void_p
    lib.ossl_ed25519_verify_many.argtypes = [vp, vp, vp, ctypes.c_size_t, vp, ctypes.c_int]
    n = pks.shape[0]
    out = np.zeros(n, dtype=np.uint8)
    m, p, s = (np.ascontiguousarray(a, dtype=np.uint8) for a in (msgs, pks, sigs))
    assert m.shape == (n, 32) and p.shape == (n, 32) and s.shape == (n, 64)
    lib.ossl_ed25519_verify_many(Oracle._p(m), Oracle._p(p), Oracle._p(s), n, Oracle._p(out), threads)
    return out.astype(bool)


_ORACLE = None


def load_oracle() -> Oracle:
    global _ORACLE
    if _ORACLE is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
        _ORACLE = Oracle(ctypes.CDLL(ORACLE_SO))
    return _ORACLE
