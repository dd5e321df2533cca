"""Host-side mirror of the reference's primary messages (/root/reference/primary/src/messages.rs)
and of Core's batched sanitisation (primary/src/core.rs:306-346), backed by the GPU message
pipeline of libnwc.so (nwc_sanitize_messages: bincode + base64 decoding, Header / Vote /
Certificate digests, committee checks and all signatures on the device).

  Header       messages.rs:13-85     author, round, payload {Digest: WorkerId}, parents {Digest},
                                     id, signature; digest(); verify(committee)
  Vote         messages.rs:104-154   id, round, origin, author, signature
  Certificate  messages.rs:168-235   header, votes [(PublicKey, Signature)]; genesis(committee)
  Committee    config/src/lib.rs:134-212  authorities {PublicKey: Authority(stake, workers)}
  DagError     primary/src/error.rs  verification failures (code + variant name)
  sanitize_many(messages, committee, gc_round, current_header) -> [DagError | None]
Wire format = bincode of `PrimaryMessage` (primary/src/primary.rs:33-38), built by `to_bytes()`.
The object-level `verify` / `digest` calls go through the same GPU batch path (a batch of one);
there is no CPU verification path.
"""
from __future__ import annotations

import ctypes
import struct
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Set, Tuple

from . import _lib
from .crypto import Digest, PublicKey, SecretKey, Signature, digest_bytes

__all__ = ["DagError", "Authority", "Committee", "Header", "Vote", "Certificate", "sanitize_many",
           "DAG_ERRORS"]

DAG_ERRORS = ["Ok", "InvalidSignature", "InvalidHeaderId", "MalformedHeader", "UnknownAuthority",
              "AuthorityReuse", "CertificateRequiresQuorum", "TooOld", "SerializationError", "UnexpectedVote",
              "UnexpectedMessage", "DecodePanic"]


class DagError(Exception):
    """primary/src/error.rs DagError: `code` is the NWC_DAG_* value, `name` the variant."""

    def __init__(self, code: int):
        self.code = int(code)
        self.name = DAG_ERRORS[self.code] if 0 <= self.code < len(DAG_ERRORS) else "Unknown"
        super().__init__(self.name)


@dataclass
class Authority:
    stake: int
    workers: Sequence[int] = (0,)


class Committee:
    """config::Committee: authorities ordered as the reference's BTreeMap<PublicKey, _>."""

    def __init__(self, authorities: Dict[PublicKey, Authority]):
        self.authorities = dict(sorted(authorities.items(), key=lambda kv: bytes(kv[0])))

    def stake(self, name: PublicKey) -> int:
        a = self.authorities.get(name)
        return a.stake if a else 0

    def quorum_threshold(self) -> int:
        return 2 * sum(a.stake for a in self.authorities.values()) // 3 + 1

    def install(self) -> None:
        """Upload keys, stakes and worker ids (nwc_set_committee_config).  Every sanitize_many call
        installs its committee: another caller may have replaced the device-side committee."""
        lib = _lib.load()
        keys = b"".join(bytes(k) for k in self.authorities)
        stakes = (ctypes.c_uint64 * max(1, len(self.authorities)))(*[a.stake for a in self.authorities.values()])
        offs, ids = [0], []
        for a in self.authorities.values():
            ids.extend(int(w) for w in a.workers)
            offs.append(len(ids))
        offs_c = (ctypes.c_uint32 * len(offs))(*offs)
        ids_c = (ctypes.c_uint32 * max(1, len(ids)))(*ids)
        _lib.check(lib.nwc_set_committee_config(_lib.buf(keys) if keys else None, stakes, len(self.authorities),
                                                offs_c, ids_c))


# ---- bincode helpers -------------------------------------------------------------------------
def _key(pk: PublicKey) -> bytes:
    s = pk.encode_base64().encode()
    return struct.pack("<Q", len(s)) + s


@dataclass
class Header:
    author: PublicKey = field(default_factory=PublicKey)
    round: int = 0
    payload: Dict[Digest, int] = field(default_factory=dict)
    parents: Set[Digest] = field(default_factory=set)
    id: Digest = field(default_factory=Digest)
    signature: Signature = field(default_factory=Signature)

    @classmethod
    def new(cls, author: PublicKey, round: int, payload: Dict[Digest, int], parents: Set[Digest],
            secret: SecretKey) -> "Header":
        """Header::new (messages.rs:24-46): id = digest(), signature over the id."""
        h = cls(author, round, dict(payload), set(parents))
        h.id = h.digest()
        h.signature = Signature.new(h.id, secret)
        return h

    def digest_input(self) -> bytes:
        b = bytes(self.author) + struct.pack("<Q", self.round)
        for d in sorted(self.payload):
            b += bytes(d) + struct.pack("<I", self.payload[d])
        for p in sorted(self.parents):
            b += bytes(p)
        return b

    def digest(self) -> Digest:
        """Hash for Header (messages.rs:70-84) -- SHA-512 on the GPU."""
        return digest_bytes(self.digest_input())

    def encode(self) -> bytes:
        b = _key(self.author) + struct.pack("<Q", self.round) + struct.pack("<Q", len(self.payload))
        for d in sorted(self.payload):
            b += bytes(d) + struct.pack("<I", self.payload[d])
        b += struct.pack("<Q", len(self.parents)) + b"".join(bytes(p) for p in sorted(self.parents))
        return b + bytes(self.id) + self.signature.flatten()

    def to_bytes(self) -> bytes:
        """bincode of PrimaryMessage::Header(self)."""
        return struct.pack("<I", 0) + self.encode()

    def verify(self, committee: Committee) -> None:
        """Header::verify (messages.rs:48-67); raises DagError."""
        _raise(sanitize_many([self.to_bytes()], committee)[0])


@dataclass
class Vote:
    id: Digest
    round: int
    origin: PublicKey
    author: PublicKey
    signature: Signature = field(default_factory=Signature)

    @classmethod
    def new(cls, header: Header, author: PublicKey, secret: SecretKey) -> "Vote":
        v = cls(header.id, header.round, header.author, author)
        v.signature = Signature.new(v.digest(), secret)
        return v

    def digest(self) -> Digest:
        """Hash for Vote (messages.rs:145-153)."""
        return digest_bytes(bytes(self.id) + struct.pack("<Q", self.round) + bytes(self.origin))

    def to_bytes(self) -> bytes:
        return (struct.pack("<I", 1) + bytes(self.id) + struct.pack("<Q", self.round) + _key(self.origin) +
                _key(self.author) + self.signature.flatten())

    def verify(self, committee: Committee) -> None:
        """Vote::verify (messages.rs:131-142); raises DagError."""
        _raise(sanitize_many([self.to_bytes()], committee)[0])


@dataclass
class Certificate:
    header: Header = field(default_factory=Header)
    votes: List[Tuple[PublicKey, Signature]] = field(default_factory=list)

    @staticmethod
    def genesis(committee: Committee) -> List["Certificate"]:
        return [Certificate(Header(author=name)) for name in committee.authorities]

    def round(self) -> int:
        return self.header.round

    def origin(self) -> PublicKey:
        return self.header.author

    def digest(self) -> Digest:
        """Hash for Certificate (messages.rs:226-234)."""
        return digest_bytes(bytes(self.header.id) + struct.pack("<Q", self.round()) + bytes(self.origin()))

    def to_bytes(self) -> bytes:
        b = struct.pack("<I", 2) + self.header.encode() + struct.pack("<Q", len(self.votes))
        for k, s in self.votes:
            b += _key(k) + s.flatten()
        return b

    def verify(self, committee: Committee) -> None:
        """Certificate::verify (messages.rs:189-215); raises DagError."""
        _raise(sanitize_many([self.to_bytes()], committee)[0])


def _raise(err: Optional[DagError]) -> None:
    if err is not None:
        raise err


def sanitize_many(messages: Sequence[bytes], committee: Committee, gc_round: int = 0,
                  current_header: Optional[Header] = None, digests: Optional[list] = None) -> List[Optional[DagError]]:
    """Core::sanitize_header / sanitize_vote / sanitize_certificate over a batch of wire messages
    (bincode PrimaryMessage bytes, as PrimaryReceiverHandler::dispatch receives them).  Returns
    None (Ok) or the DagError per message; `digests` (a list) receives each message's digest."""
    lib = _lib.load()
    committee.install()
    m = len(messages)
    if m == 0:
        return []
    offs = [0]
    for b in messages:
        offs.append(offs[-1] + len(b))
    data = b"".join(messages) or b"\0"
    offsets = (ctypes.c_uint64 * (m + 1))(*offs)
    codes = (ctypes.c_int32 * m)()
    dig = ctypes.create_string_buffer(32 * m) if digests is not None else None
    target = None
    if current_header is not None:
        target = bytes(current_header.id) + struct.pack("<Q", current_header.round) + bytes(current_header.author)
    _lib.check(lib.nwc_sanitize_messages(_lib.buf(data), offsets, m, gc_round, _lib.buf(target) if target else None,
                                         codes, dig, None))
    if digests is not None:
        raw = dig.raw   # one copy (`.raw` copies the whole buffer on every access)
        digests.extend(Digest(raw[32 * i:32 * i + 32]) for i in range(m))
    return [None if c == 0 else DagError(c) for c in codes]
