"""CPU restatement of the reference's primary-message checks -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module; the
product (libnwc.so, narwhal_amd/) never imports it.

Restates, on the wire bytes a primary receives:
  * bincode 1.3 legacy decoding of PrimaryMessage (primary/src/primary.rs:33-38, :230):
    little-endian fixint, u64 lengths/counts, u32 enum variant, trailing bytes ignored;
  * PublicKey serde = base64 string (crypto/src/lib.rs:94-112), restricted to the canonical
    44-character padded form (other base64 0.13 forms are parity-unpinned);
  * Header::digest (primary/src/messages.rs:70-84), Vote::digest (:145-153),
    Certificate::digest (:226-234): SHA-512[..32];
  * Header::verify (:48-67), Vote::verify (:131-142), Certificate::verify (:189-215) with
    Certificate::genesis / PartialEq (:173-186, :249-255), and the Core::sanitize_* prefixes
    (primary/src/core.rs:306-346): TooOld / UnexpectedVote;
  * Committee::stake / worker / quorum_threshold (config/src/lib.rs:154-212).
Signature verdicts come from a pluggable `sig` object with strict(msg, pk, sig) -> bool and
leaf(msg, pk, sig) -> bool (the Python or C restatement of dalek, oracle/).
"""
from __future__ import annotations

import base64
import hashlib
import struct
from typing import Dict, List, Optional, Sequence, Tuple

OK, INVALID_SIGNATURE, INVALID_HEADER_ID, MALFORMED_HEADER, UNKNOWN_AUTHORITY = 0, 1, 2, 3, 4
AUTHORITY_REUSE, REQUIRES_QUORUM, TOO_OLD, SERIALIZATION, UNEXPECTED_VOTE, UNEXPECTED_MESSAGE = 5, 6, 7, 8, 9, 10
NAMES = ["Ok", "InvalidSignature", "InvalidHeaderId", "MalformedHeader", "UnknownAuthority", "AuthorityReuse",
         "CertificateRequiresQuorum", "TooOld", "SerializationError", "UnexpectedVote", "UnexpectedMessage"]

B64 = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"


def sha512_32(b: bytes) -> bytes:
    return hashlib.sha512(b).digest()[:32]


# ---- committee ------------------------------------------------------------------------------
class RefCommittee:
    """config::Committee: authorities (BTreeMap<PublicKey, Authority>) with stake and worker ids."""

    def __init__(self, authorities: Dict[bytes, Tuple[int, Sequence[int]]]):
        self.auth = {bytes(k): (int(s), list(w)) for k, (s, w) in authorities.items()}

    def stake(self, name: bytes) -> int:
        return self.auth.get(name, (0, []))[0]

    def worker_ok(self, name: bytes, wid: int) -> bool:
        return name in self.auth and wid in self.auth[name][1]

    def quorum_threshold(self) -> int:
        return 2 * sum(s for s, _ in self.auth.values()) // 3 + 1


# ---- bincode decoding ---------------------------------------------------------------------
class Short(Exception):
    pass


class Rd:
    def __init__(self, b: bytes):
        self.b, self.p = b, 0

    def take(self, n: int) -> bytes:
        if n < 0 or self.p + n > len(self.b):
            raise Short()
        r = self.b[self.p:self.p + n]
        self.p += n
        return r

    def u32(self) -> int:
        return struct.unpack("<I", self.take(4))[0]

    def u64(self) -> int:
        return struct.unpack("<Q", self.take(8))[0]

    def key(self) -> bytes:
        n = self.u64()
        s = self.take(n)
        if n != 44 or s[43:44] != b"=" or any(c not in B64.encode() for c in s[:43]):
            raise Short()
        raw = base64.b64decode(s, validate=True)
        if B64.index(chr(s[42])) & 3:       # non-zero trailing bits
            raise Short()
        return raw[:32]


def parse_header(r: Rd):
    author = r.key()
    round_ = r.u64()
    P = r.u64()
    payload = [(r.take(32), r.u32()) for _ in range(P)] if P * 36 <= len(r.b) else r.take(P * 36)
    Q = r.u64()
    parents = [r.take(32) for _ in range(Q)] if Q * 32 <= len(r.b) else r.take(Q * 32)
    hid = r.take(32)
    sig = r.take(64)
    return dict(author=author, round=round_, payload=payload, parents=parents, id=hid, sig=sig)


def header_digest(h) -> bytes:
    b = h["author"] + struct.pack("<Q", h["round"])
    for d, w in h["payload"]:
        b += d + struct.pack("<I", w)
    for p in h["parents"]:
        b += p
    return sha512_32(b)


def digest72(hid: bytes, round_: int, key: bytes) -> bytes:
    return sha512_32(hid + struct.pack("<Q", round_) + key)


def decode(msg: bytes):
    """-> (kind, fields) or (None, None) on a bincode/serde error."""
    r = Rd(msg)
    try:
        v = r.u32()
        if v == 0:
            return 0, parse_header(r)
        if v == 1:
            hid = r.take(32)
            round_ = r.u64()
            origin = r.key()
            author = r.key()
            sig = r.take(64)
            return 1, dict(id=hid, round=round_, origin=origin, author=author, sig=sig)
        if v == 2:
            h = parse_header(r)
            V = r.u64()
            if V * 116 > len(msg):
                raise Short()
            votes = [(r.key(), r.take(64)) for _ in range(V)]
            return 2, dict(header=h, votes=votes)
        if v == 3:
            return 3, None
        return None, None
    except Short:
        return None, None


# ---- the checks ---------------------------------------------------------------------------
def header_verify(h, committee: RefCommittee, sig) -> int:
    """Header::verify (primary/src/messages.rs:48-67)."""
    if header_digest(h) != h["id"]:
        return INVALID_HEADER_ID
    if committee.stake(h["author"]) <= 0:
        return UNKNOWN_AUTHORITY
    for _, wid in h["payload"]:
        if not committee.worker_ok(h["author"], wid):
            return MALFORMED_HEADER
    return OK if sig.strict(h["id"], h["author"], h["sig"]) else INVALID_SIGNATURE


def certificate_verify(c, committee: RefCommittee, sig) -> int:
    """Certificate::verify (primary/src/messages.rs:189-215)."""
    h = c["header"]
    if h["id"] == bytes(32) and h["round"] == 0 and h["author"] in committee.auth:
        return OK                                    # genesis (:191-193, PartialEq :249-255)
    e = header_verify(h, committee, sig)
    if e != OK:
        return e
    weight, used = 0, set()
    for name, _ in c["votes"]:
        if name in used:
            return AUTHORITY_REUSE
        st = committee.stake(name)
        if st <= 0:
            return UNKNOWN_AUTHORITY
        used.add(name)
        weight += st
    if weight < committee.quorum_threshold():
        return REQUIRES_QUORUM
    cd = digest72(h["id"], h["round"], h["author"])
    # Signature::verify_batch (crypto/src/lib.rs:206-219) on the deterministic domain = all leaves
    return OK if all(sig.leaf(cd, k, s) for k, s in c["votes"]) else INVALID_SIGNATURE


def sanitize(msg: bytes, committee: RefCommittee, sig, gc_round: int = 0,
             vote_target: Optional[Tuple[bytes, int, bytes]] = None) -> Tuple[int, Optional[int], bytes]:
    """Core::sanitize_* on one wire message -> (code, kind, digest of the message)."""
    kind, f = decode(msg)
    if kind is None:
        return SERIALIZATION, None, bytes(32)
    if kind == 3:
        return UNEXPECTED_MESSAGE, 3, bytes(32)
    if kind == 0:
        dig = header_digest(f)
        if gc_round > f["round"]:
            return TOO_OLD, 0, dig
        return header_verify(f, committee, sig), 0, dig
    if kind == 1:
        dig = digest72(f["id"], f["round"], f["origin"])
        if vote_target is not None:
            tid, tround, torigin = vote_target
            if tround > f["round"]:
                return TOO_OLD, 1, dig
            if not (f["id"] == tid and f["origin"] == torigin and f["round"] == tround):
                return UNEXPECTED_VOTE, 1, dig
        if committee.stake(f["author"]) <= 0:
            return UNKNOWN_AUTHORITY, 1, dig
        return (OK if sig.strict(dig, f["author"], f["sig"]) else INVALID_SIGNATURE), 1, dig
    h = f["header"]
    dig = digest72(h["id"], h["round"], h["author"])
    if gc_round > h["round"]:
        return TOO_OLD, 2, dig
    return certificate_verify(f, committee, sig), 2, dig


# ---- bincode encoding (fixture construction) ------------------------------------------------
def enc_key(pk: bytes) -> bytes:
    s = base64.b64encode(pk)
    return struct.pack("<Q", len(s)) + s


def enc_header(author: bytes, round_: int, payload: Sequence[Tuple[bytes, int]], parents: Sequence[bytes],
               hid: bytes, sig: bytes) -> bytes:
    b = enc_key(author) + struct.pack("<Q", round_) + struct.pack("<Q", len(payload))
    for d, w in sorted(payload):
        b += d + struct.pack("<I", w)
    b += struct.pack("<Q", len(parents)) + b"".join(sorted(parents)) + hid + sig
    return b


def header_id(author: bytes, round_: int, payload, parents) -> bytes:
    return header_digest(dict(author=author, round=round_, payload=sorted(payload), parents=sorted(parents)))


def msg_header(hdr: bytes) -> bytes:
    return struct.pack("<I", 0) + hdr


def msg_vote(hid: bytes, round_: int, origin: bytes, author: bytes, sig: bytes) -> bytes:
    return struct.pack("<I", 1) + hid + struct.pack("<Q", round_) + enc_key(origin) + enc_key(author) + sig


def msg_certificate(hdr: bytes, votes: Sequence[Tuple[bytes, bytes]]) -> bytes:
    b = struct.pack("<I", 2) + hdr + struct.pack("<Q", len(votes))
    for k, s in votes:
        b += enc_key(k) + s
    return b
