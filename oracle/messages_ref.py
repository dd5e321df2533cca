"""CPU restatement of the reference's primary-message checks -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module; the
product (libnwc.so, narwhal_amd/) never imports it.

Restates, on the wire bytes a primary receives:
  * bincode 1.3 legacy decoding of PrimaryMessage (primary/src/primary.rs:33-38, :230):
    little-endian fixint, u64 lengths/counts, u32 enum variant, trailing bytes ignored;
  * PublicKey serde = base64 string (crypto/src/lib.rs:94-112): serde String (UTF-8), then
    `PublicKey::decode_base64` (crypto/src/lib.rs:73-79) = base64 0.13 `decode` (restated in
    b64_013_decode from its published algorithm; base64 = "0.13.0", crypto/Cargo.toml) and
    `bytes[..32]`, which panics when fewer than 32 bytes decode (reported as DECODE_PANIC);
  * Header.payload: BTreeMap<Digest, WorkerId> and Header.parents: BTreeSet<Digest>
    (primary/src/messages.rs:17-18): serde inserts the decoded entries one by one, so the header
    holds them sorted by digest bytes, duplicates dropped (a map keeps the last value);
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
DECODE_PANIC = 11   # not a DagError: the reference panics inside bincode::deserialize (primary.rs:230)
NAMES = ["Ok", "InvalidSignature", "InvalidHeaderId", "MalformedHeader", "UnknownAuthority", "AuthorityReuse",
         "CertificateRequiresQuorum", "TooOld", "SerializationError", "UnexpectedVote", "UnexpectedMessage",
         "DecodePanic"]

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


# ---- base64 0.13 decode ---------------------------------------------------------------------
def b64_013_decode(s: bytes) -> Optional[bytes]:
    """base64 0.13 `decode(input)` with the STANDARD config (standard alphabet; padding is not
    required on decode; decode_allow_trailing_bits = false) -> bytes, or None for a DecodeError.

    The crate decodes the input in 8-symbol chunks.  Every chunk but the last goes through
    `decode_chunk`, which rejects any byte outside the alphabet ('=' included).  A length of 1 or 5
    modulo 8 is InvalidLength.  The last chunk (1..8 bytes) is decoded symbol by symbol: '=' may
    only stand at a position i (within the chunk) with i % 4 >= 2 and may only be followed by '=';
    the k symbols before it give floor(6k / 8) bytes, and the bits past those must be zero
    (InvalidLastSymbol)."""
    n = len(s)
    if n == 0:
        return b""
    if n % 8 in (1, 5):
        return None
    tl = (n - 1) % 8 + 1
    head, tail = s[:n - tl], s[n - tl:]
    acc, bits, out = 0, 0, bytearray()
    for c in head:
        v = B64.find(chr(c)) if 0 < c < 128 else -1
        if v < 0:
            return None
        acc, bits = (acc << 6) | v, bits + 6
        if bits == 24:
            out += acc.to_bytes(3, "big")
            acc, bits = 0, 0
    k, pad, t = 0, False, 0
    for i, c in enumerate(tail):
        if c == ord("="):
            if i % 4 < 2:
                return None
            pad = True
            continue
        if pad:
            return None
        v = B64.find(chr(c)) if 0 < c < 128 else -1
        if v < 0:
            return None
        t, k = (t << 6) | v, k + 1
    assert k in (2, 3, 4, 6, 7, 8), k   # 0, 1, 5 are excluded by the length and padding rules
    nb = 6 * k // 8
    extra = 6 * k - 8 * nb
    if t & ((1 << extra) - 1):
        return None
    return bytes(out) + (t >> extra).to_bytes(nb, "big")


# ---- bincode decoding ---------------------------------------------------------------------
class Short(Exception):
    pass


class Panic(Exception):
    """`bytes[..32]` on a base64 decode shorter than 32 bytes (crypto/src/lib.rs:75)."""


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
        """PublicKey::deserialize: String (bincode: u64 length + UTF-8 bytes), then
        decode_base64 (crypto/src/lib.rs:73-79, 103-112)."""
        n = self.u64()
        s = self.take(n)
        try:
            s.decode("utf-8")
        except UnicodeDecodeError:
            raise Short()
        d = b64_013_decode(s)
        if d is None:
            raise Short()
        if len(d) < 32:
            raise Panic()
        return d[:32]


def parse_header(r: Rd):
    author = r.key()
    round_ = r.u64()
    P = r.u64()
    wire_payload = [(r.take(32), r.u32()) for _ in range(P)] if P * 36 <= len(r.b) else r.take(P * 36)
    Q = r.u64()
    wire_parents = [r.take(32) for _ in range(Q)] if Q * 32 <= len(r.b) else r.take(Q * 32)
    hid = r.take(32)
    sig = r.take(64)
    # BTreeMap / BTreeSet (primary/src/messages.rs:17-18): sorted, deduplicated, last value wins
    payload = {}
    for d, w in wire_payload:
        payload[d] = w
    return dict(author=author, round=round_, payload=sorted(payload.items()), parents=sorted(set(wire_parents)),
                id=hid, sig=sig)


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
    """-> (kind, fields), (None, None) on a bincode/serde error, ("panic", None) when a key's
    base64 decodes to fewer than 32 bytes before any error."""
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
            votes = []
            for _ in range(V):   # every vote takes >= 72 bytes: the loop ends at the message end
                votes.append((r.key(), r.take(64)))
            return 2, dict(header=h, votes=votes)
        if v == 3:
            return 3, None
        return None, None
    except Short:
        return None, None
    except Panic:
        return "panic", None


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
    if kind == "panic":
        return DECODE_PANIC, None, bytes(32)
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
def enc_key(pk: bytes, text: Optional[bytes] = None) -> bytes:
    """bincode of a PublicKey: its base64 string (base64::encode), or `text` verbatim."""
    s = base64.b64encode(pk) if text is None else text
    return struct.pack("<Q", len(s)) + s


def enc_header(author: bytes, round_: int, payload: Sequence[Tuple[bytes, int]], parents: Sequence[bytes],
               hid: bytes, sig: bytes, wire_order: bool = False, author_text: Optional[bytes] = None) -> bytes:
    """bincode of a Header.  Serialising a BTreeMap/BTreeSet emits sorted entries; wire_order=True
    emits them as given (duplicates and all), as a Byzantine peer may."""
    b = enc_key(author, author_text) + struct.pack("<Q", round_) + struct.pack("<Q", len(payload))
    for d, w in (payload if wire_order else sorted(payload)):
        b += d + struct.pack("<I", w)
    b += struct.pack("<Q", len(parents)) + b"".join(parents if wire_order else sorted(parents)) + hid + sig
    return b


def header_id(author: bytes, round_: int, payload, parents) -> bytes:
    """Header::digest of the canonical (BTree) form of the given entries (last value wins)."""
    canon = {}
    for d, w in payload:
        canon[d] = w
    return header_digest(dict(author=author, round=round_, payload=sorted(canon.items()),
                              parents=sorted(set(parents))))


def msg_header(hdr: bytes) -> bytes:
    return struct.pack("<I", 0) + hdr


def msg_vote(hid: bytes, round_: int, origin: bytes, author: bytes, sig: bytes) -> bytes:
    return struct.pack("<I", 1) + hid + struct.pack("<Q", round_) + enc_key(origin) + enc_key(author) + sig


def msg_certificate(hdr: bytes, votes: Sequence[Tuple[bytes, bytes]], key_texts=None) -> bytes:
    """key_texts (optional, per vote): the key's string verbatim instead of base64::encode."""
    b = struct.pack("<I", 2) + hdr + struct.pack("<Q", len(votes))
    for j, (k, s) in enumerate(votes):
        b += enc_key(k, None if key_texts is None else key_texts[j]) + s
    return b
