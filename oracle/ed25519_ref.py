"""Pure-Python restatement of the reference's Ed25519 verify / SHA-512 digest semantics.

TEST INFRASTRUCTURE ONLY -- this module is the checker, never the product path.
Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may use
anything under `oracle/` (and only as the checker). It is slow (Python big ints),
meant for small cases and for generating the committed golden fixtures.

What it restates (reference call sites, /root/reference):
  * `crypto::Signature::verify`        crypto/src/lib.rs:200-204
        -> ed25519 1.x `Signature::from_bytes` + dalek `PublicKey::from_bytes`
           + dalek 1.0.1 `PublicKey::verify_strict`             
  * `crypto::Signature::verify_batch`  crypto/src/lib.rs:206-219
        -> dalek 1.0.1 `verify_batch` (batch feature, random z_i)  
  * the per-signature bisection leaf   (not in the reference)
  * `Digest = SHA-512(bytes)[..32]`    worker/src/processor.rs:38,
                                       crypto/src/tests/crypto_tests.rs:8-12
  * signing (`Signature::new`, crypto/src/lib.rs:185-191 -> RFC 8032 sign) and
    key generation (`generate_keypair`, crypto/src/lib.rs:167-175) for fixtures.

The arithmetic lives in un-vendored crates (ed25519-dalek 1.0.1, curve25519-dalek 3.x,
ed25519 1.x, sha2 0.9 -- crypto/Cargo.toml:10); their published algorithms are
restated here from the specification in SURVEY.md Appendix A.  SHA-512 uses
`hashlib` (OpenSSL), an independent FIPS 180-4 implementation.
"""
from __future__ import annotations

import hashlib
import random
from typing import List, Optional, Sequence, Tuple

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)

Point = Tuple[int, int]  # affine (x, y); the group law below is complete for Ed25519
IDENTITY: Point = (0, 1)


def sha512(data: bytes) -> bytes:
    return hashlib.sha512(data).digest()


def digest32(data: bytes) -> bytes:
    """`Digest(Sha512::digest(bytes)[..32])` -- worker/src/processor.rs:38."""
    return sha512(data)[:32]


# ----------------------------------------------------------------------------- field
def fe_is_negative(x: int) -> bool:
    """curve25519-dalek `FieldElement::is_negative`: low bit of the canonical encoding."""
    return (x % P) & 1 == 1


def sqrt_ratio_i(u: int, v: int) -> Tuple[bool, int]:
    """curve25519-dalek 3 `FieldElement::sqrt_ratio_i`.

    Returns (was_nonzero_square, r) with r the non-negative root of u/v when it exists;
    u == 0 gives (True, 0); a non-square gives (False, r * something) -- only the flag
    matters for decompression.
    """
    u %= P
    v %= P
    v3 = v * v % P * v % P
    v7 = v3 * v3 % P * v % P
    r = (u * v3 % P) * pow(u * v7 % P, (P - 5) // 8, P) % P
    check = v * r % P * r % P
    correct = check == u
    flipped = check == (-u) % P
    flipped_i = check == (-u) * SQRT_M1 % P
    if flipped or flipped_i:
        r = r * SQRT_M1 % P
    if fe_is_negative(r):
        r = (-r) % P
    return (correct or flipped), r


# ----------------------------------------------------------------------------- group
def pt_add(p1: Point, p2: Point) -> Point:
    x1, y1 = p1
    x2, y2 = p2
    t = D * x1 % P * x2 % P * y1 % P * y2 % P
    x3 = (x1 * y2 + y1 * x2) * pow(1 + t, P - 2, P) % P
    y3 = (y1 * y2 + x1 * x2) * pow(1 - t, P - 2, P) % P
    return (x3, y3)


def pt_neg(p: Point) -> Point:
    return ((-p[0]) % P, p[1])


def pt_mul(k: int, p: Point) -> Point:
    if k < 0:
        return pt_mul(-k, pt_neg(p))
    acc = IDENTITY
    add = p
    while k:
        if k & 1:
            acc = pt_add(acc, add)
        add = pt_add(add, add)
        k >>= 1
    return acc


def on_curve(p: Point) -> bool:
    x, y = p
    return (-x * x + y * y - 1 - D * x * x % P * y * y) % P == 0


B_Y = 4 * pow(5, P - 2, P) % P
_ok, _bx = sqrt_ratio_i(B_Y * B_Y - 1, D * B_Y * B_Y + 1)
assert _ok
BASEPOINT: Point = (_bx, B_Y)  # x even (non-negative), RFC 8032
assert on_curve(BASEPOINT)


def compress(p: Point) -> bytes:
    x, y = p
    b = bytearray(y.to_bytes(32, "little"))
    if x & 1:
        b[31] |= 0x80
    return bytes(b)


def decompress(b: bytes) -> Optional[Point]:
    """curve25519-dalek 3 `CompressedEdwardsY::decompress`.

    y = the low 255 bits, NOT required < p (reduced implicitly); the sign bit negates x
    even when x == 0 (accepted, unlike RFC 8032).
    """
    assert len(b) == 32
    y = (int.from_bytes(b, "little") & ((1 << 255) - 1)) % P
    yy = y * y % P
    u = (yy - 1) % P
    v = (yy * D + 1) % P
    ok, x = sqrt_ratio_i(u, v)
    if not ok:
        return None
    if b[31] >> 7:
        x = (-x) % P
    return (x, y)


def is_small_order(p: Point) -> bool:
    """`EdwardsPoint::is_small_order` = mul_by_cofactor().is_identity()."""
    return pt_mul(8, p) == IDENTITY


# ----------------------------------------------------------------------------- scalars
def scalar_from_hash(h: bytes) -> int:
    """`Scalar::from_hash` -- 64-byte little-endian integer mod l."""
    return int.from_bytes(h, "little") % L


def sig_scalar_ok(sig: bytes) -> bool:
    """A.1: ed25519 1.x `Signature::from_bytes` (sig[63] & 0xE0 == 0) + dalek `check_scalar`
    (fast accept if sig[63] & 0xF0 == 0, else `Scalar::from_canonical_bytes`). Net: s < l."""
    if len(sig) != 64:
        return False
    if sig[63] & 0xE0:
        return False
    s = int.from_bytes(sig[32:], "little")
    if sig[63] & 0xF0 == 0:
        return True
    return s < L


# ----------------------------------------------------------------------------- verify
def verify_strict(msg: bytes, pk: bytes, sig: bytes) -> bool:
    """`crypto::Signature::verify` (crypto/src/lib.rs:200-204) -> dalek `verify_strict` (A.3)."""
    if not sig_scalar_ok(sig):
        return False
    A = decompress(pk)
    if A is None:
        return False
    R = decompress(sig[:32])
    if R is None:
        return False
    if is_small_order(R) or is_small_order(A):
        return False
    k = scalar_from_hash(sha512(sig[:32] + pk + msg))
    s = int.from_bytes(sig[32:], "little")
    Rp = pt_add(pt_mul(k, pt_neg(A)), pt_mul(s, BASEPOINT))
    return Rp == R  # group equality (dalek's projective ct_eq)


def residual(msg: bytes, pk: bytes, sig: bytes) -> Optional[Point]:
    """e = s*B - R - k*A for a parsed vote, or None if the vote fails A.1/A.2."""
    if not sig_scalar_ok(sig):
        return None
    A = decompress(pk)
    R = decompress(sig[:32])
    if A is None or R is None:
        return None
    k = scalar_from_hash(sha512(sig[:32] + pk + msg))
    s = int.from_bytes(sig[32:], "little")
    return pt_add(pt_add(pt_mul(s, BASEPOINT), pt_neg(R)), pt_neg(pt_mul(k, A)))


def has_torsion(p: Point) -> bool:
    """A point with a non-zero 8-torsion component: l * P != O (curve25519-dalek 3
    `EdwardsPoint::is_torsion_free` negated)."""
    return pt_mul(L, p) != IDENTITY


def vote_class(msg: bytes, pk: bytes, sig: bytes) -> str:
    """One vote of dalek 1.0.1 `verify_batch` (as corrected in round 2).

    dalek checks   -(sum z_i s_i mod l) B + sum z_i R_i + sum (z_i k_i mod l) A_i == O
    with random 128-bit z_i.  Writing z_i k_i = (z_i k_i mod l) + q_i l, the A-term differs from
    z_i k_i A_i by q_i (l A_i) = q_i (l T_i), T_i the 8-torsion component of A_i.  So the
    batch sum is  -sum z_i e_i - sum q_i l T_i  (e_i = s_i B - R_i - k_i A_i), and a vote is
      "err"         it fails A.1/A.2, or e_i has a prime-order component (Err w.p. 1 - 2^-125);
      "randomized"  e_i is pure torsion and (e_i != O or T_i != O): the verdict depends on
                    thread_rng through z_i and q_i = floor(z_i k_i / l);
      "ok"          e_i == O and A_i is torsion-free (identity included): deterministic Ok.
    """
    e = residual(msg, pk, sig)
    if e is None:
        return "err"
    if pt_mul(8, e) != IDENTITY:
        return "err"
    if e != IDENTITY or has_torsion(decompress(pk)):
        return "randomized"
    return "ok"


def leaf_ok(msg: bytes, pk: bytes, sig: bytes) -> bool:
    """A.5 bisection leaf = dalek `verify_batch([vote])` decided deterministically: the vote
    parses, pk and R decode, e == identity (cofactorless) and A is torsion-free.  On the
    randomized domain the build answers Err (bad vote)."""
    return vote_class(msg, pk, sig) == "ok"


def verify_batch_class(msg: bytes, votes: Sequence[Tuple[bytes, bytes]]) -> str:
    """`crypto::Signature::verify_batch` (crypto/src/lib.rs:206-219) -> dalek `verify_batch` (A.4).

    Returns "err" if any vote is "err"; else "randomized" if any vote is (the reference's
    verdict then depends on thread_rng; the build returns Err there); else "ok".
    """
    classes = [vote_class(msg, pk, sig) for pk, sig in votes]
    if "err" in classes:
        return "err"
    return "randomized" if "randomized" in classes else "ok"


def verify_batch(msg: bytes, votes: Sequence[Tuple[bytes, bytes]]) -> bool:
    """Deterministic verdict of the build: Ok iff every leaf is Ok (A.4 / A.5)."""
    return all(leaf_ok(msg, pk, sig) for pk, sig in votes)


def verify_batch_dalek_sampled(msg: bytes, votes: Sequence[Tuple[bytes, bytes]],
                               rng: random.Random) -> bool:
    """One draw of dalek 1.0.1 `verify_batch`'s equation as the crate computes it
    (crypto/src/lib.rs:218): random 128-bit z_i (thread_rng stands in for the merlin-seeded
    RNG), the basepoint coefficient -(sum z_i s_i) mod l, z_i on R_i and (z_i k_i mod l) on A_i."""
    bcoef, acc = 0, IDENTITY
    for pk, sig in votes:
        if not sig_scalar_ok(sig):
            return False
        A = decompress(pk)
        R = decompress(sig[:32])
        if A is None or R is None:
            return False
        k = scalar_from_hash(sha512(sig[:32] + pk + msg))
        s = int.from_bytes(sig[32:], "little")
        z = rng.getrandbits(128)
        bcoef = (bcoef + z * s) % L
        acc = pt_add(acc, pt_add(pt_mul(z, R), pt_mul(z * k % L, A)))
    acc = pt_add(acc, pt_mul((-bcoef) % L, BASEPOINT))
    return acc == IDENTITY


def verify_batch_dalek_z(msg: bytes, votes: Sequence[Tuple[bytes, bytes]], zs: Sequence[int]) -> bool:
    """dalek 1.0.1 `verify_batch`'s equation (crypto/src/lib.rs:218) for GIVEN 128-bit z_i, as the
    crate computes it: -(sum z_i s_i mod l) B + sum z_i R_i + sum (z_i k_i mod l) A_i == O."""
    bcoef, acc = 0, IDENTITY
    for (pk, sig), z in zip(votes, zs):
        if not sig_scalar_ok(sig):
            return False
        A = decompress(pk)
        R = decompress(sig[:32])
        if A is None or R is None:
            return False
        k = scalar_from_hash(sha512(sig[:32] + pk + msg))
        s = int.from_bytes(sig[32:], "little")
        bcoef = (bcoef + z * s) % L
        acc = pt_add(acc, pt_add(pt_mul(z, R), pt_mul(z * k % L, A)))
    acc = pt_add(acc, pt_mul((-bcoef) % L, BASEPOINT))
    return acc == IDENTITY


# The order-8 point G8 that generates E[8] (y = the fourth small-order y of SURVEY.md A.3, x even).
G8_HEX = "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05"


def torsion_dlog(p: Point) -> Optional[int]:
    """j in 0..7 with p == [j] G8, or None when p is not in E[8] (E[8] is cyclic of order 8)."""
    g = decompress(bytes.fromhex(G8_HEX))
    acc = IDENTITY
    for j in range(8):
        if acc == p:
            return j
        acc = pt_add(acc, g)
    return None


def verify_batch_z8(msg: bytes, votes: Sequence[Tuple[bytes, bytes]], zs: Sequence[int]) -> bool:
    """The same equation for the same z_i, evaluated the way the GPU resolves it
    (narwhal_amd/csrc/resolve.h): with z_i k_i = (z_i k_i mod l) + q_i l and e_i = s_i B - R_i - k_i A_i
    the left side is -sum (z_i e_i + q_i (l A_i)).  A vote that does not parse or decode, or whose
    e_i has a prime-order component, fails the equation (w.p. 1 - 2^-125; decided as Err); the
    others have e_i = [a_i] G8 and l A_i = [b_i] G8, and the equation holds iff
    sum (z_i a_i + q_i b_i) = 0 mod 8."""
    total = 0
    for (pk, sig), z in zip(votes, zs):
        e = residual(msg, pk, sig)
        if e is None or pt_mul(8, e) != IDENTITY:
            return False
        k = scalar_from_hash(sha512(sig[:32] + pk + msg))
        q = (z * k) // L
        total += z * torsion_dlog(e) + q * torsion_dlog(pt_mul(L, decompress(pk)))
    return total % 8 == 0


def batch_z(seed32: bytes, v: int) -> int:
    """The GPU's z_i (narwhal_amd/csrc/straus.h straus_z): SHA-512(seed || u64le(v))[..16], little-endian."""
    return int.from_bytes(sha512(seed32 + v.to_bytes(8, "little"))[:16], "little")


# ----------------------------------------------------------------------------- signing
def secret_expand(seed: bytes) -> Tuple[int, bytes]:
    h = sha512(seed)
    a = bytearray(h[:32])
    a[0] &= 248
    a[31] &= 127
    a[31] |= 64
    return int.from_bytes(a, "little"), h[32:]


def public_key(seed: bytes) -> bytes:
    a, _ = secret_expand(seed)
    return compress(pt_mul(a, BASEPOINT))


def sign(seed: bytes, msg: bytes) -> bytes:
    """RFC 8032 Ed25519 sign == dalek `Keypair::sign` (used by `Signature::new`)."""
    a, prefix = secret_expand(seed)
    A = compress(pt_mul(a, BASEPOINT))
    r = scalar_from_hash(sha512(prefix + msg))
    Rb = compress(pt_mul(r, BASEPOINT))
    k = scalar_from_hash(sha512(Rb + A + msg))
    s = (r + k * a) % L
    return Rb + s.to_bytes(32, "little")


# ----------------------------------------------------------------------------- small order
def small_order_points() -> List[Point]:
    """The 8 points of E[8]."""
    pts = [IDENTITY, (0, P - 1), (SQRT_M1, 0), ((-SQRT_M1) % P, 0)]
    # order-8 points: x^2 = ... solve for y with 8-torsion; find via halving (+-i,0)
    # y^2 for order-8 points satisfies: doubling (x,y) gives y'=(y^2-x^2)/(2-(y^2-x^2))... search:
    # Use the known encoding of one order-8 point and its multiples.
    t8 = decompress(bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05"))
    assert t8 is not None
    acc = IDENTITY
    for _ in range(8):
        acc = pt_add(acc, t8)
        if acc not in pts:
            pts.append(acc)
    assert len(pts) == 8 and all(pt_mul(8, q) == IDENTITY for q in pts)
    return pts
