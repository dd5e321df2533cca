"""Host-logic tests of the crypto-crate mirror that need no GPU (crypto_tests.rs:31-47)."""
import pytest

from narwhal_amd.crypto import Digest, PublicKey, SecretKey, Signature


def test_import_export_public_key():
    pk = PublicKey(bytes.fromhex("beada06126c78d98b4a1a69f6ee6189694f0f4751538da824f1adc8b14a1b562"))
    export = pk.encode_base64()
    assert PublicKey.decode_base64(export) == pk


def test_import_export_secret_key():
    sk = SecretKey(bytes(range(64)))
    assert SecretKey.decode_base64(sk.encode_base64()) == sk


def test_digest_display_and_ord():
    d = Digest(bytes(range(32)))
    assert repr(d) == "AAECAwQFBgcICQoLDA0ODxAREhMUFRYXGBkaGxwdHh8="
    assert str(d) == repr(d)[:16]
    assert Digest(bytes(32)) < d


def test_signature_default_and_flatten():
    s = Signature.default()
    assert s.flatten() == bytes(64)
    s2 = Signature.from_bytes(bytes(range(64)))
    assert s2.part1 == bytes(range(32)) and s2.part2 == bytes(range(32, 64))


def test_bad_lengths_rejected():
    with pytest.raises(ValueError):
        Digest(b"x")
    with pytest.raises(ValueError):
        PublicKey(bytes(31))
