"""Primary-message host logic without a GPU: the CPU restatement (oracle/messages_ref.py) against
the golden wire fixtures (tests/golden/messages.json; positives = the reference's own primary test
fixtures), re-derived here with the C restatement of dalek for signatures; and the host mirror's
bincode encoder (narwhal_amd/messages.py) byte-identical to the fixtures."""
import json
import os
import sys

import pytest

from tests.conftest import GOLDEN, ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))


@pytest.fixture(scope="module")
def golden_messages():
    return json.load(open(os.path.join(GOLDEN, "messages.json")))


class _CSig:
    def __init__(self, oracle):
        self.o = oracle

    def strict(self, m, pk, s):
        return self.o.verify_strict(m, pk, s)

    def leaf(self, m, pk, s):
        return self.o.leaf(m, pk, s)


def _committee(g):
    import messages_ref as mr
    c = g["committee"]
    return mr.RefCommittee({bytes.fromhex(k): (s, w) for k, s, w in zip(c["keys"], c["stakes"], c["workers"])})


def test_oracle_reproduces_golden_codes(golden_messages, oracle):
    import messages_ref as mr
    committee = _committee(golden_messages)
    sig = _CSig(oracle)
    for c in golden_messages["cases"]:
        t = c["target"]
        target = None if t is None else (bytes.fromhex(t[0]), t[1], bytes.fromhex(t[2]))
        code, kind, dig = mr.sanitize(bytes.fromhex(c["msg"]), committee, sig, c["gc_round"], target)
        assert (code, kind if kind is not None else -1, dig.hex()) == (c["code"], c["kind"], c["digest"]), c["name"]


def test_reference_fixtures_are_accepted(golden_messages):
    ref = [c for c in golden_messages["cases"] if c["name"].startswith("ref-")]
    assert len(ref) == 18 and all(c["code"] == 0 for c in ref)


def test_mirror_encoder_matches_fixtures(golden_messages):
    """narwhal_amd.messages builds the same bincode bytes as the fixtures (header(), votes(),
    certificate(), genesis) -- the mirror's wire format is the reference's."""
    import messages_ref as mr
    from narwhal_amd.crypto import Digest, PublicKey, Signature
    from narwhal_amd.messages import Certificate, Header, Vote
    by = {c["name"]: bytes.fromhex(c["msg"]) for c in golden_messages["cases"]}
    for name in ("ref-header", "ref-certificate", "ref-vote-2", "ref-genesis-1", "header-many-parents"):
        kind, f = mr.decode(by[name])
        if kind == 1:
            v = Vote(Digest(f["id"]), f["round"], PublicKey(f["origin"]), PublicKey(f["author"]),
                     Signature.from_bytes(f["sig"]))
            assert v.to_bytes() == by[name], name
            continue
        h = f if kind == 0 else f["header"]
        hdr = Header(PublicKey(h["author"]), h["round"], {Digest(d): w for d, w in h["payload"]},
                     {Digest(p) for p in h["parents"]}, Digest(h["id"]), Signature.from_bytes(h["sig"]))
        if kind == 0:
            assert hdr.to_bytes() == by[name], name
            assert mr.header_digest(h) == __import__("hashlib").sha512(hdr.digest_input()).digest()[:32]
        else:
            cert = Certificate(hdr, [(PublicKey(k), Signature.from_bytes(s)) for k, s in f["votes"]])
            assert cert.to_bytes() == by[name], name
