"""Per-wave phase times of k_verify_cold (block 0 of a 3-vote first-sight certificate), printed by
a build with -DNWC_COLD_TIMING=1 (tools/build_variant.sh cold_timing -DNWC_COLD_TIMING=1):
    NWC_LIB_PATH=narwhal_amd/variants/cold_timing.so python tools/cold_timing.py [strict]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from narwhal_amd import device  # noqa: E402

strict = len(sys.argv) > 1 and sys.argv[1] == "strict"
for rep in range(3):
    msgs = device.derive32(b"cold-timing-msg", rep, 3)
    pks, sigs = device.keygen_sign(device.derive32(b"cold-timing-seed", rep, 3), msgs)
    w = device.verify(msgs, pks, sigs, strict=strict)
    torch.cuda.synchronize()
    print("rep", rep, "verdicts", device.unpack_bits(w, 3).tolist(), flush=True)
