"""The oracle against the reference's own rx code (oracle/_ref, compiled from
/root/reference) on random frames (tests/fuzz_frames.py): the branch
ProcessPacket takes and TCPCalcChecksum's value must equal the oracle's
verdict and tcp_csum for every frame whose outcome the reference defines
(frames where it would read past the frame, and ICMP frames whose odd length
makes it read an uninitialised byte, are the documented exceptions).  This
pins the restatement beyond the committed golden vectors; it needs the
reference build, so it runs in the build container only."""
import ctypes

import numpy as np
import pytest

import oracle
from tests.fuzz_frames import fuzz_batch

V_TRUNCATED, V_ICMP = 10, 6


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("seed,aligned", [(301, True), (302, False)])
def test_oracle_equals_reference_on_random_frames(seed, aligned):
    buf, desc = fuzz_batch(3000, seed, aligned)
    want = oracle.rx_chunk(buf, desc, 0)
    R = oracle.ref()
    ret, csum = ctypes.c_int(0), ctypes.c_uint16(0)
    compared = 0
    for i, (o, L) in enumerate(zip(desc["offset"].astype(np.int64), desc["len"].astype(np.int64))):
        v = int(want["verdict"][i])
        if v == V_TRUNCATED:
            continue
        pkt = np.zeros(int(L) + 64, np.uint8)          # the reference may zero tcph->check: a copy
        pkt[:L] = buf[o:o + L]
        br = R.ref_rx_packet(pkt.ctypes.data, int(L), ctypes.byref(ret), ctypes.byref(csum))
        assert br == v, (i, int(L), br, v)
        if v in (0, 9):
            assert csum.value == int(want["tcp_csum"][i]), (i, csum.value, int(want["tcp_csum"][i]))
        compared += 1
    assert compared > 2000
