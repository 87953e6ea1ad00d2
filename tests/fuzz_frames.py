"""Random frames for the fuzz parity tests (tests/test_gpu_fuzz.py on the GPU,
tests/test_oracle_fuzz_ref.py against the reference's own code on the CPU):
random lengths (1 B to 20 000 B) and bytes, headers drawn to reach every
branch of ProcessPacket -> ProcessIPv4Packet -> ProcessTCPPacket (ethertypes,
ihl 0..15, version, tot_len shorter / longer than the frame, protocols, doff
0..15), a valid IP header checksum for most frames, valid TCP checksums from
the oracle's tx fill where they apply, then single-bit corruptions."""
import numpy as np

import oracle
from mtcp_amd import DESC_DTYPE


def fuzz_batch(n, seed, aligned):
    rng = np.random.default_rng(seed)
    k = rng.random(n)
    L = np.where(k < .3, rng.integers(1, 129, n),
                 np.where(k < .7, rng.integers(54, 1601, n),
                          np.where(k < .9, rng.integers(1600, 9001, n), rng.integers(9000, 20001, n))))
    offs = np.zeros(n, np.int64)
    pos = 0
    for i in range(n):
        if aligned:
            offs[i] = pos
            pos += (int(L[i]) + 63) & ~63
        else:
            offs[i] = ((pos + 127) & ~127) + 2 * int(rng.integers(0, 64))   # any even start
            pos = offs[i] + int(L[i])
    buf = rng.integers(0, 256, ((pos + 127) & ~127) + 128, dtype=np.uint8)

    def put(i, at, vals):
        o = offs[i] + at
        for j, v in enumerate(vals):
            if at + j < L[i]:
                buf[o + j] = v

    for i in range(n):
        r = rng.random(8)
        put(i, 12, [0x08, 0x00] if r[0] < .8 else ([0x08, 0x06] if r[0] < .85 else list(rng.integers(0, 256, 2))))
        ihl = 5 if r[1] < .75 else int(rng.integers(0, 16))
        ver = 4 if r[2] < .92 else int(rng.integers(0, 16))
        put(i, 14, [(ver << 4) | ihl])
        tl = int(L[i]) - 14
        if r[3] < .15:
            tl = max(0, tl - int(rng.integers(1, 41)))          # Ethernet padding
        elif r[3] < .25:
            tl = int(rng.integers(0, 65536))
        elif r[3] < .3:
            tl += int(rng.integers(1, 41))                         # claims more than the frame
        tl &= 0xFFFF
        put(i, 16, [tl >> 8, tl & 0xFF])
        put(i, 23, [6 if r[4] < .8 else (1 if r[4] < .9 else int(rng.integers(0, 256)))])
        T = 14 + 4 * ihl
        put(i, T + 12, [0x50 if r[5] < .7 else (0x80 if r[5] < .9 else int(rng.integers(0, 256)))])
        if ihl >= 5 and L[i] >= T and r[6] < .85:                  # a valid IP header checksum
            o = offs[i]
            buf[o + 24:o + 26] = 0
            c = oracle.ip_fast_csum(buf[o + 14:o + T].tobytes(), ihl)
            buf[o + 24], buf[o + 25] = c & 0xFF, c >> 8
    desc = np.zeros(n, dtype=DESC_DTYPE)
    desc["offset"] = offs.astype(np.uint32)
    desc["len"] = L.astype(np.uint16)
    oracle.tx_fill(buf, desc, 0)                                   # valid checksums where they apply
    flip = np.nonzero(rng.random(n) < .1)[0]
    for i in flip:                                                 # single-bit corruptions
        b = int(rng.integers(0, L[i]))
        buf[offs[i] + b] ^= np.uint8(1 << int(rng.integers(0, 8)))
    return buf, desc
