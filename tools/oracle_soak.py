#!/usr/bin/env python3
"""Oracle soak against the reference (a checking tool; build container only:
oracle/_ref is compiled from /root/reference).  Many seeds of the fuzz
frames of tests/fuzz_frames.py; for every frame whose outcome the reference
defines (not TRUNCATED: there it reads past the frame), the branch the
reference's own ProcessPacket takes and its TCPCalcChecksum value must equal
the oracle's verdict and tcp_csum — tests/test_oracle_fuzz_ref.py at scale.
Then, for the first `ub_seeds` seeds, the TRUNCATED frames themselves: the
guard-page probe (oracle/ref/ub_probe.c, -O0 and -O3 builds of the
reference) must observe the reference reading past exactly those frames.
  usage: python tools/oracle_soak.py [first_seed] [n_seeds] [frames] [workers] [ub_seeds]"""
import ctypes
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

V_TRUNCATED = 10


def ub_check(seed, frames, tmp):
    """ub_probe over one seed's frames, both builds of the reference: per frame
    the oracle's verdict and the probe's ref-UB-by-observation bit (-O0, -O3)."""
    import subprocess
    import oracle
    from mtcp_amd import DESC_DTYPE
    from tests.fuzz_frames import fuzz_batch
    buf, desc = fuzz_batch(frames, seed, bool(seed & 1))
    v = oracle.rx_chunk(buf, desc, 0)["verdict"]
    buf.tofile(os.path.join(tmp, "rx_buf.bin"))
    desc.astype(DESC_DTYPE).tofile(os.path.join(tmp, "rx_desc.bin"))
    meta = np.zeros((len(desc), 4), np.uint8)
    meta[:, 0] = v == V_TRUNCATED
    meta.tofile(os.path.join(tmp, "rx_meta.bin"))
    bits = {}
    for exe in ("ub_probe_O0", "ub_probe"):
        subprocess.run([os.path.join(ROOT, "oracle", "_ref", exe), tmp, os.path.join(tmp, "ub.bin")],
                       capture_output=True, text=True, check=True)
        bits[exe] = np.fromfile(os.path.join(tmp, "ub.bin"), np.uint8)
    return v, bits["ub_probe_O0"], bits["ub_probe"]


def oracle_branch_if_defined(seed, frames, idx):
    """The branch the reference's -O3 build takes on frames idx (they are
    TRUNCATED for the oracle; at -O3 the reference does not read past them)."""
    import oracle
    from tests.fuzz_frames import fuzz_batch
    if len(idx) == 0:
        return []
    buf, desc = fuzz_batch(frames, seed, bool(seed & 1))
    R = oracle.ref()
    ret, csum = ctypes.c_int(0), ctypes.c_uint16(0)
    out = []
    for i in idx:
        o, L = int(desc["offset"][i]), int(desc["len"][i])
        pkt = np.zeros(L + 64, np.uint8)
        pkt[:L] = buf[o:o + L]
        out.append(R.ref_rx_packet(pkt.ctypes.data, L, ctypes.byref(ret), ctypes.byref(csum)))
    return out


def one(args):
    seed, frames = args
    import oracle
    from tests.fuzz_frames import fuzz_batch
    buf, desc = fuzz_batch(frames, seed, bool(seed & 1))
    want = oracle.rx_chunk(buf, desc, 0)
    R = oracle.ref()
    ret, csum = ctypes.c_int(0), ctypes.c_uint16(0)
    compared = skipped = bad = 0
    first_bad = None
    for i, (o, L) in enumerate(zip(desc["offset"].astype(np.int64), desc["len"].astype(np.int64))):
        v = int(want["verdict"][i])
        if v == V_TRUNCATED:
            skipped += 1
            continue
        pkt = np.zeros(int(L) + 64, np.uint8)          # the reference may zero tcph->check: a copy
        pkt[:L] = buf[o:o + L]
        br = R.ref_rx_packet(pkt.ctypes.data, int(L), ctypes.byref(ret), ctypes.byref(csum))
        ok = br == v and (v not in (0, 9) or csum.value == int(want["tcp_csum"][i]))
        if not ok:
            bad += 1
            if first_bad is None:
                first_bad = {"seed": seed, "frame": i, "len": int(L), "ref": br, "oracle": v}
        compared += 1
    return compared, skipped, bad, first_bad


def main():
    first = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    count = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    frames = int(sys.argv[3]) if len(sys.argv) > 3 else 3000
    workers = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    ub_seeds = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    import oracle
    if not oracle.ref_available():
        print("oracle/_ref not built (needs /root/reference)", file=sys.stderr)
        return 2
    t0 = time.time()
    tot = {"compared": 0, "skipped_truncated": 0, "mismatches": 0}
    first_bad = None
    with mp.Pool(workers) as pool:
        for c, s, b, fb in pool.imap_unordered(one, [(sd, frames) for sd in range(first, first + count)]):
            tot["compared"] += c
            tot["skipped_truncated"] += s
            tot["mismatches"] += b
            first_bad = first_bad or fb
    # -O0 (every load the source writes, in its order) defines ref-UB: its set
    # must be the oracle's TRUNCATED set; -O3 (mTCP's flags) reads past len on
    # a subset, the difference being TCP_LEN_BAD frames whose dead header
    # loads gcc sinks (tests/test_oracle_golden.py::test_ref_ub_at_mtcp_build_flags)
    ub = {"seeds": 0, "frames": 0, "truncated": 0, "agree_O0": 0, "masked_tail_O0": 0, "write_past_len_O0": 0,
          "o3_outside_o0": 0, "o3_fewer": 0, "o3_fewer_not_tcp_len_bad": 0, "first_disagreement": None}
    if ub_seeds:
        import tempfile
        with tempfile.TemporaryDirectory() as tmp:
            for sd in range(first, first + ub_seeds):
                v, b0, b3 = ub_check(sd, frames, tmp)
                t = v == V_TRUNCATED
                u0, u3 = (b0 & 4) != 0, (b3 & 4) != 0
                ub["seeds"] += 1
                ub["frames"] += len(v)
                ub["truncated"] += int(t.sum())
                ub["agree_O0"] += int((u0 == t).sum())
                ub["masked_tail_O0"] += int(((b0 & 2) != 0).sum())
                ub["write_past_len_O0"] += int(((b0 & 8) != 0).sum())
                ub["o3_outside_o0"] += int((u3 & ~u0).sum())
                fewer = u0 & ~u3
                ub["o3_fewer"] += int(fewer.sum())
                # the oracle's verdict is TRUNCATED there; the branch the
                # reference takes at -O3 is the tot_len check's (TCP_LEN_BAD)
                oracle_ok = oracle_branch_if_defined(sd, frames, np.nonzero(fewer)[0])
                ub["o3_fewer_not_tcp_len_bad"] += int(sum(b != 8 for b in oracle_ok))
                if ub["first_disagreement"] is None and (u0 != t).any():
                    ub["first_disagreement"] = {"seed": sd, "frame": int(np.nonzero(u0 != t)[0][0])}
    print(json.dumps({"probe": "oracle_soak", "first_seed": first, "seeds": count, "frames_per_seed": frames,
                      **tot, "first_mismatch": first_bad, "ub_probe": ub,
                      "seconds": round(time.time() - t0, 1)}))
    ub_bad = (ub["frames"] != ub["agree_O0"] or ub["o3_outside_o0"] or ub["o3_fewer_not_tcp_len_bad"])
    return 1 if tot["mismatches"] or ub_bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
