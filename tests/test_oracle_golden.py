"""The C oracle against the reference's golden vectors (CPU only).

Pins oracle/mtcp_oracle.c — the parity checker for every GPU test — to the
reference's own code: verdicts of the real ProcessPacket chain
(mtcp/src/eth_in.c:9-56, ip_in.c:15-62, tcp_in.c:1138-1175), values of the
real ip_fast_csum (io_engine/include/ps.h:66-95), TCPCalcChecksum
(mtcp/src/tcp_util.c:157-190) and GetRSSHash / GetRSSCPUCore (util/rss.c,
mtcp/src/rss.c), and the Microsoft Toeplitz KATs of util/rss.c:185-189.
"""
import socket
import struct

import numpy as np
import pytest

import oracle
from tests.golden_io import compare_results, pool_case_entries, pool_entries_equal

V_TRUNCATED = 10


def test_ip_fast_csum_vectors(golden):
    c = golden.csum_ip
    got = np.array([oracle.ip_fast_csum(bytes(c["hdr"][i]), int(c["ihl"][i]))
                    for i in range(len(c))], dtype=np.uint16)
    assert np.array_equal(got, c["csum"])
    # ihl <= 4 returns the first dword unfolded (ps.h:72-73): covered above
    assert (c["ihl"] <= 4).sum() >= 16


def test_ip_fast_csum_worked_example():
    # 45 00 00 73 00 00 40 00 40 11 [00 00] c0 a8 00 01 c0 a8 00 c7 -> b8 61
    hdr = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
    assert oracle.ip_fast_csum(hdr, 5) == 0x61b8
    filled = hdr[:10] + struct.pack("<H", 0x61b8) + hdr[12:]
    assert oracle.ip_fast_csum(filled, 5) == 0


def test_tcp_checksum_vectors(golden):
    c = golden.csum_tcp
    for i in range(len(c)):
        got = oracle.tcp_calc_checksum(bytes(c["seg"][i]), int(c["len"][i]),
                                       int(c["saddr"][i]), int(c["daddr"][i]))
        assert got == c["csum"][i], (i, int(c["len"][i]))


def test_closed_form_fold():
    """a2' of SURVEY §8: ~(S mod 0xFFFF, 0 -> 0xFFFF when S > 0) for ihl >= 5."""
    rng = np.random.default_rng(7)
    for _ in range(20000):
        ihl = int(rng.integers(5, 16))
        hdr = rng.integers(0, 256, size=4 * ihl, dtype=np.uint8)
        if rng.random() < 0.05:
            hdr[:] = 0xFF
        words = hdr.view("<u2").astype(np.int64)
        s = int(words.sum())
        r = s % 0xFFFF
        if r == 0 and s > 0:
            r = 0xFFFF
        assert oracle.ip_fast_csum(hdr.tobytes(), ihl) == (~r) & 0xFFFF


def test_rss_microsoft_kat():
    """util/rss.c:173-189 (VerifyRSSHash): host-order inputs, Microsoft key."""
    src = ["66.9.149.187", "199.92.111.2", "24.19.198.95", "38.27.205.30", "153.39.163.191"]
    dst = ["161.142.100.80", "65.69.140.83", "12.22.207.184", "209.142.163.6",
           "202.188.127.2"]
    sport = [2794, 14230, 12898, 48228, 44251]
    dport = [1766, 4739, 38024, 2217, 1303]
    want = [0x51ccc178, 0xc626b0ea, 0x5c2b394a, 0xafc7327f, 0x10e828a2]
    cache = oracle.key_cache(oracle.KEY_MICROSOFT)
    for s, d, sp, dp, w in zip(src, dst, sport, dport, want):
        sip = struct.unpack("!I", socket.inet_aton(s))[0]
        dip = struct.unpack("!I", socket.inet_aton(d))[0]
        assert oracle.rss_hash(cache, sip, dip, sp, dp) == w


def test_rss_vectors_0x05(golden):
    r = golden.rss
    cache = oracle.key_cache(oracle.KEY_0X05)
    for i in range(len(r)):
        args = (int(r["sip"][i]), int(r["dip"][i]), int(r["sp"][i]), int(r["dp"][i]))
        assert oracle.rss_hash(cache, *args) == r["hash"][i]
        for nq in (1, 2, 3, 4, 7, 8, 16):
            assert oracle.rss_cpu_core(cache, *args, nq, 1) == r["util_core"][i][nq - 1]
            assert oracle.rss_cpu_core(cache, *args, nq, 0) == r["mtcp_core0"][i][nq - 1]
            assert oracle.rss_cpu_core(cache, *args, nq, 1) == r["mtcp_core1"][i][nq - 1]


def test_rx_chunk_matches_reference(golden):
    rss = oracle.rss_cfg(oracle.KEY_0X05, golden.rss_num_queues, 1)
    got = oracle.rx_chunk(golden.buf, golden.desc, 0, rss)
    bad = compare_results(got, golden)
    assert not bad, bad
    # TRUNCATED exactly where the reference would read past len
    assert np.array_equal(got["verdict"] == V_TRUNCATED, golden.meta["ref_ub"] == 1)
    # every branch of the chain is covered by the fixtures
    branches = set(golden.meta["branch"][golden.meta["ref_ub"] == 0].tolist())
    assert branches == set(range(10))


def _ub_probe(golden, name):
    """oracle/ref/ub_probe.c's per-frame byte: bit 0 the reference faulted
    with a PROT_NONE page right after the frame, bit 1 that fault was the
    masked odd trailing byte of TCPCalcChecksum (tcp_util.c:175-176), bit 2
    the reference read past len otherwise (ref-UB by observation)."""
    import os
    from tests.golden_io import GOLDEN
    p = np.fromfile(os.path.join(GOLDEN, name), dtype=np.uint8)
    assert len(p) == len(golden.desc)
    return p


def _segment_odd_at_len(golden, i):
    o, n = int(golden.desc["offset"][i]), int(golden.desc["len"][i])
    f = golden.buf[o:o + n].astype(np.int64)
    ihl, tot = f[14] & 0xF, f[16] << 8 | f[17]
    return 14 + tot == n and tot >= 4 * ihl and (tot - 4 * ihl) % 2 == 1


def test_ref_ub_is_what_the_reference_reads_past_len(golden):
    """The ref-UB set (golden_gen's, i.e. the oracle's TRUNCATED verdict) is
    exactly the set of frames for which the REFERENCE's own code reads past
    the frame: the reference's rx chain (compiled from /root/reference at -O0,
    so that every load the source writes runs in the source's order) run on
    each golden frame placed against a PROT_NONE guard page, under a SIGSEGV
    handler (oracle/ref/ub_probe.c; regenerated by `make -C oracle golden`).
    Reads: ip_fast_csum's 4*ihl bytes, one dword for ihl <= 4
    (io_engine/include/ps.h:66-95), the header fields of eth_in.c:13,
    ip_in.c:19-21 and tcp_in.c:1141-1149, TCPCalcChecksum's len bytes
    (tcp_util.c:168-176).  The one read past len that is not UB — the masked
    high byte of an odd segment's last word — is told apart by re-running
    with one readable byte of four values after the frame."""
    p = _ub_probe(golden, "rx_ub_probe.bin")
    assert np.array_equal((p & 4) != 0, golden.meta["ref_ub"] == 1)
    masked = np.nonzero(p & 2)[0]
    assert len(masked) > 100                         # odd TCP segments ending at len
    assert all(_segment_odd_at_len(golden, i) for i in masked)
    assert set(golden.meta["branch"][masked].tolist()) <= {0, 9}
    # the ICMP frames flagged 2 (icmp.c:31-33 reads an uninitialised byte of
    # a local, not past the frame) do not fault
    assert not (p[golden.meta["ref_ub"] == 2] & 4).any()


def test_ref_ub_at_mtcp_build_flags(golden):
    """The same probe through the reference built as mTCP builds it (-O3):
    the reads past len are the -O0 set minus five TCP_LEN_BAD frames whose
    20-byte TCP header passes the frame's end, where gcc sinks the tcph->seq
    / ack_seq / window loads of the declarations (tcp_in.c:1147-1149) past
    the length check (tcp_in.c:1155-1156) that makes them dead; and gcc's
    byte load for the odd trailing word reads nothing past len."""
    p0 = _ub_probe(golden, "rx_ub_probe.bin")
    p3 = _ub_probe(golden, "rx_ub_probe_o3.bin")
    ub0, ub3 = (p0 & 4) != 0, (p3 & 4) != 0
    assert not (ub3 & ~ub0).any()
    only0 = np.nonzero(ub0 & ~ub3)[0]
    assert len(only0) == 5 and (golden.meta["branch"][only0] == 8).all()
    for i in only0:
        o, n = int(golden.desc["offset"][i]), int(golden.desc["len"][i])
        ihl = int(golden.buf[o + 14]) & 0xF
        assert 14 + 4 * ihl + 13 <= n < 14 + 4 * ihl + 16     # doff inside, window past
    assert not (p3 & 2).any()


def test_ub_probe_tells_a_write_past_len_from_a_read(tmp_path):
    """A TCP frame whose header ends before the check field's end (doff 4,
    tot_len covering 16 TCP bytes, frame ending there) and whose checksum
    fails: every read of the reference is inside the frame and its branch is
    TCP_CSUM_BAD, then `tcph->check = 0` (tcp_in.c:1171) stores two bytes past
    it.  The probe reports that store (bit 3), not ref-UB, and the oracle's
    verdict is TCP_CSUM_BAD (found by tools/oracle_soak.py)."""
    import os
    import subprocess
    import oracle
    from mtcp_amd import DESC_DTYPE
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exes = [os.path.join(root, "oracle", "_ref", e) for e in ("ub_probe_O0", "ub_probe")]
    if not all(os.path.exists(e) for e in exes):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    f = np.zeros(64, np.uint8)
    f[12:14] = (0x08, 0x00)
    f[14], f[16], f[17], f[22], f[23] = 0x45, 0, 36, 64, 6
    f[26:34] = (10, 0, 0, 1, 10, 0, 0, 2)
    f[24:26] = 0
    c = oracle.ip_fast_csum(f[14:34].tobytes(), 5)
    f[24], f[25] = c & 0xFF, c >> 8
    f[34 + 12] = 0x40                                   # doff 4
    desc = np.zeros(1, dtype=DESC_DTYPE)
    desc["len"] = 50                                    # 14 + tot_len
    assert oracle.rx_chunk(f, desc, 0)["verdict"][0] == 9        # TCP_CSUM_BAD
    f.tofile(tmp_path / "rx_buf.bin")
    desc.tofile(tmp_path / "rx_desc.bin")
    np.zeros(4, np.uint8).tofile(tmp_path / "rx_meta.bin")       # not ref-UB
    for exe in exes:
        r = subprocess.run([exe, str(tmp_path), str(tmp_path / "ub.bin")], check=True,
                           capture_output=True, text=True, timeout=60)
        assert '"write_past_len": 1' in r.stdout and '"agree_with_meta": 1' in r.stdout, r.stdout
        assert np.fromfile(tmp_path / "ub.bin", np.uint8)[0] == 1 | 8


def test_ub_probe_reproduces(golden, tmp_path):
    """Where the reference build is present, re-run the probe: it writes the
    committed bytes."""
    import os
    import subprocess
    from tests.golden_io import GOLDEN
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for exe, name in (("ub_probe_O0", "rx_ub_probe.bin"), ("ub_probe", "rx_ub_probe_o3.bin")):
        path = os.path.join(root, "oracle", "_ref", exe)
        if not os.path.exists(path):
            pytest.skip("oracle/_ref not built (needs /root/reference)")
        out = tmp_path / name
        subprocess.run([path, GOLDEN, str(out)], check=True, capture_output=True, timeout=300)
        assert out.read_bytes() == open(os.path.join(GOLDEN, name), "rb").read()


def test_rx_verdicts_match_reference_return_values(golden):
    """ProcessPacket's return (ERROR -1 / FALSE 0 / TRUE 1) against the verdict."""
    ok = golden.meta["ref_ub"] == 0
    ret = golden.meta["ret"].astype(np.int32) - 1
    v = golden.expect["verdict"]
    err = np.isin(v, [3, 4, 8, 9])
    assert np.all(ret[ok & err] == -1)
    assert np.all(ret[ok & np.isin(v, [5, 7])] == 0)
    assert np.all(ret[ok & np.isin(v, [1, 2, 6])] == 1)
    # the reference zeroes tcph->check on a bad TCP checksum (tcp_in.c:1171)
    assert golden.meta["check_zeroed"][ok & (v == 9)].sum() >= (ok & (v == 9)).sum() - 1


def test_tx_fill_matches_reference(golden):
    buf = golden.buf.copy()
    n = oracle.tx_fill(buf, golden.desc, 0)
    assert n == golden.manifest["tx_filled"]
    tx = golden.tx
    for i in np.nonzero(tx["filled"])[0]:
        off = int(golden.desc["offset"][i])
        t = int(tx["T"][i])
        assert buf[off + 24:off + 26].view("<u2")[0] == tx["ip_check"][i]
        assert buf[off + t + 16:off + t + 18].view("<u2")[0] == tx["tcp_check"][i]


def _phase_even(i):            # every even start inside a 128 B line, odd ones rare
    return (2 * i) % 128


def test_rx_and_tx_at_every_even_start_match_reference(golden):
    """The golden frames moved to every even start inside a 128 B line (2-byte
    aligned starts: NET_IP_ALIGN-style buffers): the oracle's records equal
    the reference's, and its tx fills write the reference's check values."""
    from tests.repack import repack
    buf, desc = repack(golden.buf, golden.desc, 0, _phase_even)
    assert set((desc["offset"] % 4).tolist()) == {0, 2}
    rss = oracle.rss_cfg(oracle.KEY_0X05, golden.rss_num_queues, 1)
    got = oracle.rx_chunk(buf, desc, 0, rss)
    bad = compare_results(got, golden)
    assert not bad, bad
    n = oracle.tx_fill(buf, desc, 0)
    assert n == golden.manifest["tx_filled"]
    tx = golden.tx
    for i in np.nonzero(tx["filled"])[0]:
        off, t = int(desc["offset"][i]), int(tx["T"][i])
        assert buf[off + 24:off + 26].view("<u2")[0] == tx["ip_check"][i]
        assert buf[off + t + 16:off + t + 18].view("<u2")[0] == tx["tcp_check"][i]
    # an odd start is refused (BAD_DESC), as the ABI says
    d = desc[:4].copy()
    d["offset"] += 1
    assert (oracle.rx_chunk(buf, d, 0)["verdict"] == 11).all()


def test_pktgen_samples_match_fixture(golden):
    """The oracle's generator reproduces the sample bytes stored in the fixture."""
    for s in golden.manifest["samples"]:
        first, count = s["first"], s["count"]
        d = golden.desc[first:first + count].copy()
        base = int(d["offset"][0])
        end = int(d["offset"][-1]) + ((int(d["len"][-1]) + 63) & ~63)
        d["offset"] -= base
        buf = np.zeros(end - base, np.uint8)
        oracle.pktgen(buf, d, 0, s["seed"], 0)
        assert np.array_equal(buf, golden.buf[base:end]), s["name"]


def test_pktgen_corruption_rates():
    from mtcp_amd import pktgen
    n = 1 << 16
    desc, size = pktgen.layout(n, 1500, off_shift=6)
    buf = np.zeros(size, np.uint8)
    oracle.pktgen(buf, desc, 6, 2, 0)
    res = oracle.rx_chunk(buf, desc, 6)
    counts = np.bincount(res["verdict"], minlength=12)
    assert counts[0] > n * 0.99
    assert 20 < counts[9] < 120            # ~1/1024 TCP bit flips
    assert 3 < counts[4] < 40              # ~1/4096 IP header bit flips


# ---- HashFlow (mtcp/src/tcp_stream.c:56-90) --------------------
def test_hash_flow_cases(golden):
    c = golden.flow_cases
    got = np.array([oracle.hash_flow(bytes(k)) for k in c["key"]], dtype=np.uint32)
    assert np.array_equal(got, c["hash"])
    assert got.max() < 131072            # NUM_BINS_FLOWS mask (fhash.h:7)


def test_flow_bins_of_golden_rx(golden):
    # the reference's own StreamHTSearch key (tcp_in.c:1180-1186), hashed by
    # the reference's HashFlow, for every golden packet that got that far
    got = oracle.flow_bins(golden.expect)
    ok = golden.meta["ref_ub"] == 0
    assert np.array_equal(got[ok], golden.flow_bins[ok])
    assert (golden.flow_bins != 0xFFFFFFFF).sum() > 1000


# ---- CreateAddressPoolPerCore (mtcp/src/addr_pool.c:103-180) ----
def test_addr_pool_search_cases(golden):
    n = 0
    for c, saddr, sport in pool_case_entries(golden):
        got = oracle.addr_pool_search(None, int(c["core"]), int(c["nq"]), int(c["saddr_base"]),
                                      int(c["num_addr"]), int(c["daddr"]), int(c["dport"]),
                                      int(c["endian"]))
        assert pool_entries_equal(got, saddr, sport), dict(zip(c.dtype.names, c.tolist()))
        n += 1
    assert n == len(golden.pool_cases) >= 8


# ---- ICMPChecksum (mtcp/src/icmp.c:18-42) ---------------------
def test_icmp_checksum_cases(golden):
    e, m = golden.expect, golden.meta
    icmp = (e["verdict"] == 6) & (m["ref_ub"] == 0)
    got = oracle.rx_chunk(golden.buf, golden.desc, 0)
    assert np.array_equal(got["tcp_csum"][icmp], e["tcp_csum"][icmp])
    assert np.array_equal(got["payload_len"][icmp], e["payload_len"][icmp])
    # echo requests with the reference's checksum (0), corrupted copies,
    # negative lengths (~0) and odd lengths (reference UB, flagged 2)
    assert ((e["tcp_csum"] == 0) & icmp & (e["payload_len"] > 0)).sum() >= 20
    assert ((e["tcp_csum"] != 0) & icmp).sum() >= 20
    assert ((e["tcp_csum"] == 0xFFFF) & icmp).sum() >= 4
    assert ((m["ref_ub"] == 2) & (e["verdict"] == 6)).sum() >= 10
