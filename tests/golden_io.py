"""Loader for tests/golden/ (written by oracle/ref/golden_gen.c from the
reference's own code; regenerate with `make -C oracle golden`)."""
import json
import os

import numpy as np

from oracle import DESC_DTYPE, RESULT_DTYPE

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

RSS_DTYPE = np.dtype([("sip", "<u4"), ("dip", "<u4"), ("sp", "<u2"), ("dp", "<u2"),
                      ("hash", "<u4"), ("util_core", "u1", 16), ("mtcp_core0", "u1", 16),
                      ("mtcp_core1", "u1", 16)])
CSUM_IP_DTYPE = np.dtype([("hdr", "u1", 60), ("ihl", "u1"), ("pad", "u1"), ("csum", "<u2")])
CSUM_TCP_DTYPE = np.dtype([("len", "<u4"), ("saddr", "<u4"), ("daddr", "<u4"),
                           ("csum", "<u2"), ("pad", "<u2"), ("seg", "u1", 2048)])
TX_DTYPE = np.dtype([("filled", "u1"), ("pad", "u1"), ("ip_check", "<u2"),
                     ("tcp_check", "<u2"), ("T", "<u2")])
FLOW_CASE_DTYPE = np.dtype([("key", "u1", 12), ("hash", "<u4")])
POOL_CASE_DTYPE = np.dtype([("core", "<i4"), ("nq", "<i4"), ("saddr_base", "<u4"),
                            ("num_addr", "<i4"), ("daddr", "<u4"), ("dport", "<i4"),
                            ("endian", "<i4"), ("count", "<i4")])
META_DTYPE = np.dtype([("ref_ub", "u1"), ("branch", "u1"), ("ret", "u1"),
                       ("check_zeroed", "u1")])


class Golden:
    pass


def load_golden() -> Golden:
    g = Golden()
    g.manifest = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    rd = lambda name, dt: np.fromfile(os.path.join(GOLDEN, name), dtype=dt)
    g.buf = rd("rx_buf.bin", np.uint8)
    # chunk buffers are padded to a multiple of 64 B (PSIO layout)
    pad = (-g.buf.nbytes) % 64
    if pad:
        g.buf = np.concatenate([g.buf, np.zeros(pad, np.uint8)])
    g.desc = rd("rx_desc.bin", DESC_DTYPE)
    g.expect = rd("rx_expect.bin", RESULT_DTYPE)
    g.meta = rd("rx_meta.bin", META_DTYPE)
    g.tx = rd("tx_expect.bin", TX_DTYPE)
    g.rss = rd("rss_cases.bin", RSS_DTYPE)
    g.csum_ip = rd("csum_ip.bin", CSUM_IP_DTYPE)
    g.csum_tcp = rd("csum_tcp.bin", CSUM_TCP_DTYPE)
    g.rss_num_queues = g.manifest["rss_num_queues"]
    # SURVEY 8 f3/f4 (oracle/ref/golden_flow.c)
    g.flow_bins = rd("rx_flowbins.bin", np.uint32)
    g.flow_cases = rd("flow_cases.bin", FLOW_CASE_DTYPE)
    g.pool_cases = rd("pool_cases.bin", POOL_CASE_DTYPE)
    g.pool_entries = rd("pool_entries.bin", np.uint32)
    return g


def pool_case_entries(golden: Golden):
    """Yield (case, entries) with entries as ADDR_ENTRY-like (saddr net, sport net)
    arrays decoded from pool_entries.bin ((addr index << 16) | port, host order)."""
    off = 0
    for c in golden.pool_cases:
        cnt = int(c["count"])
        e = golden.pool_entries[off:off + cnt].astype(np.uint64)
        off += cnt
        base_h = int.from_bytes(int(c["saddr_base"]).to_bytes(4, "little"), "big")
        saddr_h = (base_h + (e >> np.uint64(16))).astype(np.uint32)
        port_h = (e & np.uint64(0xFFFF)).astype(np.uint16)
        yield c, saddr_h.byteswap(), port_h.byteswap()


def pool_entries_equal(got: np.ndarray, saddr_net: np.ndarray, sport_net: np.ndarray) -> bool:
    return (len(got) == len(saddr_net) and np.array_equal(got["saddr"], saddr_net)
            and np.array_equal(got["sport"], sport_net))


def compare_results(got: np.ndarray, golden: Golden, mask=None):
    """Field-by-field comparison against the reference's results, skipping the
    ref-UB frames (the reference reads past len there).  Returns a list of
    mismatch descriptions."""
    ok = golden.meta["ref_ub"] == 0
    if mask is not None:
        ok &= mask
    bad = []
    for f in RESULT_DTYPE.names:
        diff = np.nonzero((got[f] != golden.expect[f]) & ok)[0]
        if len(diff):
            i = diff[0]
            bad.append(f"{f}: {len(diff)} mismatches, first #{i}: got {got[f][i]} "
                       f"want {golden.expect[f][i]} (verdict want {golden.expect['verdict'][i]})")
    return bad
