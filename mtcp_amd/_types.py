"""numpy views of the C ABI records (include/mtcp_gpu.h)."""
import numpy as np

# struct mtcp_gpu_desc: layout-compatible with PSIO's ps_pkt_info (ps.h:181-185)
DESC_DTYPE = np.dtype([("offset", "<u4"), ("len", "<u2"), ("flags", "u1"), ("rsvd", "u1")])

# struct mtcp_gpu_result (40 B)
RESULT_DTYPE = np.dtype([
    ("saddr", "<u4"), ("daddr", "<u4"), ("sport", "<u2"), ("dport", "<u2"),
    ("seq", "<u4"), ("ack_seq", "<u4"), ("window", "<u2"), ("ip_len", "<u2"),
    ("ip_csum", "<u2"), ("tcp_csum", "<u2"), ("rss_hash", "<u4"),
    ("payload_len", "<u2"), ("ihl_doff", "u1"), ("tcp_flags", "u1"),
    ("verdict", "u1"), ("rss_queue", "u1"), ("eth_type", "<u2"),
])
assert DESC_DTYPE.itemsize == 8 and RESULT_DTYPE.itemsize == 40

# struct mtcp_gpu_result16 (16 B, MTCP_GPU_F_COMPACT): the same fields as the
# 40 B record's, for callers that act on the verdict
RESULT16_DTYPE = np.dtype([
    ("rss_hash", "<u4"), ("ip_csum", "<u2"), ("tcp_csum", "<u2"), ("payload_len", "<u2"),
    ("ip_len", "<u2"), ("ihl_doff", "u1"), ("tcp_flags", "u1"), ("verdict", "u1"),
    ("rss_queue", "u1"),
])
assert RESULT16_DTYPE.itemsize == 16


def compact_of(res: np.ndarray) -> np.ndarray:
    """The 16 B records a compact context writes, from 40 B records."""
    out = np.zeros(len(res), dtype=RESULT16_DTYPE)
    for f in RESULT16_DTYPE.names:
        out[f] = res[f]
    return out

VERDICTS = ("TCP_OK", "ETH_OTHER", "ARP", "IP_SHORT", "IP_CSUM_BAD", "IP_VERSION", "ICMP",
            "IP_PROTO_OTHER", "TCP_LEN_BAD", "TCP_CSUM_BAD", "TRUNCATED", "BAD_DESC")
RX_ERROR_VERDICTS = (3, 4, 8, 9)   # ProcessPacket ret < 0 (eth_in.c:49-53)

# struct mtcp_gpu_addr_entry: sockaddr_in address and port, network order
ADDR_ENTRY_DTYPE = np.dtype([("saddr", "<u4"), ("sport", "<u2"), ("rsvd", "<u2")])
assert ADDR_ENTRY_DTYPE.itemsize == 8

NUM_BINS_FLOWS = 131072      # mtcp/src/include/fhash.h:7
FLOW_NONE = 0xFFFFFFFF
MIN_PORT, MAX_PORT = 1025, 65536   # mtcp/src/include/addr_pool.h:7-8
