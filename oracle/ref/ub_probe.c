/*
 * ub_probe.c — TEST INFRASTRUCTURE ONLY (runs in this container).
 *
 * Which golden frames make the REFERENCE read past the frame?  golden_gen
 * marks a frame "ref-UB" (rx_meta.bin byte 0 == 1) from the oracle's
 * TRUNCATED verdict; this program decides the same question from the
 * reference's own compiled code (ref_glue.c: the real ProcessPacket ->
 * ProcessIPv4Packet -> ProcessTCPPacket -> TCPCalcChecksum chain of
 * /root/reference, -DDISABLE_HWCSUM), by observation:
 *
 *   strict   the frame's last byte abuts a PROT_NONE page (mmap + mprotect),
 *            so any read at or past p + len faults; the reference runs under a
 *            SIGSEGV handler that siglongjmps back (the fault offset is kept).
 *   slack    for a frame that faulted: the same frame with ONE more readable
 *            byte after it, run four times, that byte 0x00, 0xFF, 0x5A, 0xA5.
 *            A "masked tail" — the one read past len whose value the
 *            reference discards — is TCPCalcChecksum's odd trailing word
 *            (`sum += *w & ntohs(0xFF00)`, mtcp/src/tcp_util.c:175-176: a
 *            2-byte load whose high byte lies past an odd-length segment that
 *            ends at len; gcc -O3 turns it into a byte load, -O0 keeps it):
 *            the strict fault is at p + len, the segment is odd and ends at
 *            len, the branch reached the TCP checksum, no slack run faults and
 *            all give the same result (branch, return value, TCP checksum,
 *            ip_fast_csum, stream key).  Its result is defined.  Any other
 *            read past len counts, even when this frame's outcome happens not
 *            to depend on the byte (e.g. tot_len's low byte compared with 20).
 *
 *   write    the first access past len is a store, not a load: the
 *            `tcph->check = 0` of a TCP_CSUM_BAD frame whose TCP header is
 *            shorter than 18 bytes at the frame's end (doff < 5 and tot_len
 *            covering only 4*doff bytes: mtcp/src/tcp_in.c:1171).  Every read
 *            was inside the frame and the branch is decided: re-run with 64
 *            readable bytes after it, the branch must be TCP_CSUM_BAD.  The
 *            reference corrupts two bytes after the frame there (the GPU path
 *            writes nothing); its result is defined.
 *
 * ref-UB by observation = strict fault, not a masked tail, not a write.  The reads
 * that define it are ip_fast_csum's 4*ihl bytes (io_engine/include/ps.h:
 * 66-95), the header fields ProcessPacket / ProcessIPv4Packet /
 * ProcessTCPPacket load (eth_in.c:13, ip_in.c:19-20, tcp_in.c:1141-1152),
 * and TCPCalcChecksum's len bytes (tcp_util.c:168-176).
 *
 * usage: ub_probe GOLDEN_DIR OUT_FILE
 * OUT_FILE: one byte per golden frame — bit 0 strict fault, bit 1 masked
 * tail, bit 2 ref-UB by observation, bit 3 write past len; bits 4-7 zero.  Prints a JSON summary.
 * tests/test_oracle_golden.py::test_ref_ub_is_what_the_reference_reads_past_len
 * asserts bit 2 == (rx_meta ref_ub == 1) for every frame.
 */
#define _GNU_SOURCE
#include <setjmp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <ucontext.h>
#include <unistd.h>

#include "ref_glue.h"

#define DATA_PAGES 32                      /* 128 KiB: frames are <= 16 000 B */

static sigjmp_buf g_env;
static volatile uintptr_t g_fault_addr;
static volatile int g_fault_write;          /* the faulting access was a store */

static void on_fault(int sig, siginfo_t *si, void *uc)
{
    (void)sig;
    g_fault_addr = (uintptr_t)si->si_addr;
#ifdef REG_ERR
    /* x86-64 page-fault error code: bit 1 set for a write access */
    g_fault_write = (((ucontext_t *)uc)->uc_mcontext.gregs[REG_ERR] & 2) != 0;
#else
    g_fault_write = 0;
#endif
    siglongjmp(g_env, 1);
}

/* what golden_gen records from the reference for a frame: the branch, the
 * return value, the TCP checksum it computed, ip_fast_csum over the header
 * (golden_gen.c takes it for every IPv4 frame past the ip_len < 20 test) and
 * the stream key StreamHTSearch received */
typedef struct {
    int faulted, fault_write, br, ret;
    uint16_t csum, ip_csum;
    uint8_t key[12];
    long fault_off;
} run_t;

static int same_result(const run_t *a, const run_t *b)
{
    return a->br == b->br && a->ret == b->ret && a->csum == b->csum &&
           a->ip_csum == b->ip_csum && memcmp(a->key, b->key, 12) == 0;
}

/* Run the reference on a copy of frame (len bytes) placed so that `slack`
 * readable bytes (value v) follow it, then the guard page. */
static run_t run_ref(uint8_t *guard, const uint8_t *frame0, uint32_t len, uint32_t slack, uint8_t v)
{
    run_t r;
    uint8_t *p = guard - slack - len;
    const uint8_t *frame = p;
    volatile int faulted = 0;

    memset(&r, 0, sizeof(r));
    memcpy(p, frame0, len);
    memset(p + len, v, slack);
    g_fault_addr = 0;
    if (sigsetjmp(g_env, 1) == 0) {
        int ret = 0;
        uint16_t cs = 0;
        r.br = ref_rx_packet(p, (int)len, &ret, &cs);
        r.ret = ret;
        r.csum = cs;
        if (r.br == REF_BR_TCP_OK)
            ref_last_flow_key(r.key);
        if (r.br != REF_BR_ETH_OTHER && r.br != REF_BR_ARP && r.br != REF_BR_IP_SHORT)
            r.ip_csum = ref_ip_fast_csum(frame + 14, frame[14] & 0xF);
    } else {
        faulted = 1;
    }
    r.faulted = faulted;
    r.fault_write = faulted && g_fault_write;
    r.fault_off = faulted ? (long)((intptr_t)g_fault_addr - (intptr_t)p) : -1;
    return r;
}

/* the TCP segment [14 + 4*ihl, 14 + tot_len) has odd length and ends at len:
 * TCPCalcChecksum's last load is the 2-byte word at len - 1 */
static int odd_segment_ends_at(const uint8_t *f, uint32_t len)
{
    uint32_t ihl, tot;
    if (len < 18)
        return 0;
    ihl = f[14] & 0xF;
    tot = (uint32_t)f[16] << 8 | f[17];
    return 14 + tot == len && tot >= 4 * ihl && ((tot - 4 * ihl) & 1);
}

static void *slurp(const char *dir, const char *name, size_t *size)
{
    char path[4096];
    FILE *f;
    void *buf;
    long n;
    snprintf(path, sizeof(path), "%s/%s", dir, name);
    f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    fseek(f, 0, SEEK_END);
    n = ftell(f);
    fseek(f, 0, SEEK_SET);
    buf = malloc((size_t)n + 1);
    if (fread(buf, 1, (size_t)n, f) != (size_t)n) { perror(path); exit(1); }
    fclose(f);
    *size = (size_t)n;
    return buf;
}

int main(int argc, char **argv)
{
    size_t nb, nd, nm;
    const long pg = sysconf(_SC_PAGESIZE);
    uint8_t *buf, *map, *guard, *out;
    const ref_desc_t *desc;
    const uint8_t *meta;
    uint32_t n, i, strict = 0, masked = 0, ub = 0, agree = 0, fault_at_len = 0, writes = 0;
    struct sigaction sa;
    FILE *f;

    if (argc < 3) {
        fprintf(stderr, "usage: ub_probe GOLDEN_DIR OUT_FILE\n");
        return 1;
    }
    buf = slurp(argv[1], "rx_buf.bin", &nb);
    desc = slurp(argv[1], "rx_desc.bin", &nd);
    meta = slurp(argv[1], "rx_meta.bin", &nm);
    n = (uint32_t)(nd / sizeof(ref_desc_t));
    if (nm != 4ull * n) { fprintf(stderr, "ub_probe: rx_meta.bin size\n"); return 1; }
    out = calloc(n, 1);

    map = mmap(NULL, (size_t)(DATA_PAGES + 1) * pg, PROT_READ | PROT_WRITE,
               MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (map == MAP_FAILED) { perror("mmap"); return 1; }
    guard = map + (size_t)DATA_PAGES * pg;
    if (mprotect(guard, (size_t)pg, PROT_NONE) != 0) { perror("mprotect"); return 1; }

    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = on_fault;
    sa.sa_flags = SA_SIGINFO | SA_NODEFER;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, NULL);
    sigaction(SIGBUS, &sa, NULL);

    for (i = 0; i < n; i++) {
        const uint8_t *frame = buf + desc[i].offset;
        uint32_t len = desc[i].len;
        run_t s;
        int is_masked = 0, is_write = 0, is_ub;
        if (desc[i].offset + (size_t)len > nb || len + 64 > (uint32_t)(DATA_PAGES * pg)) {
            fprintf(stderr, "ub_probe: frame %u out of range\n", i);
            return 1;
        }
        s = run_ref(guard, frame, len, 0, 0);
        if (s.faulted && s.fault_write) {
            run_t w = run_ref(guard, frame, len, 64, 0);
            is_write = !w.faulted && w.br == REF_BR_TCP_CSUM_BAD;
            strict++;
            fault_at_len += s.fault_off == (long)len;
        } else if (s.faulted) {
            static const uint8_t fills[4] = {0x00, 0xFF, 0x5A, 0xA5};
            run_t a = run_ref(guard, frame, len, 1, fills[0]);
            int k;
            is_masked = !a.faulted && s.fault_off == (long)len && odd_segment_ends_at(frame, len) &&
                        (a.br == REF_BR_TCP_OK || a.br == REF_BR_TCP_CSUM_BAD);
            for (k = 1; k < 4 && is_masked; k++) {
                run_t b = run_ref(guard, frame, len, 1, fills[k]);
                is_masked = !b.faulted && same_result(&a, &b);
            }
            strict++;
            fault_at_len += s.fault_off == (long)len;
        }
        is_ub = s.faulted && !is_masked && !is_write;
        masked += is_masked;
        writes += is_write;
        ub += is_ub;
        agree += is_ub == (meta[4 * i] == 1);
        out[i] = (uint8_t)(s.faulted | is_masked << 1 | is_ub << 2 | is_write << 3);
    }
    f = fopen(argv[2], "wb");
    if (!f || fwrite(out, 1, n, f) != n) { perror(argv[2]); return 1; }
    fclose(f);
    printf("{\"frames\": %u, \"strict_faults\": %u, \"fault_at_len\": %u, \"masked_tail\": %u, "
           "\"write_past_len\": %u, \"ref_ub_observed\": %u, \"agree_with_meta\": %u}\n",
           n, strict, fault_at_len, masked, writes, ub, agree);
    return 0;
}
