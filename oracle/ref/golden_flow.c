/*
 * golden_flow.c — TEST INFRASTRUCTURE ONLY (oracle/_ref build, this
 * container).  Golden vectors for SURVEY §8 f3/f4 from the REFERENCE's own
 * code, compiled from /root/reference by oracle/Makefile:
 *
 *   HashFlow                  mtcp/src/tcp_stream.c:56-90 (tcp_stream.o,
 *                             linked with --gc-sections: only HashFlow's
 *                             section is kept)
 *   CreateAddressPoolPerCore  mtcp/src/addr_pool.c:103-180 and FetchAddress
 *                             :216-270 (addr_pool.o) over GetRSSCPUCore
 *                             (mtcp/src/rss.c:90-103)
 *
 * Writes into <dir>:
 *   rx_flowbins.bin   u32 per golden rx packet: HashFlow of the stream key
 *                     the reference handed to StreamHTSearch (captured by
 *                     golden_gen into rx_flowkey.bin), 0xFFFFFFFF if the
 *                     packet never got there
 *   flow_cases.bin    16 B records: 12 key bytes (tcp_stream saddr..dport in
 *                     memory order) + HashFlow
 *   pool_cases.bin    per case 8 x i32: core, num_queues, saddr_base (net),
 *                     num_addr, daddr (net), dport (net), endian, count
 *   pool_entries.bin  u32 per entry, all cases back to back:
 *                     (address index << 16) | source port (host order)
 */
#include <arpa/inet.h>
#include <netinet/in.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mtcp.h"
#include "tcp_stream.h"
#include "addr_pool.h"

struct mtcp_config CONFIG;           /* addr_pool.c reads max_concurrency */

/* io_module.c:400-415 FetchEndianType: 1 without DPDK; the cases below set it */
static int g_endian = 1;
int FetchEndianType(void) { return g_endian; }

int ref_mtcp_rss_core(uint32_t sip, uint32_t dip, uint16_t sp, uint16_t dp, int nq,
                      uint8_t endian_check);
int GetRSSCPUCore(in_addr_t sip, in_addr_t dip, in_port_t sp, in_port_t dp, int num_queues,
                  uint8_t endian_check)
{
    return ref_mtcp_rss_core(sip, dip, sp, dp, num_queues, endian_check);
}

static uint64_t g_state = 0x5EED0F10u;
static uint64_t next64(void)
{
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void *read_file(const char *dir, const char *name, size_t *size)
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

static void write_file(const char *dir, const char *name, const void *data, size_t size)
{
    char path[4096];
    FILE *f;
    snprintf(path, sizeof(path), "%s/%s", dir, name);
    f = fopen(path, "wb");
    if (!f || fwrite(data, 1, size, f) != size) { perror(path); exit(1); }
    fclose(f);
}

static uint32_t ref_hash_key(const uint8_t key[12])
{
    tcp_stream s;
    memset(&s, 0, sizeof(s));
    memcpy(&s.saddr, key, 4);
    memcpy(&s.daddr, key + 4, 4);
    memcpy(&s.sport, key + 8, 2);
    memcpy(&s.dport, key + 10, 2);
    return HashFlow(&s);
}

int main(int argc, char **argv)
{
    const char *dir = argc > 1 ? argv[1] : ".";
    size_t nk, nexp, i;
    uint8_t *keys = read_file(dir, "rx_flowkey.bin", &nk);
    uint8_t *exp = read_file(dir, "rx_expect.bin", &nexp);   /* mtcp_gpu_result, 40 B */
    size_t n = nk / 12;
    uint32_t *bins;

    if (nexp != n * 40) { fprintf(stderr, "rx_flowkey / rx_expect size mismatch\n"); return 1; }
    bins = (uint32_t *)malloc(n * 4);
    for (i = 0; i < n; i++)
        bins[i] = exp[40 * i + 36] == 0 ? ref_hash_key(keys + 12 * i) : 0xFFFFFFFFu;
    write_file(dir, "rx_flowbins.bin", bins, n * 4);

    /* random keys plus the sign-extension corners of tcp_stream.c:80 */
    {
        const int nr = 4096;
        uint8_t *rec = (uint8_t *)calloc(nr, 16);
        int r, b;
        for (r = 0; r < nr; r++) {
            uint8_t *k = rec + 16 * r;
            uint32_t h;
            uint64_t a = next64(), c = next64();
            if (r == 0) memset(k, 0x00, 12);
            else if (r == 1) memset(k, 0xFF, 12);
            else if (r == 2) memset(k, 0x80, 12);
            else if (r == 3) memset(k, 0x7F, 12);
            else if (r < 64) for (b = 0; b < 12; b++) k[b] = (uint8_t)(b == (r - 4) % 12 ? 0x80 : 0);
            else { memcpy(k, &a, 8); memcpy(k + 8, &c, 4); }
            h = ref_hash_key(k);
            memcpy(k + 12, &h, 4);
        }
        write_file(dir, "flow_cases.bin", rec, (size_t)nr * 16);
    }

    /* CreateAddressPoolPerCore, drained in order with FetchAddress */
    {
        static const int cases[][7] = {
            /* core nq num_addr endian  saddr_base_h  daddr_h     dport */
            {0, 4, 1, 1, 0x0A000100, 0x0A000001, 80},
            {3, 4, 1, 1, 0x0A000100, 0x0A000001, 80},
            {1, 8, 1, 0, 0xC0A80A0A, 0xC0A80001, 8080},
            {5, 8, 2, 1, 0xC0A80A0A, 0xC0A80001, 8080},
            {2, 3, 1, 1, 0x0A0A0A00, 0x0A0B0C0D, 443},
            {15, 16, 1, 1, 0xAC100000, 0xAC10FFFE, 5001},
            {0, 16, 3, 0, 0x0AFFFFFE, 0x01020304, 1},
            {6, 7, 1, 1, 0x7F000001, 0x7F000001, 65535},
        };
        const int nc = (int)(sizeof(cases) / sizeof(cases[0]));
        int32_t *meta = (int32_t *)calloc((size_t)nc, 8 * sizeof(int32_t));
        size_t cap = 1u << 20, used = 0;
        uint32_t *ent = (uint32_t *)malloc(cap * 4);
        int c;
        for (c = 0; c < nc; c++) {
            const int core = cases[c][0], nq = cases[c][1], num_addr = cases[c][2];
            const uint32_t base_h = (uint32_t)cases[c][4], daddr_h = (uint32_t)cases[c][5];
            const uint16_t dport_h = (uint16_t)cases[c][6];
            struct sockaddr_in dst, src;
            addr_pool_t ap;
            int32_t count = 0;
            g_endian = cases[c][3];
            CONFIG.max_concurrency = 0;
            ap = CreateAddressPoolPerCore(core, nq, htonl(base_h), num_addr, htonl(daddr_h),
                                          htons(dport_h));
            if (!ap) { fprintf(stderr, "CreateAddressPoolPerCore failed\n"); return 1; }
            memset(&dst, 0, sizeof(dst));
            dst.sin_addr.s_addr = htonl(daddr_h);
            dst.sin_port = htons(dport_h);
            for (;;) {
                memset(&src, 0, sizeof(src));        /* INADDR_ANY, INPORT_ANY */
                if (FetchAddress(ap, core, nq, &dst, &src) != 0)
                    break;
                if (used == cap) { cap *= 2; ent = (uint32_t *)realloc(ent, cap * 4); }
                ent[used++] = ((ntohl(src.sin_addr.s_addr) - base_h) << 16) | ntohs(src.sin_port);
                count++;
            }
            DestroyAddressPool(ap);
            meta[8 * c + 0] = core;
            meta[8 * c + 1] = nq;
            meta[8 * c + 2] = (int32_t)htonl(base_h);
            meta[8 * c + 3] = num_addr;
            meta[8 * c + 4] = (int32_t)htonl(daddr_h);
            meta[8 * c + 5] = (int32_t)htons(dport_h);
            meta[8 * c + 6] = cases[c][3];
            meta[8 * c + 7] = count;
        }
        write_file(dir, "pool_cases.bin", meta, (size_t)nc * 8 * sizeof(int32_t));
        write_file(dir, "pool_entries.bin", ent, used * 4);
        printf("golden_flow: %zu rx bins, 4096 flow cases, %d pool cases, %zu entries\n", n, nc,
               used);
    }
    return 0;
}
