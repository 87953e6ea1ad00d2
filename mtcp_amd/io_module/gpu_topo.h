/*
 * gpu_topo.h — which MI355X an mTCP thread's GPU context opens (part of
 * gpu_module.c, SURVEY §8 e/f2; header-only so that tests/c/topo_test.c can
 * run the same code on a faked sysfs tree).
 *
 * mTCP keeps a thread's memory on its core's NUMA node: mtcp_core_affinitize
 * binds it there (mtcp/src/cpu.c:54-79), and the DPDK backend puts each
 * port's rx queues on the NIC's socket (rte_eth_dev_socket_id(portid),
 * mtcp/src/dpdk_module.c:660-663).  The GPU a thread stages its frames to is
 * chosen the same way: a device on the thread's node, so the staging copy
 * and the H2D / D2H stay on that socket's PCIe root (measured on one GPU:
 * threads on the other socket ran 24-29 instead of 31 Mpkt/s,
 * profiles/r2/io_thread_sweep.jsonl).  Among the node's devices the node's
 * cpus are dealt round-robin (the k-th cpu of the node -> its k mod m-th
 * device), so the threads of one node spread over all of its GPUs' links.
 * A node with no device, or a topology sysfs does not show, falls back to
 * cpu mod ndev (the round-2 rule).
 *
 * Inputs: <sysfs>/devices/system/node/node<N>/cpulist (cpus of node N, the
 * kernel's "0-63,128-191" list format) and
 * <sysfs>/bus/pci/devices/<bdf>/numa_node (a device's node, -1 unknown);
 * <sysfs> is /sys, or MTCP_GPU_SYSFS in the environment (tests).
 */
#ifndef GPU_TOPO_H
#define GPU_TOPO_H

#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define GPU_TOPO_MAX_NODES 64
#define GPU_TOPO_MAX_DEVS  64

/* Is cpu in the kernel cpulist string s ("0-3,8,10-11")?  *rank receives the
 * number of listed cpus below it. */
static inline int gpu_topo_cpulist_has(const char *s, int cpu, int *rank)
{
    int below = 0, found = 0;
    while (*s) {
        char *end;
        long lo, hi;
        while (*s == ',' || isspace((unsigned char)*s))
            s++;
        if (!*s)
            break;
        lo = strtol(s, &end, 10);
        if (end == s)
            break;
        hi = lo;
        s = end;
        if (*s == '-') {
            hi = strtol(s + 1, &end, 10);
            if (end == s + 1)
                break;
            s = end;
        }
        if (cpu >= lo && cpu <= hi) {
            found = 1;
            below += (int)(cpu - lo);
        } else if (hi < cpu) {
            below += (int)(hi - lo + 1);
        }
    }
    if (rank)
        *rank = below;
    return found;
}

static inline const char *gpu_topo_sysfs(void)
{
    const char *e = getenv("MTCP_GPU_SYSFS");
    return e && *e ? e : "/sys";
}

/* NUMA node of cpu (and its rank among the node's cpus), or -1. */
static inline int gpu_topo_cpu_node(const char *sysfs, int cpu, int *rank)
{
    char path[512], buf[4096];
    int node;
    for (node = 0; node < GPU_TOPO_MAX_NODES; node++) {
        FILE *f;
        size_t n;
        snprintf(path, sizeof(path), "%s/devices/system/node/node%d/cpulist", sysfs, node);
        f = fopen(path, "r");
        if (!f)
            continue;
        n = fread(buf, 1, sizeof(buf) - 1, f);
        fclose(f);
        buf[n] = 0;
        if (gpu_topo_cpulist_has(buf, cpu, rank))
            return node;
    }
    return -1;
}

/* NUMA node of the PCI device bdf ("0000:05:00.0"), or -1. */
static inline int gpu_topo_pci_node(const char *sysfs, const char *bdf)
{
    char path[512];
    int node = -1;
    FILE *f;
    size_t i;
    char low[64];
    /* sysfs names are lower case; hipDeviceGetPCIBusId may print upper case */
    for (i = 0; bdf[i] && i + 1 < sizeof(low); i++)
        low[i] = (char)tolower((unsigned char)bdf[i]);
    low[i] = 0;
    snprintf(path, sizeof(path), "%s/bus/pci/devices/%s/numa_node", sysfs, low);
    f = fopen(path, "r");
    if (!f)
        return -1;
    if (fscanf(f, "%d", &node) != 1)
        node = -1;
    fclose(f);
    return node;
}

/*
 * The device for the mTCP thread on `cpu`, given each device's NUMA node
 * (dev_node[d], -1 unknown): the (rank mod m)-th of the m devices on the
 * cpu's node, in device order; cpu mod ndev when the cpu's node is unknown
 * or holds no device.
 */
static inline int gpu_topo_pick(int cpu, int cpu_node, int cpu_rank, int ndev, const int *dev_node)
{
    int d, m = 0, k;
    if (ndev <= 0)
        return -1;
    if (cpu_node >= 0)
        for (d = 0; d < ndev; d++)
            m += dev_node[d] == cpu_node;
    if (m == 0)
        return (cpu < 0 ? 0 : cpu) % ndev;
    k = cpu_rank % m;
    for (d = 0; d < ndev; d++)
        if (dev_node[d] == cpu_node && k-- == 0)
            return d;
    return (cpu < 0 ? 0 : cpu) % ndev;        /* not reached */
}

#endif /* GPU_TOPO_H */
