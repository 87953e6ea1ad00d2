/*
 * topo_test.c — TEST HARNESS for mtcp_amd/io_module/gpu_topo.h (the device
 * choice of gpu_module.c) on a faked sysfs tree.
 *
 *   topo_test SYSFS NCPU BDF...
 * For every cpu 0..NCPU-1 prints "cpu node rank device" (one line each),
 * with the devices' NUMA nodes read from SYSFS/bus/pci/devices/BDF/numa_node
 * exactly as gpu_module.c's gpu_pick_device reads them.
 */
#include <stdio.h>
#include <stdlib.h>

#include "../../mtcp_amd/io_module/gpu_topo.h"

int main(int argc, char **argv)
{
    int ndev, ncpu, d, cpu, dev_node[GPU_TOPO_MAX_DEVS];
    if (argc < 4) {
        fprintf(stderr, "usage: topo_test SYSFS NCPU BDF...\n");
        return 1;
    }
    ncpu = atoi(argv[2]);
    ndev = argc - 3;
    if (ndev > GPU_TOPO_MAX_DEVS) ndev = GPU_TOPO_MAX_DEVS;
    for (d = 0; d < ndev; d++)
        dev_node[d] = gpu_topo_pci_node(argv[1], argv[3 + d]);
    for (cpu = 0; cpu < ncpu; cpu++) {
        int rank = 0, node = gpu_topo_cpu_node(argv[1], cpu, &rank);
        printf("%d %d %d %d\n", cpu, node, rank, gpu_topo_pick(cpu, node, rank, ndev, dev_node));
    }
    return 0;
}
