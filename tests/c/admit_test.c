/*
 * admit_test.c — TEST HARNESS: CPU unit test of gpu_module.c's admission and
 * limit parsing (the module's static functions, so the source is included).
 *
 *   admit_test  -> one JSON line of results; tests/test_io_module.py checks it
 *
 * Admission: at most GPU_THREADS_DEFAULT (2) mTCP threads per GPU offload
 * (none where 4 or more mTCP threads share a GPU) unless MTCP_GPU_THREADS
 * says otherwise ("all": every thread); a thread's
 * slot is given back when its context fails to open or is destroyed.
 * MTCP_GPU_WAIT_TIMEOUT_MS: default 2000 ms, <= 0 no limit, clamped to the
 * 32-bit microsecond range.
 */
#include "../../mtcp_amd/io_module/gpu_module.c"
#include "../../oracle/mtcp_oracle.h"

uint16_t ip_fast_csum(const void *iph, unsigned int ihl) { return oracle_ip_fast_csum(iph, ihl); }
uint16_t TCPCalcChecksum(uint16_t *buf, uint16_t len, uint32_t saddr, uint32_t daddr)
{
    return oracle_tcp_calc_checksum(buf, len, saddr, daddr);
}
struct mtcp_config CONFIG = {1};
io_module_func netmap_module_func;

/* admit `k` threads on device `dev`; returns how many were admitted */
static int per_gpu_now = 0;   /* mTCP threads per GPU the admissions below see */

static int admit_n(int dev, int k, struct gpu_private_context *gs)
{
    int i, got = 0;
    for (i = 0; i < k; i++) {
        gs[i].slot_dev = -1;
        if (gpu_thread_admit(dev, per_gpu_now)) {
            gs[i].slot_dev = dev;
            got++;
        }
    }
    return got;
}

static void release_all(struct gpu_private_context *gs, int k)
{
    int i;
    for (i = 0; i < k; i++)
        gpu_thread_release(&gs[i]);
}

int main(void)
{
    struct gpu_private_context gs[16];
    int def16, def_other_dev, after_release, all16, zero, three;
    unsigned long long w_default, w_zero, w_neg, w_big, w_5000;
    int q_default_2, q_4, q_5, q_env8_5, q_env8_9;
    int crowd_16_on_1, crowd_16_on_8, crowd_3_on_1, crowd_4_on_1, crowd_16_on_1_k1, crowd_24_on_8;
    int per_gpu_16_8, per_gpu_17_8;

    unsetenv("MTCP_GPU_THREADS");
    def16 = admit_n(0, 16, gs);              /* default: 2 of 16 on device 0 */
    def_other_dev = admit_n(1, 4, gs + 8);   /* another device has its own 2 (overwrites gs[8..11]) */
    release_all(gs + 8, 4);
    /* the two holders on device 0 are gs[0], gs[1]: one leaves, one joins */
    gpu_thread_release(&gs[0]);
    after_release = admit_n(0, 3, gs + 12);
    release_all(gs, 16);

    setenv("MTCP_GPU_THREADS", "all", 1);
    all16 = admit_n(0, 16, gs);
    release_all(gs, 16);
    setenv("MTCP_GPU_THREADS", "0", 1);
    zero = admit_n(0, 16, gs);
    release_all(gs, 16);
    setenv("MTCP_GPU_THREADS", "3", 1);
    three = admit_n(0, 16, gs);
    release_all(gs, 16);

    /* crowded GPUs: from 4 mTCP threads per GPU (num_cores over the GPUs)
     * the default admits none; MTCP_GPU_THREADS still decides when set */
    unsetenv("MTCP_GPU_THREADS");
    CONFIG.num_cores = 16;
    per_gpu_now = gpu_threads_per_gpu(1);
    crowd_16_on_1 = admit_n(0, 16, gs);
    release_all(gs, 16);
    per_gpu_now = per_gpu_16_8 = gpu_threads_per_gpu(8);
    crowd_16_on_8 = admit_n(0, 2, gs);        /* the two threads dealt to one of 8 GPUs */
    release_all(gs, 2);
    CONFIG.num_cores = 24;
    per_gpu_now = gpu_threads_per_gpu(8);
    crowd_24_on_8 = admit_n(0, 3, gs);        /* three threads per GPU still offload two */
    release_all(gs, 3);
    CONFIG.num_cores = 17;
    per_gpu_17_8 = gpu_threads_per_gpu(8);
    CONFIG.num_cores = 3;
    per_gpu_now = gpu_threads_per_gpu(1);
    crowd_3_on_1 = admit_n(0, 3, gs);
    release_all(gs, 3);
    CONFIG.num_cores = 4;
    per_gpu_now = gpu_threads_per_gpu(1);
    crowd_4_on_1 = admit_n(0, 4, gs);
    release_all(gs, 4);
    setenv("MTCP_GPU_THREADS", "1", 1);
    CONFIG.num_cores = 16;
    per_gpu_now = gpu_threads_per_gpu(1);
    crowd_16_on_1_k1 = admit_n(0, 16, gs);
    release_all(gs, 16);
    unsetenv("MTCP_GPU_THREADS");
    CONFIG.num_cores = 0;
    per_gpu_now = 0;

    /* hardware queues: one stream per offloading thread against GPU_MAX_HW_QUEUES */
    unsetenv("GPU_MAX_HW_QUEUES");
    q_default_2 = gpu_queues_shared(2);
    q_4 = gpu_queues_shared(4);
    q_5 = gpu_queues_shared(5);
    setenv("GPU_MAX_HW_QUEUES", "8", 1);
    q_env8_5 = gpu_queues_shared(5);
    q_env8_9 = gpu_queues_shared(9);
    unsetenv("GPU_MAX_HW_QUEUES");

    unsetenv("MTCP_GPU_WAIT_TIMEOUT_MS");
    w_default = gpu_wait_us();
    setenv("MTCP_GPU_WAIT_TIMEOUT_MS", "0", 1);
    w_zero = gpu_wait_us();
    setenv("MTCP_GPU_WAIT_TIMEOUT_MS", "-7", 1);
    w_neg = gpu_wait_us();
    setenv("MTCP_GPU_WAIT_TIMEOUT_MS", "5000000", 1);    /* wrapped to ~705 s before */
    w_big = gpu_wait_us();
    setenv("MTCP_GPU_WAIT_TIMEOUT_MS", "5000", 1);
    w_5000 = gpu_wait_us();

    printf("{\"default_of_16\": %d, \"default_other_device_of_4\": %d, \"after_release_of_3\": %d, "
           "\"all_of_16\": %d, \"zero_of_16\": %d, \"three_of_16\": %d, \"count_left\": %d, "
           "\"wait_default\": %llu, \"wait_zero\": %llu, \"wait_negative\": %llu, "
           "\"wait_5000000ms\": %llu, \"wait_5000ms\": %llu, "
           "\"queues_shared\": [%d, %d, %d, %d, %d], "
           "\"crowded\": {\"16_on_1\": %d, \"16_on_8\": %d, \"3_on_1\": %d, \"4_on_1\": %d, "
           "\"16_on_1_k1\": %d, \"24_on_8\": %d, \"per_gpu_16_8\": %d, \"per_gpu_17_8\": %d}}\n",
           def16, def_other_dev, after_release, all16, zero, three, gpu_thread_count[0],
           w_default, w_zero, w_neg, w_big, w_5000, q_default_2, q_4, q_5, q_env8_5, q_env8_9,
           crowd_16_on_1, crowd_16_on_8, crowd_3_on_1, crowd_4_on_1, crowd_16_on_1_k1, crowd_24_on_8,
           per_gpu_16_8, per_gpu_17_8);
    return 0;
}
