/* Test double: the io_module_func table (mtcp/src/include/io_module.h:56-68)
 * and the dev_ioctl commands (:80-87); see mtcp.h in this directory. */
#ifndef TEST_DOUBLE_IO_MODULE_H
#define TEST_DOUBLE_IO_MODULE_H
#include <stdint.h>

#define MAX_DEVICES 16
struct mtcp_thread_context;
typedef struct io_module_func {
    void      (*load_module)(void);
    void      (*init_handle)(struct mtcp_thread_context *ctx);
    int32_t   (*link_devices)(struct mtcp_thread_context *ctx);
    void      (*release_pkt)(struct mtcp_thread_context *ctx, int ifidx, unsigned char *pkt_data, int len);
    uint8_t * (*get_wptr)(struct mtcp_thread_context *ctx, int ifidx, uint16_t len);
    int32_t   (*send_pkts)(struct mtcp_thread_context *ctx, int nif);
    uint8_t * (*get_rptr)(struct mtcp_thread_context *ctx, int ifidx, int index, uint16_t *len);
    int32_t   (*recv_pkts)(struct mtcp_thread_context *ctx, int ifidx);
    int32_t   (*select)(struct mtcp_thread_context *ctx);
    void      (*destroy_handle)(struct mtcp_thread_context *ctx);
    int32_t   (*dev_ioctl)(struct mtcp_thread_context *ctx, int nif, int cmd, void *argp);
} io_module_func;

#define PKT_TX_IP_CSUM          0x01
#define PKT_TX_TCP_CSUM         0x02
#define PKT_RX_TCP_LROSEG       0x03
#define PKT_TX_TCPIP_CSUM       0x04
#define PKT_RX_IP_CSUM          0x05
#define PKT_RX_TCP_CSUM         0x06
#define PKT_TX_TCPIP_CSUM_PEEK  0x07
#define DRV_NAME                0x08
#endif
