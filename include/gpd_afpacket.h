/*
 * gpd_afpacket.h — C-ABI of the AF_PACKET TPACKET_V3 ring ingest in front of the batched
 * decoder.
 *
 * The reference reads a TPACKET_V3 ring one packet at a time: ZeroCopyReadPacketData takes
 * the block at the ring offset, waits until the kernel hands it to user space
 * (TP_STATUS_USER), returns each packet of the block in turn through the v3wrapper's next(),
 * and hands the block back (block_status = 0) when it moves on (afpacket/afpacket.go:
 * 300-330 ZeroCopyReadPacketData, 431-455 getTPacketHeader, 457-483 pollForFirstPacket,
 * 282-287 releaseCurrentPacket; afpacket/header.go:137-195 v3wrapper).  Here every block the
 * kernel has already handed over is walked in one call: the walk fills offset / caplen
 * arrays that point INTO the ring memory, so the ring's own bytes are the batch buffer —
 * copied to HBM block by block (or read in place once the ring is registered with
 * gpd_host_register) and decoded without repacking.
 *
 * Reference interfaces each entry point replaces (paths relative to google/gopacket):
 *   gpd_tpv3_walk     the loop `for { data, ci, err := tp.ZeroCopyReadPacketData() ... }` over
 *                     the blocks currently owned by user space: block selection
 *                     (afpacket.go:445-453), the TP_STATUS_USER check (:459), the empty-block
 *                     retry (:313-316), v3wrapper getData/getLength/getTime/getIfaceIndex/
 *                     getVLAN/next (header.go:151-195), CaptureInfo (afpacket.go:318-326)
 *   gpd_tpv3_release  releaseCurrentPacket -> v3wrapper.clearStatus (afpacket.go:282-287,
 *                     header.go:162-164) for the walked blocks
 *   gpd_decode_tpv3   that loop feeding DecodingLayerParser.DecodeLayers: H2D of the walked
 *                     blocks + the walk on the device (gpd_tuning.device_walk, the default;
 *                     or on the host) + gpd_decode + D2H of results and capture info;
 *                     OptAddVLANHeader's tag insertion (header.go:74-82, 168-173) for the
 *                     packets it applies to (the host path)
 *
 * Ring layout (linux/if_packet.h; TPACKET_V3): block k starts at ring + k * block_size with a
 * struct tpacket_block_desc; its tpacket_hdr_v1 gives block_status, num_pkts and
 * offset_to_first_pkt; each packet is a struct tpacket3_hdr whose tp_mac / tp_snaplen locate
 * the frame, followed (TPACKET_ALIGN'ed) by a struct sockaddr_ll.
 */
#ifndef GPD_AFPACKET_H_
#define GPD_AFPACKET_H_
#include "gpd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A mapped TPACKET_V3 ring (afpacket options.go: blockSize, numBlocks). */
typedef struct gpd_tpv3_ring {
  uint8_t *base;        /* the mmap'ed ring */
  uint32_t block_size;  /* tp_block_size */
  uint32_t num_blocks;  /* tp_block_nr */
} gpd_tpv3_ring;

/* Per-packet capture info of a walk (CaptureInfo, afpacket.go:318-326). */
typedef struct gpd_tpv3_pkts {
  uint64_t *offset;     /* frame start relative to ring->base (packet + tp_mac) */
  uint32_t *caplen;     /* tp_snaplen (CaptureLength before any VLAN tag insertion) */
  uint32_t *wire_len;   /* tp_len (CaptureInfo.Length) */
  uint64_t *ts_ns;      /* tp_sec * 1e9 + tp_nsec (CaptureInfo.Timestamp) */
  int32_t  *ifindex;    /* sockaddr_ll.sll_ifindex (CaptureInfo.InterfaceIndex) */
  int32_t  *vlan;       /* AncillaryVLAN: tp_vlan_tci & 0xfff if TP_STATUS_VLAN_VALID, else -1 */
  uint32_t *vlan_tci;   /* hv1.tp_vlan_tci as stored (OptAddVLANHeader inserts it when != 0) */
} gpd_tpv3_pkts;        /* any pointer but offset/caplen may be NULL */

/* Walk the user-owned blocks starting at ring block `first_block`, in ring order (wrapping),
 * until a block the kernel still owns, `max_blocks` blocks, or a block whose packets would
 * pass max_n.  Fills up to max_n entries of *pk; *n_out = packets, *blocks_out = blocks
 * walked (whole blocks only; the caller releases them with gpd_tpv3_release).
 * nthreads <= 0: the cores, at most 16 (blocks are independent once their status is read). */
int gpd_tpv3_walk(const gpd_tpv3_ring *ring, uint32_t first_block, uint32_t max_blocks,
                  uint64_t max_n, const gpd_tpv3_pkts *pk, uint64_t *n_out, uint32_t *blocks_out,
                  int nthreads);
/* Hand `count` blocks from first_block on back to the kernel (block_status = 0). */
int gpd_tpv3_release(const gpd_tpv3_ring *ring, uint32_t first_block, uint32_t count);
/* Walk + decode: the walked blocks' bytes go host -> device in ring order, every packet is
 * decoded where it lies (OptAddVLANHeader packets from a tagged copy), results land in the
 * host arrays of `out` (n_out entries, in walk order).  Does not release the blocks.
 * `pk` (optional, host) receives the walk's capture info. */
int gpd_decode_tpv3(gpd_ctx *ctx, const gpd_tpv3_ring *ring, uint32_t first_block,
                    uint32_t max_blocks, int add_vlan_header, uint64_t max_n,
                    const gpd_result *out, const gpd_tpv3_pkts *pk, uint64_t *n_out,
                    uint32_t *blocks_out, int nthreads);
/* Which walk the calling thread's last successful gpd_decode_tpv3 used: 1 the device walk
 * (gpd_tuning.device_walk; the blocks walked in HBM), 0 the host walk (diagnostic). */
int gpd_decode_tpv3_last_path(void);

#ifdef __cplusplus
}
#endif
#endif /* GPD_AFPACKET_H_ */
