/*
 * gpd_defrag.h — C-ABI of the IPv4 fragment hand-off ("IPv4 fragment
 * flagging -> ip4defrag").
 *
 * The reference's consumer of IPv4 fragments is ip4defrag: for every decoded IPv4 layer the
 * application calls IPv4Defragmenter.DefragIPv4(WithTimestamp)(&ip4, t)
 * (ip4defrag/defrag.go:76-135), which
 *   1. returns the layer untouched when it needs no reassembly (dontDefrag, :162-172: DF set,
 *      or neither MoreFragments nor a fragment offset);
 *   2. rejects it with an error when securityChecks (:175-198) fail;
 *   3. otherwise files it under the key ipv4{ip.NetworkFlow(), ip.Id} (:331-342) and inserts
 *      it into that key's fragment list (stateful, BSD-right, :216-273).
 * gpd_ip4_fragments runs steps 1 and 2 and builds step 3's key for a whole decoded batch in
 * HBM, and hands over — in packet order, the order the calls would be made in — exactly the
 * packets for which step 1 does not return early, each with its key, the fields insert() and
 * build() read (FragOffset, Flags, Length, IHL, the payload's place) and step 2's verdict.
 * The stateful list insert and reassembly stay with the caller's defragmenter (out of scope,
 * DESIGN.md §9): it is called for the handed-over packets only, and every other packet skips
 * the defragmenter, as DefragIPv4 would have returned it unchanged.
 *
 * "ip" is the DecodingLayerParser's IPv4 object after the call: the last IPv4 layer in the
 * packet's decoded list (for VXLAN, the inner one).  A fragmented IPv4 layer ends the decode
 * (ip4.go:281-286: its next layer is gopacket.Fragment), so it is also the packet's last
 * network layer, the one the header offsets word (gpd.h) locates.
 *
 * Reference interfaces the entry point replaces (paths relative to google/gopacket):
 *   gpd_ip4_fragments   the per-packet DefragIPv4 pre-steps: dontDefrag + securityChecks +
 *                       newIPv4 key (ip4defrag/defrag.go:86-103,162-198,331-342), for a batch
 */
#ifndef GPD_DEFRAG_H_
#define GPD_DEFRAG_H_
#include "gpd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* verdict of one handed-over packet */
#define GPD_FRAG_INSERT     0u  /* a fragment for fragmentList.insert (defrag.go:115) */
#define GPD_FRAG_TOO_SMALL  1u  /* securityChecks: Length - IHL*4 < 8 (defrag.go:179-182,
                                   "fragment too small (handcrafted? %d < %d)") */
#define GPD_FRAG_OFFSET     2u  /* securityChecks: FragOffset > 8183 (defrag.go:185-188,
                                   "fragment offset too big (handcrafted? %d > %d)") */
#define GPD_FRAG_OVERRUN    3u  /* securityChecks: fragOffset + Length > 65535 (defrag.go:192-195).
                                   Never produced: the reference adds two uint16 values, so the
                                   sum wraps and the comparison cannot hold; kept for the text. */
#define GPD_FRAG_WHOLE      4u  /* dontDefrag after all: only for a packet whose IPv4 header
                                   starts past byte 65534 (the header offsets word saturates
                                   there, so the batch pass cannot rule it out early) */

/* One handed-over packet (32 B).  Multi-byte fields are host order except src/dst (raw). */
typedef struct gpd_ip4_frag {
  uint32_t packet;       /* index of the packet in the batch */
  uint32_t net_off;      /* offset of ip.Contents (the IPv4 header) in the packet */
  uint8_t  src[4];       /* ip.SrcIP  } the reassembly key ipv4{NetworkFlow(), Id}      */
  uint8_t  dst[4];       /* ip.DstIP  } (defrag.go:331-342)                            */
  uint16_t id;           /* ip.Id                                                      */
  uint16_t frag_offset;  /* ip.FragOffset (units of 8 bytes) */
  uint16_t length;       /* ip.Length as DecodeFromBytes leaves it (0 on the wire => len(data),
                            ip4.go:214-218) */
  uint8_t  flags;        /* ip.Flags (bit 0 MoreFragments, bit 1 DontFragment, bit 2 EvilBit) */
  uint8_t  ihl;          /* ip.IHL */
  uint32_t payload_len;  /* len(ip.Payload); it starts at net_off + 4 * ihl */
  uint8_t  verdict;      /* GPD_FRAG_* */
  uint8_t  reserved[3];
} gpd_ip4_frag;

/* The hand-off for a decoded device batch: `in` is the batch gpd_decode read and `res` its
 * results on the device (status + layers, or records; hdr_off required).  Writes the first
 * min(count, max_out) handed-over packets to out[] (device memory) in packet order and the
 * count to *count (host); synchronises `stream`.  The context must be the one (same tables,
 * decoders, options, first layer) that decoded the batch.  in->n < 2^32. */
int gpd_ip4_fragments(gpd_ctx *ctx, const gpd_batch *in, const gpd_result *res, gpd_ip4_frag *out,
                      uint64_t max_out, uint64_t *count, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GPD_DEFRAG_H_ */
