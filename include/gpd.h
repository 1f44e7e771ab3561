/*
 * gpd.h — C-ABI of the MI355X batched packet-decode engine (gopacket_amd).
 *
 * This is the drop-in boundary for gopacket's DecodingLayerParser / Flow hot
 * path.  It is batch-only: one call decodes N packets that sit in one byte
 * buffer, described by an offset array and a caplen array.  Plain pointers and
 * sizes only; no torch types.  A cgo binding over exactly these symbols is
 * shown in INTEGRATION.md.
 *
 * Reference interfaces each entry point replaces (paths relative to
 * google/gopacket):
 *   gpd_ctx_create        NewDecodingLayerParser(first, decoders...)  parser.go:222-233
 *                         + DecodingLayerParserOptions                parser.go:336-350
 *                         + snapshot of the global dispatch tables     layers/enums.go:304-345,
 *                           layers/ports.go:62-74,105-122
 *   gpd_ctx_reload_tables RegisterTCPPortLayerType / RegisterUDPPortLayerType
 *                           layers/ports.go:78-80,126-128 and writes to
 *                           EthernetTypeMetadata / IPProtocolMetadata (layers/enums.go:288)
 *   gpd_ctx_set_options   assigning parser.IgnoreUnsupported / IgnorePanic  parser.go:182-195,
 *                           336-350 (plain fields: the parser, its decoders and the tables stay)
 *   gpd_ctx_add_decoders  (*DecodingLayerParser).AddDecodingLayer       parser.go:197-202
 *   gpd_ctx_set_decoders  (*DecodingLayerParser).SetDecodingLayerContainer parser.go:236-242
 *   gpd_decode            (*DecodingLayerParser).DecodeLayers        parser.go:302-316
 *                         (loop: layers_decoder.go:60-79), fused with
 *                         TCP.ComputeChecksum                          layers/tcp.go:193-195,
 *                                                                      layers/tcpip.go:26-88
 *                         IPv4 header checksum `checksum`              layers/ip4.go:158-179
 *                         NetworkFlow().FastHash()/TransportFlow().FastHash()
 *                                                                      flows.go:60-83,167-174
 *   gpd_decode_host       the same, from host memory (pinned H2D -> kernel -> D2H pipeline);
 *                         the caller's ReadPacketData loop feeding DecodeLayers
 *                         (examples/statsassembly/main.go:171-177)
 *
 * Every per-packet output is bit-exact with the reference decoder on the
 * same bytes; see DESIGN.md §Semantics for the definition of each output.
 *
 * Threading: a context is used by one host thread at a time, as a DecodingLayerParser is
 * (it holds mutable layer state and is not goroutine-safe).  Calls on one context
 * from two threads at once are not supported (its staging slots, per-stream fallback lists
 * and tuning are unlocked); give each thread its own context.  Contexts are independent, and
 * one context may launch on several streams from its one thread.
 */
#ifndef GPD_H_
#define GPD_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPD_ABI_VERSION 10 /* 2: ICMPv4 + LLC, 12 objects, 224-B ext; 3: gpd_result.hdr_off;
                              4: gpd_ctx_set_tuning; 5: gpd_tuning.header_once,
                              gpd_tuning.device_walk, gpd_result.records; 6: outputs follow the
                              objects as a failing call leaves them; ext err_obj/err_wrote/err_off;
                              7: gpd_result.detail (error arguments and deep stacks without ext);
                              8: gpd_ctx_set_options, gpd_ctx_add_decoders, gpd_ctx_set_decoders
                              (in place: device, tables and staging kept); 9: gpd_fast_hash
                              (gpd_flow.h); 10: gpd_tuning.grid_rounds, waves_per_simd enforced */

/* ---- gopacket LayerType numbers (layertypes.go:14-154, decode.go:105-116) ---- */
#define GPD_LT_ZERO            0
#define GPD_LT_DECODE_FAILURE  1
#define GPD_LT_PAYLOAD         2
#define GPD_LT_FRAGMENT        3
#define GPD_LT_ARP             10
#define GPD_LT_DOT1Q           15
#define GPD_LT_ETHERNET        17
#define GPD_LT_ICMPV4          19
#define GPD_LT_IPV4            20
#define GPD_LT_IPV6            21
#define GPD_LT_LLC             22
#define GPD_LT_SNAP            23
#define GPD_LT_TCP             44
#define GPD_LT_UDP             45
#define GPD_LT_IPV6_HOPBYHOP   46
#define GPD_LT_IPV6_ROUTING    47
#define GPD_LT_IPV6_FRAGMENT   48
#define GPD_LT_IPV6_DEST       49
#define GPD_LT_ICMPV6          57
#define GPD_LT_DNS             107
#define GPD_LT_VXLAN           116
#define GPD_LT_STP             121
#define GPD_LT_TLS             140

/* ---- DecodingLayers this engine implements (bit = registered) ----
 * The reference registers DecodingLayer objects with the parser; here the
 * registered set is a bitmask.  Each decoder's CanDecode() set is fixed:      */
#define GPD_DEC_ETHERNET   (1u << 0)  /* {17}            layers/ethernet.go:41-62,106-112 */
#define GPD_DEC_DOT1Q      (1u << 1)  /* {15}            layers/dot1q.go:29-50            */
#define GPD_DEC_IPV4       (1u << 2)  /* {20}            layers/ip4.go:188-286            */
#define GPD_DEC_IPV6       (1u << 3)  /* {21} (+HBH)     layers/ip6.go:221-291,509-526    */
#define GPD_DEC_IPV6_EXT   (1u << 4)  /* {46,47,48,49}   IPv6ExtensionSkipper ip6.go:437-461 */
#define GPD_DEC_TCP        (1u << 5)  /* {44}            layers/tcp.go:229-314            */
#define GPD_DEC_UDP        (1u << 6)  /* {45}            layers/udp.go:30-110             */
#define GPD_DEC_VXLAN      (1u << 7)  /* {116}           layers/vxlan.go:43-78            */
#define GPD_DEC_PAYLOAD    (1u << 8)  /* {2}             gopacket.Payload base.go:55-63   */
#define GPD_DEC_FRAGMENT   (1u << 9)  /* {3}             gopacket.Fragment base.go:108-117 */
#define GPD_DEC_ICMPV4     (1u << 10) /* {19}            layers/icmp4.go:220-231,261-263  */
#define GPD_DEC_LLC        (1u << 11) /* {22}            layers/llc.go:31-52,61-69        */
#define GPD_DEC_ALL        0xFFFu

/* ---- options (DecodingLayerParserOptions, parser.go:336-350, + engine knobs) ---- */
#define GPD_OPT_IGNORE_UNSUPPORTED (1u << 0)  /* parser.IgnoreUnsupported = true */
#define GPD_OPT_IGNORE_PANIC       (1u << 1)  /* accepted; no decoder here can panic */
#define GPD_OPT_NO_CHECKSUMS       (1u << 8)  /* skip IPv4-header and L4 checksums (csum := 0, valid bits 0) */
#define GPD_OPT_NO_FLOW_HASH       (1u << 9)  /* skip FastHash (hashes := 0, valid bits 0) */
/* Every other bit is unknown: gpd_ctx_create and gpd_ctx_set_options return GPD_ERR_INVALID for
 * it (the bench's stream-only ablations live in a separately built diagnostic library). */

/* ---- per-packet status word (uint32) ----
 *  [1:0]   class: GPD_ST_OK (DecodeLayers returned nil), GPD_ST_UNSUPPORTED
 *          (UnsupportedLayerType), GPD_ST_DECODE_ERROR (a layer's DecodeFromBytes error)
 *  [2]     Truncated (parser.Truncated after the call)
 *  [3]     n_layers saturated (> 31 layers decoded)
 *  [8:4]   n_layers = len(decoded), saturating at 31
 *  [14:9]  err_code (GPD_E_*; 0 unless class == DECODE_ERROR)
 *  [15]    reserved (0)
 *  [16]    net_hash valid   (an IPv4/IPv6 layer is in decoded)
 *  [17]    tp_hash valid    (a TCP/UDP layer is in decoded)
 *  [18]    IPv4 header checksum valid (IPv4 in decoded, and len(ip4.Contents) even: after a
 *          failed Length/IHL check Contents is the whole remaining data, ip4.go:210, and an odd
 *          length makes `checksum` index past the end, ip4.go:165-167 — a panic in Go)
 *  [19]    L4 checksum valid (TCP/UDP in decoded, preceded by IPv4/IPv6)
 *  [23:20] EndpointType of NetworkFlow(): of the last IPv4/IPv6 in decoded (1 IPv4, 2 IPv6,
 *          0 none; layers/endpoints.go:20-23), whether or not hashes are computed
 *  [27:24] EndpointType of TransportFlow(): of the last TCP/UDP (4 TCP, 5 UDP, 0 none;
 *          layers/endpoints.go:29-32)
 *  [31:28] reserved (0)
 * The hashes and checksums read each layer object as the call leaves it, which is not always
 * its last successful decode: a later DecodeFromBytes of the same kind that fails may already
 * have assigned addresses / ports / BaseLayer (see gpd_ext_rec.err_wrote).                */
#define GPD_ST_OK            0u
#define GPD_ST_UNSUPPORTED   1u
#define GPD_ST_DECODE_ERROR  2u
#define GPD_STATUS_CLASS(s)      ((s) & 3u)
#define GPD_STATUS_TRUNCATED(s)  (((s) >> 2) & 1u)
#define GPD_STATUS_SATURATED(s)  (((s) >> 3) & 1u)
#define GPD_STATUS_NLAYERS(s)    (((s) >> 4) & 31u)
#define GPD_STATUS_ERRCODE(s)    (((s) >> 9) & 63u)
#define GPD_STATUS_NET_VALID(s)  (((s) >> 16) & 1u)
#define GPD_STATUS_TP_VALID(s)   (((s) >> 17) & 1u)
#define GPD_STATUS_IPCS_VALID(s) (((s) >> 18) & 1u)
#define GPD_STATUS_L4CS_VALID(s) (((s) >> 19) & 1u)
#define GPD_STATUS_NET_EPT(s)    (((s) >> 20) & 15u)
#define GPD_STATUS_TP_EPT(s)     (((s) >> 24) & 15u)

/* ---- per-packet layers word (uint64) ----
 *  [15:0]  stop type: the LayerType DecodingLayerFunc returned (nonzero => no decoder
 *          registered for it; class UNSUPPORTED unless IGNORE_UNSUPPORTED)
 *  [63:16] decoded[0..11] as 4-bit layer codes, decoded[i] at bits 16+4i (0 = none)  */
#define GPD_LAYERS_STOP(w)      ((uint32_t)((w) & 0xFFFFu))
#define GPD_LAYERS_CODE(w, i)   ((uint32_t)(((w) >> (16 + 4 * (i))) & 15u))
#define GPD_CORE_MAX_LAYERS 12
#define GPD_EXT_MAX_LAYERS  32

/* 4-bit layer codes (index into gpd_code_layertype below) */
#define GPD_C_NONE      0
#define GPD_C_ETHERNET  1
#define GPD_C_DOT1Q     2
#define GPD_C_IPV4      3
#define GPD_C_IPV6      4
#define GPD_C_IPV6_HBH  5
#define GPD_C_IPV6_RT   6
#define GPD_C_IPV6_FRAG 7
#define GPD_C_IPV6_DEST 8
#define GPD_C_TCP       9
#define GPD_C_UDP       10
#define GPD_C_VXLAN     11
#define GPD_C_PAYLOAD   12
#define GPD_C_FRAGMENT  13
#define GPD_C_ICMPV4    14
#define GPD_C_LLC       15
/* code -> LayerType: {0,17,15,20,21,46,47,48,49,44,45,116,2,3,19,22} */

/* ---- checksum word (uint32): [15:0] IPv4 header checksum as ip4.go:158 `checksum`
 *      computes it over ip4.Contents (compare with the stored field); [31:16] L4 checksum as
 *      TCP.ComputeChecksum() (tcp.go:193) / the same computeChecksum over UDP contents+payload
 *      (tcpip.go:75-88), stored checksum included: 0 <=> valid.                        */
#define GPD_CSUM_IP4(c) ((uint16_t)((c) & 0xFFFFu))
#define GPD_CSUM_L4(c)  ((uint16_t)((c) >> 16))

/* ---- decode error sites (err_code); each is one `return ...error` in the reference ---- */
enum gpd_err {
  GPD_E_NONE = 0,
  GPD_E_ETH_TOO_SMALL = 1,        /* ethernet.go:42-43  "Ethernet packet too small" */
  GPD_E_DOT1Q_TOO_SHORT = 2,      /* dot1q.go:30-32     "802.1Q tag length %d too short" (a0=len) */
  GPD_E_IP4_TOO_SHORT = 3,        /* ip4.go:189-191     "Invalid ip4 header. Length %d less than 20" */
  GPD_E_IP4_LENGTH_LT20 = 4,      /* ip4.go:220-221     "Invalid (too small) IP length (%d < 20)" (a0=Length) */
  GPD_E_IP4_IHL_LT5 = 5,          /* ip4.go:222-223     "Invalid (too small) IP header length (%d < 5)" (a0=IHL) */
  GPD_E_IP4_IHL_GT_LENGTH = 6,    /* ip4.go:224-225     "Invalid IP header length > IP length (%d > %d)" (a0=IHL,a1=Length) */
  GPD_E_IP4_HDR_TRUNC = 7,        /* ip4.go:231-232     "Not all IP header bytes available" */
  GPD_E_IP4_OPT_LT2 = 8,          /* ip4.go:257-259     "Invalid ip4 option length. Length %d less than 2" */
  GPD_E_IP4_OPT_EXCEEDS = 9,      /* ip4.go:262-264     "IP option length exceeds remaining IP header size, option type %v length %v" */
  GPD_E_IP4_OPT_LE2 = 10,         /* ip4.go:266-267     "Invalid IP option type %v length %d. Must be greater than 2" */
  GPD_E_IP6_TOO_SHORT = 11,       /* ip6.go:222-224     "Invalid ip6 header. Length %d less than 40" */
  GPD_E_IP6EXT_LT2 = 12,          /* ip6.go:419-421     "Invalid ip6-extension header. Length %d less than 2" */
  GPD_E_IP6EXT_LT_SPEC = 13,      /* ip6.go:426-427     "Invalid ip6-extension header. Length %d less than specified length %d" */
  GPD_E_IP6_TLV_LT2 = 14,         /* ip6.go:328-330     "IPv6 header option too small" */
  GPD_E_IP6_TLV_TRUNC = 15,       /* ip6.go:340-342     "IPv6 header TLV option too small" */
  GPD_E_IP6_JUMBO_TLV_LEN = 16,   /* ip6.go:67-68       "Jumbo length TLV data must have length 4" */
  GPD_E_IP6_JUMBO_TOO_SMALL = 17, /* ip6.go:71-72       "Jumbo length cannot be less than 65536" */
  GPD_E_IP6_JUMBO_AND_LEN = 18,   /* ip6.go:257-258     "IPv6 has jumbo length and IPv6 length is not 0" */
  GPD_E_IP6_LEN0_NO_JUMBO = 19,   /* ip6.go:259-260     "IPv6 length 0, but HopByHop header does not have jumbogram option" */
  GPD_E_IP6_LEN0_NOT_HBH = 20,    /* ip6.go:266-267     "IPv6 length 0, but next header is %v, not HopByHop" (a0=NextHeader) */
  GPD_E_TCP_TOO_SHORT = 21,       /* tcp.go:230-232     "Invalid TCP header. Length %d less than 20" */
  GPD_E_TCP_DOFF_LT5 = 22,        /* tcp.go:260-261     "Invalid TCP data offset %d < 5" */
  GPD_E_TCP_DOFF_GT_LEN = 23,     /* tcp.go:264-268     "TCP data offset greater than packet length" */
  GPD_E_TCP_OPT_LT2_REM = 24,     /* tcp.go:286-288     "Invalid TCP option length. Length %d less than 2" */
  GPD_E_TCP_OPT_LEN_LT2 = 25,     /* tcp.go:291-292     "Invalid TCP option length %d < 2" */
  GPD_E_TCP_OPT_EXCEEDS = 26,     /* tcp.go:293-295     "Invalid TCP option length %d exceeds remaining %d bytes" */
  GPD_E_UDP_TOO_SHORT = 27,       /* udp.go:31-33       "Invalid UDP header. Length %d less than 8" */
  GPD_E_UDP_LEN_TOO_SMALL = 28,   /* udp.go:52-53       "UDP packet too small: %d bytes" */
  GPD_E_VXLAN_TOO_SMALL = 29,     /* vxlan.go:54-56     "vxlan packet too small" */
  GPD_E_ICMP4_TOO_SMALL = 30,     /* icmp4.go:221-223   "ICMP layer less then 8 bytes for ICMPv4 packet" (sets Truncated) */
  GPD_E_LLC_TOO_SMALL = 31,       /* llc.go:32-33,42-43 "LLC header too small" */
  GPD_E_COUNT = 32
};

/* ---- layer objects: one per registered DecodingLayer (its state after the call) ---- */
enum gpd_obj {
  GPD_OBJ_ETHERNET = 0, GPD_OBJ_DOT1Q = 1, GPD_OBJ_IPV4 = 2, GPD_OBJ_IPV6 = 3,
  GPD_OBJ_IPV6_EXT = 4, GPD_OBJ_TCP = 5, GPD_OBJ_UDP = 6, GPD_OBJ_VXLAN = 7,
  GPD_OBJ_PAYLOAD = 8, GPD_OBJ_FRAGMENT = 9, GPD_OBJ_ICMPV4 = 10, GPD_OBJ_LLC = 11,
  GPD_NOBJ = 12
};

#define GPD_NOBJ_NONE 0xFFu

/* BaseLayer of one object as the call leaves it (offsets relative to the packet):
 * Contents = pkt[contents_off : contents_off+contents_len],
 * Payload  = pkt[payload_off  : payload_off+payload_len]; a nil Payload is length 0 at the end
 * of Contents.  The parser reuses one object per kind (layers_decoder.go:61-78), so this is the
 * object's last successful DecodeFromBytes in the packet — unless a later call on the same
 * object failed after assigning BaseLayer (err_wrote == 2 below), which then wins. */
typedef struct gpd_layer_rec {
  uint32_t contents_off, contents_len, payload_off, payload_len;
} gpd_layer_rec;

/* Optional extended record (224 B) — everything a Go/C++ shim needs to rebuild the
 * decoded slice, the exact error text and every layer struct by reading header bytes. */
typedef struct gpd_ext_rec {
  uint64_t layer_codes[2];  /* decoded[0..31] as 4-bit codes, decoded[i] at bit 4*(i%16) of word i/16 */
  uint32_t err_arg0;        /* first %d/%v argument of the error text (see enum gpd_err) */
  uint32_t err_arg1;        /* second argument, if any */
  uint16_t obj_valid;       /* bit k: object k decoded successfully at least once (its kind is
                               in decoded); obj[k] is then its BaseLayer as the call leaves it */
  uint8_t  err_obj;         /* decode error: object (enum gpd_obj) whose DecodeFromBytes failed;
                               GPD_NOBJ_NONE otherwise */
  uint8_t  err_wrote;       /* what that failing call assigned before it returned:
                               0 nothing (the length checks come first);
                               1 header fields read from pkt[err_off:] (TCP doff < 5: ports ..
                                 Urgent, tcp.go:234-259; LLC: DSAP .. Control, llc.go:35-39),
                                 BaseLayer unchanged;
                               2 header fields from pkt[err_off:] and BaseLayer, recorded in
                                 obj[err_obj] (IPv4 after len >= 20: Contents = data, Payload nil,
                                 ip4.go:195-210, or the header split for option errors :235-236;
                                 IPv6 after len >= 40, ip6.go:226-235; TCP doff overrun
                                 (Contents = data, tcp.go:264-268) and option errors; UDP
                                 "too small", Contents = data[:8], udp.go:35-41) */
  uint32_t err_off;         /* offset of the data the failing DecodeFromBytes was given */
  gpd_layer_rec obj[GPD_NOBJ];
} gpd_ext_rec;

/* Optional per-packet detail record (24 B; the first 24 bytes of gpd_ext_rec, same meaning):
 * what a caller needs beyond the core words to rebuild DecodeLayers' exact return values —
 * the format arguments of the decode error (parser.go:302-316 returns the layer's error, e.g.
 * ip4.go:220-225, tcp.go:260-295, udp.go:31-53) and the decoded list past the core record's
 * 12 layers.  It is written ONLY for packets whose status has class GPD_ST_DECODE_ERROR or
 * n_layers > GPD_CORE_MAX_LAYERS (saturated included); the entries of every other packet are
 * left unspecified (gpd_decode leaves them untouched).  Those packets are exactly the ones the
 * fast kernel hands to the generic decoder, so asking for detail costs the fast path nothing:
 * it never forces the generic path for the batch, as ext does.                               */
typedef struct gpd_detail {
  uint64_t layer_codes[2];  /* decoded[0..31] as 4-bit codes, decoded[i] at bit 4*(i%16) of word i/16 */
  uint32_t err_arg0;        /* first %d/%v argument of the error text (enum gpd_err), else 0 */
  uint32_t err_arg1;        /* second argument, if any, else 0 */
} gpd_detail;

/* ---- context configuration ---- */
typedef struct gpd_config {
  uint32_t first_layer;      /* LayerType the parser starts with (NewDecodingLayerParser first) */
  uint32_t decoders;         /* GPD_DEC_* mask of registered DecodingLayers */
  uint32_t options;          /* GPD_OPT_* */
  uint32_t reserved;
  /* Dispatch-table snapshot (LayerType values).  NULL => the reference defaults.
   * ethertype[65536]: EthernetTypeMetadata[t].LayerType   (enums.go:304-321)
   * ipproto[256]:     IPProtocolMetadata[p].LayerType      (enums.go:323-345)
   * tcp_port[65536]:  tcpPortLayerType[p] (0 => Payload)  (ports.go:62-74)
   * udp_port[65536]:  udpPortLayerType[p] (0 => Payload)  (ports.go:105-122)      */
  const uint16_t *ethertype;
  const uint16_t *ipproto;
  const uint16_t *tcp_port;
  const uint16_t *udp_port;
} gpd_config;

/* ---- a batch: N packets in one byte buffer ----
 * packet i = data[offset[i] : offset[i] + caplen[i]].
 * The data buffer must be readable up to round_up(data_len, 16) bytes (pad the
 * allocation); bytes past data_len never influence a result.  For gpd_decode all
 * pointers are device pointers on the context's device. */
typedef struct gpd_batch {
  const uint8_t  *data;
  uint64_t        data_len;
  const uint32_t *offset;
  const uint32_t *caplen;
  uint64_t        n;
} gpd_batch;

/* ---- header offsets word (uint32): where the flows' layers sit in the packet ----
 *  [15:0]  offset (from the packet start) of the header whose SrcIP/DstIP NetworkFlow()
 *          reads: the object of the kind of the last IPv4/IPv6 in decoded, as the call leaves
 *          it (a later failing call of that kind may have re-assigned them); 0xFFFF if none
 *  [31:16] the same for the ports TransportFlow() reads (the last TCP/UDP in decoded);
 *          0xFFFF if none
 * Offsets >= 0xFFFF saturate to 0xFFFF.  With these a caller fills the layer structs (or
 * builds the [2]Flow key tcpassembly uses) straight from the packet bytes, zero copy. */
#define GPD_HDR_NET(h) ((uint32_t)((h) & 0xFFFFu))
#define GPD_HDR_TP(h)  ((uint32_t)((h) >> 16))
#define GPD_HDR_NONE   0xFFFFu

/* One packet's five result words packed in 32 bytes (the AoS alternative to the SoA arrays). */
typedef struct gpd_record {
  uint32_t status;
  uint32_t csum;
  uint64_t layers;
  uint64_t net_hash;
  uint64_t tp_hash;
} gpd_record;

/* ---- results (caller-allocated SoA, n entries each) ----
 * status and layers are required; the others may be NULL (not written).
 * records (gpd_decode only): when non-NULL, status, layers, net_hash, tp_hash and csum must be
 * NULL and each packet's five words are written as one 32-byte gpd_record instead (one
 * stream of 2 x 16-byte stores per packet rather than five arrays); ext and hdr_off stay
 * separate arrays.  The host-memory entry points (gpd_decode_host, gpd_decode_pcap*,
 * TPACKET_V3) take the SoA form only.
 * detail (every entry point): see gpd_detail — written for decode errors and > 12-layer stacks
 * only.  ext (gpd_decode, gpd_decode_host) forces the generic decoder for the whole batch. */
typedef struct gpd_result {
  uint32_t    *status;
  uint64_t    *layers;
  uint64_t    *net_hash;   /* ip4/ip6.NetworkFlow().FastHash()   */
  uint64_t    *tp_hash;    /* tcp/udp.TransportFlow().FastHash() */
  uint32_t    *csum;
  gpd_ext_rec *ext;
  uint32_t    *hdr_off;    /* header offsets word (above) */
  gpd_record  *records;    /* AoS form of the first five (see above) */
  gpd_detail  *detail;     /* error arguments / deep stacks (ABI 7) */
} gpd_result;

typedef struct gpd_ctx gpd_ctx;

/* return codes */
#define GPD_OK            0
#define GPD_ERR_INVALID  (-1)
#define GPD_ERR_HIP      (-2)
#define GPD_ERR_NOMEM    (-3)
#define GPD_ERR_NODEVICE (-4)

int  gpd_abi_version(void);
/* Fill the four tables with the reference's defaults (any pointer may be NULL). */
void gpd_default_tables(uint16_t *ethertype, uint16_t *ipproto,
                        uint16_t *tcp_port, uint16_t *udp_port);
int  gpd_ctx_create(int device, const gpd_config *cfg, gpd_ctx **out);
int  gpd_ctx_reload_tables(gpd_ctx *ctx, const gpd_config *cfg);
/* ABI 8.  Change the options of ctx in place, as assigning the reference's IgnoreUnsupported /
 * IgnorePanic fields does (parser.go:182-195,336-350): the context keeps its device, decoder set,
 * dispatch-table snapshot (gpd_ctx_reload_tables), tuning and staging.  Takes effect on the next
 * launch; launches already enqueued keep the options they were enqueued with.  GPD_ERR_INVALID
 * on unknown bits (cfg->options of gpd_ctx_create is checked the same way). */
int  gpd_ctx_set_options(gpd_ctx *ctx, uint32_t options);
/* ABI 8.  AddDecodingLayer (parser.go:197-202): add GPD_DEC_* decoders to ctx's registered set.
 * The dispatch image is rebuilt from the context's current table snapshot (the defaults or the
 * last gpd_ctx_reload_tables), on its device; synchronous. */
int  gpd_ctx_add_decoders(gpd_ctx *ctx, uint32_t decoders);
/* ABI 8.  SetDecodingLayerContainer (parser.go:236-242): the registered set becomes exactly
 * `decoders` (the kinds whose CanDecode types the container holds), replacing the previous set;
 * rebuilt like gpd_ctx_add_decoders. */
int  gpd_ctx_set_decoders(gpd_ctx *ctx, uint32_t decoders);
int  gpd_ctx_destroy(gpd_ctx *ctx);
/* Asynchronous on `stream` (a hipStream_t; NULL = the null stream).  Device pointers. */
int  gpd_decode(gpd_ctx *ctx, const gpd_batch *in, const gpd_result *out, void *stream);
/* Host-memory batch: pinned staging, chunked double-buffered H2D -> decode -> D2H.
 * Synchronous; all pointers in `in`/`out` are host pointers.  Arrays registered with
 * gpd_host_register move by DMA without a staging copy: the packet bytes of a back-to-back
 * span, its offset and caplen arrays (then without any host pass over the descriptors), and
 * the result arrays. */
int  gpd_decode_host(gpd_ctx *ctx, const gpd_batch *in, const gpd_result *out);
int  gpd_sync(gpd_ctx *ctx, void *stream);
/* Time of the last gpd_decode kernel(s) on `stream`, measured with HIP events recorded on
 * that stream around the launch (ms); -1 if not available.  Requires gpd_ctx_set_timing(1). */
int  gpd_ctx_set_timing(gpd_ctx *ctx, int enable);
float gpd_last_kernel_ms(gpd_ctx *ctx);
/* The last timed gpd_decode split in two (synchronises its stream): the packets the fast
 * decode left to the generic decoder (IPv4 options, hop-by-hop, LLC, errors, ...; IPv4 fragments
 * decode on the fast path), the fast
 * kernel's time (each of its waves decodes its own fallback list at its end, so that time
 * includes the generic decodes) and the time after it to the end of the call (ms, ~0).  Needs a
 * timed launch that took the fast path (Ethernet first, hashed tables, no ext records). */
int  gpd_last_launch_split(gpd_ctx *ctx, uint64_t *fallback, float *fast_ms, float *list_ms);

/* Engine tuning of later launches on ctx.  None of these changes a result — every setting
 * decodes every packet bit-exactly — only how the fast kernel stages packets; the defaults
 * choose per batch from its mean frame slot.  Tests force each staging mode, and A/B
 * measurements compare them; a NULL pointer restores the defaults. */
typedef struct gpd_tuning {
  uint32_t window_bytes;  /* LDS window per wave: 0 automatic, 4096 or 8192 */
  int32_t  shift;         /* window copies shifted so network headers sit 16-B aligned in LDS:
                             -1 automatic (mean slot <= 96 B), 0 off, 1 on */
  int32_t  reg_prefix;    /* 8 KiB windows' chunk prefix sums from the registers at commit:
                             -1 automatic (mean slot > 160 B), 0 off, 1 on */
  int32_t  waves_per_simd; /* resident waves of the fast kernel per SIMD (= its 4-wave workgroups
                              per CU), enforced by the workgroup's LDS reservation: 0 automatic,
                              2, 3, 4 (4 KiB windows) or 2, 3 (8 KiB windows) */
  int32_t  header_once;   /* decode each 64-packet tile once from headers staged as its bytes
                             pass, instead of once per window: 0 off, 1 over 8 KiB windows cut at
                             packet boundaries, 2 over 8 KiB rounds of the tile's contiguous byte
                             run (packets larger than a window stay on the fast path); -1
                             automatic: 2 when the mean slot exceeds 160 B, else 0 */
  int32_t  device_walk; /* gpd_decode_pcap(_at): find the records in HBM after the raw
                               bytes arrive (gpd_pcapwalk.hip) instead of walking them on the
                               host first: -1 automatic (on), 0 off, 1 on */
  int32_t  grid_rounds; /* ABI 10: the fast kernel's grid in rounds of resident workgroups
                           (each wave takes every (grid waves)-th tile): 0 automatic, 1..8 */
  int32_t  split;       /* ABI 10: 4 KiB windows (small frames) with gpd_result.records by the
                           loader / decoder split kernel — one loading wave and seven decoding
                           waves per workgroup over an LDS ring: -1 automatic (on), 0 off, 1 on */
} gpd_tuning;
int  gpd_ctx_set_tuning(gpd_ctx *ctx, const gpd_tuning *t);
const char *gpd_last_error_string(void);

#ifdef __cplusplus
}
#endif
#endif /* GPD_H_ */
