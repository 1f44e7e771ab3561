/*
 * gpd_oracle.c — TEST INFRASTRUCTURE ONLY (parity oracle; see gpd_oracle.h).
 *
 * A deliberately plain, single-packet restatement of gopacket's
 * DecodingLayerParser over the decoder set {Ethernet, Dot1Q, IPv4, IPv6(+HBH),
 * IPv6ExtensionSkipper, TCP, UDP, VXLAN, Payload, Fragment}, written from the
 * Go source and structured like it (a slice = (off,len) into the packet).  It
 * shares no code with the HIP kernels it checks.  Each function cites the
 * reference lines it follows (paths relative to google/gopacket).
 */
#include "gpd_oracle.h"

#include <pthread.h>
#include <string.h>

typedef struct { uint32_t off, len; } sl; /* a Go []byte: pkt[off : off+len] */

enum { D_ETH, D_DOT1Q, D_IP4, D_IP6, D_IP6EXT, D_TCP, D_UDP, D_VXLAN, D_PAYLOAD, D_FRAG, D_ICMP4,
       D_LLC };

typedef struct {
  const uint8_t *pkt;
  const gpo_tables *t;
  int truncated;                /* DecodeFeedback.SetTruncated, decode.go:14-19 */
  uint32_t err, a0, a1;         /* the error returned by DecodeFromBytes */
  sl contents, payload;         /* BaseLayer set by the current DecodeFromBytes */
  uint32_t next;                /* NextLayerType() of the current layer */
  /* What a failing DecodeFromBytes already wrote into its reused object before it returned
   * (the parser keeps one object per kind, layers_decoder.go:61-78): 0 nothing, 1 header
   * fields read from data (addresses, ports...), 2 those fields and BaseLayer (contents /
   * payload above, a nil Payload as length 0 at the end of Contents). */
  int wrote;
} st;

static uint32_t be16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
static uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

static int fail(st *s, uint32_t code, uint32_t a0, uint32_t a1) {
  s->err = code; s->a0 = a0; s->a1 = a1;
  return -1;
}

/* EthernetType.LayerType(), enums_generated.go:77-79 */
static uint32_t ethertype_lt(const st *s, uint32_t et) { return s->t->ethertype[et & 0xFFFF]; }
/* IPProtocol.LayerType(), enums_generated.go:151-153 */
static uint32_t ipproto_lt(const st *s, uint32_t p) { return s->t->ipproto[p & 0xFF]; }
/* TCPPort.LayerType() / UDPPort.LayerType(), ports.go:54-60,97-103: 0 => Payload */
static uint32_t port_lt(const uint16_t *tab, uint32_t port) {
  uint32_t lt = tab[port & 0xFFFF];
  return lt != 0 ? lt : GPD_LT_PAYLOAD;
}

/* Ethernet.DecodeFromBytes, layers/ethernet.go:41-62; NextLayerType :110-112 */
static int dec_ethernet(st *s, sl d) {
  const uint8_t *p = s->pkt + d.off;
  if (d.len < 14) return fail(s, GPD_E_ETH_TOO_SMALL, 0, 0);
  uint32_t etype = be16(p + 12);
  s->contents = (sl){d.off, 14};
  s->payload = (sl){d.off + 14, d.len - 14};
  if (etype < 0x0600) {
    uint32_t length = etype;
    etype = 0; /* EthernetTypeLLC */
    int64_t cmp = (int64_t)s->payload.len - (int64_t)length;
    if (cmp < 0) s->truncated = 1;
    else if (cmp > 0) s->payload.len -= (uint32_t)cmp;
  }
  s->next = ethertype_lt(s, etype);
  return 0;
}

/* Dot1Q.DecodeFromBytes, layers/dot1q.go:29-40; NextLayerType :48-50 */
static int dec_dot1q(st *s, sl d) {
  const uint8_t *p = s->pkt + d.off;
  if (d.len < 4) { s->truncated = 1; return fail(s, GPD_E_DOT1Q_TOO_SHORT, d.len, 0); }
  s->contents = (sl){d.off, 4};
  s->payload = (sl){d.off + 4, d.len - 4};
  s->next = ethertype_lt(s, be16(p + 2));
  return 0;
}

/* IPv4.DecodeFromBytes, layers/ip4.go:188-275; NextLayerType :281-286 */
static int dec_ipv4(st *s, sl d) {
  const uint8_t *p = s->pkt + d.off;
  if (d.len < 20) { s->truncated = 1; return fail(s, GPD_E_IP4_TOO_SHORT, d.len, 0); }
  /* ip4.go:195-210: every header field, then BaseLayer{Contents: data} (Payload nil), are set
   * before the Length/IHL checks; a later error leaves them so */
  s->wrote = 2;
  s->contents = d;
  s->payload = (sl){d.off + d.len, 0};
  uint32_t flagsfrags = be16(p + 6);
  uint32_t ihl = p[0] & 0x0F;
  uint32_t length = be16(p + 2);
  uint32_t flags = flagsfrags >> 13, fragoff = flagsfrags & 0x1FFF;
  uint32_t proto = p[9];
  if (length == 0) length = (uint16_t)d.len;          /* ip4.go:214-218, uint16(len(data)) */
  if (length < 20) return fail(s, GPD_E_IP4_LENGTH_LT20, length, 0);
  if (ihl < 5) return fail(s, GPD_E_IP4_IHL_LT5, ihl, 0);
  if (ihl * 4 > length) return fail(s, GPD_E_IP4_IHL_GT_LENGTH, ihl, length);
  uint32_t dlen = d.len;
  if ((int64_t)dlen - (int64_t)length > 0) {
    dlen = length;                                      /* data = data[:ip.Length] */
  } else if ((int64_t)dlen - (int64_t)length < 0) {
    s->truncated = 1;
    if (ihl * 4 > dlen) return fail(s, GPD_E_IP4_HDR_TRUNC, 0, 0);
  }
  s->contents = (sl){d.off, ihl * 4};
  s->payload = (sl){d.off + ihl * 4, dlen - ihl * 4};
  /* options walk, ip4.go:238-273 */
  uint32_t o = 20, end = ihl * 4;
  while (o < end) {
    uint32_t rem = end - o;
    uint32_t otype = p[o];
    if (otype == 0) break;                              /* end of options: Padding = rest */
    if (otype == 1) { o += 1; continue; }
    if (rem < 2) { s->truncated = 1; return fail(s, GPD_E_IP4_OPT_LT2, rem, 0); }
    uint32_t olen = p[o + 1];
    if (rem < olen) { s->truncated = 1; return fail(s, GPD_E_IP4_OPT_EXCEEDS, otype, olen); }
    if (olen <= 2) return fail(s, GPD_E_IP4_OPT_LE2, otype, olen);
    o += olen;
  }
  if ((flags & 1) != 0 || fragoff != 0) s->next = GPD_LT_FRAGMENT;
  else s->next = ipproto_lt(s, proto);
  return 0;
}

/* decodeIPv6ExtensionBase, layers/ip6.go:418-432 (returns ActualLength) */
static int ip6_ext_base(st *s, sl d, uint32_t *nh, uint32_t *actual) {
  const uint8_t *p = s->pkt + d.off;
  if (d.len < 2) { s->truncated = 1; return fail(s, GPD_E_IP6EXT_LT2, d.len, 0); }
  *nh = p[0];
  *actual = (uint32_t)p[1] * 8 + 8;
  if (d.len < *actual) return fail(s, GPD_E_IP6EXT_LT_SPEC, d.len, *actual);
  return 0;
}

/* IPv6.DecodeFromBytes, layers/ip6.go:221-278, with IPv6HopByHop.DecodeFromBytes :509-526,
 * decodeIPv6HeaderTLVOption :327-346 and getIPv6HopByHopJumboLength :54-76;
 * NextLayerType :286-291 */
static int dec_ipv6(st *s, sl d) {
  const uint8_t *p = s->pkt + d.off;
  if (d.len < 40) { s->truncated = 1; return fail(s, GPD_E_IP6_TOO_SHORT, d.len, 0); }
  uint32_t length = be16(p + 4);
  uint32_t nh = p[6];
  /* ip6.go:226-235: fields and BaseLayer{data[:40], data[40:]} before the HBH / length errors */
  s->wrote = 2;
  s->contents = (sl){d.off, 40};
  s->payload = (sl){d.off + 40, d.len - 40};
  int have_hbh = 0;
  uint32_t hbh_nh = 0;
  if (nh == 0) { /* IPProtocolIPv6HopByHop */
    sl hd = s->payload;
    uint32_t actual;
    if (ip6_ext_base(s, hd, &hbh_nh, &actual)) return -1;
    const uint8_t *h = s->pkt + hd.off;
    int found = 0;
    uint32_t jdata = 0, jlen = 0;
    for (uint32_t off = 2; off < actual;) {
      uint32_t rem = hd.len - off;                      /* data[offset:] is the whole rest */
      if (rem < 2) { s->truncated = 1; return fail(s, GPD_E_IP6_TLV_LT2, 0, 0); }
      uint32_t otype = h[off], act;
      if (otype == 0) {
        act = 1;                                        /* Pad1: OptionType 0, no data */
      } else {
        uint32_t olen = h[off + 1];
        act = olen + 2;
        if (rem < act) { s->truncated = 1; return fail(s, GPD_E_IP6_TLV_TRUNC, 0, 0); }
        if (otype == 0xC2 && !found) { found = 1; jdata = off + 2; jlen = olen; }
      }
      off += act;
    }
    have_hbh = 1;
    uint32_t jumbo_len = 0;
    int jumbo = 0;
    if (found) {
      if (jlen != 4) return fail(s, GPD_E_IP6_JUMBO_TLV_LEN, 0, 0);
      jumbo_len = be32(h + jdata);
      if (jumbo_len <= 65535) return fail(s, GPD_E_IP6_JUMBO_TOO_SMALL, 0, 0);
      jumbo = 1;
    }
    if (jumbo && length == 0) {
      uint32_t pend = jumbo_len;
      if (pend > s->payload.len) { s->truncated = 1; pend = s->payload.len; }
      s->payload.len = pend;                            /* still starts at the HBH header */
      s->next = ipproto_lt(s, hbh_nh);
      return 0;
    } else if (jumbo && length != 0) {
      return fail(s, GPD_E_IP6_JUMBO_AND_LEN, 0, 0);
    } else if (!jumbo && length == 0) {
      return fail(s, GPD_E_IP6_LEN0_NO_JUMBO, 0, 0);
    } else {
      s->payload.off += actual;
      s->payload.len -= actual;
    }
  }
  if (length == 0) return fail(s, GPD_E_IP6_LEN0_NOT_HBH, nh, 0);
  uint32_t pend = length;
  if (pend > s->payload.len) { s->truncated = 1; pend = s->payload.len; }
  s->payload.len = pend;
  s->next = ipproto_lt(s, have_hbh ? hbh_nh : nh);
  return 0;
}

/* IPv6ExtensionSkipper.DecodeFromBytes, layers/ip6.go:443-451; NextLayerType :459-461 */
static int dec_ip6ext(st *s, sl d) {
  uint32_t nh, actual;
  if (ip6_ext_base(s, d, &nh, &actual)) return -1;
  s->contents = (sl){d.off, actual};
  s->payload = (sl){d.off + actual, d.len - actual};
  s->next = ipproto_lt(s, nh);
  return 0;
}

/* TCP.DecodeFromBytes, layers/tcp.go:229-302; NextLayerType :308-314 */
static int dec_tcp(st *s, sl d) {
  const uint8_t *p = s->pkt + d.off;
  if (d.len < 20) { s->truncated = 1; return fail(s, GPD_E_TCP_TOO_SHORT, d.len, 0); }
  uint32_t sport = be16(p), dport = be16(p + 2);
  uint32_t doff = p[12] >> 4;
  s->wrote = 1;  /* tcp.go:234-259: ports .. Urgent; BaseLayer untouched by the doff error */
  if (doff < 5) return fail(s, GPD_E_TCP_DOFF_LT5, doff, 0);
  uint32_t ds = doff * 4;
  s->wrote = 2;
  if (ds > d.len) {  /* tcp.go:264-268: Payload = nil, Contents = data */
    s->contents = d;
    s->payload = (sl){d.off + d.len, 0};
    s->truncated = 1;
    return fail(s, GPD_E_TCP_DOFF_GT_LEN, 0, 0);
  }
  s->contents = (sl){d.off, ds};
  s->payload = (sl){d.off + ds, d.len - ds};
  for (uint32_t o = 20; o < ds;) {                      /* OPTIONS loop, tcp.go:274-300 */
    uint32_t rem = ds - o, olen;
    uint32_t kind = p[o];
    if (kind == 0) break;                               /* EndList: Padding = rest */
    if (kind == 1) {
      olen = 1;
    } else {
      if (rem < 2) { s->truncated = 1; return fail(s, GPD_E_TCP_OPT_LT2_REM, rem, 0); }
      olen = p[o + 1];
      if (olen < 2) return fail(s, GPD_E_TCP_OPT_LEN_LT2, olen, 0);
      if (olen > rem) { s->truncated = 1; return fail(s, GPD_E_TCP_OPT_EXCEEDS, olen, rem); }
    }
    o += olen;
  }
  uint32_t lt = port_lt(s->t->tcp_port, dport);
  if (lt == GPD_LT_PAYLOAD) lt = port_lt(s->t->tcp_port, sport);
  s->next = lt;
  return 0;
}

/* UDP.DecodeFromBytes, layers/udp.go:30-56; NextLayerType :105-110 */
static int dec_udp(st *s, sl d) {
  const uint8_t *p = s->pkt + d.off;
  if (d.len < 8) { s->truncated = 1; return fail(s, GPD_E_UDP_TOO_SHORT, d.len, 0); }
  uint32_t sport = be16(p), dport = be16(p + 2), length = be16(p + 4);
  /* udp.go:35-41: ports, Length, Checksum, BaseLayer{Contents: data[:8]} (Payload nil) before
   * the "too small" error */
  s->wrote = 2;
  s->contents = (sl){d.off, 8};
  s->payload = (sl){d.off + 8, 0};
  if (length >= 8) {
    uint32_t hlen = length;
    if (hlen > d.len) { s->truncated = 1; hlen = d.len; }
    s->payload = (sl){d.off + 8, hlen - 8};
  } else if (length == 0) {
    s->payload = (sl){d.off + 8, d.len - 8};
  } else {
    return fail(s, GPD_E_UDP_LEN_TOO_SMALL, length, 0);
  }
  uint32_t lt = port_lt(s->t->udp_port, dport);
  if (lt == GPD_LT_PAYLOAD) lt = port_lt(s->t->udp_port, sport);
  s->next = lt;
  return 0;
}

/* VXLAN.DecodeFromBytes, layers/vxlan.go:53-78; NextLayerType :48-50 */
static int dec_vxlan(st *s, sl d) {
  if (d.len < 8) return fail(s, GPD_E_VXLAN_TOO_SMALL, 0, 0);
  s->contents = (sl){d.off, 8};
  s->payload = (sl){d.off + 8, d.len - 8};
  s->next = GPD_LT_ETHERNET;
  return 0;
}

/* ICMPv4.DecodeFromBytes, layers/icmp4.go:220-231; NextLayerType :261-263 (always Payload) */
static int dec_icmp4(st *s, sl d) {
  if (d.len < 8) { s->truncated = 1; return fail(s, GPD_E_ICMP4_TOO_SMALL, 0, 0); }
  s->contents = (sl){d.off, 8};
  s->payload = (sl){d.off + 8, d.len - 8};
  s->next = GPD_LT_PAYLOAD;
  return 0;
}

/* LLC.DecodeFromBytes, layers/llc.go:31-52; NextLayerType :61-69 */
static int dec_llc(st *s, sl d) {
  const uint8_t *p = s->pkt + d.off;
  if (d.len < 3) return fail(s, GPD_E_LLC_TOO_SMALL, 0, 0);
  s->wrote = 1;  /* llc.go:35-39: DSAP .. Control before the second length check */
  uint32_t dsap = p[0] & 0xFE, ssap = p[1] & 0xFE, control = p[2];
  uint32_t hl = 3;
  if ((control & 0x1) == 0 || (control & 0x3) == 0x1) {
    if (d.len < 4) return fail(s, GPD_E_LLC_TOO_SMALL, 0, 0);
    hl = 4;
  }
  s->contents = (sl){d.off, hl};
  s->payload = (sl){d.off + hl, d.len - hl};
  if (dsap == 0xAA && ssap == 0xAA) s->next = GPD_LT_SNAP;
  else if (dsap == 0x42 && ssap == 0x42) s->next = GPD_LT_STP;
  else s->next = GPD_LT_ZERO;
  return 0;
}

/* Payload / Fragment DecodeFromBytes, base.go:60-63,115-117: the whole data; LayerPayload
 * is nil and NextLayerType is Zero, base.go:42,57,99,112 */
static int dec_rest(st *s, sl d) {
  s->contents = d;
  s->payload = (sl){d.off + d.len, 0};
  s->next = GPD_LT_ZERO;
  return 0;
}

/* The registered container: LayerType -> DecodingLayer (DecodingLayerMap, parser.go:147-164),
 * filled from each decoder's CanDecode() (layertypes.go:193-198 for the skipper class). */
static int lookup(uint32_t typ, uint32_t mask) {
  switch (typ) {
    case GPD_LT_ETHERNET: return (mask & GPD_DEC_ETHERNET) ? D_ETH : -1;
    case GPD_LT_DOT1Q: return (mask & GPD_DEC_DOT1Q) ? D_DOT1Q : -1;
    case GPD_LT_IPV4: return (mask & GPD_DEC_IPV4) ? D_IP4 : -1;
    case GPD_LT_IPV6: return (mask & GPD_DEC_IPV6) ? D_IP6 : -1;
    case GPD_LT_IPV6_HOPBYHOP: case GPD_LT_IPV6_ROUTING:
    case GPD_LT_IPV6_FRAGMENT: case GPD_LT_IPV6_DEST:
      return (mask & GPD_DEC_IPV6_EXT) ? D_IP6EXT : -1;
    case GPD_LT_TCP: return (mask & GPD_DEC_TCP) ? D_TCP : -1;
    case GPD_LT_UDP: return (mask & GPD_DEC_UDP) ? D_UDP : -1;
    case GPD_LT_VXLAN: return (mask & GPD_DEC_VXLAN) ? D_VXLAN : -1;
    case GPD_LT_PAYLOAD: return (mask & GPD_DEC_PAYLOAD) ? D_PAYLOAD : -1;
    case GPD_LT_FRAGMENT: return (mask & GPD_DEC_FRAGMENT) ? D_FRAG : -1;
    case GPD_LT_ICMPV4: return (mask & GPD_DEC_ICMPV4) ? D_ICMP4 : -1;
    case GPD_LT_LLC: return (mask & GPD_DEC_LLC) ? D_LLC : -1;
    default: return -1;
  }
}

static uint32_t code_of(uint32_t typ) {
  switch (typ) {
    case GPD_LT_ETHERNET: return GPD_C_ETHERNET;
    case GPD_LT_DOT1Q: return GPD_C_DOT1Q;
    case GPD_LT_IPV4: return GPD_C_IPV4;
    case GPD_LT_IPV6: return GPD_C_IPV6;
    case GPD_LT_IPV6_HOPBYHOP: return GPD_C_IPV6_HBH;
    case GPD_LT_IPV6_ROUTING: return GPD_C_IPV6_RT;
    case GPD_LT_IPV6_FRAGMENT: return GPD_C_IPV6_FRAG;
    case GPD_LT_IPV6_DEST: return GPD_C_IPV6_DEST;
    case GPD_LT_TCP: return GPD_C_TCP;
    case GPD_LT_UDP: return GPD_C_UDP;
    case GPD_LT_VXLAN: return GPD_C_VXLAN;
    case GPD_LT_PAYLOAD: return GPD_C_PAYLOAD;
    case GPD_LT_FRAGMENT: return GPD_C_FRAGMENT;
    case GPD_LT_ICMPV4: return GPD_C_ICMPV4;
    case GPD_LT_LLC: return GPD_C_LLC;
    default: return GPD_C_NONE;
  }
}

static const int obj_of_dec[] = {GPD_OBJ_ETHERNET, GPD_OBJ_DOT1Q, GPD_OBJ_IPV4, GPD_OBJ_IPV6,
                                 GPD_OBJ_IPV6_EXT, GPD_OBJ_TCP, GPD_OBJ_UDP, GPD_OBJ_VXLAN,
                                 GPD_OBJ_PAYLOAD, GPD_OBJ_FRAGMENT, GPD_OBJ_ICMPV4, GPD_OBJ_LLC};

/* ip4.go:158-179 `checksum`: bytes 10-11 read as zero, fold `for csum > 0xffff`, invert. */
uint16_t gpo_ip4_header_checksum(const uint8_t *b, uint32_t len) {
  uint32_t csum = 0;
  for (uint32_t i = 0; i + 1 < len; i += 2) { /* contents are IHL*4 bytes: even */
    uint32_t hi = (i == 10) ? 0 : b[i];
    uint32_t lo = (i + 1 == 11) ? 0 : b[i + 1];
    csum += hi << 8;
    csum += lo;
  }
  while (csum > 65535) csum = (csum >> 16) + (uint32_t)(uint16_t)csum;
  return (uint16_t)~csum;
}

/* tcpipChecksum, layers/tcpip.go:52-70 (uint32 arithmetic wraps like Go's) */
uint16_t gpo_tcpip_checksum(const uint8_t *data, uint32_t len, uint32_t csum) {
  int64_t length = (int64_t)len - 1;
  for (int64_t i = 0; i < length; i += 2) {
    csum += (uint32_t)data[i] << 8;
    csum += (uint32_t)data[i + 1];
  }
  if (len % 2 == 1) csum += (uint32_t)data[length] << 8;
  while (csum > 0xffff) csum = (csum >> 16) + (csum & 0xffff);
  return (uint16_t)~csum;
}

/* (*IPv4).pseudoheaderChecksum, layers/tcpip.go:26-35 */
uint32_t gpo_pseudo_v4(const uint8_t *s4, const uint8_t *d4) {
  uint32_t csum = 0;
  csum += ((uint32_t)s4[0] + (uint32_t)s4[2]) << 8;
  csum += (uint32_t)s4[1] + (uint32_t)s4[3];
  csum += ((uint32_t)d4[0] + (uint32_t)d4[2]) << 8;
  csum += (uint32_t)d4[1] + (uint32_t)d4[3];
  return csum;
}

/* (*IPv6).pseudoheaderChecksum, layers/tcpip.go:37-48 */
uint32_t gpo_pseudo_v6(const uint8_t *s16, const uint8_t *d16) {
  uint32_t csum = 0;
  for (int i = 0; i < 16; i += 2) {
    csum += (uint32_t)s16[i] << 8;
    csum += (uint32_t)s16[i + 1];
    csum += (uint32_t)d16[i] << 8;
    csum += (uint32_t)d16[i + 1];
  }
  return csum;
}

/* fnvHash, flows.go:60-70 */
uint64_t gpo_fnv_hash(const uint8_t *s, uint32_t len) {
  uint64_t h = 14695981039346656037ULL;
  for (uint32_t i = 0; i < len; i++) {
    h ^= (uint64_t)s[i];
    h *= 1099511628211ULL;
  }
  return h;
}

/* Flow.FastHash, flows.go:167-174 (on a NewFlow, flows.go:214-224) */
uint64_t gpo_flow_fasthash(uint32_t ept, const uint8_t *src, uint32_t slen, const uint8_t *dst,
                           uint32_t dlen) {
  uint64_t h = gpo_fnv_hash(src, slen) + gpo_fnv_hash(dst, dlen);
  h ^= (uint64_t)ept;
  h *= 1099511628211ULL;
  return h;
}

/* Endpoint.FastHash, flows.go:78-83 */
uint64_t gpo_endpoint_fasthash(uint32_t ept, const uint8_t *raw, uint32_t len) {
  uint64_t h = gpo_fnv_hash(raw, len);
  h ^= (uint64_t)ept;
  h *= 1099511628211ULL;
  return h;
}

void gpo_decode_packet(const uint8_t *pkt, uint32_t caplen, uint32_t first, uint32_t mask,
                       uint32_t options, const gpo_tables *t, uint32_t *status_out,
                       uint64_t *layers_out, uint64_t *net_hash_out, uint64_t *tp_hash_out,
                       uint32_t *csum_out, uint32_t *hdr_off_out, gpd_ext_rec *ext) {
  st s;
  memset(&s, 0, sizeof s);
  s.pkt = pkt;
  s.t = t;
  int obj_ok[GPD_NOBJ] = {0};     /* the kind is in decoded (one successful call at least) */
  gpd_layer_rec obj[GPD_NOBJ];    /* each object's BaseLayer as the call leaves it */
  uint32_t fbase[GPD_NOBJ];       /* where its header fields (addresses, ports) were read */
  memset(obj, 0, sizeof obj);
  memset(fbase, 0, sizeof fbase);
  int err_obj = -1, err_wrote = 0;
  uint32_t err_off = 0;
  uint32_t ncount = 0;
  uint64_t core_codes = 0, ext_codes[2] = {0, 0};
  int last_net = -1, last_tp = -1, tp_net = -1; /* object ids */
  uint32_t stop = GPD_LT_ZERO, klass = GPD_ST_OK;

  /* DecodeLayers (parser.go:302-316) -> LayersDecoder closure (layers_decoder.go:60-79) */
  int dec = lookup(first, mask);
  if (dec < 0) {
    stop = first; /* layers_decoder.go:12-17: returns (first, nil) without touching decoded */
  } else {
    uint32_t typ = first;
    sl data = {0, caplen};
    for (;;) {
      int rc;
      s.wrote = 0;
      switch (dec) {
        case D_ETH: rc = dec_ethernet(&s, data); break;
        case D_DOT1Q: rc = dec_dot1q(&s, data); break;
        case D_IP4: rc = dec_ipv4(&s, data); break;
        case D_IP6: rc = dec_ipv6(&s, data); break;
        case D_IP6EXT: rc = dec_ip6ext(&s, data); break;
        case D_TCP: rc = dec_tcp(&s, data); break;
        case D_UDP: rc = dec_udp(&s, data); break;
        case D_VXLAN: rc = dec_vxlan(&s, data); break;
        case D_ICMP4: rc = dec_icmp4(&s, data); break;
        case D_LLC: rc = dec_llc(&s, data); break;
        default: rc = dec_rest(&s, data); break;
      }
      if (rc) {
        /* The failing call's object keeps what it wrote before returning (ip4.go:195-210,
         * ip6.go:226-235, tcp.go:234-268, udp.go:35-41, llc.go:35-39) */
        klass = GPD_ST_DECODE_ERROR;
        err_obj = obj_of_dec[dec];
        err_off = data.off;
        err_wrote = s.wrote;
        if (s.wrote >= 1) fbase[err_obj] = data.off;
        if (s.wrote == 2) {
          obj[err_obj].contents_off = s.contents.off;
          obj[err_obj].contents_len = s.contents.len;
          obj[err_obj].payload_off = s.payload.off;
          obj[err_obj].payload_len = s.payload.len;
        }
        break;
      }
      /* *decoded = append(*decoded, typ) */
      uint32_t code = code_of(typ);
      if (ncount < GPD_CORE_MAX_LAYERS) core_codes |= (uint64_t)code << (16 + 4 * ncount);
      if (ncount < GPD_EXT_MAX_LAYERS) ext_codes[ncount / 16] |= (uint64_t)code << (4 * (ncount % 16));
      ncount++;
      int o = obj_of_dec[dec];
      obj_ok[o] = 1;
      obj[o].contents_off = s.contents.off;
      obj[o].contents_len = s.contents.len;
      obj[o].payload_off = s.payload.off;
      obj[o].payload_len = s.payload.len;
      fbase[o] = data.off;
      if (o == GPD_OBJ_IPV4 || o == GPD_OBJ_IPV6) last_net = o;
      if (o == GPD_OBJ_TCP || o == GPD_OBJ_UDP) { last_tp = o; tp_net = last_net; }
      typ = s.next;
      data = s.payload;
      if (data.len == 0) break;
      dec = lookup(typ, mask);
      if (dec < 0) { stop = typ; break; }
    }
  }
  if (klass != GPD_ST_DECODE_ERROR && stop != GPD_LT_ZERO)
    klass = (options & GPD_OPT_IGNORE_UNSUPPORTED) ? GPD_ST_OK : GPD_ST_UNSUPPORTED;

  uint32_t status = klass | ((uint32_t)s.truncated << 2);
  uint32_t nl = ncount > 31 ? 31 : ncount;
  status |= (ncount > 31 ? 1u : 0u) << 3;
  status |= nl << 4;
  if (klass == GPD_ST_DECODE_ERROR) status |= s.err << 9;

  uint64_t nh = 0, th = 0;
  uint32_t csum = 0;
  /* EndpointTypes of the flows' layers (layers/endpoints.go:20-32), hashed or not */
  if (last_net >= 0) status |= (last_net == GPD_OBJ_IPV4 ? 1u : 2u) << 20;
  if (last_tp >= 0) status |= (last_tp == GPD_OBJ_TCP ? 4u : 5u) << 24;
  if (!(options & GPD_OPT_NO_FLOW_HASH)) {
    if (last_net >= 0) {  /* ip4/ip6.NetworkFlow() over SrcIP/DstIP as last written */
      const uint8_t *c = pkt + fbase[last_net];
      if (last_net == GPD_OBJ_IPV4) nh = gpo_flow_fasthash(1, c + 12, 4, c + 16, 4);
      else nh = gpo_flow_fasthash(2, c + 8, 16, c + 24, 16);
      status |= 1u << 16;
    }
    if (last_tp >= 0) {  /* tcp/udp.TransportFlow() over sPort/dPort as last written */
      const uint8_t *c = pkt + fbase[last_tp];
      uint32_t ept = last_tp == GPD_OBJ_TCP ? 4 : 5;
      th = gpo_flow_fasthash(ept, c, 2, c + 2, 2);
      status |= 1u << 17;
    }
  }
  if (!(options & GPD_OPT_NO_CHECKSUMS)) {
    /* checksum(ip4.Contents): after a failed Length/IHL check Contents is all of that call's
     * data (ip4.go:210); an odd length makes `checksum` index past the end (ip4.go:165-167),
     * a Go panic, so that case reports no value (bit 18 clear) */
    if (obj_ok[GPD_OBJ_IPV4] && (obj[GPD_OBJ_IPV4].contents_len & 1u) == 0) {
      csum |= gpo_ip4_header_checksum(pkt + obj[GPD_OBJ_IPV4].contents_off,
                                      obj[GPD_OBJ_IPV4].contents_len);
      status |= 1u << 18;
    }
    if (last_tp >= 0 && tp_net >= 0) {
      /* tcp.SetNetworkLayerForChecksum(net); tcp.ComputeChecksum() (tcp.go:193-195,
       * tcpip.go:75-88): append(Contents, Payload...) with the pseudo-header of `net` */
      const gpd_layer_rec *r = &obj[last_tp];
      const uint8_t *nc = pkt + fbase[tp_net];
      uint32_t ps = tp_net == GPD_OBJ_IPV4 ? gpo_pseudo_v4(nc + 12, nc + 16)
                                          : gpo_pseudo_v6(nc + 8, nc + 24);
      uint32_t length = r->contents_len + r->payload_len;
      ps += last_tp == GPD_OBJ_TCP ? 6u : 17u;
      ps += length & 0xffff;
      ps += length >> 16;
      csum |= (uint32_t)gpo_tcpip_checksum(pkt + r->contents_off, length, ps) << 16;
      status |= 1u << 19;
    }
  }

  *status_out = status;
  *layers_out = core_codes | (stop & 0xFFFFu);
  if (net_hash_out) *net_hash_out = nh;
  if (tp_hash_out) *tp_hash_out = th;
  if (csum_out) *csum_out = csum;
  if (hdr_off_out) { /* gpd.h header offsets word: the objects NetworkFlow/TransportFlow read */
    uint32_t a = last_net >= 0 ? fbase[last_net] : 0xFFFFu;
    uint32_t b = last_tp >= 0 ? fbase[last_tp] : 0xFFFFu;
    *hdr_off_out = (a < 0xFFFFu ? a : 0xFFFFu) | ((b < 0xFFFFu ? b : 0xFFFFu) << 16);
  }
  if (ext) {
    memset(ext, 0, sizeof *ext);
    ext->layer_codes[0] = ext_codes[0];
    ext->layer_codes[1] = ext_codes[1];
    ext->err_obj = GPD_NOBJ_NONE;
    if (klass == GPD_ST_DECODE_ERROR) {
      ext->err_arg0 = s.a0;
      ext->err_arg1 = s.a1;
      ext->err_obj = (uint8_t)err_obj;
      ext->err_wrote = (uint8_t)err_wrote;
      ext->err_off = err_off;
    }
    uint32_t valid = 0;
    for (int o = 0; o < GPD_NOBJ; o++) {
      if (obj_ok[o]) valid |= 1u << o;
      if (obj_ok[o] || (o == err_obj && err_wrote == 2)) ext->obj[o] = obj[o];
    }
    ext->obj_valid = (uint16_t)valid;
  }
}

typedef struct {
  const uint8_t *data; const uint32_t *offset, *caplen;
  uint64_t lo, hi;
  uint32_t first, decoders, options;
  const gpo_tables *t;
  uint32_t *status; uint64_t *layers, *net_hash, *tp_hash; uint32_t *csum, *hdr_off;
  gpd_ext_rec *ext;
} job;

static void run_job(const job *j) {
  for (uint64_t i = j->lo; i < j->hi; i++) {
    gpo_decode_packet(j->data + j->offset[i], j->caplen[i], j->first, j->decoders, j->options,
                      j->t, &j->status[i], &j->layers[i],
                      j->net_hash ? &j->net_hash[i] : 0, j->tp_hash ? &j->tp_hash[i] : 0,
                      j->csum ? &j->csum[i] : 0, j->hdr_off ? &j->hdr_off[i] : 0,
                      j->ext ? &j->ext[i] : 0);
  }
}

static void *job_main(void *arg) { run_job((const job *)arg); return 0; }

void gpo_decode_batch(const uint8_t *data, const uint32_t *offset, const uint32_t *caplen,
                      uint64_t n, uint32_t first, uint32_t decoders, uint32_t options,
                      const gpo_tables *t, uint32_t *status, uint64_t *layers,
                      uint64_t *net_hash, uint64_t *tp_hash, uint32_t *csum,
                      uint32_t *hdr_off, gpd_ext_rec *ext, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  job jobs[256];
  pthread_t th[256];
  for (int k = 0; k < nthreads; k++) {
    job j = {data, offset, caplen, n * k / nthreads, n * (k + 1) / nthreads,
             first, decoders, options, t, status, layers, net_hash, tp_hash, csum, hdr_off, ext};
    jobs[k] = j;
  }
  if (nthreads == 1) { run_job(&jobs[0]); return; }
  for (int k = 0; k < nthreads; k++) pthread_create(&th[k], 0, job_main, &jobs[k]);
  for (int k = 0; k < nthreads; k++) pthread_join(th[k], 0);
}
