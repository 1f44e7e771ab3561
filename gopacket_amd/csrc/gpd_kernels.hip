// gpd_kernels.hip — MI355X (gfx950) batched DecodingLayerParser kernels.
//
// One wavefront lane per packet.  A wave owns a tile of 64 consecutive packet
// indices; the byte range those packets occupy in the batch buffer is staged
// HBM -> LDS with 16-byte LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
// instruction, fully coalesced) into the wave's private LDS window, and every
// lane then runs the DecodingLayerParser loop for its packet out of LDS.  The
// decode loop, the IPv4 header checksum, the TCP/UDP pseudo-header checksum and
// both flow FastHashes are fused: header bytes are read from HBM exactly once.
// Packets that do not fit one window are handled in further windows of the
// same tile; a packet larger than a window is decoded straight from global
// memory (same code, other byte source).
//
// Semantics follow the reference (paths relative to google/gopacket):
//   loop ............ layers_decoder.go:60-79, parser.go:302-316
//   Ethernet ........ layers/ethernet.go:41-62,110-112
//   Dot1Q ........... layers/dot1q.go:29-50
//   IPv4 ............ layers/ip4.go:188-286
//   IPv6 (+HBH) ..... layers/ip6.go:54-76,221-291,327-346,418-432,509-526
//   ExtSkipper ...... layers/ip6.go:443-461
//   TCP ............. layers/tcp.go:229-314
//   UDP ............. layers/udp.go:30-110
//   VXLAN ........... layers/vxlan.go:48-78
//   Payload/Fragment  base.go:55-63,108-117
//   checksums ....... layers/ip4.go:158-179, layers/tcpip.go:26-88, layers/tcp.go:193-195
//   FastHash ........ flows.go:60-83,167-174
// DESIGN.md §Semantics defines every output word.
#include <hip/hip_runtime.h>

#include "gpd_internal.h"

namespace gpd {

constexpr int kWaves = 4;           // waves per workgroup
constexpr int kBlock = 64 * kWaves; // threads per workgroup

extern __shared__ __attribute__((aligned(16))) uint8_t g_lds[];

// ---------------------------------------------------------------- byte sources
// LDS window: absolute LDS byte addresses.
struct LdsSrc {
  uint32_t base;  // LDS address of the packet's first byte
  __device__ __forceinline__ uint32_t dw(uint32_t a) const {  // a 4-aligned
    return *reinterpret_cast<const uint32_t *>(g_lds + a);
  }
  __device__ __forceinline__ uint32_t u8(uint32_t rel) const { return g_lds[base + rel]; }
  __device__ __forceinline__ uint32_t abs(uint32_t rel) const { return base + rel; }
  __device__ __forceinline__ uint4 q(uint32_t a) const {  // a 16-aligned
    return *reinterpret_cast<const uint4 *>(g_lds + a);
  }
};

// Global memory: byte offsets into the batch buffer (16-aligned base pointer).
struct GlbSrc {
  const uint8_t *data;
  uint64_t base;  // offset of the packet's first byte
  __device__ __forceinline__ uint32_t dw(uint64_t a) const {
    return *reinterpret_cast<const uint32_t *>(data + a);
  }
  __device__ __forceinline__ uint32_t u8(uint32_t rel) const { return data[base + rel]; }
  __device__ __forceinline__ uint64_t abs(uint32_t rel) const { return base + rel; }
  __device__ __forceinline__ uint4 q(uint64_t a) const {
    return *reinterpret_cast<const uint4 *>(data + a);
  }
};

// N little-endian words holding packet bytes [rel, rel+4N) (unaligned start).
template <int N, class S>
__device__ __forceinline__ void load_words(const S &s, uint32_t rel, uint32_t (&w)[N]) {
  auto A = s.abs(rel);
  auto Al = A & ~decltype(A)(3);
  uint32_t sh = (uint32_t)(A & 3);
  uint32_t a[N + 1];
#pragma unroll
  for (int k = 0; k <= N; k++) a[k] = s.dw(Al + 4 * k);
#pragma unroll
  for (int k = 0; k < N; k++) w[k] = __builtin_amdgcn_alignbyte(a[k + 1], a[k], sh);
}

template <int N>
__device__ __forceinline__ uint32_t byte_at(const uint32_t (&w)[N], int o) {
  return (w[o >> 2] >> (8 * (o & 3))) & 0xFFu;
}
template <int N>
__device__ __forceinline__ uint32_t be16_at(const uint32_t (&w)[N], int o) {
  return (byte_at(w, o) << 8) | byte_at(w, o + 1);
}

// ---------------------------------------------------------------- tables
__device__ __forceinline__ uint32_t page_lookup(const uint16_t *T, uint32_t dir, uint32_t key) {
  uint32_t page = T[dir + (key >> 8)];
  return T[kTabPages + page * 256u + (key & 0xFFu)];
}
__device__ __forceinline__ uint32_t ethertype_lt(const uint16_t *T, uint32_t et) {
  return page_lookup(T, kTabEthDir, et);  // enums_generated.go:77-79
}
__device__ __forceinline__ uint32_t ipproto_lt(const uint16_t *T, uint32_t p) {
  return T[kTabIpProto + (p & 0xFFu)];    // enums_generated.go:151-153
}
__device__ __forceinline__ uint32_t port_lt(const uint16_t *T, uint32_t dir, uint32_t port) {
  uint32_t lt = page_lookup(T, dir, port);  // ports.go:54-60,97-103
  return lt ? lt : (uint32_t)GPD_LT_PAYLOAD;
}

enum Dec : int { D_ETH, D_DOT1Q, D_IP4, D_IP6, D_IP6EXT, D_TCP, D_UDP, D_VXLAN, D_PAYLOAD, D_FRAG, D_NONE };

// DecodingLayerMap lookup over the registered set (parser.go:147-164).
__device__ __forceinline__ int lookup(uint32_t typ, uint32_t mask) {
  int d;
  switch (typ) {
    case GPD_LT_ETHERNET: d = D_ETH; break;
    case GPD_LT_DOT1Q: d = D_DOT1Q; break;
    case GPD_LT_IPV4: d = D_IP4; break;
    case GPD_LT_IPV6: d = D_IP6; break;
    case GPD_LT_IPV6_HOPBYHOP: case GPD_LT_IPV6_ROUTING:
    case GPD_LT_IPV6_FRAGMENT: case GPD_LT_IPV6_DEST: d = D_IP6EXT; break;
    case GPD_LT_TCP: d = D_TCP; break;
    case GPD_LT_UDP: d = D_UDP; break;
    case GPD_LT_VXLAN: d = D_VXLAN; break;
    case GPD_LT_PAYLOAD: d = D_PAYLOAD; break;
    case GPD_LT_FRAGMENT: d = D_FRAG; break;
    default: return D_NONE;
  }
  return (mask >> d) & 1u ? d : (int)D_NONE;
}

__device__ __forceinline__ uint32_t code_of(uint32_t typ) {
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
    default: return GPD_C_FRAGMENT;
  }
}

// ---------------------------------------------------------------- checksums / hashes
// Exact (mod 2^32) sum of the big-endian 16-bit words of packet bytes [rel, rel+len)
// as tcpipChecksum accumulates them (tcpip.go:57-65; an odd last byte counts <<8):
// S = 256*E + O with E/O the byte sums at even/odd positions of the range.
template <class S>
__device__ __forceinline__ uint32_t be16_sum(const S &s, uint32_t rel, uint32_t len) {
  if (len == 0) return 0;
  auto A = s.abs(rel);
  auto C = A & ~decltype(A)(15);
  auto Cend = (A + len + 15) & ~decltype(A)(15);
  const uint32_t even_w = (A & 1) ? 0x01000100u : 0x00010001u;
  const uint32_t odd_w = (A & 1) ? 0x00010001u : 0x01000100u;
  uint32_t E = 0, O = 0;
  // first and last chunk carry a byte mask, the interior is straight
  const auto last = Cend - 16;
  for (; C < Cend; C += 16) {
    uint4 v = s.q(C);
    uint32_t x[4] = {v.x, v.y, v.z, v.w};
    if (C < A || C == last) {
      int64_t lo = (int64_t)A - (int64_t)C;             // first valid byte in chunk
      int64_t hi = (int64_t)(A + len) - (int64_t)C;     // one past last valid byte
#pragma unroll
      for (int j = 0; j < 4; j++) {
        int64_t l = lo - 4 * j, h = hi - 4 * j;
        l = l < 0 ? 0 : (l > 4 ? 4 : l);
        h = h < 0 ? 0 : (h > 4 ? 4 : h);
        uint64_t m = ((1ull << (8 * h)) - 1ull) & ~((1ull << (8 * l)) - 1ull);
        x[j] &= (uint32_t)m;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      E = __builtin_amdgcn_udot4(x[j], even_w, E, false);
      O = __builtin_amdgcn_udot4(x[j], odd_w, O, false);
    }
  }
  return (E << 8) + O;
}

__device__ __forceinline__ uint16_t fold_not(uint32_t csum) {
  while (csum > 0xFFFFu) csum = (csum >> 16) + (csum & 0xFFFFu);
  return (uint16_t)~csum;
}

constexpr uint64_t kFnvBasis = 14695981039346656037ULL;  // flows.go:69
constexpr uint64_t kFnvPrime = 1099511628211ULL;         // flows.go:70

// FNV-1a over the bytes of little-endian word w (lowest byte first), flows.go:60-67.
__device__ __forceinline__ uint64_t fnv_word(uint64_t h, uint32_t w, int nbytes) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    if (j < nbytes) {
      h ^= (uint64_t)((w >> (8 * j)) & 0xFFu);
      h *= kFnvPrime;
    }
  }
  return h;
}
// Flow.FastHash, flows.go:167-174
__device__ __forceinline__ uint64_t flow_mix(uint64_t hs, uint64_t hd, uint32_t ept) {
  uint64_t h = hs + hd;
  h ^= (uint64_t)ept;
  return h * kFnvPrime;
}

// ---------------------------------------------------------------- one packet
struct Out {
  uint32_t status;
  uint64_t layers;
  uint64_t net_hash, tp_hash;
  uint32_t csum;
};

#define GPD_FAIL(code, x0, x1) \
  do { err = (code); a0 = (x0); a1 = (x1); goto fail; } while (0)

template <bool EXT, class S>
__device__ __forceinline__ Out decode_packet(const S &s, uint32_t caplen, const uint16_t *T,
                                             uint32_t first, uint32_t mask, uint32_t options,
                                             gpd_ext_rec *ext) {
  uint32_t truncated = 0, err = 0, a0 = 0, a1 = 0;
  uint32_t ncount = 0;
  uint64_t codes = 0, ecodes0 = 0, ecodes1 = 0;
  uint32_t stop = 0, klass = GPD_ST_OK;
  // final (last successful) state of the objects the fused outputs read
  uint32_t ip4_off = 0, ip4_hl = 0, ip6_off = 0;
  uint32_t tcp_off = 0, tcp_tot = 0, udp_off = 0, udp_tot = 0;
  uint32_t last_net = 0, last_tp = 0, tp_net = 0;  // net: 1 v4, 2 v6; tp: 1 TCP, 2 UDP
  uint32_t obj_valid = 0;
  gpd_layer_rec rec[EXT ? GPD_NOBJ : 1];

  uint32_t typ = first;
  int dec = lookup(typ, mask);
  uint32_t off = 0, len = caplen;
  if (dec == D_NONE) {
    stop = typ;  // layers_decoder.go:12-17
  } else {
    for (;;) {
      uint32_t c_off = off, c_len, p_off, p_len, next;
      switch (dec) {
        case D_ETH: {  // ethernet.go:41-62
          if (len < 14) GPD_FAIL(GPD_E_ETH_TOO_SMALL, 0, 0);
          uint32_t w[1];
          load_words(s, off + 12, w);
          uint32_t et = ((w[0] & 0xFFu) << 8) | ((w[0] >> 8) & 0xFFu);
          c_len = 14; p_off = off + 14; p_len = len - 14;
          if (et < 0x0600u) {
            if (p_len < et) truncated = 1;
            else p_len = et;
            et = 0;  // EthernetTypeLLC
          }
          next = ethertype_lt(T, et);
          break;
        }
        case D_DOT1Q: {  // dot1q.go:29-40
          if (len < 4) { truncated = 1; GPD_FAIL(GPD_E_DOT1Q_TOO_SHORT, len, 0); }
          uint32_t w[1];
          load_words(s, off, w);
          c_len = 4; p_off = off + 4; p_len = len - 4;
          next = ethertype_lt(T, be16_at(w, 2));
          break;
        }
        case D_IP4: {  // ip4.go:188-286
          if (len < 20) { truncated = 1; GPD_FAIL(GPD_E_IP4_TOO_SHORT, len, 0); }
          uint32_t w[3];
          load_words(s, off, w);  // bytes 0..11 (version/IHL .. protocol)
          uint32_t ihl = byte_at(w, 0) & 0x0Fu;
          uint32_t length = be16_at(w, 2);
          uint32_t ff = be16_at(w, 6);
          uint32_t proto = byte_at(w, 9);
          if (length == 0) length = len & 0xFFFFu;  // uint16(len(data))
          if (length < 20) GPD_FAIL(GPD_E_IP4_LENGTH_LT20, length, 0);
          if (ihl < 5) GPD_FAIL(GPD_E_IP4_IHL_LT5, ihl, 0);
          if (ihl * 4 > length) GPD_FAIL(GPD_E_IP4_IHL_GT_LENGTH, ihl, length);
          uint32_t dlen = len;
          if (len > length) {
            dlen = length;
          } else if (len < length) {
            truncated = 1;
            if (ihl * 4 > len) GPD_FAIL(GPD_E_IP4_HDR_TRUNC, 0, 0);
          }
          c_len = ihl * 4; p_off = off + c_len; p_len = dlen - c_len;
          for (uint32_t q = 20; q < c_len;) {  // options, ip4.go:240-273
            uint32_t rem = c_len - q;
            uint32_t t = s.u8(off + q);
            if (t == 0) break;
            if (t == 1) { q += 1; continue; }
            if (rem < 2) { truncated = 1; GPD_FAIL(GPD_E_IP4_OPT_LT2, rem, 0); }
            uint32_t ol = s.u8(off + q + 1);
            if (rem < ol) { truncated = 1; GPD_FAIL(GPD_E_IP4_OPT_EXCEEDS, t, ol); }
            if (ol <= 2) GPD_FAIL(GPD_E_IP4_OPT_LE2, t, ol);
            q += ol;
          }
          next = ((ff >> 13) & 1u) || (ff & 0x1FFFu) ? (uint32_t)GPD_LT_FRAGMENT : ipproto_lt(T, proto);
          break;
        }
        case D_IP6: {  // ip6.go:221-291
          if (len < 40) { truncated = 1; GPD_FAIL(GPD_E_IP6_TOO_SHORT, len, 0); }
          uint32_t w[2];
          load_words(s, off + 4, w);  // bytes 4..11: payload length, next header
          uint32_t length = be16_at(w, 0);
          uint32_t nh = byte_at(w, 2);
          c_len = 40; p_off = off + 40; p_len = len - 40;
          uint32_t use_nh = nh;
          if (nh == 0) {  // hop-by-hop parsed inside IPv6
            uint32_t hlen = p_len, hoff = p_off;
            if (hlen < 2) { truncated = 1; GPD_FAIL(GPD_E_IP6EXT_LT2, hlen, 0); }
            uint32_t hnh = s.u8(hoff), actual = s.u8(hoff + 1) * 8u + 8u;
            if (hlen < actual) GPD_FAIL(GPD_E_IP6EXT_LT_SPEC, hlen, actual);
            bool found = false;
            uint32_t jd = 0, jl = 0;
            for (uint32_t q = 2; q < actual;) {  // ip6.go:516-524 over data[offset:]
              uint32_t rem = hlen - q;
              if (rem < 2) { truncated = 1; GPD_FAIL(GPD_E_IP6_TLV_LT2, 0, 0); }
              uint32_t t = s.u8(hoff + q), act = 1;
              if (t != 0) {
                uint32_t ol = s.u8(hoff + q + 1);
                act = ol + 2;
                if (rem < act) { truncated = 1; GPD_FAIL(GPD_E_IP6_TLV_TRUNC, 0, 0); }
                if (t == 0xC2u && !found) { found = true; jd = q + 2; jl = ol; }
              }
              q += act;
            }
            uint32_t jumbo_len = 0;
            bool jumbo = false;
            if (found) {  // getIPv6HopByHopJumboLength, ip6.go:54-76
              if (jl != 4) GPD_FAIL(GPD_E_IP6_JUMBO_TLV_LEN, 0, 0);
              jumbo_len = (s.u8(hoff + jd) << 24) | (s.u8(hoff + jd + 1) << 16) |
                          (s.u8(hoff + jd + 2) << 8) | s.u8(hoff + jd + 3);
              if (jumbo_len <= 65535u) GPD_FAIL(GPD_E_IP6_JUMBO_TOO_SMALL, 0, 0);
              jumbo = true;
            }
            use_nh = hnh;
            if (jumbo && length == 0) {
              if (jumbo_len > p_len) truncated = 1;
              else p_len = jumbo_len;  // payload still starts at the HBH header (ip6.go:255)
              next = ipproto_lt(T, use_nh);
              break;
            } else if (jumbo) {
              GPD_FAIL(GPD_E_IP6_JUMBO_AND_LEN, 0, 0);
            } else if (length == 0) {
              GPD_FAIL(GPD_E_IP6_LEN0_NO_JUMBO, 0, 0);
            }
            p_off += actual;
            p_len -= actual;
          }
          if (length == 0) GPD_FAIL(GPD_E_IP6_LEN0_NOT_HBH, nh, 0);
          if (length > p_len) truncated = 1;
          else p_len = length;
          next = ipproto_lt(T, use_nh);
          break;
        }
        case D_IP6EXT: {  // ip6.go:418-432,443-461
          if (len < 2) { truncated = 1; GPD_FAIL(GPD_E_IP6EXT_LT2, len, 0); }
          uint32_t w[1];
          load_words(s, off, w);
          uint32_t actual = byte_at(w, 1) * 8u + 8u;
          if (len < actual) GPD_FAIL(GPD_E_IP6EXT_LT_SPEC, len, actual);
          c_len = actual; p_off = off + actual; p_len = len - actual;
          next = ipproto_lt(T, byte_at(w, 0));
          break;
        }
        case D_TCP: {  // tcp.go:229-314
          if (len < 20) { truncated = 1; GPD_FAIL(GPD_E_TCP_TOO_SHORT, len, 0); }
          uint32_t w[4];
          load_words(s, off, w);  // bytes 0..15: ports .. flags
          uint32_t doff = byte_at(w, 12) >> 4;
          if (doff < 5) GPD_FAIL(GPD_E_TCP_DOFF_LT5, doff, 0);
          uint32_t ds = doff * 4;
          if (ds > len) { truncated = 1; GPD_FAIL(GPD_E_TCP_DOFF_GT_LEN, 0, 0); }
          c_len = ds; p_off = off + ds; p_len = len - ds;
          for (uint32_t q = 20; q < ds;) {  // OPTIONS, tcp.go:274-300
            uint32_t rem = ds - q;
            uint32_t k = s.u8(off + q), ol = 1;
            if (k == 0) break;
            if (k != 1) {
              if (rem < 2) { truncated = 1; GPD_FAIL(GPD_E_TCP_OPT_LT2_REM, rem, 0); }
              ol = s.u8(off + q + 1);
              if (ol < 2) GPD_FAIL(GPD_E_TCP_OPT_LEN_LT2, ol, 0);
              if (ol > rem) { truncated = 1; GPD_FAIL(GPD_E_TCP_OPT_EXCEEDS, ol, rem); }
            }
            q += ol;
          }
          uint32_t lt = port_lt(T, kTabTcpDir, be16_at(w, 2));
          if (lt == GPD_LT_PAYLOAD) lt = port_lt(T, kTabTcpDir, be16_at(w, 0));
          next = lt;
          break;
        }
        case D_UDP: {  // udp.go:30-56,105-110
          if (len < 8) { truncated = 1; GPD_FAIL(GPD_E_UDP_TOO_SHORT, len, 0); }
          uint32_t w[2];
          load_words(s, off, w);
          uint32_t length = be16_at(w, 4);
          c_len = 8; p_off = off + 8;
          if (length >= 8) {
            uint32_t hlen = length;
            if (hlen > len) { truncated = 1; hlen = len; }
            p_len = hlen - 8;
          } else if (length == 0) {
            p_len = len - 8;
          } else {
            GPD_FAIL(GPD_E_UDP_LEN_TOO_SMALL, length, 0);
          }
          uint32_t lt = port_lt(T, kTabUdpDir, be16_at(w, 2));
          if (lt == GPD_LT_PAYLOAD) lt = port_lt(T, kTabUdpDir, be16_at(w, 0));
          next = lt;
          break;
        }
        case D_VXLAN: {  // vxlan.go:53-78
          if (len < 8) GPD_FAIL(GPD_E_VXLAN_TOO_SMALL, 0, 0);
          c_len = 8; p_off = off + 8; p_len = len - 8;
          next = GPD_LT_ETHERNET;
          break;
        }
        default: {  // Payload / Fragment: all of it; LayerPayload nil; next Zero
          c_len = len; p_off = off + len; p_len = 0;
          next = GPD_LT_ZERO;
          break;
        }
      }
      // *decoded = append(*decoded, typ)
      {
        uint64_t code = code_of(typ);
        if (ncount < GPD_CORE_MAX_LAYERS) codes |= code << (16 + 4 * ncount);
        if (EXT) {
          if (ncount < 16) ecodes0 |= code << (4 * ncount);
          else if (ncount < 32) ecodes1 |= code << (4 * (ncount - 16));
        }
        ncount++;
      }
      obj_valid |= 1u << dec;  // Dec order == enum gpd_obj order
      if (EXT) {
#pragma unroll
        for (int k = 0; k < GPD_NOBJ; k++)
          if (k == dec) rec[k] = gpd_layer_rec{c_off, c_len, p_off, p_len};
      }
      if (dec == D_IP4) { ip4_off = c_off; ip4_hl = c_len; last_net = 1; }
      else if (dec == D_IP6) { ip6_off = c_off; last_net = 2; }
      else if (dec == D_TCP) { tcp_off = c_off; tcp_tot = c_len + p_len; last_tp = 1; tp_net = last_net; }
      else if (dec == D_UDP) { udp_off = c_off; udp_tot = c_len + p_len; last_tp = 2; tp_net = last_net; }
      typ = next;
      off = p_off;
      len = p_len;
      if (len == 0) break;  // layers_decoder.go:71-73
      dec = lookup(typ, mask);
      if (dec == D_NONE) { stop = typ; break; }
    }
  }
  goto done;
fail:
  klass = GPD_ST_DECODE_ERROR;
done:
  if (klass != GPD_ST_DECODE_ERROR && stop != 0)
    klass = (options & GPD_OPT_IGNORE_UNSUPPORTED) ? GPD_ST_OK : GPD_ST_UNSUPPORTED;

  uint32_t st = klass | (truncated << 2);
  st |= (ncount > 31 ? 1u : 0u) << 3;
  st |= (ncount > 31 ? 31u : ncount) << 4;
  if (klass == GPD_ST_DECODE_ERROR) st |= err << 9;

  uint64_t nhash = 0, thash = 0;
  uint32_t cs = 0;
  if (!(options & GPD_OPT_NO_FLOW_HASH)) {
    if (last_net == 1) {  // ip4.NetworkFlow(), ip4.go:63-65
      uint32_t w[2];
      load_words(s, ip4_off + 12, w);
      nhash = flow_mix(fnv_word(kFnvBasis, w[0], 4), fnv_word(kFnvBasis, w[1], 4), 1u);
      st |= (1u << 16) | (1u << 20);
    } else if (last_net == 2) {  // ip6.NetworkFlow(), ip6.go:49-51
      uint32_t w[8];
      load_words(s, ip6_off + 8, w);
      uint64_t hs = kFnvBasis, hd = kFnvBasis;
#pragma unroll
      for (int k = 0; k < 4; k++) { hs = fnv_word(hs, w[k], 4); hd = fnv_word(hd, w[k + 4], 4); }
      nhash = flow_mix(hs, hd, 2);
      st |= (1u << 16) | (2u << 20);
    }
    if (last_tp) {  // tcp/udp.TransportFlow(), tcp.go:331-333, udp.go:123-125
      uint32_t w[1];
      load_words(s, last_tp == 1 ? tcp_off : udp_off, w);
      uint32_t ept = last_tp == 1 ? 4u : 5u;
      thash = flow_mix(fnv_word(kFnvBasis, w[0], 2), fnv_word(kFnvBasis, w[0] >> 16, 2), ept);
      st |= (1u << 17) | (ept << 24);
    }
  }
  if (!(options & GPD_OPT_NO_CHECKSUMS)) {
    if (obj_valid & (1u << D_IP4)) {  // checksum(ip4.Contents), ip4.go:158-179
      uint32_t sum = be16_sum(s, ip4_off, 10) + be16_sum(s, ip4_off + 12, ip4_hl - 12);
      cs |= fold_not(sum);
      st |= 1u << 18;
    }
    if (last_tp && tp_net) {  // tcp.ComputeChecksum(), tcp.go:193-195 / tcpip.go:75-88
      uint32_t ps;
      if (tp_net == 1) {
        uint32_t w[2];
        load_words(s, ip4_off + 12, w);
        ps = __builtin_amdgcn_udot4(w[0], 0x00010001u, 0, false) * 256u +
             __builtin_amdgcn_udot4(w[0], 0x01000100u, 0, false) +
             __builtin_amdgcn_udot4(w[1], 0x00010001u, 0, false) * 256u +
             __builtin_amdgcn_udot4(w[1], 0x01000100u, 0, false);
      } else {
        ps = be16_sum(s, ip6_off + 8, 32);
      }
      uint32_t toff = last_tp == 1 ? tcp_off : udp_off;
      uint32_t tot = last_tp == 1 ? tcp_tot : udp_tot;
      ps += last_tp == 1 ? 6u : 17u;
      ps += tot & 0xFFFFu;
      ps += tot >> 16;
      cs |= (uint32_t)fold_not(ps + be16_sum(s, toff, tot)) << 16;
      st |= 1u << 19;
    }
  }
  Out o;
  o.status = st;
  o.layers = codes | (stop & 0xFFFFu);
  o.net_hash = nhash;
  o.tp_hash = thash;
  o.csum = cs;
  if (EXT) {
    gpd_ext_rec e;
    e.layer_codes[0] = ecodes0;
    e.layer_codes[1] = ecodes1;
    e.err_arg0 = klass == GPD_ST_DECODE_ERROR ? a0 : 0;
    e.err_arg1 = klass == GPD_ST_DECODE_ERROR ? a1 : 0;
    e.obj_valid = (uint16_t)obj_valid;
    e.pad0 = 0;
    e.pad1 = 0;
#pragma unroll
    for (int k = 0; k < GPD_NOBJ; k++)
      e.obj[k] = (obj_valid >> k) & 1u ? rec[k] : gpd_layer_rec{0, 0, 0, 0};
    *ext = e;
  }
  return o;
}

// ---------------------------------------------------------------- wave helpers
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

__device__ __forceinline__ void store_out(const KParams &P, uint64_t i, const Out &o) {
  P.status[i] = o.status;
  P.layers[i] = o.layers;
  if (P.net_hash) P.net_hash[i] = o.net_hash;
  if (P.tp_hash) P.tp_hash[i] = o.tp_hash;
  if (P.csum) P.csum[i] = o.csum;
}

// ---------------------------------------------------------------- kernel
template <int STAGE, bool EXT>
__global__ __launch_bounds__(kBlock) void decode_kernel(KParams P) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t stage = wave * STAGE;  // this wave's LDS window
  const uint64_t ntiles = (P.n + 63) / 64;
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;

  for (uint64_t t = (uint64_t)blockIdx.x * kWaves + wave; t < ntiles; t += nwaves) {
    const uint64_t i = t * 64 + lane;
    const bool valid = i < P.n;
    const uint32_t off = valid ? P.offset[i] : 0u;
    const uint32_t len = valid ? P.caplen[i] : 0u;
    bool pending = valid;
    Out o;
    gpd_ext_rec *ext = EXT && valid ? P.ext + i : nullptr;

    // a packet that can never fit a window is decoded from global memory
    if (pending && len > (uint32_t)STAGE - 15u) {
      o = decode_packet<EXT>(GlbSrc{P.data, off}, len, P.tables, P.first, P.decoders, P.options, ext);
      store_out(P, i, o);
      pending = false;
    }
    while (__any(pending)) {
      // window starts at the first pending packet (16-aligned); covers every pending packet
      // that lies wholly inside [base, base + STAGE)
      const uint32_t first_lane = __builtin_ctzll(__ballot(pending));
      const uint32_t base = (uint32_t)__shfl((int)off, first_lane) & ~15u;
      const uint64_t win_end = (uint64_t)base + STAGE;
      const bool in = pending && off >= base && (uint64_t)off + len <= win_end;
      const uint32_t need = wave_max(in ? (uint32_t)((uint64_t)off + len - base) : 0u);
      const uint32_t nbytes = (need + 15u) & ~15u;
      // 16-byte LDS-DMA, 1 KiB per wave instruction, LDS destination lane-linear
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      for (uint32_t c = 0; c < nbytes; c += 1024u) {
        const uint32_t b = c + lane * 16u;
        if (b < nbytes)
          __builtin_amdgcn_global_load_lds(
              (const void *)(P.data + base + b),
              (__attribute__((address_space(3))) void *)(g_lds + stage + c), 16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (in) {
        o = decode_packet<EXT>(LdsSrc{stage + (off - base)}, len, P.tables, P.first, P.decoders,
                               P.options, ext);
        store_out(P, i, o);
        pending = false;
      }
    }
  }
}

template <int STAGE, bool EXT>
static hipError_t launch_t(const KParams &P, hipStream_t stream, int num_cus) {
  const uint64_t ntiles = (P.n + 63) / 64;
  uint64_t blocks = (ntiles + kWaves - 1) / kWaves;
  const uint64_t cap = (uint64_t)num_cus * 16;  // grid-stride beyond 16 workgroups per CU
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return hipSuccess;
  const size_t lds = (size_t)STAGE * kWaves + 64;  // +64: tail reads past the last window stay in bounds
  hipLaunchKernelGGL((decode_kernel<STAGE, EXT>), dim3((unsigned)blocks), dim3(kBlock), lds, stream, P);
  return hipGetLastError();
}

hipError_t launch_decode(const KParams &P, hipStream_t stream, int num_cus) {
  if (P.ext) return launch_t<8192, true>(P, stream, num_cus);
  return launch_t<8192, false>(P, stream, num_cus);
}

}  // namespace gpd
