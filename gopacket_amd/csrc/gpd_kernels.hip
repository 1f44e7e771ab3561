// gpd_kernels.hip — MI355X (gfx950) batched DecodingLayerParser kernels.
//
// One wavefront lane per packet.  A wave owns a tile of 64 consecutive packet
// indices; the byte range those packets occupy in the batch buffer is staged
// HBM -> LDS with 16-byte LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
// instruction, fully coalesced) into one of the wave's two LDS windows, and every
// lane runs the DecodingLayerParser loop for its packet out of LDS while the next
// tile's bytes are already in flight into the other window (double buffering).
// The decode loop, the IPv4 header checksum, the TCP/UDP pseudo-header checksum
// and both flow FastHashes are fused, so packet bytes leave HBM exactly once.
//
// LDS windows are XOR-free "slot rotated": 16-byte slot g of a window is stored at
// slot (g & ~15) | ((g + (g >> 4)) & 15), so lanes walking packets at a power-of-two
// stride (64 B, 128 B...) spread over the LDS banks instead of piling on two.
// Packets that do not fit the first window are decoded in further windows of the
// same tile; a packet larger than a window is decoded straight from global memory
// (same code, other byte source).  Dispatch tables are sparse hashes held in LDS.
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

#include <cstdlib>

#include "gpd_internal.h"

namespace gpd {

constexpr uint32_t kDiagSkipDecode = 1u << 31;  // internal diagnostic option (bench --ablate nodecode)
constexpr uint32_t kDiagNoWait = 1u << 30;      // internal diagnostic: skip the per-tile DMA wait

extern __shared__ __attribute__((aligned(16))) uint8_t g_lds[];

__device__ __forceinline__ uint32_t lds_u32(uint32_t a) {
  return *reinterpret_cast<const uint32_t *>(g_lds + a);
}

// ---------------------------------------------------------------- byte sources
// Logical window byte x -> physical LDS byte (slot rotation inside 256-byte blocks).
__device__ __forceinline__ uint32_t swz_slot(uint32_t g) { return (g & ~15u) | ((g + (g >> 4)) & 15u); }
__device__ __forceinline__ uint32_t unswz_slot(uint32_t s) { return (s & ~15u) | ((s - (s >> 4)) & 15u); }

struct LdsSrc {
  uint32_t buf;  // LDS byte address of the window
  uint32_t pos;  // logical offset of the packet's first byte in the window
  __device__ __forceinline__ uint32_t abs(uint32_t rel) const { return pos + rel; }
  __device__ __forceinline__ uint32_t phys(uint32_t x) const {
    return buf + (swz_slot(x >> 4) << 4) + (x & 15u);
  }
  __device__ __forceinline__ uint32_t dw(uint32_t x) const { return lds_u32(phys(x)); }  // x 4-aligned
  __device__ __forceinline__ uint32_t u8(uint32_t rel) const { return g_lds[phys(pos + rel)]; }
  __device__ __forceinline__ uint4 q(uint32_t x) const {  // x 16-aligned
    return *reinterpret_cast<const uint4 *>(g_lds + buf + (swz_slot(x >> 4) << 4));
  }
};

// Global memory: byte offsets into the batch buffer (16-aligned base pointer).
struct GlbSrc {
  const uint8_t *data;
  uint64_t pos;  // offset of the packet's first byte
  __device__ __forceinline__ uint64_t abs(uint32_t rel) const { return pos + rel; }
  __device__ __forceinline__ uint32_t dw(uint64_t a) const {
    return *reinterpret_cast<const uint32_t *>(data + a);
  }
  __device__ __forceinline__ uint32_t u8(uint32_t rel) const { return data[pos + rel]; }
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
enum Dec : uint32_t {
  D_ETH, D_DOT1Q, D_IP4, D_IP6, D_IP6EXT, D_TCP, D_UDP, D_VXLAN, D_PAYLOAD, D_FRAG, D_NONE = 15
};

struct TE {        // a dispatch-table result
  uint32_t lt;     // LayerType (0: none / unknown)
  uint32_t ent;    // its type-LUT entry: decoder id (15 = not registered) | layer code << 4
};

template <bool PAGES>
struct Tab {
  const uint16_t *pages;
  uint32_t eth_base, tcp_base, udp_base, eth_bits, tcp_bits, udp_bits;

  // type LUT (registered set applied by the host)
  __device__ __forceinline__ uint32_t lut(uint32_t t) const { return t < 128 ? g_lds[t] : 0xFFu; }
  __device__ __forceinline__ TE proto(uint32_t p) const {  // enums_generated.go:151-153
    const uint32_t v = lds_u32(4 * (kHashLutWords + (p & 0xFFu)));
    return TE{v & 0xFFFFu, v >> 16};
  }
  __device__ __forceinline__ TE hash(uint32_t base, uint32_t bits, uint32_t key) const {
    const uint32_t mask = (1u << bits) - 1;
    uint32_t h = key_hash(key, bits);
    for (;;) {  // linear probing; an empty slot ends it (the host bounds probes at 8)
      const uint32_t v = lds_u32(4 * (base + h));
      if (v == 0) return TE{0u, 0xFFu};
      if ((v >> 16) == key) return TE{(v >> 8) & 0xFFu, v & 0xFFu};
      h = (h + 1) & mask;
    }
  }
  __device__ __forceinline__ TE page(uint32_t dir, uint32_t key) const {
    const uint32_t pg = pages[dir + (key >> 8)];
    const uint32_t lt = pages[kTabPages + pg * 256u + (key & 0xFFu)];
    return TE{lt, lut(lt)};
  }
  __device__ __forceinline__ TE eth(uint32_t et) const {  // enums_generated.go:77-79
    return PAGES ? page(kTabEthDir, et) : hash(eth_base, eth_bits, et);
  }
  __device__ __forceinline__ TE tcp(uint32_t port) const {  // ports.go:54-60 (raw)
    return PAGES ? page(kTabTcpDir, port) : hash(tcp_base, tcp_bits, port);
  }
  __device__ __forceinline__ TE udp(uint32_t port) const {  // ports.go:97-103 (raw)
    return PAGES ? page(kTabUdpDir, port) : hash(udp_base, udp_bits, port);
  }
};

// TCP/UDP NextLayerType: dst port table, else src port table; 0 => Payload
// (tcp.go:308-314, udp.go:105-110).  Both lookups are issued together.
__device__ __forceinline__ TE ports_next(TE d, TE s, uint32_t payload_ent) {
  d = d.lt ? d : TE{(uint32_t)GPD_LT_PAYLOAD, payload_ent};
  s = s.lt ? s : TE{(uint32_t)GPD_LT_PAYLOAD, payload_ent};
  return d.lt != GPD_LT_PAYLOAD ? d : s;
}

// ---------------------------------------------------------------- checksums / hashes
// Exact (mod 2^32) sum of the big-endian 16-bit words of packet bytes [rel, rel+len)
// as tcpipChecksum accumulates them (tcpip.go:57-65; an odd last byte counts <<8):
// S = 256*E + O with E/O the byte sums at even/odd positions of the range, taken
// with v_dot4_u32_u8 against 0/1 byte weights that also carry the edge masks.
template <class S>
__device__ __forceinline__ uint32_t be16_sum(const S &s, uint32_t rel, uint32_t len) {
  auto A = s.abs(rel);
  const auto end = A + len;
  const uint32_t ew = (A & 1) ? 0x01000100u : 0x00010001u;
  const uint32_t ow = ew ^ 0x01010101u;
  uint32_t E = 0, O = 0;
  for (auto C = A & ~decltype(A)(15); C < end; C += 16) {
    const uint4 v = s.q(C);
    const uint32_t x[4] = {v.x, v.y, v.z, v.w};
    const uint32_t lo = A > C ? (uint32_t)(A - C) : 0u;
    const uint32_t hi = end - C < 16 ? (uint32_t)(end - C) : 16u;
    const uint32_t m16 = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t bm = (((m16 >> (4 * j)) & 15u) * 0x00204081u) & 0x01010101u;
      E = __builtin_amdgcn_udot4(x[j], ew & bm, E, false);
      O = __builtin_amdgcn_udot4(x[j], ow & bm, O, false);
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

// FNV-1a over the low `nbytes` bytes of little-endian word w, flows.go:60-67.
// h * prime = h * 0x1b3 + (h << 40) (fnvPrime = 2^40 + 0x1b3).
__device__ __forceinline__ uint64_t fnv_word(uint64_t h, uint32_t w, int nbytes) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    if (j < nbytes) {
      h ^= (uint64_t)((w >> (8 * j)) & 0xFFu);
      h = h * 0x1b3ull + (h << 40);
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

template <bool EXT, bool PAGES, class S>
__device__ __forceinline__ Out decode_packet(const S &s, uint32_t caplen, const Tab<PAGES> &T,
                                             uint32_t first, uint32_t options, gpd_ext_rec *ext) {
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
  uint32_t ent = T.lut(typ);
  uint32_t dec = ent & 15u;
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
          next = T.eth(et).lt;
          break;
        }
        case D_DOT1Q: {  // dot1q.go:29-40
          if (len < 4) { truncated = 1; GPD_FAIL(GPD_E_DOT1Q_TOO_SHORT, len, 0); }
          uint32_t w[1];
          load_words(s, off, w);
          c_len = 4; p_off = off + 4; p_len = len - 4;
          next = T.eth(be16_at(w, 2)).lt;
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
          next = ((ff >> 13) & 1u) || (ff & 0x1FFFu) ? (uint32_t)GPD_LT_FRAGMENT : T.proto(proto).lt;
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
              next = T.proto(use_nh).lt;
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
          next = T.proto(use_nh).lt;
          break;
        }
        case D_IP6EXT: {  // ip6.go:418-432,443-461
          if (len < 2) { truncated = 1; GPD_FAIL(GPD_E_IP6EXT_LT2, len, 0); }
          uint32_t w[1];
          load_words(s, off, w);
          uint32_t actual = byte_at(w, 1) * 8u + 8u;
          if (len < actual) GPD_FAIL(GPD_E_IP6EXT_LT_SPEC, len, actual);
          c_len = actual; p_off = off + actual; p_len = len - actual;
          next = T.proto(byte_at(w, 0)).lt;
          break;
        }
        case D_TCP: {  // tcp.go:229-314
          if (len < 20) { truncated = 1; GPD_FAIL(GPD_E_TCP_TOO_SHORT, len, 0); }
          uint32_t w[4];
          load_words(s, off, w);  // bytes 0..15: ports .. flags
          const TE ld = T.tcp(be16_at(w, 2)), ls = T.tcp(be16_at(w, 0));
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
          next = ports_next(ld, ls, 0).lt;
          break;
        }
        case D_UDP: {  // udp.go:30-56,105-110
          if (len < 8) { truncated = 1; GPD_FAIL(GPD_E_UDP_TOO_SHORT, len, 0); }
          uint32_t w[2];
          load_words(s, off, w);
          const TE ld = T.udp(be16_at(w, 2)), ls = T.udp(be16_at(w, 0));
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
          next = ports_next(ld, ls, 0).lt;
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
        const uint64_t code = ent >> 4;
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
          if ((uint32_t)k == dec) rec[k] = gpd_layer_rec{c_off, c_len, p_off, p_len};
      }
      if (dec == D_IP4) { ip4_off = c_off; ip4_hl = c_len; last_net = 1; }
      else if (dec == D_IP6) { ip6_off = c_off; last_net = 2; }
      else if (dec == D_TCP) { tcp_off = c_off; tcp_tot = c_len + p_len; last_tp = 1; tp_net = last_net; }
      else if (dec == D_UDP) { udp_off = c_off; udp_tot = c_len + p_len; last_tp = 2; tp_net = last_net; }
      typ = next;
      off = p_off;
      len = p_len;
      if (len == 0) break;  // layers_decoder.go:71-73
      ent = T.lut(typ);
      dec = ent & 15u;
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
  uint32_t v4[2] = {0, 0};  // ip4 src/dst words, shared by the net hash and the pseudo-header
  if (last_net == 1 || (last_tp && tp_net == 1)) load_words(s, ip4_off + 12, v4);
  if (!(options & GPD_OPT_NO_FLOW_HASH)) {
    if (last_net == 1) {  // ip4.NetworkFlow(), ip4.go:63-65
      nhash = flow_mix(fnv_word(kFnvBasis, v4[0], 4), fnv_word(kFnvBasis, v4[1], 4), 1u);
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
      uint32_t h[5];
      load_words(s, ip4_off, h);
      h[2] &= 0x0000FFFFu;  // bytes 10-11 read as zero
      uint32_t E = 0, O = 0;
#pragma unroll
      for (int k = 0; k < 5; k++) {
        E = __builtin_amdgcn_udot4(h[k], 0x00010001u, E, false);
        O = __builtin_amdgcn_udot4(h[k], 0x01000100u, O, false);
      }
      uint32_t sum = (E << 8) + O;
      if (ip4_hl > 20) sum += be16_sum(s, ip4_off + 20, ip4_hl - 20);
      cs |= fold_not(sum);
      st |= 1u << 18;
    }
    if (last_tp && tp_net) {  // tcp.ComputeChecksum(), tcp.go:193-195 / tcpip.go:75-88
      uint32_t ps;
      if (tp_net == 1) {
        ps = (__builtin_amdgcn_udot4(v4[0], 0x00010001u, 0, false) +
              __builtin_amdgcn_udot4(v4[1], 0x00010001u, 0, false)) * 256u +
             __builtin_amdgcn_udot4(v4[0], 0x01000100u, 0, false) +
             __builtin_amdgcn_udot4(v4[1], 0x01000100u, 0, false);
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

// ---------------------------------------------------------------- fast path
// Straight-line decode of the stacks that carry nearly all traffic:
//   Ethernet [Dot1Q]{0,2} (IPv4 with IHL 5 | IPv6 without hop-by-hop) (TCP | UDP) [Payload]
// for a 16-byte-aligned packet in an LDS window, with Ethernet as the first layer.  The
// first 80 bytes come in with five ds_read_b128 (conflict-free on the rotated window) and
// every header field is extracted at a compile-time offset.  It returns false — having
// written nothing — as soon as a packet leaves that envelope (options on IPv4, fragments,
// HBH, VXLAN, any decode error, unusual table mappings...), and the caller then runs the
// generic decoder, so results are those of decode_packet in every case.
template <int O, int N>
__device__ __forceinline__ uint32_t word_at(const uint32_t (&h)[N]) {
  static_assert(O / 4 + 1 < N || O % 4 == 0, "window");
  if constexpr (O % 4 == 0) return h[O / 4];
  else return __builtin_amdgcn_alignbyte(h[O / 4 + 1], h[O / 4], O % 4);
}
template <int O, int N>
__device__ __forceinline__ uint32_t fbyte(const uint32_t (&h)[N]) {
  return (h[O / 4] >> (8 * (O % 4))) & 0xFFu;
}
template <int O, int N>
__device__ __forceinline__ uint32_t fbe16(const uint32_t (&h)[N]) {
  return (fbyte<O>(h) << 8) | fbyte<O + 1>(h);
}

struct Fast {
  uint32_t truncated, ncount, stop, net, tp;  // net: 1 v4 / 2 v6; tp: 1 TCP / 2 UDP
  uint64_t codes;
  uint32_t cs;        // ip4 header checksum (low 16)
  uint32_t ps;        // pseudo-header partial sum of the network layer
  uint64_t nhash;
};

struct FastCtx {        // wave-uniform facts about the registered set
  uint32_t eth_code;    // layer code of Ethernet
  uint32_t dq_code;     // layer code of Dot1Q
  bool dq;              // Dot1Q registered
  uint32_t pl_ent;      // LUT entry of Payload
};

// Transport at compile-time offset T4 with `tl` bytes available (the network payload).
template <int T4, bool PAGES>
__device__ __forceinline__ bool fast_tp(const LdsSrc &s, const uint32_t (&h)[20], uint32_t tl,
                                        uint32_t dec, uint32_t code, const Tab<PAGES> &T,
                                        const FastCtx &F, Fast &f, uint32_t &seg_sum,
                                        uint32_t &seg_len, uint64_t &thash) {
  TE next;
  uint32_t plen;
  if (dec == D_TCP) {  // tcp.go:229-314
    if (tl < 20) return false;
    const uint32_t doff = fbyte<T4 + 12>(h) >> 4;
    if (doff < 5) return false;
    const uint32_t ds = doff * 4;
    if (ds > tl) return false;
    for (uint32_t q = 20; q < ds;) {  // OPTIONS, tcp.go:274-300 (errors -> generic path)
      const uint32_t k = s.u8(T4 + q);
      if (k == 0) break;
      uint32_t ol = 1;
      if (k != 1) {
        if (ds - q < 2) return false;
        ol = s.u8(T4 + q + 1);
        if (ol < 2 || ol > ds - q) return false;
      }
      q += ol;
    }
    next = ports_next(T.tcp(fbe16<T4 + 2>(h)), T.tcp(fbe16<T4>(h)), F.pl_ent);
    plen = tl - ds;
    seg_len = tl;
  } else {  // UDP, udp.go:30-56
    if (tl < 8) return false;
    const uint32_t length = fbe16<T4 + 4>(h);
    uint32_t hl;
    if (length >= 8) {
      hl = length;
      if (hl > tl) { f.truncated = 1; hl = tl; }
    } else if (length == 0) {
      hl = tl;
    } else {
      return false;
    }
    next = ports_next(T.udp(fbe16<T4 + 2>(h)), T.udp(fbe16<T4>(h)), F.pl_ent);
    plen = hl - 8;
    seg_len = hl;
  }
  const uint32_t w = word_at<T4>(h);
  thash = flow_mix(fnv_word(kFnvBasis, w, 2), fnv_word(kFnvBasis, w >> 16, 2), dec == D_TCP ? 4u : 5u);
  seg_sum = be16_sum(s, T4, seg_len);
  f.tp = dec == D_TCP ? 1u : 2u;
  f.codes |= (uint64_t)code << (16 + 4 * f.ncount);
  f.ncount++;
  if (plen == 0) return true;
  if ((next.ent & 15u) == D_NONE) { f.stop = next.lt; return true; }
  if ((next.ent & 15u) != D_PAYLOAD) return false;  // e.g. VXLAN, a registered app layer
  f.codes |= (uint64_t)(next.ent >> 4) << (16 + 4 * f.ncount);  // Payload consumes the rest
  f.ncount++;
  return true;
}

// Network layer at compile-time offset L3; `typ` is the LayerType Ethernet/Dot1Q chose.
template <int L3, bool PAGES>
__device__ __forceinline__ bool fast_l3(const LdsSrc &s, const uint32_t (&h)[20], uint32_t len,
                                        TE typ, const Tab<PAGES> &T, const FastCtx &F, Fast &f,
                                        uint32_t &seg_sum, uint32_t &seg_len, uint64_t &thash) {
  const uint32_t ent = typ.ent;
  const uint32_t dec = ent & 15u;
  const uint32_t dl = len - L3;
  TE next;
  uint32_t plen;
  if (dec == D_IP4) {  // ip4.go:188-286
    if (dl < 20) return false;
    const uint32_t w0 = word_at<L3>(h), w1 = word_at<L3 + 4>(h), w2 = word_at<L3 + 8>(h);
    const uint32_t w3 = word_at<L3 + 12>(h), w4 = word_at<L3 + 16>(h);
    if ((w0 & 0x0Fu) != 5u) return false;  // IHL != 5: options walk in the generic path
    const uint32_t length = ((w0 >> 8) & 0xFF00u) | (w0 >> 24);
    if (length < 20) return false;          // 0 (TSO rule) or an error: generic path
    const uint32_t ff = ((w1 >> 8) & 0xFF00u) | (w1 >> 24);
    if (ff & 0x3FFFu) return false;         // MF or fragment offset: Fragment, generic path
    uint32_t dlen = dl;
    if (dl > length) dlen = length;
    else if (dl < length) f.truncated = 1;
    plen = dlen - 20;
    next = T.proto((w2 >> 8) & 0xFFu);
    // checksum(ip4.Contents), ip4.go:158-179 (bytes 10-11 as zero)
    const uint32_t w2z = w2 & 0x0000FFFFu;
    uint32_t E = __builtin_amdgcn_udot4(w0, 0x00010001u, 0, false);
    uint32_t O = __builtin_amdgcn_udot4(w0, 0x01000100u, 0, false);
    E = __builtin_amdgcn_udot4(w1, 0x00010001u, E, false);
    O = __builtin_amdgcn_udot4(w1, 0x01000100u, O, false);
    E = __builtin_amdgcn_udot4(w2z, 0x00010001u, E, false);
    O = __builtin_amdgcn_udot4(w2z, 0x01000100u, O, false);
    uint32_t Ea = __builtin_amdgcn_udot4(w3, 0x00010001u, 0, false);
    uint32_t Oa = __builtin_amdgcn_udot4(w3, 0x01000100u, 0, false);
    Ea = __builtin_amdgcn_udot4(w4, 0x00010001u, Ea, false);
    Oa = __builtin_amdgcn_udot4(w4, 0x01000100u, Oa, false);
    f.cs = fold_not(((E + Ea) << 8) + O + Oa);
    f.ps = (Ea << 8) + Oa;  // src + dst words of the pseudo-header, tcpip.go:26-35
    f.nhash = flow_mix(fnv_word(kFnvBasis, w3, 4), fnv_word(kFnvBasis, w4, 4), 1u);
    f.net = 1;
  } else if (dec == D_IP6) {  // ip6.go:221-278 without hop-by-hop
    if constexpr (L3 > 18) {
      return false;  // transport header would pass the 80-byte register window
    } else {
      if (dl < 40) return false;
      const uint32_t w1 = word_at<L3 + 4>(h);
      const uint32_t nh = (w1 >> 16) & 0xFFu;
      if (nh == 0) return false;
      const uint32_t length = ((w1 & 0xFFu) << 8) | ((w1 >> 8) & 0xFFu);
      if (length == 0) return false;
      plen = dl - 40;
      if (length > plen) f.truncated = 1;
      else plen = length;
      next = T.proto(nh);
      uint64_t hs = kFnvBasis, hd = kFnvBasis;
      uint32_t E = 0, O = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t a = k == 0 ? word_at<L3 + 8>(h) : k == 1 ? word_at<L3 + 12>(h)
                         : k == 2 ? word_at<L3 + 16>(h) : word_at<L3 + 20>(h);
        const uint32_t b = k == 0 ? word_at<L3 + 24>(h) : k == 1 ? word_at<L3 + 28>(h)
                         : k == 2 ? word_at<L3 + 32>(h) : word_at<L3 + 36>(h);
        hs = fnv_word(hs, a, 4);
        hd = fnv_word(hd, b, 4);
        E = __builtin_amdgcn_udot4(a, 0x00010001u, E, false);
        O = __builtin_amdgcn_udot4(a, 0x01000100u, O, false);
        E = __builtin_amdgcn_udot4(b, 0x00010001u, E, false);
        O = __builtin_amdgcn_udot4(b, 0x01000100u, O, false);
      }
      f.ps = (E << 8) + O;  // tcpip.go:37-48
      f.nhash = flow_mix(hs, hd, 2u);
      f.net = 2;
    }
  } else {
    return false;
  }
  f.codes |= (uint64_t)(ent >> 4) << (16 + 4 * f.ncount);
  f.ncount++;
  if (plen == 0) return true;
  const uint32_t d2 = next.ent & 15u;
  if (d2 == D_NONE) { f.stop = next.lt; return true; }
  if (d2 != D_TCP && d2 != D_UDP) return false;
  if (dec == D_IP4)
    return fast_tp<L3 + 20>(s, h, plen, d2, next.ent >> 4, T, F, f, seg_sum, seg_len, thash);
  if constexpr (L3 <= 18)
    return fast_tp<L3 + 40>(s, h, plen, d2, next.ent >> 4, T, F, f, seg_sum, seg_len, thash);
  return false;
}

template <bool PAGES>
__device__ __forceinline__ bool fast_decode(const LdsSrc &s, uint32_t len, const Tab<PAGES> &T,
                                            const FastCtx &F, uint32_t options, Out &o) {
  if (len < 14) return false;
  uint32_t h[20];
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const uint4 v = s.q(s.pos + 16 * k);
    h[4 * k] = v.x; h[4 * k + 1] = v.y; h[4 * k + 2] = v.z; h[4 * k + 3] = v.w;
  }
  Fast f{0, 1, 0, 0, 0, 0, 0, 0, 0};
  f.codes = (uint64_t)F.eth_code << 16;     // Ethernet, ethernet.go:41-62
  const uint32_t et = fbe16<12>(h);
  if (et < 0x0600u) return false;            // 802.3 length framing: generic path
  TE typ = T.eth(et);
  uint32_t seg_sum = 0, seg_len = 0;
  uint64_t thash = 0;
  bool ok;
  if (typ.lt == GPD_LT_DOT1Q && F.dq) {  // dot1q.go:29-50
    if (len < 18) return false;
    f.codes |= (uint64_t)F.dq_code << 20;
    f.ncount = 2;
    typ = T.eth(fbe16<16>(h));
    if (typ.lt == GPD_LT_DOT1Q) {
      if (len < 22) return false;
      f.codes |= (uint64_t)F.dq_code << 24;
      f.ncount = 3;
      typ = T.eth(fbe16<20>(h));
      if (typ.lt == GPD_LT_DOT1Q) return false;
      if (len == 22) return false;  // empty Dot1Q payload: generic path ends the loop there
      ok = fast_l3<22>(s, h, len, typ, T, F, f, seg_sum, seg_len, thash);
    } else {
      if (len == 18) return false;
      ok = fast_l3<18>(s, h, len, typ, T, F, f, seg_sum, seg_len, thash);
    }
  } else {
    if (len == 14) return false;
    ok = fast_l3<14>(s, h, len, typ, T, F, f, seg_sum, seg_len, thash);
  }
  if (!ok) return false;
  // status / layers / hashes / checksums exactly as decode_packet composes them
  uint32_t klass = GPD_ST_OK;
  if (f.stop != 0 && !(options & GPD_OPT_IGNORE_UNSUPPORTED)) klass = GPD_ST_UNSUPPORTED;
  uint32_t st = klass | (f.truncated << 2) | (f.ncount << 4);
  uint64_t nh = 0, th = 0;
  uint32_t cs = 0;
  if (!(options & GPD_OPT_NO_FLOW_HASH)) {
    nh = f.nhash;
    st |= (1u << 16) | (f.net << 20);
    if (f.tp) {
      th = thash;
      st |= (1u << 17) | ((f.tp == 1 ? 4u : 5u) << 24);
    }
  }
  if (!(options & GPD_OPT_NO_CHECKSUMS)) {
    if (f.net == 1) { cs = f.cs; st |= 1u << 18; }
    if (f.tp) {
      uint32_t ps = f.ps + (f.tp == 1 ? 6u : 17u) + (seg_len & 0xFFFFu) + (seg_len >> 16);
      cs |= (uint32_t)fold_not(ps + seg_sum) << 16;
      st |= 1u << 19;
    }
  }
  o.status = st;
  o.layers = f.codes | (f.stop & 0xFFFFu);
  o.net_hash = nh;
  o.tp_hash = th;
  o.csum = cs;
  return true;
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

// The first LDS window of a tile: starts at the first packet that fits a window
// (16-aligned) and covers every packet lying wholly inside [base, base + STAGE).
struct Window {
  uint32_t base, nbytes;
};

template <int STAGE>
__device__ __forceinline__ Window plan_window(bool pending, uint32_t off, uint32_t len) {
  Window w{0, 0};
  const uint64_t m = __ballot(pending);
  if (m == 0) return w;
  const uint32_t first_lane = __builtin_ctzll(m);
  w.base = (uint32_t)__shfl((int)off, first_lane) & ~15u;
  const bool in = pending && off >= w.base && (uint64_t)off + len <= (uint64_t)w.base + STAGE;
  const uint32_t need = wave_max(in ? (uint32_t)((uint64_t)off + len - w.base) : 0u);
  w.nbytes = (need + 15u) & ~15u;
  return w;
}

// One 16-byte LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes land at LDS
// lds_base + 16 l.  Issued from inline asm so the compiler's waitcnt pass does not see it:
// otherwise it cannot tell the in-flight DMA into the other window from this window's
// ds_reads and drains it (vmcnt(0)) before the first one, serialising the prefetch.  Every
// wait on these loads is therefore explicit (s_waitcnt vmcnt(0) before a window is read).
__device__ __forceinline__ void glds16(const uint8_t *gsrc, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_base))
      : "memory");
}

// The window into LDS `buf`: wave instruction c writes physical slots [64c, 64c+64); lane
// l's source is the logical slot that rotates onto slot 64c+l.
__device__ __forceinline__ void issue_window(const uint8_t *data, const Window &w, uint32_t buf,
                                             uint32_t lane) {
  for (uint32_t c = 0; c < w.nbytes; c += 1024u) {
    const uint32_t g = unswz_slot((c >> 4) + lane);
    if ((g << 4) < w.nbytes) glds16(data + w.base + (g << 4), buf + c);
  }
}

// ---------------------------------------------------------------- kernel
// WAVES waves per workgroup; MINW = waves per SIMD the register allocation must allow.
template <int STAGE, bool EXT, bool PAGES, int WAVES, int MINW>
__global__ __launch_bounds__(64 * WAVES, MINW) void decode_kernel(KParams P) {
  constexpr int kWaves = WAVES, kBlock = 64 * WAVES;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = threadIdx.x >> 6;
  // stage the dispatch-table image (LUT, ipproto, hashes) into LDS
  for (uint32_t k = threadIdx.x; k < P.image_words; k += kBlock)
    reinterpret_cast<uint32_t *>(g_lds)[k] = P.image[k];
  __syncthreads();
  const Tab<PAGES> T{P.pages, P.eth_base, P.tcp_base, P.udp_base, P.eth_bits, P.tcp_bits, P.udp_bits};
  const uint32_t img = (P.image_words * 4u + 15u) & ~15u;
  const uint32_t bufs = img + wave * 2u * STAGE;
  const uint64_t ntiles = (P.n + 63) / 64;
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint32_t fits = (uint32_t)STAGE - 15u;  // a packet of <= fits bytes always fits a window
  // the fast path assumes Ethernet first (DecodingLayerParser built with LayerTypeEthernet)
  const bool fast_ok = !PAGES && P.first == GPD_LT_ETHERNET && (T.lut(GPD_LT_ETHERNET) & 15u) == D_ETH;
  const FastCtx F{T.lut(GPD_LT_ETHERNET) >> 4, T.lut(GPD_LT_DOT1Q) >> 4,
                  (T.lut(GPD_LT_DOT1Q) & 15u) == D_DOT1Q, T.lut(GPD_LT_PAYLOAD)};

  uint64_t t = (uint64_t)blockIdx.x * kWaves + wave;
  if (t >= ntiles) return;
  uint32_t cur = 0;
  uint64_t i = t * 64 + lane;
  bool valid = i < P.n;
  uint32_t off = valid ? P.offset[i] : 0u, len = valid ? P.caplen[i] : 0u;
  Window W = plan_window<STAGE>(valid && len <= fits, off, len);
  issue_window(P.data, W, bufs, lane);
  // descriptors of the next tile
  uint64_t tn = t + nwaves;
  uint64_t in_ = tn * 64 + lane;
  bool valid_n = tn < ntiles && in_ < P.n;
  uint32_t off_n = valid_n ? P.offset[in_] : 0u, len_n = valid_n ? P.caplen[in_] : 0u;

  for (;;) {
    // this tile's window and the next tile's descriptors were issued one decode ago
    if (!(P.options & kDiagNoWait)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const bool has_next = tn < ntiles;
    Window Wn{0, 0};
    if (has_next) {  // next tile's first window streams in while this tile decodes
      Wn = plan_window<STAGE>(valid_n && len_n <= fits, off_n, len_n);
      issue_window(P.data, Wn, bufs + (cur ^ 1u) * STAGE, lane);
    }
    // descriptors two tiles ahead
    const uint64_t tnn = tn + nwaves;
    const uint64_t inn = tnn * 64 + lane;
    const bool valid_nn = tnn < ntiles && inn < P.n;
    const uint32_t off_nn = valid_nn ? P.offset[inn] : 0u, len_nn = valid_nn ? P.caplen[inn] : 0u;

    const uint32_t buf = bufs + cur * STAGE;
    gpd_ext_rec *ext = EXT && valid ? P.ext + i : nullptr;
    bool pending = valid;
    Out o;
    if (pending && len > fits) {  // larger than a window: straight from global memory
      o = decode_packet<EXT>(GlbSrc{P.data, off}, len, T, P.first, P.options, ext);
      store_out(P, i, o);
      pending = false;
    }
    bool firstw = true;
    while (__any(pending)) {
      if (!firstw) {  // further windows of this tile (rare: tiles wider than a window)
        W = plan_window<STAGE>(pending, off, len);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue_window(P.data, W, buf, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      firstw = false;
      const bool in = pending && off >= W.base && (uint64_t)off + len <= (uint64_t)W.base + STAGE;
      if (in && (P.options & kDiagSkipDecode)) {  // diagnostics: data movement only
        o = Out{g_lds[buf + ((off - W.base) & ~15u)], 0, 0, 0, 0};
        store_out(P, i, o);
        pending = false;
      } else if (in) {
        const LdsSrc src{buf, off - W.base};
        bool done = false;
        if (!EXT && fast_ok && (src.pos & 15u) == 0) done = fast_decode<PAGES>(src, len, T, F, P.options, o);
        if (!done) o = decode_packet<EXT>(src, len, T, P.first, P.options, ext);
        store_out(P, i, o);
        pending = false;
      }
    }
    if (!has_next) break;
    t = tn;
    i = in_;
    valid = valid_n;
    off = off_n;
    len = len_n;
    W = Wn;
    tn = tnn;
    in_ = inn;
    valid_n = valid_nn;
    off_n = off_nn;
    len_n = len_nn;
    cur ^= 1u;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

template <int STAGE, bool EXT, bool PAGES, int WAVES, int MINW>
static hipError_t launch_t(const KParams &P, hipStream_t stream, int num_cus) {
  const uint64_t ntiles = (P.n + 63) / 64;
  const size_t img = (P.image_words * 4u + 15u) & ~15u;
  const size_t lds = img + (size_t)STAGE * 2 * WAVES + 320;  // slack: rotated reads past a window end
  const uint64_t per_cu = (160u * 1024u) / lds;               // resident workgroups per CU (LDS)
  uint64_t blocks = (ntiles + WAVES - 1) / WAVES;
  const uint64_t cap = (uint64_t)num_cus * (per_cu ? per_cu : 1) * 4;  // a few tiles per wave
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((decode_kernel<STAGE, EXT, PAGES, WAVES, MINW>), dim3((unsigned)blocks),
                     dim3(64 * WAVES), lds, stream, P);
  return hipGetLastError();
}

// Geometry variants (diagnostic selector GPD_GEOM: 0 = 4 waves/WG, 1 = 2 waves/WG with a
// 5-waves-per-SIMD register budget, 2 = 4 waves/WG with that budget, 3 = 2 waves/WG).
static int geom() {
  static int g = -1;
  if (g < 0) {
    const char *e = getenv("GPD_GEOM");
    g = e ? atoi(e) : 0;
  }
  return g;
}

template <bool EXT, bool PAGES>
static hipError_t launch_s(const KParams &P, hipStream_t stream, int num_cus) {
  const int g = geom();
  switch (P.stage) {
    case 4096:
      if (g == 1) return launch_t<4096, EXT, PAGES, 2, 5>(P, stream, num_cus);
      if (g == 2) return launch_t<4096, EXT, PAGES, 4, 5>(P, stream, num_cus);
      if (g == 3) return launch_t<4096, EXT, PAGES, 2, 1>(P, stream, num_cus);
      return launch_t<4096, EXT, PAGES, 4, 1>(P, stream, num_cus);
    default:
      if (g == 1) return launch_t<8192, EXT, PAGES, 2, 5>(P, stream, num_cus);
      if (g == 2) return launch_t<8192, EXT, PAGES, 4, 5>(P, stream, num_cus);
      if (g == 3) return launch_t<8192, EXT, PAGES, 2, 1>(P, stream, num_cus);
      return launch_t<8192, EXT, PAGES, 4, 1>(P, stream, num_cus);
  }
}

hipError_t launch_decode(const KParams &P, hipStream_t stream, int num_cus) {
  if (P.ext) return P.use_pages ? launch_s<true, true>(P, stream, num_cus)
                                : launch_s<true, false>(P, stream, num_cus);
  return P.use_pages ? launch_s<false, true>(P, stream, num_cus)
                     : launch_s<false, false>(P, stream, num_cus);
}

}  // namespace gpd

#ifdef GPD_ISA_PROBE
// Instruction-count probe (not built into libgpd.so): the fast path alone on one packet.
namespace gpd {
__global__ void probe_fast(KParams P) {
  const uint32_t pos = P.offset[threadIdx.x], len = P.caplen[threadIdx.x];
  const Tab<false> T{P.pages, P.eth_base, P.tcp_base, P.udp_base, P.eth_bits, P.tcp_bits, P.udp_bits};
  Out o{};
  const FastCtx F{1, 2, true, 0xC8};
  const bool ok = fast_decode<false>(LdsSrc{0, pos}, len, T, F, P.options, o);
  const uint32_t i = threadIdx.x;
  if (ok) store_out(P, i, o);
}
}  // namespace gpd
#endif
