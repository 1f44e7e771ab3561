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

#include <algorithm>

#include "gpd_internal.h"

namespace gpd {

constexpr uint64_t kGridRounds = 4;  // a launch covers at most 4 rounds of resident workgroups
// The two diagnostic bits (bench --ablate nodecode / nowait) exist only in the diagnostic
// library (libgpd_diag.so, built with -DGPD_DIAG): there the runtime accepts them; in the
// shipped libgpd.so they are refused by gpd_ctx_set_options / gpd_ctx_create and every branch
// that reads them compiles away (kDiagBuild false => both constants 0).
#ifdef GPD_DIAG
constexpr bool kDiagBuild = true;
#else
constexpr bool kDiagBuild = false;
#endif
constexpr uint32_t kDiagSkipDecodeBit = 1u << 31, kDiagNoWaitBit = 1u << 30;
constexpr uint32_t kDiagSkipDecode = kDiagBuild ? kDiagSkipDecodeBit : 0u;  // stream only, no decode
constexpr uint32_t kDiagNoWait = kDiagBuild ? kDiagNoWaitBit : 0u;          // skip the per-tile DMA wait
constexpr uint32_t kDiagNtLoad = 1u << 29;      // A/B: window LDS-DMA with the nt cache policy
constexpr uint32_t kDiagNtStore = 1u << 28;     // A/B: result stores with the nt cache policy
constexpr uint32_t kShiftWindows = 1u << 27;    // internal: register-staged windows copied shifted
constexpr uint32_t kRegPrefix = 1u << 26;       // internal: 8 KiB windows of long frames (IMIX)
constexpr uint32_t kHeaderOnce = 1u << 25;      // internal: 8 KiB windows decoded once per tile (seg_pass)
constexpr uint32_t kRounds = 1u << 24;          // internal: header-once over 8 KiB rounds (ro_kernel)
constexpr uint32_t kDiagMask = kDiagSkipDecodeBit | kDiagNoWaitBit | kDiagNtLoad | kDiagNtStore | kShiftWindows |
                               kRegPrefix | kHeaderOnce | kRounds;
// A/B builds only (GPD_EXTRA_CFLAGS=-DGPD_EXP=..., tools/ab_exp.sh): a fast-path variant under
// test reads kExp inside an `#if GPD_EXP` block; the shipped library has none.
#ifndef GPD_EXP
#define GPD_EXP 0
#endif
[[maybe_unused]] constexpr uint32_t kExp = GPD_EXP;

extern __shared__ __attribute__((aligned(16))) uint8_t g_lds[];

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

#ifdef GPD_PHASE_TIMING
// Diagnostic build only (libgpd_phase.so): per-phase shader-clock totals of the fast kernel's
// loop, summed over waves; read back with gpd_diag_phase().
__device__ unsigned long long g_phase[8];
#define PH_DECL uint64_t ph_t = __builtin_amdgcn_s_memtime(), ph_acc[6] = {0, 0, 0, 0, 0, 0};
#define PH_MARK(k)                                      \
  do {                                                  \
    const uint64_t ph_n = __builtin_amdgcn_s_memtime(); \
    ph_acc[k] += ph_n - ph_t;                           \
    ph_t = ph_n;                                        \
  } while (0)
#define PH_FLUSH                                                              \
  do {                                                                        \
    if (lane == 0)                                                            \
      for (int k = 0; k < 6; k++) atomicAdd(&g_phase[k], (unsigned long long)ph_acc[k]); \
  } while (0)
#else
#define PH_DECL
#define PH_MARK(k) do {} while (0)
#define PH_FLUSH do {} while (0)
#endif

__device__ __forceinline__ uint32_t lds_u32(uint32_t a) {
  return *reinterpret_cast<const uint32_t *>(g_lds + a);
}

// ---------------------------------------------------------------- byte sources
// Logical window byte x -> physical LDS byte (slot rotation inside 256-byte blocks).
__device__ __forceinline__ uint32_t swz_slot(uint32_t g) { return (g & ~15u) | ((g + (g >> 4)) & 15u); }
__device__ __forceinline__ uint32_t unswz_slot(uint32_t s) { return (s & ~15u) | ((s - (s >> 4)) & 15u); }

// SWZ: the window's 16-byte slots are rotated (see the file comment); otherwise linear.
template <bool SWZ>
struct LdsSrc {
  uint32_t buf;  // LDS byte address of the window
  uint32_t pos;  // logical offset of the packet's first byte in the window
  __device__ __forceinline__ uint32_t abs(uint32_t rel) const { return pos + rel; }
  __device__ __forceinline__ uint32_t phys(uint32_t x) const {
    return SWZ ? buf + (swz_slot(x >> 4) << 4) + (x & 15u) : buf + x;
  }
  __device__ __forceinline__ uint32_t dw(uint32_t x) const { return lds_u32(phys(x)); }  // x 4-aligned
  __device__ __forceinline__ uint32_t u8(uint32_t rel) const { return g_lds[phys(pos + rel)]; }
  __device__ __forceinline__ uint4 q(uint32_t x) const {  // x 16-aligned
    return *reinterpret_cast<const uint4 *>(g_lds + phys(x));
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

// A fallback packet whose first K bytes (from its 16-aligned global start) a lane staged in
// its own LDS slot: reads below that bound come from LDS, the rest (long segments' checksums)
// from global memory.  The generic decoder's chain of dependent header reads then costs LDS
// latency instead of HBM latency (rs_kernel's end-of-wave fallback lists).
template <uint32_t K>
struct HybSrc {
  const uint8_t *data;
  uint64_t pos;    // global offset of the packet's first byte
  uint64_t gbase;  // pos & ~15: global offset of slot byte 0
  uint32_t slot;   // LDS address of the lane's slot
  __device__ __forceinline__ uint64_t abs(uint32_t rel) const { return pos + rel; }
  __device__ __forceinline__ uint32_t dw(uint64_t a) const {
    return a - gbase < K ? lds_u32(slot + (uint32_t)(a - gbase)) : *reinterpret_cast<const uint32_t *>(data + a);
  }
  __device__ __forceinline__ uint32_t u8(uint32_t rel) const {
    const uint64_t a = pos + rel;
    return a - gbase < K ? (uint32_t)g_lds[slot + (uint32_t)(a - gbase)] : (uint32_t)data[a];
  }
  __device__ __forceinline__ uint4 q(uint64_t a) const {
    return a - gbase < K ? *reinterpret_cast<const uint4 *>(g_lds + slot + (uint32_t)(a - gbase))
                         : *reinterpret_cast<const uint4 *>(data + a);
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
  D_ETH, D_DOT1Q, D_IP4, D_IP6, D_IP6EXT, D_TCP, D_UDP, D_VXLAN, D_PAYLOAD, D_FRAG, D_ICMP4,
  D_LLC, D_NONE = 15
};

struct TE {        // a dispatch-table result
  uint32_t lt;     // LayerType (0: none / unknown)
  uint32_t ent;    // its type-LUT entry: decoder id (15 = not registered) | layer code << 4
};

template <bool PAGES>
struct Tab {
  const uint16_t *pages;
  uint32_t eth_base, tcp_base, udp_base, eth_bits, tcp_bits, udp_bits, eth_mult, tcp_mult, udp_mult;

  // type LUT (registered set applied by the host)
  __device__ __forceinline__ uint32_t lut(uint32_t t) const { return t < 128 ? g_lds[t] : 0xFFu; }
  __device__ __forceinline__ TE proto(uint32_t p) const {  // enums_generated.go:151-153
    const uint32_t v = lds_u32(4 * (kHashLutWords + (p & 0xFFu)));
    return TE{v & 0xFFFFu, v >> 16};
  }
  // Raw slot of `key` in a two-way bucketed hash: LayerType << 8 | LUT entry in the low 16
  // bits (0x00FF on a miss: LayerType 0, not registered).  One ds_read_b64, no loop.
  __device__ __forceinline__ uint32_t bucket(uint32_t base, uint32_t mult, uint32_t bits,
                                             uint32_t key) const {
    const uint32_t b = __builtin_amdgcn_ubfe(key * mult, 16 - bits, bits);
    const uint2 v = *reinterpret_cast<const uint2 *>(g_lds + 4 * base + 8 * b);
    return (v.x >> 16) == key ? v.x : ((v.y >> 16) == key ? v.y : 0xFFu);
  }
  __device__ __forceinline__ TE hash(uint32_t base, uint32_t mult, uint32_t bits, uint32_t key) const {
    const uint32_t r = bucket(base, mult, bits, key);
    return TE{(r >> 8) & 0xFFu, r & 0xFFu};
  }
  __device__ __forceinline__ TE page(uint32_t dir, uint32_t key) const {
    const uint32_t pg = pages[dir + (key >> 8)];
    const uint32_t lt = pages[kTabPages + pg * 256u + (key & 0xFFu)];
    return TE{lt, lut(lt)};
  }
  __device__ __forceinline__ TE eth(uint32_t et) const {  // enums_generated.go:77-79
    return PAGES ? page(kTabEthDir, et) : hash(eth_base, eth_mult, eth_bits, et);
  }
  __device__ __forceinline__ TE tcp(uint32_t port) const {  // ports.go:54-60 (raw)
    return PAGES ? page(kTabTcpDir, port) : hash(tcp_base, tcp_mult, tcp_bits, port);
  }
  __device__ __forceinline__ TE udp(uint32_t port) const {  // ports.go:97-103 (raw)
    return PAGES ? page(kTabUdpDir, port) : hash(udp_base, udp_mult, udp_bits, port);
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

// FNV-1a (flows.go:60-67) with fnvPrime = 2^40 + 0x1b3: h * prime = h * 0x1b3 + (h << 40), the
// 64-bit state as two words (one 32x32->64 multiply per byte).
struct H64 {
  uint32_t lo, hi;
};
__device__ __forceinline__ H64 fnv_mulp(H64 h) {
  const uint64_t p = (uint64_t)h.lo * 0x1b3u;
  return H64{(uint32_t)p, h.hi * 0x1b3u + (uint32_t)(p >> 32) + (h.lo << 8)};
}
constexpr uint64_t kFnvC0 = (kFnvBasis & ~0xFFull) * kFnvPrime;  // (basis with byte 0 cleared) * prime
// fnvHash of the NB low bytes of w (byte 0 first), from the basis
template <int NB>
__device__ __forceinline__ H64 fnv_start(uint32_t w) {
  static_assert(NB == 2 || NB == 4, "fnv_start<2|4>");
  // byte 0 in closed form: (basis ^ b) * prime = C0 + c * 0x1b3 + (c << 40), c = b ^ 0x25
  const uint32_t c = (w & 0xFFu) ^ (uint32_t)(kFnvBasis & 0xFFu);
  const uint64_t r = (uint64_t)c * 0x1b3u + kFnvC0;
  H64 x{(uint32_t)r, (uint32_t)(r >> 32) + (c << 8)};
#pragma unroll
  for (int j = 1; j < NB; j++) {
    x.lo ^= (w >> (8 * j)) & 0xFFu;
    x = fnv_mulp(x);
  }
  return x;
}
__device__ __forceinline__ H64 fnv_more(H64 x, uint32_t w) {  // four more bytes
#pragma unroll
  for (int j = 0; j < 4; j++) {
    x.lo ^= (w >> (8 * j)) & 0xFFu;
    x = fnv_mulp(x);
  }
  return x;
}
// Flow.FastHash, flows.go:167-174
__device__ __forceinline__ uint64_t flow_fast(H64 s, H64 d, uint32_t ept) {
  const uint64_t sum = (((uint64_t)s.hi << 32) | s.lo) + (((uint64_t)d.hi << 32) | d.lo);
  const H64 x = fnv_mulp(H64{(uint32_t)sum ^ ept, (uint32_t)(sum >> 32)});
  return ((uint64_t)x.hi << 32) | x.lo;
}

// ---------------------------------------------------------------- one packet
struct Out {
  uint32_t status;
  uint64_t layers;
  uint64_t net_hash, tp_hash;
  uint32_t csum;
  uint32_t hoff;  // gpd.h header offsets word
};

__device__ __forceinline__ uint32_t hdr_word(bool net, uint32_t net_off, bool tp, uint32_t tp_off) {
  return (net ? min(net_off, 0xFFFFu) : 0xFFFFu) | ((tp ? min(tp_off, 0xFFFFu) : 0xFFFFu) << 16);
}

#define GPD_FAIL(code, x0, x1) \
  do { err = (code); a0 = (x0); a1 = (x1); goto fail; } while (0)

template <bool EXT, bool PAGES, class S>
__device__ __forceinline__ Out decode_packet(const S &s, uint32_t caplen, const Tab<PAGES> &T,
                                             uint32_t first, uint32_t options, gpd_ext_rec *ext,
                                             gpd_detail *det = nullptr) {
  uint32_t truncated = 0, err = 0, a0 = 0, a1 = 0;
  uint32_t ncount = 0;
  // decoded[0..11] in `codes` (the core word), [12..15] in hcodes, [16..31] in ecodes1
  uint64_t codes = 0, ecodes1 = 0;
  uint32_t hcodes = 0;
  uint32_t stop = 0, klass = GPD_ST_OK;
  // final state of the objects the fused outputs read: where their addresses / ports were read
  // (ip4_off, ip6_off, tcp_poff, udp_off) and their Contents+Payload (ip4_hl, tcp_off/tcp_tot,
  // udp_off/udp_tot) — the last successful decode of each kind, or what a failing call of that
  // kind assigned after it (the fail block)
  uint32_t ip4_off = 0, ip4_hl = 0, ip6_off = 0;
  uint32_t tcp_off = 0, tcp_tot = 0, tcp_poff = 0, udp_off = 0, udp_tot = 0;
  uint32_t err_dec = GPD_NOBJ_NONE, err_wrote = 0;
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
        case D_ICMP4: {  // icmp4.go:220-231; NextLayerType :261-263
          if (len < 8) { truncated = 1; GPD_FAIL(GPD_E_ICMP4_TOO_SMALL, 0, 0); }
          c_len = 8; p_off = off + 8; p_len = len - 8;
          next = GPD_LT_PAYLOAD;
          break;
        }
        case D_LLC: {  // llc.go:31-52; NextLayerType :61-69
          if (len < 3) GPD_FAIL(GPD_E_LLC_TOO_SMALL, 0, 0);
          const uint32_t dsap = s.u8(off) & 0xFEu, ssap = s.u8(off + 1) & 0xFEu;
          const uint32_t ctl = s.u8(off + 2);
          c_len = 3;
          if (!(ctl & 1u) || (ctl & 3u) == 1u) {  // two-byte control field
            if (len < 4) GPD_FAIL(GPD_E_LLC_TOO_SMALL, 0, 0);
            c_len = 4;
          }
          p_off = off + c_len; p_len = len - c_len;
          next = (dsap == 0xAAu && ssap == 0xAAu) ? (uint32_t)GPD_LT_SNAP
               : (dsap == 0x42u && ssap == 0x42u) ? (uint32_t)GPD_LT_STP : (uint32_t)GPD_LT_ZERO;
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
        else if (ncount < 16) hcodes |= (uint32_t)code << (4 * (ncount - GPD_CORE_MAX_LAYERS));
        else if (ncount < 32) ecodes1 |= code << (4 * (ncount - 16));
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
      else if (dec == D_TCP) { tcp_off = tcp_poff = c_off; tcp_tot = c_len + p_len; last_tp = 1; tp_net = last_net; }
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
  {
    // What the failing DecodeFromBytes assigned to its reused object before returning
    // (gpd.h gpd_ext_rec.err_wrote): header fields from `off` (1), and BaseLayer too (2).
    uint32_t ec_len = 0, ep_off = 0, ep_len = 0;
    if (dec == D_IP4 && err != GPD_E_IP4_TOO_SHORT) {  // ip4.go:195-210, 235-236
      err_wrote = 2;
      ec_len = len; ep_off = off + len;                // Contents = data, Payload nil
      if (err >= GPD_E_IP4_OPT_LT2) {                  // options: the header split stands
        uint32_t w[1];
        load_words(s, off, w);
        uint32_t length = be16_at(w, 2);
        if (length == 0) length = len & 0xFFFFu;
        ec_len = (byte_at(w, 0) & 0x0Fu) * 4u;
        ep_off = off + ec_len;
        ep_len = min(len, length) - ec_len;
      }
    } else if (dec == D_IP6 && err != GPD_E_IP6_TOO_SHORT) {  // ip6.go:226-235
      err_wrote = 2;
      ec_len = 40; ep_off = off + 40; ep_len = len - 40;
    } else if (dec == D_TCP && err != GPD_E_TCP_TOO_SHORT) {  // tcp.go:234-268
      err_wrote = err == GPD_E_TCP_DOFF_LT5 ? 1u : 2u;
      ec_len = len; ep_off = off + len;                // doff overrun: Contents = data
      if (err >= GPD_E_TCP_OPT_LT2_REM) {              // options: the header split stands
        ec_len = (s.u8(off + 12) >> 4) * 4u;
        ep_off = off + ec_len;
        ep_len = len - ec_len;
      }
    } else if (dec == D_UDP && err == GPD_E_UDP_LEN_TOO_SMALL) {  // udp.go:35-41
      err_wrote = 2;
      ec_len = 8; ep_off = off + 8;                    // Contents = data[:8], Payload nil
    } else if (dec == D_LLC && len >= 3) {             // llc.go:35-39
      err_wrote = 1;
    }
    err_dec = dec;
    if (err_wrote && ((obj_valid >> dec) & 1u)) {  // only kinds in decoded feed the outputs
      if (dec == D_IP4) { ip4_off = off; ip4_hl = ec_len; }
      else if (dec == D_IP6) ip6_off = off;
      else if (dec == D_TCP) {
        tcp_poff = off;
        if (err_wrote == 2) { tcp_off = off; tcp_tot = ec_len + ep_len; }
      } else if (dec == D_UDP) { udp_off = off; udp_tot = 8; }
    }
    if (EXT && err_wrote == 2) {
#pragma unroll
      for (int k = 0; k < GPD_NOBJ; k++)
        if ((uint32_t)k == dec) rec[k] = gpd_layer_rec{off, ec_len, ep_off, ep_len};
    }
  }
done:
  if (klass != GPD_ST_DECODE_ERROR && stop != 0)
    klass = (options & GPD_OPT_IGNORE_UNSUPPORTED) ? GPD_ST_OK : GPD_ST_UNSUPPORTED;

  uint32_t st = klass | (truncated << 2);
  st |= (ncount > 31 ? 1u : 0u) << 3;
  st |= (ncount > 31 ? 31u : ncount) << 4;
  if (klass == GPD_ST_DECODE_ERROR) st |= err << 9;

  uint64_t nhash = 0, thash = 0;
  uint32_t cs = 0;
  st |= (last_net << 20) | (last_tp ? (last_tp == 1 ? 4u : 5u) << 24 : 0u);  // endpoint types
  uint32_t v4[2] = {0, 0};  // ip4 src/dst words, shared by the net hash and the pseudo-header
  if (last_net == 1 || (last_tp && tp_net == 1)) load_words(s, ip4_off + 12, v4);
  if (!(options & GPD_OPT_NO_FLOW_HASH)) {
    if (last_net == 1) {  // ip4.NetworkFlow(), ip4.go:63-65
      nhash = flow_fast(fnv_start<4>(v4[0]), fnv_start<4>(v4[1]), 1u);
      st |= 1u << 16;
    } else if (last_net == 2) {  // ip6.NetworkFlow(), ip6.go:49-51
      uint32_t w[8];
      load_words(s, ip6_off + 8, w);
      const H64 hs = fnv_more(fnv_more(fnv_more(fnv_start<4>(w[0]), w[1]), w[2]), w[3]);
      const H64 hd = fnv_more(fnv_more(fnv_more(fnv_start<4>(w[4]), w[5]), w[6]), w[7]);
      nhash = flow_fast(hs, hd, 2u);
      st |= 1u << 16;
    }
    if (last_tp) {  // tcp/udp.TransportFlow(), tcp.go:331-333, udp.go:123-125
      uint32_t w[1];
      load_words(s, last_tp == 1 ? tcp_poff : udp_off, w);
      uint32_t ept = last_tp == 1 ? 4u : 5u;
      thash = flow_fast(fnv_start<2>(w[0]), fnv_start<2>(w[0] >> 16), ept);
      st |= 1u << 17;
    }
  }
  if (!(options & GPD_OPT_NO_CHECKSUMS)) {
    // checksum(ip4.Contents), ip4.go:158-179; an odd-length Contents (a failed Length/IHL
    // check keeps all of data) makes `checksum` index past the end: a panic, no value
    if ((obj_valid & (1u << D_IP4)) && !(ip4_hl & 1u)) {
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
  o.hoff = hdr_word(last_net != 0, last_net == 1 ? ip4_off : ip6_off, last_tp != 0,
                    last_tp == 1 ? tcp_poff : udp_off);
  // decoded[0..15] as the ext / detail records hold them (the core word's 12 codes + hcodes)
  const uint64_t ecodes0 = (codes >> 16) | ((uint64_t)hcodes << 48);
  if (det && (klass == GPD_ST_DECODE_ERROR || ncount > GPD_CORE_MAX_LAYERS)) {  // gpd.h gpd_detail
    gpd_detail d;
    d.layer_codes[0] = ecodes0;
    d.layer_codes[1] = ecodes1;
    d.err_arg0 = klass == GPD_ST_DECODE_ERROR ? a0 : 0;
    d.err_arg1 = klass == GPD_ST_DECODE_ERROR ? a1 : 0;
    *det = d;
  }
  if (EXT) {
    gpd_ext_rec e;
    e.layer_codes[0] = ecodes0;
    e.layer_codes[1] = ecodes1;
    e.err_arg0 = klass == GPD_ST_DECODE_ERROR ? a0 : 0;
    e.err_arg1 = klass == GPD_ST_DECODE_ERROR ? a1 : 0;
    e.obj_valid = (uint16_t)obj_valid;
    e.err_obj = (uint8_t)err_dec;  // Dec order == enum gpd_obj order
    e.err_wrote = (uint8_t)err_wrote;
    e.err_off = klass == GPD_ST_DECODE_ERROR ? off : 0;
#pragma unroll
    for (int k = 0; k < GPD_NOBJ; k++)
      e.obj[k] = ((obj_valid >> k) & 1u) || ((uint32_t)k == err_dec && err_wrote == 2)
                     ? rec[k] : gpd_layer_rec{0, 0, 0, 0};
    *ext = e;
  }
  return o;
}

// ---------------------------------------------------------------- fast path
// Straight-line decode of the stacks that carry nearly all traffic:
//   Ethernet [Dot1Q]{0,2} (IPv4 with IHL 5 | IPv6 without hop-by-hop) (TCP | UDP | ICMPv4)
//     [Payload | VXLAN + the same stack once more]
// for a packet in an LDS window, with Ethernet as the first layer.  Header offsets are
// runtime values and every header is read straight from LDS at its own byte address
// (gfx950 DS instructions take unaligned addresses), so one code path serves every tag
// count and both VXLAN passes.  The parse only records where the objects the fused outputs
// read ended up (the last IPv4 header, the last network layer, the last transport); the
// checksums and hashes are computed once at the end from LDS.  A lane whose packet leaves
// the envelope (IPv4 options, fragments, hop-by-hop, any decode error, unusual table
// mappings...) returns false having written nothing, and the packet goes to the generic
// decoder, so the results are those of decode_packet in every case.
//
// Instruction economy (the kernel is VALU-issue bound once the bytes are in LDS):
//  * checksums are summed in the little-endian domain with v_dot2_u32_u16 (one op per
//    4 bytes, no byte shuffles) and converted once at the end (fold_le_not);
//  * FNV-1a multiplies use the 2^40 + 0x1b3 split, with the first byte from the basis in
//    closed form;
//  * table lookups are one ds_read_b64 of a two-way bucket and two compares.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t dot2(uint32_t x, uint32_t w, uint32_t acc) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, x), __builtin_bit_cast(u16x2, w), acc,
                                false);
}

// LDS reads at any byte address
struct __attribute__((packed, aligned(1))) U128 {
  uint32_t x, y, z, w;
};
__device__ __forceinline__ U128 ld128(uint32_t a) { return *reinterpret_cast<const U128 *>(g_lds + a); }

// big-endian 16-bit value of bytes (0,1) / (2,3) of a little-endian word
__device__ __forceinline__ uint32_t be_lo(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0C0C0001u); }
__device__ __forceinline__ uint32_t be_hi(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0C0C0203u); }

// ~fold(S) (tcpip.go:66-69) from the little-endian-domain sum S' of the same 16-bit words:
// the one's-complement sum of byte-swapped words is the byte-swapped sum (RFC 1071 §2(B)),
// exactly — an all-zero input gives 0 in both domains, anything else a value in
// [1, 0xFFFF] congruent mod 0xFFFF — as long as neither sum wraps 2^32 (true for the
// <= 16 KiB a fast-path packet spans).  Two folds bring any u32 to <= 0xFFFF.
__device__ __forceinline__ uint32_t fold_le_not(uint32_t s) {
  s = (s >> 16) + (s & 0xFFFFu);
  s = (s >> 16) + (s & 0xFFFFu);
  return __builtin_amdgcn_perm(0u, ~s, 0x0C0C0001u);  // byte-swap the low half, high half 0
}

// FNV-1a (flows.go:60-67) on (lo, hi) halves.  h * fnvPrime with fnvPrime = 2^40 + 0x1b3:
// lo' = lo * 0x1b3, hi' = hi * 0x1b3 + carry + (lo << 8) (mod 2^32).
struct FastCtx {        // wave-uniform facts about the registered set and the options
  uint32_t mult;        // the fixed-layout hash multiplier
  uint32_t pl_raw;      // Payload as a raw slot: LayerType 2 << 8 | its LUT entry
  uint32_t unsup;       // status class of a nonzero stop type (IgnoreUnsupported -> OK)
  uint32_t fr_ent;      // Fragment's LUT entry (decoder id D_FRAG when registered, else 15)
};

// Lookup in a fixed-layout bucket hash (gpd_internal.h kFix*): raw slot, 0x00FF on a miss.
__device__ __forceinline__ uint32_t fix_bucket_at(uint32_t base, uint32_t mult, uint32_t key) {
  const uint32_t b = __builtin_amdgcn_ubfe(__umul24(key, mult), 16 - kFixBits, kFixBits);
  const uint2 v = *reinterpret_cast<const uint2 *>(g_lds + 8 * (base / 2 + b));
  return (v.x >> 16) == key ? v.x : ((v.y >> 16) == key ? v.y : 0xFFu);
}
template <uint32_t BASE>
__device__ __forceinline__ uint32_t fix_bucket(uint32_t mult, uint32_t key) {
  return fix_bucket_at(BASE, mult, key);
}

// TCP/UDP NextLayerType on raw slots (tcp.go:308-314, udp.go:105-110): the dst-port entry
// unless it is 0 or Payload, else the src-port entry (0 => Payload).
__device__ __forceinline__ uint32_t ports_next_raw(uint32_t rd, uint32_t rs, uint32_t pl_raw) {
  const uint32_t s = (rs & 0xFF00u) ? rs : pl_raw;
  return (rd & 0xFD00u) ? rd : s;
}

// Is this one of the EtherTypes the default tables map to Dot1Q?  Only a guess that lets the
// network header be fetched early; the table lookup still decides, and a packet whose
// lookups disagree with a guess goes to the generic decoder.
__device__ __forceinline__ uint32_t tag_type(uint32_t et) {
  return (et == 0x8100u || et == 0x88A8u) ? 1u : 0u;
}

// The 64 bytes from a network header on (it and the first 16 bytes after it need <= 56),
// as four ds_read_b128 at the header's own byte address.  Misaligned, each costs ~3.6x an
// aligned one on gfx950, but aligned dword reads of the same bytes are slower still when
// packets sit at power-of-two strides (bank conflicts: tools/micro/lds_align.hip).
__device__ __forceinline__ void load64(uint32_t (&W)[16], uint32_t a) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const U128 q = ld128(a + 16 * k);
    W[4 * k] = q.x; W[4 * k + 1] = q.y; W[4 * k + 2] = q.z; W[4 * k + 3] = q.w;
  }
}

// A long transport segment left to the wave-cooperative sum (COOP): its partial LE-domain
// sum (pseudo-header, head and tail chunks) and the aligned 16-byte chunks [a, b) of the
// window between them, whose sum is a difference of the window's chunk prefix sums.
struct Seg {
  uint32_t part, a, b;
};

// Inclusive prefix sum over the 64 lanes: row shifts 1/2/4/8, then row broadcasts 15 / 31.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return v;
}

// P[c] = LE-domain sum of the window's 16-byte chunks below c, for c in [0, STAGE/16],
// written to LDS at pfx.  Lane l sums chunks [K l, K l + K), K = STAGE/1024; bytes past the
// window's end only reach entries beyond it.
template <int STAGE>
__device__ __forceinline__ void window_prefix(uint32_t buf, uint32_t pfx, uint32_t lane) {
  constexpr int K = STAGE / 1024;
  uint32_t c[K];
#pragma unroll
  for (int j = 0; j < K; j++) {
    const uint4 q = *reinterpret_cast<const uint4 *>(g_lds + buf + 16u * K * lane + 16u * j);
    c[j] = dot2(q.w, 0x00010001u, dot2(q.z, 0x00010001u,
                dot2(q.y, 0x00010001u, dot2(q.x, 0x00010001u, 0u))));
  }
  uint32_t run = 0;
#pragma unroll
  for (int j = 0; j < K; j++) {
    const uint32_t v = c[j];
    c[j] = run;  // exclusive within the block
    run += v;
  }
  const uint32_t incl = wave_incl_scan(run), base = incl - run;
  uint4 *d = reinterpret_cast<uint4 *>(g_lds + pfx + 4u * K * lane);
#pragma unroll
  for (int j = 0; j < K / 4; j++)
    d[j] = uint4{base + c[4 * j], base + c[4 * j + 1], base + c[4 * j + 2], base + c[4 * j + 3]};
  if (lane == 63u) *reinterpret_cast<uint32_t *>(g_lds + pfx + 4u * K * 64u) = incl;
}

// TCP options the walk (tcp.go:274-300) accepts without reading them byte by byte: none, or
// exactly NOP, NOP, Timestamps (kind 8, length 10) — what established connections carry.  w:
// the first four option bytes (TCP header bytes 20..23) as a little-endian word.
__device__ __forceinline__ bool tcp_opts_quick(uint32_t hl, uint32_t w) {
  return hl == 20u || (hl == 32u && w == 0x0A080101u);
}

// Header-once decode (rs_kernel HO, windows of long frames): a tile of 64 such packets spans
// several windows, and a straight-line decode per window would run with the few lanes whose
// packets that window holds.  Instead, in the window that holds a packet, seg_pass keeps
// the bytes the decode reads in the lane's registers and sums the transport segment the
// decode will checksum; after the tile's last window fast_decode<HO> runs once for all 64
// lanes from those registers.
struct Hdr {
  uint32_t e1, e2, e3;  // frame bytes 12..23: EtherType and up to two tags (ld128(p + 8).y/z/w)
  uint32_t W[16];       // the 64 bytes from the network header on
  uint32_t pos;         // tp_off | tp_len << 16 of the segment summed (0xFFFFFFFF: none)
  uint32_t sum;         // its LE-domain byte sum, pseudo-header not included
  uint32_t ok;          // its TCP options parse (tcp.go:274-300); 2: a VXLAN payload follows
};

// The LE-domain sum s + bytes [S, S + len) of the window, read as its first 16-byte chunk, the
// whole chunks after it and the ragged tail (TCP.ComputeChecksum's loop, tcpip.go:52-88).
__device__ __forceinline__ uint32_t seg_sum_chunks(uint32_t S, uint32_t len, uint32_t s) {
  const U128 c0 = ld128(S), ct = ld128(S + (len & ~15u));
  const uint32_t w0 = len >= 16u ? 0x00010001u : 0u;  // first whole chunk
  s = dot2(c0.x, w0, s);
  s = dot2(c0.y, w0, s);
  s = dot2(c0.z, w0, s);
  s = dot2(c0.w, w0, s);
  const uint32_t r8 = (len & 15u) * 8u;  // ragged tail: an odd last byte is its half's low byte
  uint64_t lo = ((uint64_t)ct.y << 32) | ct.x, hi = ((uint64_t)ct.w << 32) | ct.z;
  lo = r8 >= 64u ? lo : (r8 ? (lo << (64u - r8)) >> (64u - r8) : 0ull);
  hi = r8 > 64u ? (hi << (128u - r8)) >> (128u - r8) : 0ull;
  s = dot2((uint32_t)lo, 0x00010001u, s);
  s = dot2((uint32_t)(lo >> 32), 0x00010001u, s);
  s = dot2((uint32_t)hi, 0x00010001u, s);
  s = dot2((uint32_t)(hi >> 32), 0x00010001u, s);
  const uint32_t xt = len & ~15u;
  for (uint32_t x = 16; x < xt; x += 16u) {
    const U128 q = ld128(S + x);
    s = dot2(q.x, 0x00010001u, s);
    s = dot2(q.y, 0x00010001u, s);
    s = dot2(q.z, 0x00010001u, s);
    s = dot2(q.w, 0x00010001u, s);
  }
  return s;
}

// hdr_parse: the first round trip of fast_decode (the Ethernet and network header bytes) kept
// in h, and the transport segment that fast_decode's guesses lead to (IPv4 IHL 5 / IPv6 by the
// version nibble, TCP / UDP by the protocol number, UDP Length): h.pos and (l4, seg); false
// when there is none.  Reads the packet's first 128 bytes at most (a TCP options walk).
// fast_decode<HO> confirms the guesses with the dispatch tables and uses the segment's sum only
// when its own transport segment is exactly h.pos (else the packet takes the generic decoder).
// With VXLAN registered (vxreg), a UDP segment whose ports lead to it is flagged (h.ok = 2) for
// the full decode in the window that holds it: its inner headers are not staged.
__device__ __forceinline__ bool hdr_parse(uint32_t p, uint32_t len, Hdr &h, const FastCtx &F, bool vxreg,
                                          uint32_t &l4_out, uint32_t &seg_out) {
  h.pos = 0xFFFFFFFFu;
  h.sum = 0;
  h.ok = 0;
  if (len < 15u) return false;
  const U128 e = ld128(p + 8);
  h.e1 = e.y;
  h.e2 = e.z;
  h.e3 = e.w;
  const uint32_t et0 = be_lo(e.y), et1 = be_lo(e.z);
  const uint32_t t1 = tag_type(et0), t2 = t1 & tag_type(et1);
  const uint32_t l3 = 14 + 4 * (t1 + t2);
  load64(h.W, p + l3);  // one trip after the tags are known (no speculative untagged read)
  if (et0 < 0x0600u) return false;
  if (len < l3 + 20u) return false;
  const uint32_t *W = h.W;
  const uint32_t ver = (W[0] >> 4) & 15u;
  const bool v4 = ver == 4u;
  const uint32_t dl = len - l3;
  const uint32_t length = v4 ? be_hi(W[0]) : be_lo(W[1]);
  uint32_t plen;
  if (v4) {
    if ((W[0] & 0x0Fu) != 5u || length < 20u) return false;
    plen = (dl > length ? length : dl) - 20u;
  } else {
    if (ver != 6u || dl < 40u) return false;
    plen = (length > dl - 40u) ? dl - 40u : length;
  }
  const uint32_t proto = v4 ? ((W[2] >> 8) & 0xFFu) : ((W[1] >> 16) & 0xFFu);
  const uint32_t g = proto == 6u ? 1u : (proto == 17u ? 2u : 0u);
  if (!g) return false;
  const uint32_t ty = v4 ? W[6] : W[11], tw = v4 ? W[8] : W[13];
  const uint32_t l4 = l3 + (v4 ? 20u : 40u);
  const uint32_t ulen = be_lo(ty);
  const uint32_t seg = (g == 2u && ulen >= 8u && ulen <= plen) ? ulen : plen;
  if (vxreg && g == 2u) {  // ports -> VXLAN (udp.go:108-110 NextLayerType by port)
    const uint32_t tx = v4 ? W[5] : W[10];
    const uint32_t rd = fix_bucket_at(kFixUdpBase, F.mult, be_hi(tx));
    const uint32_t rs = fix_bucket_at(kFixUdpBase, F.mult, be_lo(tx));
    if ((ports_next_raw(rd, rs, F.pl_raw) & 15u) == D_VXLAN) {
      h.ok = 2;
      return false;
    }
  }
  if (g == 1u) {  // the options walk of fast_decode, on the guess
    const uint32_t hl = ((tw >> 4) & 15u) * 4u;
    uint32_t ok = (plen >= 20u && hl >= 20u && hl <= plen) ? 1u : 0u;
    for (uint32_t q = 20; ok && !tcp_opts_quick(hl, v4 ? W[10] : W[15]) && q < hl;) {
      const uint32_t k = g_lds[p + l4 + q];
      if (k == 0) break;
      uint32_t ol = 1;
      if (k != 1) {
        if (hl - q < 2) { ok = 0; break; }
        ol = g_lds[p + l4 + q + 1];
        if (ol < 2 || ol > hl - q) { ok = 0; break; }
      }
      q += ol;
    }
    h.ok = ok;
  }
  h.pos = l4 | (seg << 16);
  l4_out = l4;
  seg_out = seg;
  return true;
}

// seg_pass (the per-window header-once step): hdr_parse, and the transport segment it guessed
// summed from this window: its head and tail here, the whole chunks between left to the
// window's chunk prefix sums (sg) when it is long and even-aligned.
template <bool COOP>
__device__ __forceinline__ void seg_pass(uint32_t p, uint32_t len, uint32_t buf, Hdr &h, Seg &sg,
                                         const FastCtx &F, bool vxreg) {
  uint32_t l4, seg;
  if (!hdr_parse(p, len, h, F, vxreg, l4, seg)) return;
  const uint32_t S = p + l4;
  if (COOP && seg >= 64u && !(S & 1u)) {
    // head [S, A) and tail [B, E) from their aligned chunks; [A, B) from the prefix sums
    const uint32_t E = S + seg, A = (S + 15u) & ~15u, B = E & ~15u;
    uint32_t s = 0;
    if (A > S) {
      const uint4 q = *reinterpret_cast<const uint4 *>(g_lds + A - 16u);
      const uint32_t h8 = (S & 15u) * 8u;
      uint64_t lo = ((uint64_t)q.y << 32) | q.x, hi = ((uint64_t)q.w << 32) | q.z;
      lo = h8 >= 64u ? 0ull : (lo >> h8) << h8;
      hi = h8 > 64u ? (hi >> (h8 - 64u)) << (h8 - 64u) : hi;
      s = dot2((uint32_t)lo, 0x00010001u, s);
      s = dot2((uint32_t)(lo >> 32), 0x00010001u, s);
      s = dot2((uint32_t)hi, 0x00010001u, s);
      s = dot2((uint32_t)(hi >> 32), 0x00010001u, s);
    }
    if (E > B) {
      const uint4 q = *reinterpret_cast<const uint4 *>(g_lds + B);
      const uint32_t r8 = (E & 15u) * 8u;
      uint64_t lo = ((uint64_t)q.y << 32) | q.x, hi = ((uint64_t)q.w << 32) | q.z;
      lo = r8 >= 64u ? lo : (lo << (64u - r8)) >> (64u - r8);
      hi = r8 > 64u ? (hi << (128u - r8)) >> (128u - r8) : 0ull;
      s = dot2((uint32_t)lo, 0x00010001u, s);
      s = dot2((uint32_t)(lo >> 32), 0x00010001u, s);
      s = dot2((uint32_t)hi, 0x00010001u, s);
      s = dot2((uint32_t)(hi >> 32), 0x00010001u, s);
    }
    sg = Seg{s, (A - buf) >> 4, (B - buf) >> 4};  // the caller adds P[b] - P[a] into h.sum
    return;
  }
  h.sum = seg_sum_chunks(S, seg, 0u);
}

// p: LDS address of the packet's first byte; len: its length.  CS / HASH: the fused
// checksums / flow hashes are requested (GPD_OPT_NO_CHECKSUMS / _NO_FLOW_HASH clear).
// Two dependent LDS round trips per pass (three for tagged frames): (1) the Ethernet header
// and the 64 bytes after it; (2) every table lookup — EtherType, protocol, ports, each on
// a guess read from the bytes (IPv4/IPv6 by the version nibble, TCP/UDP by the protocol
// number).  The lookups then confirm the guesses; a packet they contradict goes to the
// generic decoder.  Hashes and the IPv4 header checksum are computed from registers as
// each layer is accepted, so VXLAN's second pass overwrites them exactly as the reused
// layer objects are overwritten (A11); the transport checksum reads its segment's edge
// chunks once more after the parse.
// COOP: a long even-aligned segment's whole middle chunks are left to window_prefix (sg).
// HO: the header-once decode — no window is read: the header bytes and the segment sum come
// from seg_pass (*h), one pass (a VXLAN payload takes the generic decoder).
template <bool CS, bool HASH, bool COOP, bool HO = false, bool AL = false>
__device__ __forceinline__ bool fast_decode(uint32_t p, uint32_t len, const FastCtx &F, Out &o,
                                            uint32_t buf, Seg &sg, const Hdr *h = nullptr) {
  uint64_t codes = 0, nh = 0, th = 0;
  uint32_t nc = 0, trunc = 0, stop = 0;
  uint32_t net = 0, tp = 0, ip4 = 0, ipcs = 0;
  uint32_t tp_off = 0, tp_len = 0, tp_pl = 0;  // the last transport; its proto + length terms
  uint32_t tp_kind = 0, ps4 = 0, ps6 = 0;      // its network object kind; each kind's addresses
  uint32_t net_off = 0;                        // the last network header
  uint32_t b = 0, lim = len;                   // this pass's Ethernet offset; end of its data
  // AL (unshifted 8 KiB windows, frames of ~65..160 B): a VXLAN frame's inner Ethernet bytes
  // 8..23 come from the outer pass's registers when it is IPv4 (IHL 5) / UDP / VXLAN — one
  // misaligned LDS read fewer per pass (VXLAN -1.8 %; in the other kernels the longer live
  // range costs 1-5 %, measured A/B on one box)
  constexpr bool reg_e = !HO && AL;
  uint32_t ie1 = 0, ie2 = 0, ie3 = 0, have_ie = 0;
  auto put = [&](uint32_t code) { codes |= (uint64_t)code << (16 + 4 * nc); nc++; };
  for (int pass = 0; pass < (HO ? 1 : 2); pass++) {
    // ---- round trip 1: Ethernet header (ethernet.go:41-62) and the bytes after it
    if (lim < b + 15u) return false;  // too small, or an empty payload: generic path
    U128 e;  // bytes 8..23: EtherType and up to two tags
    uint32_t W[16];
    if (HO) {
      e.x = 0;
      e.y = h->e1;
      e.z = h->e2;
      e.w = h->e3;
#pragma unroll
      for (int k = 0; k < 16; k++) W[k] = h->W[k];
    } else if (reg_e && have_ie) {
      e.x = 0;
      e.y = ie1;
      e.z = ie2;
      e.w = ie3;
      load64(W, p + b + 14);
    } else {
      e = ld128(p + b + 8);
      load64(W, p + b + 14);
    }
    const uint32_t et0 = be_lo(e.y), et1 = be_lo(e.z), et2 = be_lo(e.w);
    if (et0 < 0x0600u) {  // 802.3 length framing
      // header-once tile decode only (the per-window kernels leave it to the generic decoder):
      // Ethernet's payload is Length bytes (ethernet.go:53-58), then LLC (llc.go:31-52) from the
      // staged bytes 14..16, then its next layer (llc.go:61-69) — which must stop the decode
      if (!HO || b != 0u) return false;
      const uint32_t re = fix_bucket<kFixEthBase>(F.mult, 0u);  // EthernetTypeLLC
      if ((re & 15u) != D_LLC) return false;
      uint32_t pl = lim - 14u;
      if (pl < et0) trunc = 1;
      else pl = et0;
      if (pl < 3u) return false;  // "LLC header too small": the generic decoder
      const uint32_t dsap = (e.y >> 16) & 0xFEu, ssap = (e.y >> 24) & 0xFEu, ctl = e.z & 0xFFu;
      uint32_t cl = 3;
      if (!(ctl & 1u) || (ctl & 3u) == 1u) {  // two-byte control field
        if (pl < 4u) return false;
        cl = 4;
      }
      put(GPD_C_ETHERNET);
      put((re >> 4) & 15u);
      if (pl == cl) break;  // layers_decoder.go:71-73
      const uint32_t nt = (dsap == 0xAAu && ssap == 0xAAu) ? (uint32_t)GPD_LT_SNAP
                        : (dsap == 0x42u && ssap == 0x42u) ? (uint32_t)GPD_LT_STP : (uint32_t)GPD_LT_ZERO;
      if ((reinterpret_cast<const uint8_t *>(g_lds)[nt] & 15u) != D_NONE) return false;
      stop = nt;
      break;
    }
    const uint32_t t1 = tag_type(et0), t2 = t1 & tag_type(et1);
    const uint32_t l3 = b + 14 + 4 * (t1 + t2);
    if (t1 && !HO) load64(W, p + l3);  // tagged: the network header is further in
    // ---- guesses from the bytes
    const uint32_t ver = (W[0] >> 4) & 15u;
    const bool v4 = ver == 4u;
    const uint32_t proto = v4 ? ((W[2] >> 8) & 0xFFu) : ((W[1] >> 16) & 0xFFu);
    const uint32_t g = proto == 6u ? 1u : (proto == 17u ? 2u : 0u);  // TCP / UDP
    const uint32_t tx = v4 ? W[5] : W[10], ty = v4 ? W[6] : W[11], tw = v4 ? W[8] : W[13];
    const uint32_t l4 = l3 + (v4 ? 20u : 40u);
    const uint32_t dl = lim - l3;
    const uint32_t length = v4 ? be_hi(W[0]) : be_lo(W[1]);  // IPv4 total / IPv6 payload
    uint32_t plen;                                             // the network payload
    if (v4) plen = (dl > length ? length : dl) - 20u;
    else plen = (length > dl - 40u) ? dl - 40u : length;
    const uint32_t ulen = be_lo(ty);
    const uint32_t seg = (g == 2u && ulen >= 8u && ulen <= plen) ? ulen : plen;
    // ---- round trip 2: all lookups
    const uint32_t r0 = fix_bucket<kFixEthBase>(F.mult, et0);
    uint32_t r1 = 0, r2 = 0;
    if (t1) {
      r1 = fix_bucket<kFixEthBase>(F.mult, et1);
      r2 = fix_bucket<kFixEthBase>(F.mult, et2);
    }
    // the network layer's next: the protocol table, or Fragment when an IPv4 header has MF or a
    // fragment offset (ip4.go:281-286) — LayerType | LUT entry << 16 either way
    const uint32_t pv = (v4 && (be_hi(W[1]) & 0x3FFFu)) ? (uint32_t)GPD_LT_FRAGMENT | (F.fr_ent << 16)
                                                      : lds_u32(4 * (kHashLutWords + proto));
    const uint32_t pbase = g == 1u ? kFixTcpBase : kFixUdpBase;
    const uint32_t rd = fix_bucket_at(pbase, F.mult, be_hi(tx));
    const uint32_t rs = fix_bucket_at(pbase, F.mult, be_lo(tx));
    // ---- Ethernet / Dot1Q (dot1q.go:29-50), confirming the tag guesses
    put(GPD_C_ETHERNET);
    if (((r0 & 15u) == D_DOT1Q) != (t1 != 0)) return false;
    uint32_t r = r0;
    if (t1) {
      if (lim <= b + 18u) return false;
      put(GPD_C_DOT1Q);
      if (((r1 & 15u) == D_DOT1Q) != (t2 != 0)) return false;
      r = r1;
      if (t2) {
        if (lim <= b + 22u || (r2 & 15u) == D_DOT1Q) return false;
        put(GPD_C_DOT1Q);
        r = r2;
      }
    }
    const uint32_t dec = r & 15u;
    if (dec == D_NONE) { stop = (r >> 8) & 0xFFu; break; }
    uint32_t ps;  // pseudo-header address words of this network layer (LE domain)
    if (dec == D_IP4) {  // ip4.go:188-286, IHL 5 only
      // IHL != 5 (options), Length 0 (TSO rule) or < 20 (error): generic path
      if (!v4 || dl < 20u || (W[0] & 0x0Fu) != 5u || length < 20u) return false;
      if (dl < length) trunc = 1;
      ps = dot2(W[4], 0x00010001u, dot2(W[3], 0x00010001u, 0u));
      if (CS) {  // checksum(ip4.Contents), ip4.go:158-179 (bytes 10-11 left out)
        ipcs = fold_le_not(dot2(W[2], 0x00000001u, dot2(W[1], 0x00010001u,
                           dot2(W[0], 0x00010001u, ps))));
        ip4 = 1;
      }
      if (HASH) nh = flow_fast(fnv_start<4>(W[3]), fnv_start<4>(W[4]), 1u);  // ip4.go:63-65
      ps4 = ps;
      net = 1;
      net_off = l3;
      put(GPD_C_IPV4);
      lim = l3 + 20u + plen;  // Length trims the payload (and Ethernet padding)
    } else if (dec == D_IP6) {  // ip6.go:221-278 without hop-by-hop
      if (ver != 6u || dl < 40u || proto == 0u || length == 0u) return false;
      if (length > dl - 40u) trunc = 1;
      ps = 0;
#pragma unroll
      for (int k = 2; k < 10; k++) ps = dot2(W[k], 0x00010001u, ps);  // tcpip.go:37-48
      if (HASH) {  // ip6.go:49-51
        const H64 hs = fnv_more(fnv_more(fnv_more(fnv_start<4>(W[2]), W[3]), W[4]), W[5]);
        const H64 hd = fnv_more(fnv_more(fnv_more(fnv_start<4>(W[6]), W[7]), W[8]), W[9]);
        nh = flow_fast(hs, hd, 2u);
      }
      ps6 = ps;
      net = 2;
      net_off = l3;
      put(GPD_C_IPV6);
      lim = l3 + 40u + plen;
    } else {
      return false;
    }
    if (plen == 0) break;
    // ---- transport, confirming the protocol guess
    const uint32_t d4 = (pv >> 16) & 15u;
    if (d4 == D_NONE) { stop = pv & 0xFFFFu; break; }
    // ICMPv4 (icmp4.go:220-231, next layer Payload :261-263) and gopacket.Fragment (base.go:108-117:
    // all of the rest, nothing after) share one exit: a separate Fragment exit made the compiler
    // add ~110 register moves to the loop (tools/isa_count.py)
    if (d4 == D_ICMP4 || d4 == D_FRAG) {
      const bool ic = d4 == D_ICMP4;
      if (ic && plen < 8u) return false;  // "ICMP layer less then 8 bytes": generic path
      put(ic ? GPD_C_ICMPV4 : GPD_C_FRAGMENT);
      if (!ic || plen == 8u) break;
      if ((F.pl_raw & 15u) == D_PAYLOAD) put(GPD_C_PAYLOAD);
      else stop = GPD_LT_PAYLOAD;
      break;
    }
    if (!((d4 == D_TCP && g == 1u) || (d4 == D_UDP && g == 2u))) return false;
    uint32_t hl;
    if (g == 1u) {  // tcp.go:229-314
      hl = ((tw >> 4) & 15u) * 4u;
      if (plen < 20u || hl < 20u || hl > plen) return false;
      if (HO && !h->ok) return false;
      // OPTIONS, tcp.go:274-300 (errors -> generic path)
      for (uint32_t q = 20; !HO && !tcp_opts_quick(hl, v4 ? W[10] : W[15]) && q < hl;) {
        const uint32_t k = g_lds[p + l4 + q];
        if (k == 0) break;
        uint32_t ol = 1;
        if (k != 1) {
          if (hl - q < 2) return false;
          ol = g_lds[p + l4 + q + 1];
          if (ol < 2 || ol > hl - q) return false;
        }
        q += ol;
      }
      put(GPD_C_TCP);
    } else {  // UDP, udp.go:30-56 (Length 0: the rest; 1..7: error)
      if (plen < 8u || (ulen != 0u && ulen < 8u)) return false;
      if (ulen > plen) trunc = 1;
      hl = 8;
      lim = l4 + seg;
      put(GPD_C_UDP);
    }
    tp = g;
    if (HASH) th = flow_fast(fnv_start<2>(tx), fnv_start<2>(tx >> 16), g == 1u ? 4u : 5u);
    // pseudo-header protocol and length as LE-domain words (seg < 2^16 in a window); the
    // addresses are added at the end from the network object of this kind as the call
    // leaves it (SetNetworkLayerForChecksum(&ip4) reads the reused object: for VXLAN whose
    // inner pass stops before a transport, the inner header's addresses)
    tp_pl = (g == 1u ? 0x0600u : 0x1100u) + __builtin_amdgcn_perm(0u, seg, 0x0C0C0001u);
    tp_kind = net;
    tp_off = l4;
    tp_len = seg;
    const uint32_t pl4 = seg - hl;
    if (pl4 == 0) break;
    const uint32_t next = ports_next_raw(rd, rs, F.pl_raw), nd = next & 15u;
    if (nd == D_NONE) { stop = (next >> 8) & 0xFFu; break; }
    if (nd == D_PAYLOAD) { put(GPD_C_PAYLOAD); break; }  // Payload consumes the rest
    if (HO || nd != D_VXLAN || pass == 1 || pl4 < 8u) return false;
    put(GPD_C_VXLAN);  // vxlan.go:53-78; its payload is an Ethernet frame (A11: two passes)
    b = l4 + hl + 8;
    if (pl4 == 8u) break;
    if (reg_e) {  // IPv4 (IHL 5) / UDP / VXLAN: the inner bytes 8..23 are W[11..14]
      have_ie = (v4 && g == 2u) ? 1u : 0u;
      ie1 = W[12];
      ie2 = W[13];
      ie3 = W[14];
    }
  }

  // ---- outputs, composed exactly as decode_packet does
  const uint32_t tp_ps = tp_pl + (tp_kind == 1u ? ps4 : ps6);
  uint32_t st = (stop ? F.unsup : GPD_ST_OK) | (trunc << 2) | (nc << 4);
  uint32_t cs = 0;
  st |= (net << 20) | (tp ? (tp == 1 ? 4u : 5u) << 24 : 0u);  // endpoint types (gpd.h)
  if (HASH) st |= (net ? 1u << 16 : 0u) | (tp ? 1u << 17 : 0u);
  sg.b = 0;
  if (HO) {
    if (CS) {  // the segment seg_pass summed must be this transport's
      if (tp && h->pos != (tp_off | (tp_len << 16))) return false;
      cs = (ip4 ? ipcs : 0u) | (tp ? fold_le_not(tp_ps + h->sum) << 16 : 0u);
      st |= (ip4 ? 1u << 18 : 0u) | (tp ? 1u << 19 : 0u);
    }
  } else if (COOP && CS && tp && tp_len >= 64u && !((p + tp_off) & 1u)) {
    // head [S, A) and tail [B, E) from their aligned chunks; [A, B) from the prefix sums
    const uint32_t S = p + tp_off, E = S + tp_len, A = (S + 15u) & ~15u, B = E & ~15u;
    uint32_t s = tp_ps;
    if (A > S) {  // keep bytes from S & 15 on
      const uint4 q = *reinterpret_cast<const uint4 *>(g_lds + A - 16u);
      const uint32_t h8 = (S & 15u) * 8u;
      uint64_t lo = ((uint64_t)q.y << 32) | q.x, hi = ((uint64_t)q.w << 32) | q.z;
      lo = h8 >= 64u ? 0ull : (lo >> h8) << h8;
      hi = h8 > 64u ? (hi >> (h8 - 64u)) << (h8 - 64u) : hi;
      s = dot2((uint32_t)lo, 0x00010001u, s);
      s = dot2((uint32_t)(lo >> 32), 0x00010001u, s);
      s = dot2((uint32_t)hi, 0x00010001u, s);
      s = dot2((uint32_t)(hi >> 32), 0x00010001u, s);
    }
    if (E > B) {  // keep bytes below E & 15
      const uint4 q = *reinterpret_cast<const uint4 *>(g_lds + B);
      const uint32_t r8 = (E & 15u) * 8u;
      uint64_t lo = ((uint64_t)q.y << 32) | q.x, hi = ((uint64_t)q.w << 32) | q.z;
      lo = r8 >= 64u ? lo : (lo << (64u - r8)) >> (64u - r8);
      hi = r8 > 64u ? (hi << (128u - r8)) >> (128u - r8) : 0ull;
      s = dot2((uint32_t)lo, 0x00010001u, s);
      s = dot2((uint32_t)(lo >> 32), 0x00010001u, s);
      s = dot2((uint32_t)hi, 0x00010001u, s);
      s = dot2((uint32_t)(hi >> 32), 0x00010001u, s);
    }
    sg = Seg{s, (A - buf) >> 4, (B - buf) >> 4};
    o.status = st | (ip4 ? 1u << 18 : 0u) | (1u << 19);
    o.layers = codes | (stop & 0xFFFFu);
    o.net_hash = HASH ? nh : 0;
    o.tp_hash = HASH ? th : 0;
    o.csum = ip4 ? ipcs : 0u;  // the transport half is added by the caller
    o.hoff = hdr_word(net != 0, net_off, tp != 0, tp_off);
    return true;
  } else if (AL && CS && tp && !((p + tp_off) & 1u)) {
    // AL (unshifted 8 KiB windows, VXLAN-sized frames): the same sum from aligned 16-byte
    // chunks, head [S, A) and tail [B, E) masked and the whole chunks between as they are — an
    // aligned DS read costs ~1/3.6 of a misaligned one (VXLAN -3.4 %; with shifted copies of
    // small frames the header reads are aligned already and the masking cost pcap64 +1 %,
    // measured A/B on one box)
    const uint32_t S = p + tp_off, E = S + tp_len, A = (S + 15u) & ~15u, B = E & ~15u;
    uint32_t s = tp_ps;
    if (A > S) {
      const uint4 q = *reinterpret_cast<const uint4 *>(g_lds + A - 16u);
      const uint32_t h8 = (S & 15u) * 8u;
      const uint32_t e8 = E < A ? (A - E) * 8u : 0u;  // a segment ending inside its head chunk
      uint64_t lo = ((uint64_t)q.y << 32) | q.x, hi = ((uint64_t)q.w << 32) | q.z;
      lo = h8 >= 64u ? 0ull : (lo >> h8) << h8;
      hi = h8 > 64u ? (hi >> (h8 - 64u)) << (h8 - 64u) : hi;
      if (e8) {  // drop the e8 top bits of (hi, lo)
        hi = e8 >= 64u ? 0ull : (hi << e8) >> e8;
        lo = e8 > 64u ? (lo << (e8 - 64u)) >> (e8 - 64u) : lo;
      }
      s = dot2((uint32_t)lo, 0x00010001u, s);
      s = dot2((uint32_t)(lo >> 32), 0x00010001u, s);
      s = dot2((uint32_t)hi, 0x00010001u, s);
      s = dot2((uint32_t)(hi >> 32), 0x00010001u, s);
    }
    for (uint32_t x = A; x < B; x += 16u) {
      const uint4 q = *reinterpret_cast<const uint4 *>(g_lds + x);
      s = dot2(q.x, 0x00010001u, s);
      s = dot2(q.y, 0x00010001u, s);
      s = dot2(q.z, 0x00010001u, s);
      s = dot2(q.w, 0x00010001u, s);
    }
    if (E > B && B >= A) {
      const uint4 q = *reinterpret_cast<const uint4 *>(g_lds + B);
      const uint32_t r8 = (E & 15u) * 8u;
      uint64_t lo = ((uint64_t)q.y << 32) | q.x, hi = ((uint64_t)q.w << 32) | q.z;
      lo = r8 >= 64u ? lo : (lo << (64u - r8)) >> (64u - r8);
      hi = r8 > 64u ? (hi << (128u - r8)) >> (128u - r8) : 0ull;
      s = dot2((uint32_t)lo, 0x00010001u, s);
      s = dot2((uint32_t)(lo >> 32), 0x00010001u, s);
      s = dot2((uint32_t)hi, 0x00010001u, s);
      s = dot2((uint32_t)(hi >> 32), 0x00010001u, s);
    }
    cs = (ip4 ? ipcs : 0u) | (fold_le_not(s) << 16);
    st |= (ip4 ? 1u << 18 : 0u) | (1u << 19);
  } else if (CS) {
    // TCP.ComputeChecksum(), tcp.go:193-195 / tcpip.go:52-88 over the last transport.  Its
    // first and ragged-last 16-byte chunks are read here, once, after the parse (holding
    // them through the parse would cost 16 VGPRs, a wave per SIMD).
    const U128 c0 = ld128(p + tp_off), ct = ld128(p + tp_off + (tp_len & ~15u));
    uint32_t s = tp_ps;
    const uint32_t w0 = tp_len >= 16u ? 0x00010001u : 0u;  // first whole chunk
    s = dot2(c0.x, w0, s);
    s = dot2(c0.y, w0, s);
    s = dot2(c0.z, w0, s);
    s = dot2(c0.w, w0, s);
    // ragged tail: the first tp_len % 16 bytes of ct (an odd last byte is the low byte of
    // its half)
    const uint32_t r8 = (tp_len & 15u) * 8u;
    uint64_t lo = ((uint64_t)ct.y << 32) | ct.x, hi = ((uint64_t)ct.w << 32) | ct.z;
    lo = r8 >= 64u ? lo : (r8 ? (lo << (64u - r8)) >> (64u - r8) : 0ull);
    hi = r8 > 64u ? (hi << (128u - r8)) >> (128u - r8) : 0ull;
    s = dot2((uint32_t)lo, 0x00010001u, s);
    s = dot2((uint32_t)(lo >> 32), 0x00010001u, s);
    s = dot2((uint32_t)hi, 0x00010001u, s);
    s = dot2((uint32_t)(hi >> 32), 0x00010001u, s);
    const uint32_t xt = tp_len & ~15u;
    for (uint32_t x = 16; x < xt; x += 16u) {  // whole chunks after the first (long segments)
      const U128 q = ld128(p + tp_off + x);
      s = dot2(q.x, 0x00010001u, s);
      s = dot2(q.y, 0x00010001u, s);
      s = dot2(q.z, 0x00010001u, s);
      s = dot2(q.w, 0x00010001u, s);
    }
    cs = (ip4 ? ipcs : 0u) | (tp ? fold_le_not(s) << 16 : 0u);
    st |= (ip4 ? 1u << 18 : 0u) | (tp ? 1u << 19 : 0u);
  }
  o.status = st;
  o.layers = codes | (stop & 0xFFFFu);
  o.net_hash = HASH ? nh : 0;
  o.tp_hash = HASH ? th : 0;
  o.csum = cs;
  o.hoff = hdr_word(net != 0, net_off, tp != 0, tp_off);
  return true;
}

// ---------------------------------------------------------------- wave helpers
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

__device__ __forceinline__ void store_out(const KParams &P, uint32_t i, const Out &o) {
  if (P.rec) {  // one 32-B gpd_record: {status, csum, layers} and {net_hash, tp_hash}
    v4u32 *r = reinterpret_cast<v4u32 *>(P.rec + i);
    const v4u32 a = {o.status, o.csum, (uint32_t)o.layers, (uint32_t)(o.layers >> 32)};
    const v4u32 b = {(uint32_t)o.net_hash, (uint32_t)(o.net_hash >> 32), (uint32_t)o.tp_hash,
                     (uint32_t)(o.tp_hash >> 32)};
    __builtin_nontemporal_store(a, r);
    __builtin_nontemporal_store(b, r + 1);
    if (P.hdr_off) __builtin_nontemporal_store(o.hoff, P.hdr_off + i);
    return;
  }
  if (P.options & kDiagNtStore) {
    __builtin_nontemporal_store(o.status, P.status + i);
    __builtin_nontemporal_store(o.layers, P.layers + i);
    if (P.net_hash) __builtin_nontemporal_store(o.net_hash, P.net_hash + i);
    if (P.tp_hash) __builtin_nontemporal_store(o.tp_hash, P.tp_hash + i);
    if (P.csum) __builtin_nontemporal_store(o.csum, P.csum + i);
    if (P.hdr_off) __builtin_nontemporal_store(o.hoff, P.hdr_off + i);
    return;
  }
  P.status[i] = o.status;
  P.layers[i] = o.layers;
  if (P.net_hash) P.net_hash[i] = o.net_hash;
  if (P.tp_hash) P.tp_hash[i] = o.tp_hash;
  if (P.csum) P.csum[i] = o.csum;
  if (P.hdr_off) P.hdr_off[i] = o.hoff;
}

// A window of the batch buffer: bytes [base, base + nbytes) (base 16-aligned).
struct Window {
  uint32_t base, nbytes;
  uint32_t shift;  // rs_kernel: LDS byte of global byte x is buf + shift + (x - base)
};

// A window starts at the first pending packet (rounded down to 16) and covers every pending
// packet lying wholly inside [base, base + STAGE).  Packets normally sit in lane order, so
// the last covered lane's end is the extent; a full wave maximum only runs when some lane
// proves otherwise.
template <int STAGE>
__device__ __forceinline__ Window plan_window(bool pending, uint32_t off, uint32_t end, uint32_t l3m = 14u) {
  Window w{0, 0, 0};
  const uint64_t m = __ballot(pending);
  if (m == 0) return w;
  const uint32_t first = __builtin_amdgcn_readlane(off, (int)__builtin_ctzll(m));
  w.base = first & ~15u;
  // the shift that puts the first packet's byte l3m (mod 16: where the wave's last network
  // header sat, 14 for an untagged frame) on a 16-byte LDS boundary: misaligned DS reads
  // cost ~3.6x aligned ones (tools/micro/lds_align)
  w.shift = (32u - ((first & 15u) + l3m)) & 15u;
  const bool in = pending && off >= w.base && end - w.base <= (uint32_t)STAGE;
  const uint32_t x = in ? end - w.base : 0u;
  const uint64_t mi = __ballot(in);  // nonzero: the first pending lane is in
  uint32_t need = __builtin_amdgcn_readlane(x, 63 - (int)__builtin_clzll(mi));  // last lane in
  if (__any(x > need)) need = __builtin_amdgcn_readfirstlane(wave_max(x));
  w.nbytes = (need + 15u) & ~15u;
  return w;
}

// 16-byte LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes from gbase + voff land at LDS
// lds + 16 l.  Issued from inline asm so the compiler's waitcnt pass does not see it:
// otherwise it cannot tell the in-flight DMA into the other window from this window's
// ds_reads and drains it (vmcnt(0)) before the first one, serialising the prefetch.  Every
// wait on these loads is therefore explicit (a counted s_waitcnt vmcnt before a window is
// read; loads, stores and LDS-DMA retire in issue order, MI355X_MICROARCH.md).
__device__ __forceinline__ void glds16(const uint8_t *gbase, uint32_t voff, uint32_t lds,
                                       bool nt = false) {
  uint32_t keep;
  if (nt) {
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2 nt\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(gbase), "s"(lds)
        : "memory");
    return;
  }
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(gbase), "s"(lds)
      : "memory");
}

// 4-byte LDS-DMA (global_load_lds_dword): lane l's word from gbase + voff lands at LDS lds + 4 l.
__device__ __forceinline__ void glds4(const void *gbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(gbase), "s"(lds)
      : "memory");
}

// Per-lane source offsets of a window: wave instruction c writes physical slots
// [64c, 64c+64); lane l's source is the logical slot that lands on slot 64c + l — for the
// rotated layout that depends on c mod 4 only (four per-lane constants).
template <bool SWZ>
struct DmaLanes {
  uint32_t voff[4];
  __device__ __forceinline__ explicit DmaLanes(uint32_t lane) {
#pragma unroll
    for (int j = 0; j < 4; j++)
      voff[j] = SWZ ? 16u * ((lane & 48u) + ((lane - (lane >> 4) - 4u * j) & 15u)) : 16u * lane;
  }
};

template <bool SWZ>
__device__ __forceinline__ void issue_window(const uint8_t *data, const Window &w, uint32_t buf,
                                             const DmaLanes<SWZ> &L, bool nt = false) {
  for (uint32_t c4 = 0; c4 < w.nbytes; c4 += 4096u) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t c = c4 + 1024u * j;
      if (c >= w.nbytes) break;
      if (c + 1024u <= w.nbytes || c + L.voff[j] < w.nbytes)
        glds16(data + w.base + c, L.voff[j], buf + c, nt);
    }
  }
}

// ---------------------------------------------------------------- kernel
// Counted wait for this tile's window: everything but the last tile's result stores.
__device__ __forceinline__ void wait_window(uint32_t nstores) {
  switch (nstores) {
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// LDS bytes per wave: two windows, two descriptor slots, and (fast kernel, windows of 8 KiB
// and more) the stage/16 + 1 chunk prefix sums of the cooperative segment checksum.
__host__ __device__ constexpr uint32_t wave_lds_bytes(int stage, bool fast) {
  return 2u * stage + 1024u + ((fast && stage >= 8192) ? (uint32_t)stage / 4u + 16u : 0u);
}

// WAVES waves per workgroup; each wave owns 64-packet tiles t, t + W, ... (grid stride).  A
// tile's bytes are staged through LDS windows of STAGE bytes (a tile of large packets takes
// several), and the window is the pipeline unit: per wave, LDS holds two window buffers
// and two descriptor slots (the 64 offsets and caplens of a tile), all filled by LDS-DMA,
// so the loop has no compiler-visible global loads and every wait is an explicit, counted
// one.  Iteration k:
//   wait for window k -> plan and issue window k+1 (the rest of this tile, or the next
//   tile's first window, whose descriptors arrived two tiles ago; then the descriptors two
//   tiles further on) -> decode window k's packets from LDS -> when window k ended its
//   tile, store the tile's 64 results.
// !FAST: the generic decoder for every packet (the FAST form is retired: see rs_kernel).
template <int STAGE, bool FAST, bool EXT, bool PAGES, bool SWZ, int WAVES, bool CS = true,
          bool HASH = true, int MINW = 1>
__global__ __launch_bounds__(64 * WAVES, MINW) void decode_kernel(KParams P) {
  // The fast path is rs_kernel, whose waves decode their own fallback lists; this loop's FAST
  // form appended to one shared counter and is no longer launched.
  static_assert(!FAST, "decode_kernel<FAST> predates the per-wave fallback regions");
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // stage the dispatch-table image (LUT, ipproto, hashes) into LDS
  for (uint32_t k = threadIdx.x; k < P.image_words; k += 64 * WAVES)
    reinterpret_cast<uint32_t *>(g_lds)[k] = P.image[k];
  __syncthreads();
  const Tab<PAGES> T{P.pages,    P.eth_base, P.tcp_base, P.udp_base, P.eth_bits,
                     P.tcp_bits, P.udp_bits, P.eth_mult, P.tcp_mult, P.udp_mult};
  constexpr bool COOP = FAST && STAGE >= 8192;  // long segments: wave-cooperative checksum
  const uint32_t img = (P.image_words * 4u + 15u) & ~15u;
  const uint32_t bufs = img + wave * wave_lds_bytes(STAGE, FAST);
  const uint32_t dslots = bufs + 2u * STAGE;  // two slots of 64 offsets + 64 caplens
  const uint32_t pfx = dslots + 1024u;        // COOP: 513 chunk prefix sums
  const uint32_t n = P.n_dev ? min((uint32_t)P.n, *P.n_dev) : (uint32_t)P.n;  // <= kMaxLaunchPackets
  const uint32_t ntiles = (n + 63u) >> 6;
  const uint32_t nwaves = gridDim.x * WAVES;
  const uint32_t dlen = (uint32_t)P.data_len;
  const uint32_t fits = (uint32_t)STAGE - 15u;  // a packet of <= fits bytes always fits a window
  const uint32_t options = P.options & ~kDiagMask;
  const bool nt = P.options & kDiagNtLoad;
  const uint32_t nst = EXT ? 0u : P.nstores;  // result stores per tile (EXT: drain fully)
  const DmaLanes<SWZ> L(lane);

  uint32_t tp = blockIdx.x * WAVES + wave;  // the planner's tile
  if (tp >= ntiles) return;
  auto desc_issue = [&](uint32_t u, uint32_t slot) -> uint32_t {  // descriptors of tile u
    if (u >= ntiles) return 0u;
    if (u * 64u + lane < n) {
      glds4(P.offset + u * 64u, 4u * lane, dslots + slot * 512u);
      glds4(P.caplen + u * 64u, 4u * lane, dslots + slot * 512u + 256u);
    }
    return 2u;  // VMEM instructions issued
  };
  // per-lane flags are kept as 0/1 words (VGPRs), not lane masks (SGPR pairs)
  auto desc_read = [&](uint32_t u, uint32_t slot, uint32_t &off, uint32_t &end) -> uint32_t {
    const uint32_t v = u * 64u + lane < n ? 1u : 0u;
    const uint32_t o = v ? min(lds_u32(dslots + slot * 512u + 4u * lane), dlen) : 0u;
    const uint32_t l = v ? min(lds_u32(dslots + slot * 512u + 256u + 4u * lane), dlen - o) : 0u;
    off = o;  // a packet reaching past data_len is clamped to the buffer
    end = o + l;
    return v;
  };
  auto covered = [&](const Window &w, uint32_t pend, uint32_t off, uint32_t end) -> uint32_t {
    return (pend && off >= w.base && end - w.base <= (uint32_t)STAGE) ? 1u : 0u;
  };

  // prologue: descriptors of the first two tiles, then the first window
  desc_issue(tp, 0);
  desc_issue(tp + nwaves, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint32_t slot = 0;  // descriptor slot of the planner's tile
  uint32_t off_p, end_p;
  uint32_t valid_p = desc_read(tp, slot, off_p, end_p);
  uint32_t pend_p = (valid_p && end_p - off_p <= fits) ? 1u : 0u;  // still to be given a window
  const uint32_t big0 = valid_p & (pend_p ^ 1u);
  Window Wd = plan_window<STAGE>(pend_p != 0, off_p, end_p);
  uint32_t cov_d = covered(Wd, pend_p, off_p, end_p);
  pend_p &= cov_d ^ 1u;
  issue_window<SWZ>(P.data, Wd, bufs, L, nt);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read before it is restaged
  uint32_t nwait = desc_issue(tp + 2u * nwaves, slot);

  // decode state: the window in flight belongs to tile td
  uint32_t td = tp, off_d = off_p, end_d = end_p;
  uint32_t valid_d = valid_p, big_d = big0;
  bool first_d = true;
  uint32_t cur = 0;  // buffer of the window to decode
  Out res{0, 0, 0, 0, 0, 0};
  PH_DECL
  for (;;) {
    PH_MARK(5);  // loop overhead / tail of the previous iteration
    // window cur landed: wait for all but the VMEM instructions issued after it
    if (!(P.options & kDiagNoWait)) {
      switch (nwait) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      }
    }
    PH_MARK(0);  // waiting for the window
    // ---- plan and issue the next window
    Window Wn{0, 0, 0};
    uint32_t cov_n = 0;
    bool has_next = false, new_tile = false;
    if (__any(pend_p != 0)) {  // more of the planner's tile
      Wn = plan_window<STAGE>(pend_p != 0, off_p, end_p);
      has_next = true;
    } else if (tp + nwaves < ntiles) {  // the next tile's first window
      tp += nwaves;
      slot ^= 1u;
      valid_p = desc_read(tp, slot, off_p, end_p);
      pend_p = (valid_p && end_p - off_p <= fits) ? 1u : 0u;
      Wn = plan_window<STAGE>(pend_p != 0, off_p, end_p);
      has_next = new_tile = true;
    }
    nwait = 0;
    if (has_next) {
      cov_n = covered(Wn, pend_p, off_p, end_p);
      pend_p &= cov_n ^ 1u;
      issue_window<SWZ>(P.data, Wn, bufs + (cur ^ 1u) * STAGE, L, nt);
      if (new_tile) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read before it is restaged
        nwait = desc_issue(tp + 2u * nwaves, slot);
      }
    }
    PH_MARK(1);  // planning and issuing the next window
    // ---- decode window cur (tile td, the lanes it covers)
    const uint32_t i = td * 64u + lane;
    const uint32_t clen = end_d - off_d;
    if (first_d && big_d)  // larger than a window
      res = decode_packet<EXT>(GlbSrc{P.data, off_d}, clen, T, P.first, options, EXT ? P.ext + i : nullptr,
                               P.detail ? P.detail + i : nullptr);
    const uint32_t buf = bufs + cur * STAGE;
    Seg sg{0, 0, 0};
    if (cov_d && (P.options & kDiagSkipDecode)) {  // diagnostics: data movement only
      res = Out{g_lds[buf + ((off_d - Wd.base) & ~15u)], 0, 0, 0, 0, 0};
    } else if (cov_d) {
      const LdsSrc<SWZ> src{buf, off_d - Wd.base};
      res = decode_packet<EXT>(src, clen, T, P.first, options, EXT ? P.ext + i : nullptr,
                               P.detail ? P.detail + i : nullptr);
    }
    PH_MARK(2);  // decode
    if constexpr (COOP) {  // long segments of this window: chunk prefix sums, shared
      if (__any(sg.b > sg.a)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        window_prefix<STAGE>(buf, pfx, lane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (sg.b > sg.a) {
          const uint32_t mid = lds_u32(pfx + 4u * sg.b) - lds_u32(pfx + 4u * sg.a);
          res.csum |= fold_le_not(sg.part + mid) << 16;
        }
      }
    }
    PH_MARK(3);  // cooperative checksum
    // ---- the tile is complete when the next window belongs to another tile (or none)
    if (!has_next || new_tile) {
      if (valid_d) store_out(P, i, res);
      nwait += nst;
    }
    PH_MARK(4);  // result stores, fallback list
    if (!has_next) {
      if constexpr (FAST) PH_FLUSH;
      break;
    }
    if (new_tile) {
      td = tp;
      off_d = off_p;
      end_d = end_p;
      valid_d = valid_p;
      big_d = (valid_p && end_p - off_p > fits) ? 1u : 0u;
      first_d = true;
    } else {
      first_d = false;
    }
    Wd = Wn;
    cov_d = cov_n;
    cur ^= 1u;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of the freed buffer done
  }
}

// The end of a fast wave: its fallback list — the generic DecodingLayerParser loop
// (decode_packet), one lane per listed packet, its bytes read from global memory — here, at the
// end of the wave, overlapped with the other waves' streaming.  (A second kernel over the lists
// cost a launch boundary, ~5 us per launch, even when every list is empty.)  The live state of
// the streaming loop is dead by now, so the generic decoder's registers do not raise the
// kernel's.  Each round first stages every listed packet's first K bytes in the lane's slot of
// the (now idle) window buffer `buf` with independent 16-byte loads, so the decoder's dependent
// header reads hit LDS (HybSrc); bytes past the slot (long segments) still come from global
// memory.
template <uint32_t K, bool CS = true, bool HASH = true>
__device__ __forceinline__ void decode_fallback_list(const KParams &P, uint32_t buf, uint32_t fb_start, uint32_t fb_c,
                                                     uint32_t lane, uint32_t dlen, uint32_t options) {
#if GPD_EXP & 8
  return;  // (A/B diagnostic build, tools/mix_diag.sh: the generic decodes skipped, wrong results)
#endif
#if GPD_EXP & 64
  options |= GPD_OPT_NO_FLOW_HASH;  // (A/B diagnostic: the generic decodes' hashes skipped)
#endif
#if GPD_EXP & 128
  options |= GPD_OPT_NO_CHECKSUMS;  // (A/B diagnostic: the generic decodes' checksums skipped)
#endif
  const uint32_t tot = fb_c;
  if (tot) {
    __threadfence_block();  // the entries other lanes of this wave stored
    const Tab<false> T{P.pages,    P.eth_base, P.tcp_base, P.udp_base, P.eth_bits,
                       P.tcp_bits, P.udp_bits, P.eth_mult, P.tcp_mult, P.udp_mult};
    const uint32_t slot = buf + K * lane;
    // readable bound of the batch contract (gpd.h gpd_batch: round_up(data_len, 16)): every
    // 16-byte chunk below it is whole, so no staging load reaches past it
    const uint64_t rlim = ((uint64_t)dlen + 15u) & ~15ull;
    // round j's descriptors and first K bytes; the next round's are fetched before this round
    // decodes (registers are free at the wave's end), so their three dependent global loads
    // (list entry, descriptor, bytes) overlap the decode instead of preceding it
    struct Fetch {
      uint32_t fi, off, len;
      v4u32 c[K / 16u];
    };
    auto fetch = [&](uint32_t j, Fetch &f) {
      const bool live = j < tot;
      const uint64_t e = live ? P.fb_list[fb_start + j] : 0ull;
      f.fi = (uint32_t)e;
      f.off = (uint32_t)(e >> 32);  // (clamped to dlen when listed)
      f.len = live ? min(P.caplen[f.fi], dlen - f.off) : 0u;
      const uint64_t gb = (uint64_t)f.off & ~15ull;
#pragma unroll
      for (uint32_t k = 0; k < K / 16u; k++)
        f.c[k] = (live && gb + 16u * k < rlim) ? *reinterpret_cast<const v4u32 *>(P.data + gb + 16u * k)
                                                : v4u32{0u, 0u, 0u, 0u};
    };
    Fetch cur;
    fetch(lane, cur);
    for (uint32_t j = lane; j - lane < tot; j += 64u) {
      const bool live = j < tot;
#pragma unroll
      for (uint32_t k = 0; k < K / 16u; k++) *reinterpret_cast<v4u32 *>(g_lds + slot + 16u * k) = cur.c[k];
      Fetch nxt;
      if (j + 64u - lane < tot) fetch(j + 64u, nxt);  // (wave-uniform)
      const uint32_t fi = cur.fi, off = cur.off, len = cur.len;
      const uint64_t gb = (uint64_t)off & ~15ull;
      // a round whose packets all lie inside their slots reads LDS only (no per-read bound)
      const bool all_in = __all(!live || (off & 15u) + len <= K);
#if GPD_EXP & 32
      if (live) {  // (A/B diagnostic: fetch, stage and store only)
        Out o{cur.c[0].x + (uint32_t)all_in, 0, 0, 0, 0, 0};
        store_out(P, fi, o);
      }
      cur = nxt;
      continue;
#endif
      if (live) {
        gpd_detail *det = P.detail ? P.detail + fi : nullptr;
        if (all_in)
          store_out(P, fi, decode_packet<false>(LdsSrc<false>{slot, off & 15u}, len, T, P.first, options, nullptr, det));
        else
          store_out(P, fi, decode_packet<false>(HybSrc<K>{P.data, off, gb, slot}, len, T, P.first, options, nullptr, det));
      }
      cur = nxt;
    }
  }
}

// ---------------------------------------------------------------- register-staged fast loop

// LDS bytes per wave of rs_kernel: one window (the next one waits in VGPRs), plus the chunk
// prefix sums of the cooperative checksum for windows of 8 KiB and more.
__host__ __device__ constexpr uint32_t rs_wave_lds_bytes(int stage) {
  return (uint32_t)stage + 16u + (stage >= 8192 ? (uint32_t)stage / 4u + 16u : 0u);
}

// Copy a register-staged window into LDS shifted up by s = 16 - 4Q - r bytes (0 < s < 16),
// with aligned ds_write_b128 only: LDS chunk m holds bytes [16m - s, 16m - s + 16) of the
// window, i.e. bytes [16 - s, 32 - s) of (chunk m-1 | chunk m).  Chunk m-1 of lane l is lane
// l-1's chunk (DPP wave_shr:1), lane 0 takes lane 63's of the previous 1-KiB row; one extra
// chunk past the window's end takes the last row's tail.
template <int Q, int NC, bool SUMS, typename V>
__device__ __forceinline__ void commit_shifted(const V (&wv)[NC], uint32_t buf, uint32_t lane, uint32_t r,
                                               uint32_t (&cs)[NC]) {
  uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0;  // lane 63's chunk of the previous row
#pragma unroll
  for (int j = 0; j <= NC; j++) {
    uint32_t D[8];
    if (j < NC) {
      D[4] = wv[j].x; D[5] = wv[j].y; D[6] = wv[j].z; D[7] = wv[j].w;
    } else {
      D[4] = D[5] = D[6] = D[7] = 0u;
    }
    D[0] = (uint32_t)__builtin_amdgcn_update_dpp((int)b0, (int)D[4], 0x138, 0xF, 0xF, false);
    D[1] = (uint32_t)__builtin_amdgcn_update_dpp((int)b1, (int)D[5], 0x138, 0xF, 0xF, false);
    D[2] = (uint32_t)__builtin_amdgcn_update_dpp((int)b2, (int)D[6], 0x138, 0xF, 0xF, false);
    D[3] = (uint32_t)__builtin_amdgcn_update_dpp((int)b3, (int)D[7], 0x138, 0xF, 0xF, false);
    V out;
    out.x = __builtin_amdgcn_alignbyte(D[Q + 1], D[Q], r);
    out.y = __builtin_amdgcn_alignbyte(D[Q + 2], D[Q + 1], r);
    out.z = __builtin_amdgcn_alignbyte(D[Q + 3], D[Q + 2], r);
    out.w = __builtin_amdgcn_alignbyte(D[Q + 4], D[Q + 3], r);
    if (j < NC || lane == 0u) *reinterpret_cast<V *>(g_lds + buf + 1024u * j + 16u * lane) = out;
    if (SUMS && j < NC)
      cs[j] = dot2(out.w, 0x00010001u, dot2(out.z, 0x00010001u, dot2(out.y, 0x00010001u, dot2(out.x, 0x00010001u, 0u))));
    if (j < NC) {
      b0 = (uint32_t)__builtin_amdgcn_readlane((int)D[4], 63);
      b1 = (uint32_t)__builtin_amdgcn_readlane((int)D[5], 63);
      b2 = (uint32_t)__builtin_amdgcn_readlane((int)D[6], 63);
      b3 = (uint32_t)__builtin_amdgcn_readlane((int)D[7], 63);
    }
  }
}

// P[c] (see window_prefix) from the LE-domain sums of the chunks as committed: LDS chunk
// 64 j + l is row j of lane l, so each row is one wave prefix scan on top of the rows below.
template <int NC>
__device__ __forceinline__ void rows_prefix(const uint32_t (&cs)[NC], uint32_t pfx, uint32_t lane) {
  uint32_t base = 0;
#pragma unroll
  for (int j = 0; j < NC; j++) {
    const uint32_t incl = wave_incl_scan(cs[j]);
    *reinterpret_cast<uint32_t *>(g_lds + pfx + 4u * (64u * j + lane)) = base + incl - cs[j];
    base += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  }
  if (lane == 0u) *reinterpret_cast<uint32_t *>(g_lds + pfx + 4u * 64u * NC) = base;
}

// The fast path's streaming loop with the window staged through registers: a window's bytes
// are loaded with plain 16-byte-per-lane loads (nt: read once) into VGPRs while the previous
// window is decoded out of the wave's single LDS buffer, then copied into that buffer with
// ds_write_b128 at the top of the next iteration.  Descriptors are register loads two tiles
// ahead.  Every load is compiler-visible, so each wait is the compiler's, placed at the first
// use.  Measured on this part (tools/micro/hbm_mix.hip): the decode kernel's 72-B-read /
// 32-B-write traffic shape streams at ~6.0 TB/s through registers against ~5.2 TB/s through
// LDS-DMA, and one LDS buffer per wave (instead of two) frees LDS for more waves.
// Iteration k:  commit window k (VGPR -> LDS)  ->  store the results of the tile the previous
// window finished (deferred one iteration, so that after the next window's loads nothing else
// is issued and the wait at the next commit covers exactly those loads)  ->  plan and load
// window k+1  ->  decode window k from LDS.
template <int STAGE, bool CS, bool HASH, int MINW, bool DEFER = false, bool RPFX = true, bool HO = false,
          bool AL = false, bool DIAG = kDiagBuild>
__global__ __launch_bounds__(256, MINW) void rs_kernel(KParams P) {
  constexpr int WAVES = 4;
  constexpr int NC = STAGE / 1024;              // 16-byte chunks per lane per window
  constexpr bool COOP = STAGE >= 8192;          // long segments: wave-cooperative checksum
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint32_t k = threadIdx.x; k < P.image_words; k += 64 * WAVES)
    reinterpret_cast<uint32_t *>(g_lds)[k] = P.image[k];
  __syncthreads();
  const uint32_t img = (P.image_words * 4u + 15u) & ~15u;
  const uint32_t buf = img + wave * rs_wave_lds_bytes(STAGE);
  const uint32_t pfx = buf + STAGE + 16u;
  const uint32_t n = P.n_dev ? min((uint32_t)P.n, *P.n_dev) : (uint32_t)P.n;
  const uint32_t ntiles = (n + 63u) >> 6;
  const uint32_t nwaves = gridDim.x * WAVES;
  const uint32_t dlen = (uint32_t)P.data_len;
  const uint32_t fits = (uint32_t)STAGE - 15u;
  const uint32_t options = P.options & ~kDiagMask;
  const FastCtx F{P.eth_mult, ((uint32_t)GPD_LT_PAYLOAD << 8) | (reinterpret_cast<const uint8_t *>(g_lds)[GPD_LT_PAYLOAD]),
                  (options & GPD_OPT_IGNORE_UNSUPPORTED) ? GPD_ST_OK : GPD_ST_UNSUPPORTED,
                  reinterpret_cast<const uint8_t *>(g_lds)[GPD_LT_FRAGMENT]};

  uint32_t tp = blockIdx.x * WAVES + wave;  // the planner's tile
  // Fallback list: wave w (tiles w, w + nwaves, ...) owns the region of 64 x its tile count
  // that starts after the regions of waves 0..w-1, so its appends need no atomic (a shared
  // counter took one same-address atomic per tile with leftovers; on the traffic mix that is
  // every tile, serialised at the memory side); the wave decodes its region after its tiles.
  const uint32_t gw = tp;
  const uint32_t fb_start = 64u * (gw * (ntiles / nwaves) + min(gw, ntiles % nwaves));
  uint32_t fb_c = 0;
  if (tp >= ntiles) {
    if (lane == 0u) P.fb_wcount[gw] = 0u;
    return;
  }
  auto dload = [&](uint32_t u, uint32_t &o, uint32_t &c) {  // descriptors of tile u
    const uint32_t i = u * 64u + lane;
    o = c = 0;
    if (u < ntiles && i < n) {
      o = __builtin_nontemporal_load(P.offset + i);
      c = __builtin_nontemporal_load(P.caplen + i);
    }
  };
  auto dread = [&](uint32_t u, uint32_t o_raw, uint32_t c_raw, uint32_t &off, uint32_t &end) -> uint32_t {
    const uint32_t v = u * 64u + lane < n ? 1u : 0u;
    const uint32_t o = v ? min(o_raw, dlen) : 0u;
    const uint32_t l = v ? min(c_raw, dlen - o) : 0u;
    off = o;  // a packet reaching past data_len is clamped to the buffer
    end = o + l;
    return v;
  };
  auto covered = [&](const Window &w, uint32_t pend, uint32_t off, uint32_t end) -> uint32_t {
    return (pend && off >= w.base && end - w.base <= (uint32_t)STAGE) ? 1u : 0u;
  };
  // Window loads are unconditional (a chunk past the window's end re-reads its first 16
  // bytes, a cached line), so every lane's registers come from this window's loads and the
  // compiler needs no merge of older values: its only wait is at the commit.
  v4u32 wv[NC];
  const bool ntl = (P.options & kDiagNtLoad) != 0;  // read-once policy (default on; A/B knob)
  auto wload = [&](const Window &w) {
#pragma unroll
    for (int j = 0; j < NC; j++) {
      const uint32_t c = 1024u * j + 16u * lane;
      const v4u32 *a = reinterpret_cast<const v4u32 *>(P.data + w.base + (c < w.nbytes ? c : 0u));
      wv[j] = ntl ? __builtin_nontemporal_load(a) : *a;
    }
    __builtin_amdgcn_sched_barrier(0);  // issue them here, ahead of the decode
  };
  // Shifted copies pay for themselves where windows hold many small frames; the host sets
  // the bit from the batch's mean slot (measured: tools/ab_shift.sh).
  const bool noshift = AL || (P.options & kShiftWindows) == 0;  // (AL: launched for unshifted windows only)
  auto wshift = [&](const Window &w) -> uint32_t { return noshift ? 0u : w.shift; };
  // COOP: the chunk prefix sums of a window are computed from the registers as it is
  // committed when the wave's previous window needed them (`pfx_pred`); otherwise, if this
  // window turns out to need them, window_prefix reads them back from LDS.
  bool pfx_pred = COOP, pfx_done = false;
  auto wcommit = [&](const Window &w) {
    const uint32_t sh = wshift(w);
    uint32_t cs[NC];
    pfx_done = false;
    const bool sums = COOP && RPFX && pfx_pred && sh == 0u;
    if (sh == 0u) {
#pragma unroll
      for (int j = 0; j < NC; j++)
        *reinterpret_cast<v4u32 *>(g_lds + buf + 1024u * j + 16u * lane) = wv[j];
      if (sums) {
#pragma unroll
        for (int j = 0; j < NC; j++)
          cs[j] = dot2(wv[j].w, 0x00010001u, dot2(wv[j].z, 0x00010001u,
                       dot2(wv[j].y, 0x00010001u, dot2(wv[j].x, 0x00010001u, 0u))));
      }
    } else {
      // (shifted windows leave the prefix to window_prefix: measured, pcap64 +2 % otherwise)
      const uint32_t o = 16u - sh, r = o & 3u;
      switch (o >> 2) {
        case 0: commit_shifted<0, NC, false>(wv, buf, lane, r, cs); break;
        case 1: commit_shifted<1, NC, false>(wv, buf, lane, r, cs); break;
        case 2: commit_shifted<2, NC, false>(wv, buf, lane, r, cs); break;
        default: commit_shifted<3, NC, false>(wv, buf, lane, r, cs); break;
      }
    }
    if (sums) {
      rows_prefix<NC>(cs, pfx, lane);
      pfx_done = true;
    }
  };

  // prologue: this tile's descriptors (waited for), the next two tiles' in flight
  uint32_t o_a, c_a, o_b, c_b, off_p, end_p;
  {
    uint32_t o0, c0;
    dload(tp, o0, c0);
    dload(tp + nwaves, o_a, c_a);
    dload(tp + 2u * nwaves, o_b, c_b);
    (void)dread(tp, o0, c0, off_p, end_p);
  }
  uint32_t valid_p = tp * 64u + lane < n ? 1u : 0u;
  uint32_t pend_p = (valid_p && end_p - off_p <= fits) ? 1u : 0u;
  uint32_t l3m = 14u;  // network header offset mod 16 the window shift aims at (learned)
  Window Wd = plan_window<STAGE>(pend_p != 0, off_p, end_p, l3m);
  uint32_t cov_d = covered(Wd, pend_p, off_p, end_p);
  pend_p &= cov_d ^ 1u;
  wload(Wd);
  uint32_t td = tp, off_d = off_p, end_d = end_p, valid_d = valid_p;
  uint32_t big_d = valid_p & ((end_p - off_p <= fits) ? 0u : 1u);
  bool first_d = true;
  Out res{0, 0, 0, 0, 0, 0};
  uint32_t fb = 0;
  Hdr hh{};          // HO: the lane's packet as seg_pass staged it
  uint32_t got = 0;  // HO: ... in one of this tile's windows (2: decoded there in full)
  const bool vxreg = (P.decoders & GPD_DEC_VXLAN) != 0;
  // results of a finished tile, stored one iteration later
  bool st_pending = false;
  uint32_t st_i = 0, st_valid = 0;
  Out st_res{0, 0, 0, 0, 0, 0};
  PH_DECL
  for (;;) {
    PH_MARK(5);  // loop overhead / tail of the previous iteration
    // Wait order: every load issued in the previous iteration (descriptors two tiles ahead,
    // then window k) is older than anything the wait below could over-cover, so the
    // compiler's vmcnt at the first use of window k's registers costs nothing extra.
    wcommit(Wd);  // window k: registers -> LDS (the compiler waits for its loads here)
    PH_MARK(0);  // waiting for the window (and copying it)
    // ---- plan the next window (the next tile's descriptors landed long ago)
    Window Wn{0, 0, 0};
    uint32_t cov_n = 0;
    bool has_next = false, new_tile = false;
    if (__any(pend_p != 0)) {  // more of the planner's tile
      has_next = true;
    } else if (tp + nwaves < ntiles) {  // the next tile's first window
      tp += nwaves;
      valid_p = dread(tp, o_a, c_a, off_p, end_p);
      o_a = o_b;
      c_a = c_b;
      pend_p = (valid_p && end_p - off_p <= fits) ? 1u : 0u;
      has_next = new_tile = true;
    }
    // ---- the previous tile's results (a fallback lane's entry is rewritten later), issued
    // before the next loads so that nothing follows those loads until their wait
    if (DEFER && st_pending) {
      if (st_valid) store_out(P, st_i, st_res);
      st_pending = false;
    }
    if (new_tile) dload(tp + 2u * nwaves, o_b, c_b);
    if (has_next) {
      Wn = plan_window<STAGE>(pend_p != 0, off_p, end_p, l3m);
      cov_n = covered(Wn, pend_p, off_p, end_p);
      pend_p &= cov_n ^ 1u;
      wload(Wn);
    }
    PH_MARK(1);  // stores of the previous tile, planning and issuing the next window
    // ---- decode window k (tile td, the lanes it covers)
    const uint32_t i = td * 64u + lane;
    if (first_d && big_d) fb = 1;  // larger than a window: the generic decoder
    Seg sg{0, 0, 0};
    if (DIAG && cov_d && (P.options & kDiagSkipDecode)) {  // diagnostics: data movement only
      res = Out{g_lds[buf + ((off_d - Wd.base) & ~15u)], 0, 0, 0, 0, 0};
    } else if (cov_d) {
      if (HO) {
        seg_pass<COOP>(buf + wshift(Wd) + (off_d - Wd.base), end_d - off_d, buf, hh, sg, F, vxreg);
        got = 1;
      } else if (!fast_decode<CS, HASH, COOP, false, AL>(buf + wshift(Wd) + (off_d - Wd.base), end_d - off_d, F,
                                                          res, buf, sg)) {
        fb = 1;
      }
    }
    const uint64_t vxm = HO ? __ballot(cov_d && hh.ok == 2u) : 0ull;
    if (HO && vxm) {  // VXLAN: its inner headers are not staged
      // A few VXLAN lanes go to the generic decoder: the per-window two-pass decode would run
      // for the whole wave in every window that holds one (on the traffic mix, 5 % VXLAN,
      // nearly every window: 0.44 ms against 0.29 without VXLAN registered).  Many lanes
      // (VXLAN-heavy long-frame traffic) decode in full while their window is here.
      if (cov_d && hh.ok == 2u) {
        got = 2;
        if (__popcll(vxm) <= 16) {
          fb = 1;
        } else if (!fast_decode<CS, HASH, COOP, false, AL>(buf + wshift(Wd) + (off_d - Wd.base), end_d - off_d,
                                                            F, res, buf, sg)) {
          fb = 1;
        }
      }
    }
    if constexpr (!AL) {  // learn where this wave's network headers sit (mod 16) for the next windows' shift
      const uint32_t no = res.hoff & 0xFFFFu;
      const uint64_t hm = __ballot(cov_d && no != 0xFFFFu);
      if (hm) l3m = (uint32_t)__builtin_amdgcn_readlane((int)no, (int)__builtin_ctzll(hm)) & 15u;
    }
    PH_MARK(2);  // decode
    if constexpr (COOP) {  // long segments of this window: chunk prefix sums, shared
      pfx_pred = __any(sg.b > sg.a);
      if (pfx_pred) {
        if (!pfx_done) window_prefix<STAGE>(buf, pfx, lane);
        if (sg.b > sg.a) {
          const uint32_t mid = lds_u32(pfx + 4u * sg.b) - lds_u32(pfx + 4u * sg.a);
          if (HO && got == 1u) hh.sum = sg.part + mid;
          else res.csum |= fold_le_not(sg.part + mid) << 16;
        }
      }
    }
    PH_MARK(3);  // cooperative checksum
    // ---- the tile is complete when the next window belongs to another tile (or none)
    if (!has_next || new_tile) {
      if (HO && got == 1u) {  // the tile's one decode, from the staged headers
        Seg none{0, 0, 0};
        if (!fast_decode<CS, HASH, COOP, true>(0u, end_d - off_d, F, res, buf, none, &hh)) fb = 1;
      }
      got = 0;
      const uint64_t m = __ballot(fb != 0);  // the tile's leftovers go to the fallback list
      if (m) {
        if (fb) P.fb_list[fb_start + fb_c + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = ((uint64_t)off_d << 32) | i;
        fb_c += (uint32_t)__popcll(m);
      }
      const uint32_t keep = valid_d && !fb;  // a listed packet is stored once, by its decode below
      fb = 0;
      if (DEFER) {
        st_pending = true;
        st_i = i;
        st_valid = keep;
        st_res = res;
      } else if (keep) {
        store_out(P, i, res);
      }
    }
    PH_MARK(4);  // fallback list (and this tile's stores when not deferred)
    if (!has_next) {
      if (DEFER && st_valid) store_out(P, st_i, st_res);
      PH_FLUSH;
      break;
    }
    if (new_tile) {
      td = tp;
      off_d = off_p;
      end_d = end_p;
      valid_d = valid_p;
      big_d = (valid_p && end_p - off_p > fits) ? 1u : 0u;
      first_d = true;
    } else {
      first_d = false;
    }
    Wd = Wn;
    cov_d = cov_n;
  }
  if (lane == 0u) P.fb_wcount[gw] = fb_c;  // (gpd_last_launch_split's count)
  decode_fallback_list<(uint32_t)STAGE / 64u, CS, HASH>(P, buf, fb_start, fb_c, lane, dlen, options);
}

// ---------------------------------------------------------------- round-based header-once loop
// ro_kernel (gpd_tuning.header_once = 2): the header-once decode of long frames, with each
// 64-packet tile's bytes streamed as ONE contiguous run in rounds of 8 KiB — the traffic shape
// of the attainable probe — instead of windows cut at packet boundaries (IMIX: 3.35 windows of
// 6.8 KiB per 22.7-KiB tile, 21 % of each window's loads re-reading its first chunk).
//  * A packet's header (its first <= 128 bytes) is staged in the round that holds them; the
//    previous round's last 144 bytes stay in front of the window, so a header may straddle the
//    boundary.
//  * Its transport segment [S, E) is summed from the tile's running chunk prefix sums G: the
//    masked head chunk and G(A) where the header is staged, G(B) and the masked tail chunk in
//    the round that holds B (A = S rounded up, B = E rounded down to 16) — one compare per
//    pending lane per round until then.  So a segment may span any number of rounds, and a
//    packet larger than a window stays on the fast path.  An odd-aligned segment is summed in
//    the other byte order (RFC 1071 §2(B)) and swapped back.
//  * The straight-line decode runs once per tile from the staged headers (fast_decode<HO>).
//  * A tile whose packets do not lie nearly back to back (a shuffled or scattered layout: the
//    run much longer than its bytes) is left to the generic decoder whole.
constexpr uint32_t kRoStage = 8192;
constexpr uint32_t kRoCarry = 144;    // bytes of the previous round kept in front of the window
constexpr uint32_t kRoPfxCarry = 12;  // prefix words kept in front of the prefix array (9 used)
constexpr uint32_t kRoHdr = 128;      // header bytes a packet's staging (hdr_parse) reads at most
__host__ __device__ constexpr uint32_t ro_wave_lds_bytes() {
  return kRoCarry + kRoStage + 16u + 4u * kRoPfxCarry + 4u * (kRoStage / 16u + 1u) + 12u;
}
static_assert(ro_wave_lds_bytes() % 16u == 0u, "ro_kernel: 16-byte aligned wave regions");

// LE-domain sum s + bytes [lo, hi) of the aligned 16-byte LDS chunk at a (0 <= lo <= hi <= 16).
__device__ __forceinline__ uint32_t chunk_part(uint32_t a, uint32_t lo, uint32_t hi, uint32_t s) {
  const uint4 q = *reinterpret_cast<const uint4 *>(g_lds + a);
  const uint32_t l8 = lo * 8u, h8 = hi * 8u;
  const uint64_t keep_lo = (l8 >= 64u ? 0ull : ~0ull << l8) & (h8 >= 64u ? ~0ull : (1ull << h8) - 1ull);
  const uint64_t keep_hi = (l8 >= 64u ? ~0ull << (l8 - 64u) : ~0ull) &
                           (h8 <= 64u ? 0ull : (h8 >= 128u ? ~0ull : (1ull << (h8 - 64u)) - 1ull));
  const uint64_t x = ((((uint64_t)q.y << 32) | q.x) & keep_lo), y = ((((uint64_t)q.w << 32) | q.z) & keep_hi);
  s = dot2((uint32_t)x, 0x00010001u, s);
  s = dot2((uint32_t)(x >> 32), 0x00010001u, s);
  s = dot2((uint32_t)y, 0x00010001u, s);
  return dot2((uint32_t)(y >> 32), 0x00010001u, s);
}

// min / sum over the wave (all 64 lanes take part)
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
  return v;
}

template <bool CS, bool HASH, int MINW>
__global__ __launch_bounds__(256, MINW) void ro_kernel(KParams P) {
  constexpr int WAVES = 4;
  constexpr int NC = (int)kRoStage / 1024;  // 16-byte chunks per lane per round
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint32_t k = threadIdx.x; k < P.image_words; k += 64 * WAVES)
    reinterpret_cast<uint32_t *>(g_lds)[k] = P.image[k];
  __syncthreads();
  const uint32_t img = (P.image_words * 4u + 15u) & ~15u;
  const uint32_t buf = img + wave * ro_wave_lds_bytes() + kRoCarry;  // the round's window
  const uint32_t pfx = buf + kRoStage + 16u + 4u * kRoPfxCarry;      // its chunk prefix sums P[0..512]
  const uint32_t n = P.n_dev ? min((uint32_t)P.n, *P.n_dev) : (uint32_t)P.n;
  const uint32_t ntiles = (n + 63u) >> 6;
  const uint32_t nwaves = gridDim.x * WAVES;
  const uint32_t dlen = (uint32_t)P.data_len;
  const uint32_t options = P.options & ~kDiagMask;
  const FastCtx F{P.eth_mult, ((uint32_t)GPD_LT_PAYLOAD << 8) | (reinterpret_cast<const uint8_t *>(g_lds)[GPD_LT_PAYLOAD]),
                  (options & GPD_OPT_IGNORE_UNSUPPORTED) ? GPD_ST_OK : GPD_ST_UNSUPPORTED,
                  reinterpret_cast<const uint8_t *>(g_lds)[GPD_LT_FRAGMENT]};
  const bool vxreg = (P.decoders & GPD_DEC_VXLAN) != 0;

  uint32_t tp = blockIdx.x * WAVES + wave;  // the planner's tile
  const uint32_t gw = tp;  // this wave's fallback region (see rs_kernel)
  const uint32_t fb_start = 64u * (gw * (ntiles / nwaves) + min(gw, ntiles % nwaves));
  uint32_t fb_c = 0;
  if (tp >= ntiles) {
    if (lane == 0u) P.fb_wcount[gw] = 0u;
    return;
  }
  auto dload = [&](uint32_t u, uint32_t &o, uint32_t &c) {  // descriptors of tile u
    const uint32_t i = u * 64u + lane;
    o = c = 0;
    if (u < ntiles && i < n) {
      o = __builtin_nontemporal_load(P.offset + i);
      c = __builtin_nontemporal_load(P.caplen + i);
    }
  };
  auto dread = [&](uint32_t u, uint32_t o_raw, uint32_t c_raw, uint32_t &off, uint32_t &end) -> uint32_t {
    const uint32_t v = u * 64u + lane < n ? 1u : 0u;
    const uint32_t o = v ? min(o_raw, dlen) : 0u;
    const uint32_t l = v ? min(c_raw, dlen - o) : 0u;
    off = o;  // a packet reaching past data_len is clamped to the buffer
    end = o + l;
    return v;
  };
  auto fb_append = [&](uint32_t i, uint32_t off, uint32_t fb) {  // the tile's leftovers: the fallback list
    const uint64_t m = __ballot(fb != 0);
    if (m) {
      if (fb) P.fb_list[fb_start + fb_c + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = ((uint64_t)off << 32) | i;
      fb_c += (uint32_t)__popcll(m);
    }
  };
  // A tile's byte run [t0, t0 + 8192 nr): its packets' extent, in nr rounds; nr = 0 when the
  // packets are not nearly back to back (or hold no bytes): the tile goes to the fallback list.
  uint32_t t0_p = 0, t1_p = 0, nr_p = 0;
  auto tile_plan = [&](uint32_t valid, uint32_t off, uint32_t end) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane(wave_min(valid ? (off & ~15u) : 0xFFFFFFFFu));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(wave_max(valid ? end : 0u));
    const uint32_t bytes = __builtin_amdgcn_readfirstlane(wave_sum(valid ? min(end - off, 1u << 24) : 0u));
    t0_p = lo;
    t1_p = hi;
    const uint32_t nr = (uint32_t)(((uint64_t)(hi - lo) + kRoStage - 1u) / kRoStage);
    // (a header's round is kept in 16 bits of the lane state: a run of more than 0xFFFF rounds,
    // 512 MiB, goes to the fallback list too)
    nr_p = (hi > lo && (uint64_t)(hi - lo) <= 2ull * bytes + kRoStage && nr <= 0xFFFFu) ? nr : 0u;
  };
  v4u32 wv[NC];
  auto rload = [&](uint32_t base, uint32_t nbytes) {  // one round's bytes into the registers
#pragma unroll
    for (int j = 0; j < NC; j++) {
      const uint32_t c = 1024u * j + 16u * lane;
      wv[j] = __builtin_nontemporal_load(reinterpret_cast<const v4u32 *>(P.data + base + (c < nbytes ? c : 0u)));
    }
    __builtin_amdgcn_sched_barrier(0);  // issue them here, ahead of the decode
  };

  // prologue: the first tile that has rounds (tiles without go to the fallback list whole)
  uint32_t o_a, c_a, o_b, c_b, off_p, end_p, valid_p;
  {
    uint32_t o0, c0;
    dload(tp, o0, c0);
    dload(tp + nwaves, o_a, c_a);
    dload(tp + 2u * nwaves, o_b, c_b);
    valid_p = dread(tp, o0, c0, off_p, end_p);
  }
  tile_plan(valid_p, off_p, end_p);
  bool any = true;
  while (nr_p == 0u) {
    fb_append(tp * 64u + lane, off_p, valid_p);
    if (tp + nwaves >= ntiles) { any = false; break; }
    tp += nwaves;
    valid_p = dread(tp, o_a, c_a, off_p, end_p);
    o_a = o_b;
    c_a = c_b;
    dload(tp + 2u * nwaves, o_b, c_b);
    tile_plan(valid_p, off_p, end_p);
  }
  if (any) {
    uint32_t rp = 0;  // the planner's round of tile tp
    rload(t0_p, min(kRoStage, ((t1_p - t0_p) + 15u) & ~15u));
    // decode state: round rd of tile td (its run from t0_d, nr_d rounds)
    uint32_t td = tp, t0_d = t0_p, nr_d = nr_p, rd = 0;
    uint32_t off_d = off_p, end_d = end_p;
    uint32_t base = 0;  // G at the round's start: the sum of the tile's earlier rounds' chunks
    // per lane, packed (registers bound the waves per SIMD): ls = its header's round (bits 0-15)
    // | staged | tail pending | odd segment start | fallback | tail bytes (20-23) | valid (24);
    // tB: the pending tail's B (tile-relative); part: the segment's partial sum
    constexpr uint32_t kStaged = 1u << 16, kPend = 1u << 17, kOdd = 1u << 18, kFb = 1u << 19, kValid = 1u << 24;
    uint32_t ls = valid_p ? kValid : 0u, tB = 0, part = 0;
    Hdr hh;  // (written where the header is staged; read only for a staged lane)
    for (;;) {
      // ---- the previous round's last bytes and prefix words in front of this round's
      if (rd > 0u) {
        if (lane < 9u) {
          const v4u32 q = *reinterpret_cast<const v4u32 *>(g_lds + buf + kRoStage - 144u + 16u * lane);
          const uint32_t pc = lds_u32(pfx + 4u * (503u + lane)) - lds_u32(pfx + 4u * 512u);
          *reinterpret_cast<v4u32 *>(g_lds + buf - 144u + 16u * lane) = q;
          *reinterpret_cast<uint32_t *>(g_lds + pfx - 36u + 4u * lane) = pc;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      // ---- commit round rd: registers -> LDS, and its chunk prefix sums from the registers
      {
        uint32_t cs[NC];
#pragma unroll
        for (int j = 0; j < NC; j++) {
          *reinterpret_cast<v4u32 *>(g_lds + buf + 1024u * j + 16u * lane) = wv[j];
          cs[j] = dot2(wv[j].w, 0x00010001u, dot2(wv[j].z, 0x00010001u,
                       dot2(wv[j].y, 0x00010001u, dot2(wv[j].x, 0x00010001u, 0u))));
        }
        rows_prefix<NC>(cs, pfx, lane);
      }
      // ---- plan and load the next round (the rest of this tile, or the next tile with rounds)
      bool has_next = false, new_tile = false;
      if (rp + 1u < nr_p) {
        rp++;
        has_next = true;
      } else {
        while (tp + nwaves < ntiles) {
          tp += nwaves;
          valid_p = dread(tp, o_a, c_a, off_p, end_p);
          o_a = o_b;
          c_a = c_b;
          dload(tp + 2u * nwaves, o_b, c_b);
          tile_plan(valid_p, off_p, end_p);
          if (nr_p) {
            rp = 0;
            has_next = new_tile = true;
            break;
          }
          fb_append(tp * 64u + lane, off_p, valid_p);
        }
      }
      if (has_next) {
        const uint32_t rb = t0_p + kRoStage * rp;
        rload(rb, min(kRoStage, (t1_p - rb + 15u) & ~15u));
      }
      // ---- round rd of tile td
      const uint32_t R0 = t0_d + kRoStage * rd;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the committed round is readable)
      if (rd == 0u && (ls & kValid)) {
        const uint32_t need = max(min(off_d + kRoHdr, end_d), off_d + 1u);
        ls = kValid | ((need - 1u - t0_d) / kRoStage);
      }
      const bool here = (ls & kValid) && (ls & 0xFFFFu) == rd;
      if (here) {  // stage the header; the segment's head, and its tail if in this round
        const uint32_t pl = buf + off_d - R0;  // (>= buf - 128: the carry)
        uint32_t l4 = 0, seg = 0;
        ls |= kStaged;
        if (hdr_parse(pl, end_d - off_d, hh, F, vxreg, l4, seg) && CS) {
          const uint32_t S = pl + l4, E = S + seg, A = (S + 15u) & ~15u, B = E & ~15u;
          ls |= (S & 1u) ? kOdd : 0u;
          if (E <= A) {  // the whole segment inside its first chunk
            part = (A > S) ? chunk_part(A - 16u, S & 15u, E - (A - 16u), 0u) : 0u;
          } else {
            part = (A > S) ? chunk_part(A - 16u, S & 15u, 16u, 0u) : 0u;
            part -= base + lds_u32(pfx + 4u * (uint32_t)((int32_t)(A - buf) >> 4));
            if (E > B ? B < buf + kRoStage : B <= buf + kRoStage) {
              // (B may lie in the carry, in front of buf: a frame whose header round is set by
              // its 128 header bytes while its segment ends before the round, e.g. a short IP
              // packet in a long frame)
              part += base + lds_u32(pfx + 4u * (uint32_t)((int32_t)(B - buf) >> 4));
              if (E > B) part = chunk_part(B, 0u, E - B, part);
            } else {
              ls |= kPend | ((E - B) << 20);
              tB = B - buf + R0 - t0_d;
            }
          }
        }
        // VXLAN frames (their inner headers are not staged) take the generic decoder: a second
        // straight-line decode in the loop would cost the kernel its third wave per SIMD
        if (hh.ok == 2u) ls |= kFb;
      } else if (ls & kPend) {  // a segment's tail in this round?
        const uint32_t rel = tB - (R0 - t0_d), tl = (ls >> 20) & 15u;
        if (tl ? rel < kRoStage : rel <= kRoStage) {
          part += base + lds_u32(pfx + 4u * (rel >> 4));
          if (tl) part = chunk_part(buf + rel, 0u, tl, part);
          ls &= ~kPend;
        }
      }
      base += lds_u32(pfx + 4u * 512u);
      // ---- the tile is complete after its last round: one decode from the staged headers
      if (rd + 1u == nr_d) {
        Out res;
        uint32_t fb = 0;
        if ((ls & (kStaged | kPend | kFb)) == kStaged) {
          // an odd-aligned segment's sum is in the other byte order: folded and swapped back
          const uint32_t f1 = (part >> 16) + (part & 0xFFFFu), f2 = (f1 >> 16) + (f1 & 0xFFFFu);
          hh.sum = (ls & kOdd) ? __builtin_amdgcn_perm(0u, f2, 0x0C0C0001u) : part;
          Seg none{0, 0, 0};
          if (!fast_decode<CS, HASH, true, true>(0u, end_d - off_d, F, res, buf, none, &hh)) fb = 1;
        } else {
          fb = 1;
        }
        const uint32_t i = td * 64u + lane;
        const uint32_t valid = (ls & kValid) ? 1u : 0u;
        fb_append(i, off_d, valid ? fb : 0u);
        if (valid && !fb) store_out(P, i, res);
      }
      if (!has_next) break;
      if (new_tile) {
        td = tp;
        t0_d = t0_p;
        nr_d = nr_p;
        rd = 0;
        off_d = off_p;
        end_d = end_p;
        ls = valid_p ? kValid : 0u;
        base = 0;
      } else {
        rd++;
      }
    }
  }
  if (lane == 0u) P.fb_wcount[gw] = fb_c;  // (gpd_last_launch_split's count)
  decode_fallback_list<kRoStage / 64u, CS, HASH>(P, buf, fb_start, fb_c, lane, dlen, options);
}

// ---------------------------------------------------------------- loader / decoder split (round 6)
// sp_kernel (gpd_tuning.split): 4 KiB windows of small frames with the two jobs of a wave split
// between waves.  A workgroup is 8 waves: wave 0 only LOADS — each tile's 64 offsets and caplens
// by LDS-DMA kSpAhead tiles ahead, then its window (planned from them) by LDS-DMA, a steady
// kSpAhead + 1 windows in flight per workgroup — into a ring of kSpSlots slots; waves 1..7 only
// DECODE, tile g of the workgroup by wave 1 + g mod 7, straight from its slot.  In LDS:
// ready[s] = tile + 1 once the tile's window landed in slot s, freed[s] = the slot's use count once
// its decoder is done with it.  Every wait is an explicit counted vmcnt (the loader's VMEM
// instructions are all LDS-DMA, so the compiler inserts none) and every spin is capped (a capped
// spin leaves the tile to the fallback list, never a wrong result or a hang).  Measured why
// (tools/micro/stream_split.hip, profiles/r06/micro/): one loader per workgroup keeps the request
// stream steady while the decode runs on seven waves, where the register loop's waves each
// alternate a burst of loads with a stretch of decode.
// A packet the tile's one window does not cover (the tile's bytes exceed 4 KiB) goes to the
// decoder wave's fallback list, decoded after the barrier that ends the ring.
constexpr int kSpWaves = 8;                                 // 1 loader + 7 decoders
constexpr uint32_t kSpDec = kSpWaves - 1;
constexpr uint32_t kSpSlots = 12;                           // ring slots per workgroup
constexpr uint32_t kSpAhead = 3;                            // tiles in flight ahead of the oldest (6 deeper: slower)
constexpr uint32_t kSpWin = 4096, kSpPad = 128;             // window, read-past pad
constexpr uint32_t kSpDesc = kSpWin + kSpPad;               // 64 offsets + 64 caplens
constexpr uint32_t kSpHdr = kSpDesc + 512;                  // {base, nbytes}
constexpr uint32_t kSpSlotBytes = kSpHdr + 16;
constexpr uint32_t kSpSpinCap = 1u << 22;
__host__ __device__ constexpr uint32_t sp_lds_bytes() { return kSpSlots * kSpSlotBytes + 8u * kSpSlots + 16u; }
static_assert(kSpSlots >= kSpAhead + 1u + kSpDec + 1u, "sp ring: in flight + decoding + one");

// min / max over the 64 lanes without LDS (the loader's critical path): DPP row shifts within each
// row of 16, then the row broadcasts, the result in lane 63
__device__ __forceinline__ uint32_t dpp_min(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x111, 0xF, 0xF, false));  // row_shr:1
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x112, 0xF, 0xF, false));  // row_shr:2
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x114, 0xF, 0xF, false));  // row_shr:4
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x118, 0xF, 0xF, false));  // row_shr:8
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x142, 0xA, 0xF, false));  // row_bcast:15
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint32_t dpp_max(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ uint32_t *sp_word(uint32_t a) {
  return static_cast<uint32_t *>(__builtin_assume_aligned(g_lds + a, 4));
}
__device__ __forceinline__ uint32_t sp_ld(uint32_t a) {  // (every lane reads the same word: uniform)
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(sp_word(a), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void sp_st(uint32_t a, uint32_t v) {
  __hip_atomic_store(sp_word(a), v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <bool CS, bool HASH>
__global__ __launch_bounds__(64 * kSpWaves, 4) void sp_kernel(KParams P) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint32_t k = threadIdx.x; k < P.image_words; k += 64 * kSpWaves)
    reinterpret_cast<uint32_t *>(g_lds)[k] = P.image[k];
  const uint32_t img = (P.image_words * 4u + 15u) & ~15u;
  const uint32_t ring = img, ready = ring + kSpSlots * kSpSlotBytes, freed = ready + 4u * kSpSlots;
  const uint32_t abort = freed + 4u * kSpSlots;  // set by a loader whose slot wait hit the cap
  if (threadIdx.x <= 2u * kSpSlots) *sp_word(ready + 4u * threadIdx.x) = 0u;
  __syncthreads();
  const uint32_t n = P.n_dev ? min((uint32_t)P.n, *P.n_dev) : (uint32_t)P.n;
  const uint32_t ntiles = (n + 63u) >> 6;
  const uint32_t nb = gridDim.x, b = blockIdx.x;
  const uint32_t dlen = (uint32_t)P.data_len;
  const uint32_t options = P.options & ~kDiagMask;
  // this workgroup's tiles: one contiguous run, t = c0 + g, g < G.  (Against the grid-strided
  // order t = b + g nb, where the whole grid reads one 2-MiB stretch at a time: faster in 71 of
  // 80 (box, buffer placement) pairs, by 1-3 %, at most 1 % slower in the rest;
  // tools/mode_probe.py, DESIGN.md §5 sp_kernel.)
  const uint32_t q = ntiles / nb, r = ntiles % nb;
  const uint32_t G = q + (b < r ? 1u : 0u);
  const uint32_t c0 = b * q + min(b, r);
  auto tile_of = [&](uint32_t g) { return c0 + g; };
  auto slot_at = [&](uint32_t g) { return ring + (g % kSpSlots) * kSpSlotBytes; };
  if (wave == 0u) {
    __builtin_amdgcn_s_setprio(3);  // the loader is every decoder's critical path: it issues first
    // ---- the loader.  Issue order per tile g: desc(g) (two DMAs), window(g) (four).  The window
    // is planned from three scalar loads issued kSpAhead tiles earlier (the first packet's offset,
    // the last packet's offset and caplen: packets in lane order, as batches are laid out; a
    // packet outside the window goes to its decoder's fallback list), so the loader's vector
    // memory stream holds only its DMAs and every wait on it is the counted one below.
    typedef const __attribute__((address_space(4))) uint32_t *cu32;
    const cu32 soff = reinterpret_cast<cu32>(reinterpret_cast<uintptr_t>(P.offset));
    const cu32 scap = reinterpret_cast<cu32>(reinterpret_cast<uintptr_t>(P.caplen));
    struct Plan {
      uint32_t o0, ol, cl;
    };
    // Each scalar plan load fetches its own 128-B line from HBM, which the descriptor DMA then
    // fetches again (profiles/r06/micro/desc_plan_ab/).  When the batch averages >= 63 bytes per
    // packet a tile's packets span ~4 KiB anyway: the window is then always 4 KiB (capped at the
    // batch end) and one load, the first packet's offset, plans it.
    const bool fixedw = (uint64_t)dlen >= 63ull * n;
    auto plan_load = [&](uint32_t g) -> Plan {  // (uniform: scalar loads)
      const uint32_t t = tile_of(g), i0 = t * 64u, il = min(i0 + 63u, n - 1u);
      if (fixedw) return Plan{soff[i0], 0u, 0u};
      return Plan{soff[i0], soff[il], scap[il]};
    };
    Plan pl[kSpAhead];
#pragma unroll
    for (uint32_t k = 0; k < kSpAhead; k++) pl[k] = k < G ? plan_load(k) : Plan{0, 0, 0};
    uint32_t sig = 0;  // tiles signalled ready
    bool stop = false;
    // tile g's plan sits in pl[g mod kSpAhead] (the inner loop unrolled: no register moves, and each
    // plan is read before the next prefetch into its registers is issued — scalar loads return out
    // of order, so any wait on them is lgkmcnt(0))
    for (uint32_t g0 = 0; g0 < G && !stop; g0 += kSpAhead) {
#pragma unroll
      for (uint32_t kk = 0; kk < kSpAhead; kk++) {
        const uint32_t g = g0 + kk;
        if (g >= G || stop) break;
        const uint32_t s = slot_at(g), t = tile_of(g);
        if (g >= kSpSlots) {  // the slot's previous tile must be decoded
          const uint32_t need = g / kSpSlots;
          if (sp_ld(freed + 4u * (g % kSpSlots)) < need) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // whatever landed goes out first
            for (; sig < g; sig++)
              if (lane == 0u) sp_st(ready + 4u * (sig % kSpSlots), sig + 1u);
            uint32_t spins = 0;
            while (sp_ld(freed + 4u * (g % kSpSlots)) < need && ++spins < kSpSpinCap) __builtin_amdgcn_s_sleep(1);
            if (spins >= kSpSpinCap) {  // (never expected) stop loading: the decoders send every
              if (lane == 0u) sp_st(abort, 1u);  // tile not signalled to the fallback list
              stop = true;
              break;
            }
          }
        }
        // plan: [base, base + nbytes), base the first packet rounded down to 16, to the last
        // packet's end (at most 4 KiB)
        const uint32_t o0 = min(pl[kk].o0, dlen), ol = min(pl[kk].ol, dlen), el = ol + min(pl[kk].cl, dlen - ol);
        const uint32_t base = __builtin_amdgcn_readfirstlane(o0 & ~15u);
        const uint32_t nbytes = __builtin_amdgcn_readfirstlane(
            fixedw ? min((dlen - base + 15u) & ~15u, kSpWin) : el > base ? min((el - base + 15u) & ~15u, kSpWin) : 0u);
        pl[kk] = g + kSpAhead < G ? plan_load(g + kSpAhead) : Plan{0, 0, 0};
        if (lane == 0u) {
          *sp_word(s + kSpHdr) = base;
          *sp_word(s + kSpHdr + 4u) = nbytes;
        }
        const uint32_t ii = min(t * 64u + lane, n - 1u);  // (a lane past n loads entry n - 1)
        glds4(P.offset, 4u * ii, s + kSpDesc);
        glds4(P.caplen, 4u * ii, s + kSpDesc + 256u);
        // a chunk past nbytes re-reads the window's first (inside the batch contract's readable
        // bound, and never read by a decoder)
        const uint8_t *src = P.data + base;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t c = 1024u * j + 16u * lane;
          glds16(src, c < nbytes ? c : 0u, s + 1024u * j, true);
        }
        // with kSpAhead + 1 tiles in flight, tiles <= g - kSpAhead have landed: tell their
        // decoders (after a slot wait's flush they may have been told already)
        if (g >= kSpAhead && sig + kSpAhead <= g) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * kSpAhead) : "memory");
          for (; sig + kSpAhead <= g; sig++)
            if (lane == 0u) sp_st(ready + 4u * (sig % kSpSlots), sig + 1u);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (; sig < G; sig++)
      if (lane == 0u) sp_st(ready + 4u * (sig % kSpSlots), sig + 1u);
  }
  // ---- the decoders
  const uint32_t d = wave - 1u;
  uint32_t fb_c = 0, fb_start = 0, gdec = 0;
  if (wave != 0u) {
    const uint32_t qq = G / kSpDec, rr = G % kSpDec;
    fb_start = 64u * (b * q + min(b, r) + d * qq + min(d, rr));  // tiles of earlier workgroups, then of earlier decoders
    gdec = b * kSpDec + d;
    const FastCtx F{P.eth_mult, ((uint32_t)GPD_LT_PAYLOAD << 8) | (reinterpret_cast<const uint8_t *>(g_lds)[GPD_LT_PAYLOAD]),
                    (options & GPD_OPT_IGNORE_UNSUPPORTED) ? GPD_ST_OK : GPD_ST_UNSUPPORTED,
                    reinterpret_cast<const uint8_t *>(g_lds)[GPD_LT_FRAGMENT]};
    const uint32_t fits = kSpWin - 15u;
    for (uint32_t g = d; g < G; g += kSpDec) {
      const uint32_t s = slot_at(g), t = tile_of(g), i = t * 64u + lane;
      uint32_t spins = 0;
      while (sp_ld(ready + 4u * (g % kSpSlots)) != g + 1u && ++spins < kSpSpinCap) {
        if ((spins & 15u) == 0u && sp_ld(abort)) break;
        __builtin_amdgcn_s_sleep(2);
      }
      // (a capped spin or an aborted loader: the whole tile to the fallback list)
      const bool ok = sp_ld(ready + 4u * (g % kSpSlots)) == g + 1u;
      const uint32_t base = lds_u32(s + kSpHdr), nbytes = lds_u32(s + kSpHdr + 4u);
      const uint32_t valid = i < n ? 1u : 0u;
      const uint32_t off = valid ? min(lds_u32(s + kSpDesc + 4u * lane), dlen) : 0u;
      const uint32_t end = valid ? off + min(lds_u32(s + kSpDesc + 256u + 4u * lane), dlen - off) : 0u;
      const bool cov = ok && valid && off >= base && end - base <= nbytes && end - off <= fits;
      uint32_t fb = valid && !cov ? 1u : 0u;
      Out res{0, 0, 0, 0, 0, 0};
      Seg sg{0, 0, 0};
      // (AL: the windows are unshifted, so the aligned-chunk transport sum; -5 % against the plain
      // decoder here, profiles/r06/micro/split_kernel_ab.txt)
      if (cov && !fast_decode<CS, HASH, false, false, true>(s + (off - base), end - off, F, res, s, sg)) fb = 1;
      if (lane == 0u) sp_st(freed + 4u * (g % kSpSlots), g / kSpSlots + 1u);  // (release: the reads above first)
      const uint64_t m = __ballot(fb != 0);
      if (m) {
        if (fb) P.fb_list[fb_start + fb_c + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = ((uint64_t)off << 32) | i;
        fb_c += (uint32_t)__popcll(m);
      }
      if (valid && !fb) store_out(P, i, res);
    }
  }
  __syncthreads();  // the ring is idle: its slots stage the fallback rounds
  if (wave != 0u) {
    if (lane == 0u) P.fb_wcount[gdec] = fb_c;  // (gpd_last_launch_split's count)
    decode_fallback_list<kSpWin / 64u, CS, HASH>(P, slot_at(d), fb_start, fb_c, lane, dlen, options);
  }
}

template <int STAGE, bool FAST, bool EXT, bool PAGES, bool SWZ, int WAVES, bool CS = true,
          bool HASH = true, int MINW = 1>
static hipError_t launch_t(const KParams &P, hipStream_t stream, int num_cus) {
  const uint64_t ntiles = (P.n + 63) / 64;
  const size_t img = (P.image_words * 4u + 15u) & ~15u;
  const size_t lds = img + (size_t)wave_lds_bytes(STAGE, FAST) * WAVES + 64;  // + slack
  const uint64_t per_cu = (160u * 1024u) / lds;                       // resident workgroups per CU
  uint64_t blocks = (ntiles + WAVES - 1) / WAVES;
  const uint64_t cap = (uint64_t)num_cus * (per_cu ? per_cu : 1) * kGridRounds;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((decode_kernel<STAGE, FAST, EXT, PAGES, SWZ, WAVES, CS, HASH, MINW>), dim3((unsigned)blocks),
                     dim3(64 * WAVES), lds, stream, P);
  return hipGetLastError();
}

template <int STAGE, bool CS, bool HASH, int MINW, bool DEFER = false, bool RPFX = true, bool HO = false,
          bool AL = false, bool DIAG = false>
static hipError_t launch_rs(KParams &P, hipStream_t stream, int num_cus) {
  const uint64_t ntiles = (P.n + 63) / 64;
  size_t lds = ((P.image_words * 4u + 15u) & ~15u) + 4 * (size_t)rs_wave_lds_bytes(STAGE) + 64;
  uint64_t per_cu = std::max<uint64_t>(1, std::min<uint64_t>((160u * 1024u) / lds, MINW));
  // gpd_tuning.waves_per_simd: at most that many workgroups per CU, by reserving 1/W of the
  // CU's LDS per workgroup (the kernel's registers alone would admit 4)
  if (P.waves) {
    lds = std::max<size_t>(lds, ((160u * 1024u) / P.waves) & ~(size_t)2047u);  // (LDS granules: 3 x 54,608 B do not fit)
    per_cu = std::max<uint64_t>(1, std::min<uint64_t>((160u * 1024u) / lds, P.waves));
  }
  uint64_t blocks = (ntiles + 3) / 4;
  // rounds of resident workgroups: the AL kernel (VXLAN-sized frames) runs one — each wave's
  // tiles four times longer — measured 2.2 % faster than four (and 1.6 % than two) on config
  // 4; config 2, IMIX, pcap64 and the traffic mix keep four (one: +1-2 %, two: within noise;
  // tools/ab_rounds.sh, profiles/r03/rounds_ab/)
  const uint64_t rounds = P.rounds ? P.rounds : (AL ? 1u : kGridRounds);
  const uint64_t cap = (uint64_t)num_cus * per_cu * rounds;
  if (blocks > cap) blocks = cap;
  P.fb_waves = (uint32_t)blocks * 4u;
  if (blocks == 0) return hipSuccess;
  if (P.fb_waves > (uint32_t)num_cus * kMaxFastWavesPerCU) return hipErrorInvalidValue;
  hipLaunchKernelGGL((rs_kernel<STAGE, CS, HASH, MINW, DEFER, RPFX, HO, AL, DIAG>), dim3((unsigned)blocks), dim3(256), lds, stream, P);
  return hipGetLastError();
}

// The fast path: the register-staged loop (rs_kernel), its register bound setting the waves
// per SIMD (VGPRs <= 512 / MINW): 4 for 4 KiB windows, 3 for 8 KiB — what LDS admits, no
// spills.  The register-computed chunk prefix pays off for long frames only (IMIX -3 %); with
// small frames (pcap records, VXLAN) its extra registers and code cost 1-2 %.
template <bool CS, bool HASH, int MINW>
static hipError_t launch_ro(KParams &P, hipStream_t stream, int num_cus) {
  const uint64_t ntiles = (P.n + 63) / 64;
  size_t lds = ((P.image_words * 4u + 15u) & ~15u) + 4 * (size_t)ro_wave_lds_bytes() + 64;
  uint64_t per_cu = std::max<uint64_t>(1, std::min<uint64_t>((160u * 1024u) / lds, MINW));
  if (P.waves) {  // (as launch_rs: the LDS reservation caps the resident workgroups per CU)
    lds = std::max<size_t>(lds, ((160u * 1024u) / P.waves) & ~(size_t)2047u);  // (LDS granules: 3 x 54,608 B do not fit)
    per_cu = std::max<uint64_t>(1, std::min<uint64_t>((160u * 1024u) / lds, P.waves));
  }
  uint64_t blocks = (ntiles + 3) / 4;
  const uint64_t cap = (uint64_t)num_cus * per_cu * (P.rounds ? P.rounds : kGridRounds);
  if (blocks > cap) blocks = cap;
  P.fb_waves = (uint32_t)blocks * 4u;
  if (blocks == 0) return hipSuccess;
  if (P.fb_waves > (uint32_t)num_cus * kMaxFastWavesPerCU) return hipErrorInvalidValue;
  hipLaunchKernelGGL((ro_kernel<CS, HASH, MINW>), dim3((unsigned)blocks), dim3(256), lds, stream, P);
  return hipGetLastError();
}

// The loader / decoder split (sp_kernel): 8-wave workgroups, two per CU (LDS), one round of
// them by default (gpd_tuning.grid_rounds more).
template <bool CS, bool HASH>
static hipError_t launch_sp(KParams &P, hipStream_t stream, int num_cus) {
  const uint64_t ntiles = (P.n + 63) / 64;
  const size_t lds = ((P.image_words * 4u + 15u) & ~15u) + (size_t)sp_lds_bytes() + 64;
  const uint64_t per_cu = std::max<uint64_t>(1, std::min<uint64_t>((160u * 1024u) / lds, 2));
  const uint64_t blocks = std::min<uint64_t>(ntiles, (uint64_t)num_cus * per_cu * (P.rounds ? P.rounds : 1u));
  P.fb_waves = (uint32_t)blocks * kSpDec;
  if (blocks == 0) return hipSuccess;
  if (P.fb_waves > (uint32_t)num_cus * kMaxFastWavesPerCU) return hipErrorInvalidValue;
  hipLaunchKernelGGL((sp_kernel<CS, HASH>), dim3((unsigned)blocks), dim3(64 * kSpWaves), lds, stream, P);
  return hipGetLastError();
}

template <bool CS, bool HASH>
static hipError_t launch_fast(KParams &P, hipStream_t stream, int num_cus) {
  // One register budget per kernel (4 waves per SIMD for 4 KiB windows, 3 for 8 KiB windows
  // and rounds: what each kernel's VGPRs admit without spills); gpd_tuning.waves_per_simd caps
  // the residency below that through the LDS reservation (launch_rs / launch_ro), it does not
  // pick another instantiation.
  if (P.options & kRounds)  // header-once over 8 KiB rounds of each tile's run (ro_kernel)
    return launch_ro<CS, HASH, 3>(P, stream, num_cus);
  if constexpr (kDiagBuild) {  // libgpd_diag.so: the skeleton (no decode) instantiations
    if (P.options & kDiagSkipDecode) {
      if (P.stage == 4096) return launch_rs<4096, CS, HASH, 4, false, true, false, false, true>(P, stream, num_cus);
      if (P.options & kHeaderOnce) return launch_rs<8192, CS, HASH, 3, false, true, true, false, true>(P, stream, num_cus);
      if (P.options & kRegPrefix) return launch_rs<8192, CS, HASH, 3, false, true, false, false, true>(P, stream, num_cus);
      if (!(P.options & kShiftWindows))
        return launch_rs<8192, CS, HASH, 3, false, false, false, true, true>(P, stream, num_cus);
      return launch_rs<8192, CS, HASH, 3, false, false, false, false, true>(P, stream, num_cus);
    }
  }
  // (the split kernel writes gpd_records: with the five SoA arrays its seven decoders per
  // workgroup ran 0.397 ms against the register loop's 0.319 on config 2, same box)
  if (P.stage == 4096 && P.split && P.rec) return launch_sp<CS, HASH>(P, stream, num_cus);
  if (P.stage == 4096) return launch_rs<4096, CS, HASH, 4>(P, stream, num_cus);
  if (P.options & kHeaderOnce) return launch_rs<8192, CS, HASH, 3, false, true, true>(P, stream, num_cus);
  if (P.options & kRegPrefix) return launch_rs<8192, CS, HASH, 3>(P, stream, num_cus);
  // unshifted windows of mid-sized frames (VXLAN's 128 B): the aligned-chunk transport checksum
  // and the inner Ethernet bytes from registers (fast_decode AL); shifted windows (pcap records,
  // 65..96-B slots) keep the plain kernel, where both cost ~1 % (measured A/B)
  // (every shipped kernel is compiled without the skeleton diagnostic's branch: round 4
  // measured config 4 -2.2 %, pcap64 -0.7 %; round 6 the 4 KiB kernels too)
  if (!(P.options & kShiftWindows)) return launch_rs<8192, CS, HASH, 3, false, false, false, true>(P, stream, num_cus);
  return launch_rs<8192, CS, HASH, 3, false, false>(P, stream, num_cus);
}

// The generic decoder over LDS windows (ext records, other first layers, PAGES tables): the
// windows' 16-byte slots rotated (swizzled) against bank conflicts.
template <bool EXT, bool PAGES>
static hipError_t launch_s(const KParams &P, hipStream_t stream, int num_cus) {
  if (P.stage == 4096) return launch_t<4096, false, EXT, PAGES, true, 4>(P, stream, num_cus);
  return launch_t<8192, false, EXT, PAGES, true, 4>(P, stream, num_cus);
}

// ---------------------------------------------------------------- IPv4 fragment hand-off
// include/gpd_defrag.h: the packets for which IPv4Defragmenter.DefragIPv4 does not return the
// layer unchanged (dontDefrag, ip4defrag/defrag.go:162-172), in packet order, with the key and
// securityChecks verdict (:175-198).  Four launches: per-2048-packet candidate counts (and one
// candidate bit per packet), their exclusive scan, the candidates' packet indices in order, and
// one record per candidate.

// Can packet i's IPv4 object (as the call leaves it: the last IPv4 in decoded, or a later IPv4
// call that failed after assigning its fields) be a fragment?  From the result words first: a fragmented IPv4 layer ends the decode (ip4.go:281-286, its next layer is
// gopacket.Fragment, which decodes nothing further), so decoded ends [.., IPv4, Fragment], or
// [.., IPv4] with Fragment unregistered (stop type 3) or the payload empty (stop 0).  Then the
// flags/offset word of the header (ip4.go:193,200-201), which also rules out DF (:164-166).
__device__ __forceinline__ bool frag_candidate(const KParams &P, uint32_t i) {
  uint32_t st;
  uint64_t lw;
  if (P.rec) {
    st = P.rec[i].status;
    lw = P.rec[i].layers;
  } else {
    st = P.status[i];
    lw = P.layers[i];
  }
  if (GPD_STATUS_NET_EPT(st) != 1u) return false;  // the last network layer is not IPv4
  const uint32_t nl = GPD_STATUS_NLAYERS(st);
  // After a decode error the ip4 object may hold a later, failed IPv4 header (ip4.go:195-210
  // assign its fields before the Length/IHL checks) wherever decoded ends: the header decides.
  if (GPD_STATUS_CLASS(st) != GPD_ST_DECODE_ERROR && nl <= GPD_CORE_MAX_LAYERS &&
      !GPD_STATUS_SATURATED(st)) {
    const uint32_t last = GPD_LAYERS_CODE(lw, nl - 1), stop = GPD_LAYERS_STOP(lw);
    const bool maybe = (last == GPD_C_FRAGMENT && nl >= 2 && GPD_LAYERS_CODE(lw, nl - 2) == GPD_C_IPV4) ||
                       (last == GPD_C_IPV4 && (stop == 0 || stop == GPD_LT_FRAGMENT));
    if (!maybe) return false;
  }
  const uint32_t net = GPD_HDR_NET(P.hdr_off[i]);
  if (net == GPD_HDR_NONE) return true;  // header past byte 65534: the record pass decides
  const uint32_t dlen = (uint32_t)P.data_len;
  const uint32_t off = min(P.offset[i], dlen);
  const uint8_t *h = P.data + off + net;  // a decoded IPv4 header: 20 bytes inside the packet
  const uint32_t flags = h[6] >> 5, fo = ((h[6] & 0x1Fu) << 8) | h[7];
  if (flags & 2u) return false;  // IPv4DontFragment
  return (flags & 1u) || fo != 0;
}

// Packets per counting workgroup: 8 rounds of 256 lanes; bit l of mask word w is packet 64w + l.
constexpr uint32_t kFragBlock = 2048;

__global__ __launch_bounds__(256) void frag_count_kernel(FragArgs A) {
  __shared__ uint32_t wsum[4];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint32_t base = blockIdx.x * kFragBlock;
  uint32_t c = 0;
#pragma unroll 2
  for (uint32_t r = 0; r < kFragBlock / 256u; ++r) {
    const uint32_t i = base + r * 256u + threadIdx.x;
    const uint64_t m = __ballot(i < A.P.n && frag_candidate(A.P, i));
    if (lane == 0 && base + r * 256u + w * 64u < A.P.n) A.mask[(base + r * 256u) / 64u + w] = m;
    c += (uint32_t)__popcll(m);
  }
  if (lane == 0) wsum[w] = c;
  __syncthreads();
  if (threadIdx.x == 0) A.blk[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// One workgroup: exclusive scan of the per-block counts in place, 1024 at a time (coalesced);
// blk[nblk] = the total.
__global__ __launch_bounds__(1024) void frag_scan_kernel(FragArgs A) {
  __shared__ uint32_t wtot[16];
  __shared__ uint32_t carry;
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  if (t == 0) carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < A.nblk; c0 += 1024u) {
    const uint32_t k = c0 + t;
    const uint32_t v = k < A.nblk ? A.blk[k] : 0u;
    uint32_t x = v;  // inclusive scan within the wave
#pragma unroll
    for (uint32_t d = 1; d < 64u; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if (lane == 63u) wtot[w] = x;
    __syncthreads();
    uint32_t before = carry;
    for (uint32_t j = 0; j < w; ++j) before += wtot[j];
    if (k < A.nblk) A.blk[k] = before + x - v;
    __syncthreads();
    if (t == 1023u) carry = before + x;
    __syncthreads();
  }
  if (t == 0) A.blk[A.nblk] = carry;
}

// The candidates' packet indices in order, from the mask words: 32 words per block, one lane
// each; a lane writes its word's set bits (fragments are rare: usually nothing at all).
__global__ __launch_bounds__(64) void frag_index_kernel(FragArgs A) {
  const uint32_t lane = threadIdx.x;
  const uint32_t wi = blockIdx.x * (kFragBlock / 64u) + lane;
  const uint32_t nw = (A.P.n + 63u) / 64u;
  const uint64_t m = (lane < kFragBlock / 64u && wi < nw) ? A.mask[wi] : 0ull;
  if (__ballot(m != 0ull) == 0ull) return;
  uint32_t x = (uint32_t)__popcll(m), v = x;
#pragma unroll
  for (uint32_t d = 1; d < 64u; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  uint32_t r = A.blk[blockIdx.x] + x - v;
  for (uint64_t b = m; b; b &= b - 1ull) A.idx[r++] = wi * 64u + (uint32_t)__builtin_ctzll(b);
}

// One lane per candidate: the generic decoder re-runs the packet for the IPv4 object's exact
// state (its Contents/Payload, so a TSO Length of 0 and truncation come out as the reference
// leaves them), then dontDefrag and securityChecks on it.
template <bool PAGES>
__global__ __launch_bounds__(256) void frag_record_kernel(FragArgs A) {
  const KParams &P = A.P;
  const uint32_t cnt = min(A.blk[A.nblk], A.max_out);
  if (cnt <= blockIdx.x * 256u) return;
  for (uint32_t k = threadIdx.x; k < P.image_words; k += 256) reinterpret_cast<uint32_t *>(g_lds)[k] = P.image[k];
  __syncthreads();
  const Tab<PAGES> T{P.pages,    P.eth_base, P.tcp_base, P.udp_base, P.eth_bits,
                     P.tcp_bits, P.udp_bits, P.eth_mult, P.tcp_mult, P.udp_mult};
  const uint32_t dlen = (uint32_t)P.data_len;
  const uint32_t options = P.options & ~kDiagMask;
  for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < cnt; j += gridDim.x * 256u) {
    const uint32_t i = A.idx[j];
    const uint32_t off = min(P.offset[i], dlen), len = min(P.caplen[i], dlen - off);
    gpd_ext_rec e;
    decode_packet<true>(GlbSrc{P.data, off}, len, T, P.first, options, &e);
    const gpd_layer_rec o = e.obj[GPD_OBJ_IPV4];
    gpd_ip4_frag r{};
    r.packet = i;
    r.verdict = GPD_FRAG_WHOLE;
    if (e.obj_valid & (1u << GPD_OBJ_IPV4)) {
      const uint8_t *h = P.data + off + o.contents_off;
      const uint32_t raw_len = ((uint32_t)h[2] << 8) | h[3], ff = ((uint32_t)h[6] << 8) | h[7];
      r.net_off = o.contents_off;
      for (int b = 0; b < 4; ++b) {
        r.src[b] = h[12 + b];
        r.dst[b] = h[16 + b];
      }
      r.id = (uint16_t)(((uint32_t)h[4] << 8) | h[5]);
      r.flags = (uint8_t)(ff >> 13);
      r.frag_offset = (uint16_t)(ff & 0x1FFFu);
      r.ihl = h[0] & 0x0Fu;
      // ip4.go:214-218: Length 0 => len(data); the decode then keeps all of data, so it is
      // Contents + Payload
      r.length = (uint16_t)(raw_len ? raw_len : o.contents_len + o.payload_len);
      r.payload_len = o.payload_len;
      const bool dont = (r.flags & 2u) || (!(r.flags & 1u) && r.frag_offset == 0);  // defrag.go:162-172
      const uint16_t frag_size = (uint16_t)(r.length - (uint16_t)(r.ihl * 4u));        // :176
      if (dont) r.verdict = GPD_FRAG_WHOLE;
      else if (frag_size < 8u) r.verdict = GPD_FRAG_TOO_SMALL;                           // :179
      else if (r.frag_offset > 8183u) r.verdict = GPD_FRAG_OFFSET;                       // :185
      else if ((uint16_t)(r.frag_offset * 8u + r.length) > 65535u) r.verdict = GPD_FRAG_OVERRUN;  // :192, uint16
      else r.verdict = GPD_FRAG_INSERT;
    }
    A.out[j] = r;
  }
}

hipError_t launch_ip4_frag(const FragArgs &A, hipStream_t stream, int num_cus) {
  if (A.nblk == 0) return hipSuccess;
  hipLaunchKernelGGL(frag_count_kernel, dim3(A.nblk), dim3(256), 0, stream, A);
  hipLaunchKernelGGL(frag_scan_kernel, dim3(1), dim3(1024), 0, stream, A);
  hipLaunchKernelGGL(frag_index_kernel, dim3(A.nblk), dim3(64), 0, stream, A);
  if (A.max_out == 0) return hipGetLastError();
  const size_t lds = (A.P.image_words * 4u + 15u) & ~15u;
  const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)num_cus * 2, (A.max_out + 255u) / 256u);
  if (A.P.use_pages) hipLaunchKernelGGL(frag_record_kernel<true>, dim3(grid), dim3(256), lds, stream, A);
  else hipLaunchKernelGGL(frag_record_kernel<false>, dim3(grid), dim3(256), lds, stream, A);
  return hipGetLastError();
}

bool fast_eligible(const KParams &P) {
  // the fast kernel: Ethernet first and registered, hashed tables, no extended records
  return !P.ext && !P.use_pages && P.fixed && P.first == GPD_LT_ETHERNET &&
         (P.decoders & GPD_DEC_ETHERNET);
}

hipError_t launch_decode(const KParams &P0, hipStream_t stream, int num_cus, hipEvent_t mid,
                         uint32_t *fb_waves) {
  KParams P = P0;
  P.fb_waves = 0;
  if (P.n > kMaxLaunchPackets) return hipErrorInvalidValue;
  if (fast_eligible(P)) {
    if (!P.fb_list || !P.fb_wcount) return hipErrorInvalidValue;
    hipError_t e;
    const bool cs = !(P.options & GPD_OPT_NO_CHECKSUMS), hash = !(P.options & GPD_OPT_NO_FLOW_HASH);
    e = cs ? (hash ? launch_fast<true, true>(P, stream, num_cus)
                   : launch_fast<true, false>(P, stream, num_cus))
           : (hash ? launch_fast<false, true>(P, stream, num_cus)
                   : launch_fast<false, false>(P, stream, num_cus));
    if (e != hipSuccess) return e;
    if (fb_waves) *fb_waves = P.fb_waves;
    if (mid && (e = hipEventRecord(mid, stream)) != hipSuccess) return e;
    return hipSuccess;  // (each fast wave decodes its own fallback list: one launch)
  }
  if (P.ext) return P.use_pages ? launch_s<true, true>(P, stream, num_cus)
                                : launch_s<true, false>(P, stream, num_cus);
  return P.use_pages ? launch_s<false, true>(P, stream, num_cus)
                     : launch_s<false, false>(P, stream, num_cus);
}

}  // namespace gpd

#ifdef GPD_PHASE_TIMING
extern "C" int gpd_diag_phase(unsigned long long *out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gpd::g_phase), 6 * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(gpd::g_phase), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

#ifdef GPD_ISA_PROBE
// Instruction-count probe (not built into libgpd.so): the fast path alone on one packet.
namespace gpd {
__global__ void probe_fast(KParams P) {
  const uint32_t pos = P.offset[threadIdx.x], len = P.caplen[threadIdx.x];
  const Tab<false> T{P.pages,    P.eth_base, P.tcp_base, P.udp_base, P.eth_bits,
                     P.tcp_bits, P.udp_bits, P.eth_mult, P.tcp_mult, P.udp_mult};
  Out o{};
  const FastCtx F{P.eth_mult, 0x2C8, 1, 0xD9};
  (void)T;
  Seg sg{0, 0, 0};
  if (fast_decode<true, true, false>(pos, len, F, o, 0, sg)) store_out(P, threadIdx.x, o);
}
}  // namespace gpd
#endif
