// gpd_runtime.cpp — host runtime behind the C-ABI in include/gpd.h.
//
// Owns the per-(thread, GPU) context: the snapshot of the dispatch tables in
// device memory (the reference reads mutable package globals on every packet,
// layers/enums.go:288-345, layers/ports.go:62-128; a context freezes them at
// creation like a parser built from them), the registered-decoder mask and
// options (parser.go:182-195, 336-350), HIP timing events, and the pinned
// staging used by gpd_decode_host.
#include <hip/hip_runtime.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cerrno>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "gpd_internal.h"

namespace {

thread_local char g_err[512] = "";

int set_err(int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}

}  // namespace

int gpd::set_error(int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}

namespace {

#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return set_err(GPD_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));        \
  } while (0)

// Reference defaults, restated as data: layers/enums.go:304-345, layers/ports.go:62-74,105-122.
const uint32_t kEtherDefaults[][2] = {
    {0x0000, 22}, {0x0800, 20}, {0x86DD, 21}, {0x0806, 10}, {0x8100, 15}, {0x880B, 25},
    {0x8863, 26}, {0x8864, 26}, {0x9000, 12}, {0x2000, 11}, {0x01A2, 61}, {0x88CC, 58},
    {0x8847, 24}, {0x8848, 24}, {0x888E, 56}, {0x88A8, 15}, {0x6558, 17}, {0x88BE, 145}};
const uint32_t kProtoDefaults[][2] = {
    {4, 20},  {6, 44},  {17, 45}, {1, 19},  {58, 57},  {132, 28}, {41, 21}, {94, 20},
    {97, 16}, {27, 27}, {47, 18}, {0, 46},  {43, 47},  {44, 48},  {60, 49}, {89, 123},
    {51, 50}, {50, 51}, {136, 52}, {137, 24}, {59, 2}, {2, 62}, {112, 119}};
const uint32_t kTcpDefaults[][2] = {{53, 107}, {443, 140}, {502, 141}, {636, 140},
                                    {989, 140}, {990, 140}, {992, 140}, {993, 140},
                                    {994, 140}, {995, 140}, {5061, 140}};
const uint32_t kUdpDefaults[][2] = {{53, 107},   {123, 117},  {4789, 116}, {67, 118},
                                    {68, 118},   {546, 134},  {547, 134},  {666, 147},
                                    {1000, 149}, {5060, 133}, {6343, 114}, {6081, 120},
                                    {3784, 122}, {2152, 129}, {623, 142},  {1812, 146}};

template <size_t N>
void fill(uint16_t *t, size_t size, const uint32_t (&e)[N][2]) {
  memset(t, 0, size * sizeof(uint16_t));
  for (size_t k = 0; k < N; k++) t[e[k][0]] = (uint16_t)e[k][1];
}

// Two-level page encoding of the three 64K tables (see gpd_internal.h).
std::vector<uint16_t> encode_tables(const uint16_t *eth, const uint16_t *proto,
                                    const uint16_t *tcp, const uint16_t *udp) {
  std::vector<uint16_t> out(gpd::kTabPages + 256, 0);  // page 0 = zeros
  std::memcpy(out.data() + gpd::kTabIpProto, proto, 256 * sizeof(uint16_t));
  std::map<std::vector<uint16_t>, uint16_t> pages;
  pages[std::vector<uint16_t>(256, 0)] = 0;
  auto encode = [&](const uint16_t *t, uint32_t dir) {
    for (uint32_t hi = 0; hi < 256; hi++) {
      std::vector<uint16_t> pg(t + hi * 256, t + hi * 256 + 256);
      auto it = pages.find(pg);
      uint16_t idx;
      if (it == pages.end()) {
        idx = (uint16_t)pages.size();
        pages[pg] = idx;
        out.insert(out.end(), pg.begin(), pg.end());
      } else {
        idx = it->second;
      }
      out[dir + hi] = idx;
    }
  };
  encode(eth, gpd::kTabEthDir);
  encode(tcp, gpd::kTabTcpDir);
  encode(udp, gpd::kTabUdpDir);
  return out;
}

// Decoder id per LayerType for the registered set (the DecodingLayerMap of parser.go:147-164,
// filled from each decoder's CanDecode, layertypes.go:193-198 for the extension class) and
// the 4-bit code the `layers` word uses for it (include/gpd.h GPD_C_*).
void type_lut(uint32_t decoders, uint8_t lut[128]) {
  struct E { uint32_t lt, dec, code; };
  static const E kMap[] = {{17, 0, 1},  {15, 1, 2},  {20, 2, 3},  {21, 3, 4},  {46, 4, 5},
                           {47, 4, 6},  {48, 4, 7},  {49, 4, 8},  {44, 5, 9},  {45, 6, 10},
                           {116, 7, 11}, {2, 8, 12}, {3, 9, 13}, {19, 10, 14}, {22, 11, 15}};
  memset(lut, 0xFF, 128);
  for (const E &e : kMap)
    if (decoders & (1u << e.dec)) lut[e.lt] = (uint8_t)(e.dec | (e.code << 4));
}

// Two-way bucketed hash of the nonzero entries of a 64K table: 2^bits buckets of two u32
// slots {key << 16 | LayerType << 8 | lut[LayerType]}, bucket = key_hash(key, mult, bits).
// The multiplier is searched so that no bucket holds more than two keys, which makes every
// device lookup one ds_read_b64 and two compares (no probe loop).  Unused slots hold a key
// absent from the table with "LayerType 0, not registered", so they read as a miss.
struct HashKeys {
  std::vector<uint32_t> keys;
  uint32_t empty = 0;
  bool ok = false;  // every LayerType < 256 and some key absent
};
HashKeys hash_keys(const uint16_t *t) {
  HashKeys h;
  std::vector<uint8_t> present(65536, 0);
  for (uint32_t k = 0; k < 65536; k++) {
    if (t[k] >= 256) return h;
    if (t[k]) { h.keys.push_back(k); present[k] = 1; }
  }
  uint32_t absent = 0;
  while (absent < 65536 && present[absent]) absent++;
  if (absent == 65536) return h;
  h.empty = (absent << 16) | 0xFFu;
  h.ok = true;
  return h;
}
bool fill_hash(const HashKeys &h, const uint16_t *t, const uint8_t lut[128], uint32_t mult,
               uint32_t bits, std::vector<uint32_t> &slots) {
  const uint32_t nb = 1u << bits;
  if (h.keys.size() > 2 * nb) return false;
  slots.assign(2 * nb, h.empty);
  std::vector<uint8_t> fill(nb, 0);
  for (uint32_t k : h.keys) {
    const uint32_t b = gpd::key_hash(k, mult, bits);
    if (fill[b] == 2) return false;
    slots[2 * b + fill[b]++] = (k << 16) | ((uint32_t)t[k] << 8) | (t[k] < 128 ? lut[t[k]] : 0xFFu);
  }
  return true;
}
uint32_t next_mult(uint32_t m) { return ((m * 2654435761u + 0x9E37u) & 0xFFFFu) | 1u; }

// Any layout: the smallest bits (<= max_words) with some multiplier.
bool build_hash(const uint16_t *t, const uint8_t lut[128], uint32_t max_words,
                std::vector<uint32_t> &slots, uint32_t &mult_out, uint32_t &bits_out) {
  const HashKeys h = hash_keys(t);
  if (!h.ok) return false;
  for (uint32_t bits = 2; bits <= 15 && (2u << bits) <= max_words; bits++) {
    uint32_t mult = 40503u;  // golden-ratio start, then a fixed odd sequence
    for (int attempt = 0; attempt < 512; attempt++, mult = next_mult(mult)) {
      if (fill_hash(h, t, lut, mult, bits, slots)) {
        mult_out = mult;
        bits_out = bits;
        return true;
      }
    }
  }
  return false;
}

// The fixed layout the fast kernel compiles in (gpd_internal.h kFix*): 2^kFixBits buckets
// per table at fixed bases, one multiplier shared by the three tables.
bool build_fixed(const uint16_t *eth, const uint16_t *tcp, const uint16_t *udp,
                 const uint8_t lut[128], std::vector<uint32_t> &he, std::vector<uint32_t> &ht,
                 std::vector<uint32_t> &hu, uint32_t &mult_out) {
  const HashKeys ke = hash_keys(eth), kt = hash_keys(tcp), ku = hash_keys(udp);
  if (!ke.ok || !kt.ok || !ku.ok) return false;
  uint32_t mult = 40503u;
  for (int attempt = 0; attempt < 4096; attempt++, mult = next_mult(mult)) {
    if (fill_hash(ke, eth, lut, mult, gpd::kFixBits, he) &&
        fill_hash(kt, tcp, lut, mult, gpd::kFixBits, ht) &&
        fill_hash(ku, udp, lut, mult, gpd::kFixBits, hu)) {
      mult_out = mult;
      return true;
    }
  }
  return false;
}

}  // namespace

struct gpd_ctx {
  int device = 0;
  int num_cus = 256;
  uint32_t first = GPD_LT_ETHERNET;
  uint32_t decoders = GPD_DEC_ALL;
  uint32_t options = 0;
  // the dispatch tables last loaded (LayerType values): AddDecodingLayer rebuilds the LDS image
  // from them, as the reference's parser reads the live tables at each decode
  std::vector<uint16_t> t_eth, t_proto, t_tcp, t_udp;
  uint32_t *d_image = nullptr;  // LUT + ipproto (+ hashes)
  uint16_t *d_pages = nullptr;  // PAGES fallback
  uint32_t image_words = 0, use_pages = 0;
  uint32_t eth_base = 0, tcp_base = 0, udp_base = 0, eth_bits = 0, tcp_bits = 0, udp_bits = 0;
  uint32_t eth_mult = 0, tcp_mult = 0, udp_mult = 0;
  bool fixed = false;  // tables in the fixed layout the fast kernel compiles in
  // fast-kernel fallback lists, one per stream the context is used on (count + indices)
  struct Fallback {
    uint32_t *d = nullptr;   // two flags (words 0 and 64), then the list
    uint32_t *wc = nullptr;  // two arrays of per-wave counts (one per parity)
    uint64_t cap = 0;
    uint32_t parity = 0;
  };
  std::map<hipStream_t, Fallback> fallback;
  // device scratch that grows on demand and lives with the context (ctx_scratch)
  struct Scratch {
    void *d = nullptr;
    size_t bytes = 0;
  } scratch[16];
  gpd_tuning tune{0, -1, -1, 0, -1, -1, 0, -1};  // gpd_ctx_set_tuning (all automatic by default)
  bool timing = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, evm = nullptr;
  bool timed = false;
  bool timed_split = false;           // evm marks the fast kernel's end in the timed launch
  const uint32_t *timed_fb_wc = nullptr;  // its per-wave fallback counts (device)
  uint32_t timed_fb_waves = 0;
  // gpd_decode_host staging (two slots)
  struct Slot {
    hipStream_t stream = nullptr;
    uint8_t *h_data = nullptr, *d_data = nullptr;
    uint32_t *h_off = nullptr, *h_len = nullptr, *d_off = nullptr, *d_len = nullptr;
    uint32_t *h_status = nullptr, *d_status = nullptr, *h_csum = nullptr, *d_csum = nullptr;
    uint64_t *h_layers = nullptr, *d_layers = nullptr, *h_nh = nullptr, *d_nh = nullptr;
    uint64_t *h_th = nullptr, *d_th = nullptr;
    uint32_t *h_hoff = nullptr, *d_hoff = nullptr;
    gpd_ext_rec *h_ext = nullptr, *d_ext = nullptr;
    gpd_detail *h_det = nullptr, *d_det = nullptr;
    uint32_t *d_pw = nullptr;  // the device pcap walk's per-segment arrays (5 x kPwMaxSeg)
    uint8_t *d_tw = nullptr, *h_tw = nullptr;  // the device TPACKET_V3 walk's tables + results
    hipStream_t stream_out = nullptr;          // its D2H (gpd_decode_tpv3, gpd_decode_host)
    // gpd_decode_host: the chunk's H2D done (host staging reusable), decoded, results back
    hipEvent_t ev_in = nullptr, ev_dec = nullptr, ev_out = nullptr;
    uint64_t lo = 0, hi = 0;  // packet range in flight
    bool busy = false;
    bool direct = false;      // its results go straight into the caller's (registered) arrays
  } slot[2];  // (a third slot measured 6-9 % slower on config 2's host path, r04)
  uint64_t slot_bytes = 0, slot_pkts = 0;
  gpd::PwCtl *d_pw_ctl = nullptr, *h_pw_ctl = nullptr;  // one control block per slot
  hipEvent_t ev_pw[2] = {nullptr, nullptr};            // a slot's chunk walked (and its block read back)
  hipStream_t tw_in = nullptr;  // TPACKET_V3 groups' bytes H2D, one after another
  hipEvent_t ev_tw[4] = {};     // TPACKET_V3 group k & 3's results back
  hipEvent_t ev_twdec[4] = {};  // ... decoded
  hipEvent_t ev_twin[2] = {}; // a slot's group bytes H2D done (its staging copy reusable)
  // host ranges pinned with gpd_host_register (H2D reads them in place)
  std::vector<std::pair<const uint8_t *, uint64_t>> registered;
  bool is_registered(const uint8_t *p, uint64_t n) const {
    for (const auto &r : registered)
      if (p >= r.first && p + n <= r.first + r.second) return true;
    return false;
  }
};

// Host-side copies of the staging pipeline run on up to 16 threads: fn(lo, hi) over [0, n).
template <class F>
static void par_for(uint64_t n, uint64_t grain, F fn) {
  static const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const uint64_t T = std::min<uint64_t>(hw, (n + grain - 1) / grain);
  if (T <= 1) {
    fn(0, n);
    return;
  }
  std::vector<std::thread> th;
  for (uint64_t t = 1; t < T; t++) th.emplace_back([&, t] { fn(n * t / T, n * (t + 1) / T); });
  fn(0, n / T);
  for (auto &x : th) x.join();
}

static void par_memcpy(void *dst, const void *src, uint64_t bytes) {
  par_for(bytes, 4u << 20, [&](uint64_t lo, uint64_t hi) {
    std::memcpy(static_cast<uint8_t *>(dst) + lo, static_cast<const uint8_t *>(src) + lo, hi - lo);
  });
}

namespace gpd {
int ctx_device(const gpd_ctx *ctx) { return ctx->device; }
int ctx_num_cus(const gpd_ctx *ctx) { return ctx->num_cus; }
void *ctx_scratch(gpd_ctx *ctx, int slot, size_t bytes) {
  if (slot < 0 || slot >= 16) return nullptr;
  auto &sc = ctx->scratch[slot];
  if (sc.bytes < bytes) {
    if (sc.d) (void)hipFree(sc.d);
    sc.d = nullptr;
    sc.bytes = 0;
    const size_t want = bytes + bytes / 4;  // headroom: a slightly larger walk reuses it
    if (hipMalloc(&sc.d, want) != hipSuccess) return nullptr;
    sc.bytes = want;
  }
  return sc.d;
}
}  // namespace gpd

extern "C" {

int gpd_abi_version(void) { return GPD_ABI_VERSION; }

const char *gpd_last_error_string(void) { return g_err; }

void gpd_default_tables(uint16_t *ethertype, uint16_t *ipproto, uint16_t *tcp_port,
                        uint16_t *udp_port) {
  if (ethertype) fill(ethertype, 65536, kEtherDefaults);
  if (ipproto) fill(ipproto, 256, kProtoDefaults);
  if (tcp_port) fill(tcp_port, 65536, kTcpDefaults);
  if (udp_port) fill(udp_port, 65536, kUdpDefaults);
}

// The LDS image (and the PAGES blob when the tables do not hash) from ctx's decoder mask and
// its table snapshot.
// Builds the dispatch image (and the PAGES blob) of `decoders` over the given tables into new
// device buffers; only when every step succeeded are they swapped into ctx (the old ones
// freed), so a failed rebuild leaves the context exactly as it was.  The callers
// commit their decoder mask / table snapshot after a GPD_OK only.
static int build_image(gpd_ctx *ctx, uint32_t decoders, const std::vector<uint16_t> &eth,
                       const std::vector<uint16_t> &proto, const std::vector<uint16_t> &tcp,
                       const std::vector<uint16_t> &udp) {
  // LDS image: LUT (32 words) + ipproto with LUT entries (256 words) + the three hashes
  std::vector<uint32_t> img(gpd::kHashLutWords + gpd::kHashProtoWords, 0);
  uint8_t *lut = reinterpret_cast<uint8_t *>(img.data());
  type_lut(decoders, lut);
  for (uint32_t p = 0; p < 256; p++) {
    const uint32_t lt = proto[p];
    img[gpd::kHashLutWords + p] = lt | ((lt < 128 ? lut[lt] : 0xFFu) << 16);
  }
  std::vector<uint32_t> he, ht, hu;
  const uint32_t room = gpd::kHashMaxWords - (uint32_t)img.size();
  uint32_t me = 0, mt = 0, mu = 0, be = 0, bt = 0, bu = 0;
  const bool fixed = build_fixed(eth.data(), tcp.data(), udp.data(), lut, he, ht, hu, me);
  bool hashed = fixed;
  if (fixed) {
    mt = mu = me;
    be = bt = bu = gpd::kFixBits;
  } else {
    hashed = build_hash(eth.data(), lut, room / 2, he, me, be) &&
             build_hash(tcp.data(), lut, room / 4, ht, mt, bt) &&
             build_hash(udp.data(), lut, room / 4, hu, mu, bu);
  }
  uint32_t eth_base = 0, tcp_base = 0, udp_base = 0;
  std::vector<uint16_t> blob;
  if (hashed) {  // every hash starts on an 8-byte boundary (ds_read_b64 buckets)
    auto put = [&](const std::vector<uint32_t> &h, uint32_t &base) {
      if (img.size() & 1) img.push_back(0);
      base = (uint32_t)img.size();
      img.insert(img.end(), h.begin(), h.end());
    };
    put(he, eth_base);
    put(ht, tcp_base);
    put(hu, udp_base);
    if (fixed && (eth_base != gpd::kFixEthBase || tcp_base != gpd::kFixTcpBase || udp_base != gpd::kFixUdpBase))
      return set_err(GPD_ERR_INVALID, "internal: fixed table layout mismatch");
  } else {
    blob = encode_tables(eth.data(), proto.data(), tcp.data(), udp.data());
  }
  gpd::DeviceScope dscope_;
  HIP_TRY(dscope_.set(ctx->device));
  uint32_t *d_image = nullptr;
  uint16_t *d_pages = nullptr;
  hipError_t e = hipMalloc(&d_image, img.size() * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemcpy(d_image, img.data(), img.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (e == hipSuccess && !hashed) e = hipMalloc(&d_pages, blob.size() * sizeof(uint16_t));
  if (e == hipSuccess && !hashed)
    e = hipMemcpy(d_pages, blob.data(), blob.size() * sizeof(uint16_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (d_image) (void)hipFree(d_image);
    if (d_pages) (void)hipFree(d_pages);
    return set_err(e == hipErrorOutOfMemory ? GPD_ERR_NOMEM : GPD_ERR_HIP, "dispatch image: %s",
                   hipGetErrorString(e));
  }
  if (ctx->d_image) (void)hipFree(ctx->d_image);
  if (ctx->d_pages) (void)hipFree(ctx->d_pages);
  ctx->d_image = d_image;
  ctx->d_pages = d_pages;
  ctx->image_words = (uint32_t)img.size();
  ctx->fixed = fixed;
  ctx->use_pages = hashed ? 0 : 1;
  if (hashed) {
    ctx->eth_base = eth_base; ctx->eth_bits = be; ctx->eth_mult = me;
    ctx->tcp_base = tcp_base; ctx->tcp_bits = bt; ctx->tcp_mult = mt;
    ctx->udp_base = udp_base; ctx->udp_bits = bu; ctx->udp_mult = mu;
  }
  return GPD_OK;
}

int gpd_ctx_reload_tables(gpd_ctx *ctx, const gpd_config *cfg) {
  if (!ctx || !cfg) return set_err(GPD_ERR_INVALID, "gpd_ctx_reload_tables: null argument");
  std::vector<uint16_t> eth(65536, 0), proto(256, 0), tcp(65536, 0), udp(65536, 0);
  gpd_default_tables(eth.data(), proto.data(), tcp.data(), udp.data());
  if (cfg->ethertype) std::memcpy(eth.data(), cfg->ethertype, 65536 * 2);
  if (cfg->ipproto) std::memcpy(proto.data(), cfg->ipproto, 256 * 2);
  if (cfg->tcp_port) std::memcpy(tcp.data(), cfg->tcp_port, 65536 * 2);
  if (cfg->udp_port) std::memcpy(udp.data(), cfg->udp_port, 65536 * 2);
  const int rc = build_image(ctx, ctx->decoders, eth, proto, tcp, udp);
  if (rc != GPD_OK) return rc;  // the context keeps its previous snapshot and image
  ctx->t_eth.swap(eth);
  ctx->t_proto.swap(proto);
  ctx->t_tcp.swap(tcp);
  ctx->t_udp.swap(udp);
  return GPD_OK;
}

// Options the caller may set: the reference's two fields and the engine knobs (bits 24-29
// are the runtime's own launch flags).  The diagnostic library (libgpd_diag.so, -DGPD_DIAG)
// also takes bench.py's two ablation bits (30: no DMA wait, 31: no decode), which give wrong
// results by design; the shipped libgpd.so refuses them like any unknown bit (gpd.h).
#ifdef GPD_DIAG
static constexpr uint32_t kDiagOptions = (1u << 30) | (1u << 31);
#else
static constexpr uint32_t kDiagOptions = 0;
#endif
static constexpr uint32_t kUserOptions = GPD_OPT_IGNORE_UNSUPPORTED | GPD_OPT_IGNORE_PANIC |
                                         GPD_OPT_NO_CHECKSUMS | GPD_OPT_NO_FLOW_HASH | kDiagOptions;

int gpd_ctx_set_options(gpd_ctx *ctx, uint32_t options) {
  if (!ctx) return set_err(GPD_ERR_INVALID, "gpd_ctx_set_options: ctx is NULL");
  if (options & ~kUserOptions)
    return set_err(GPD_ERR_INVALID, "gpd_ctx_set_options: unknown option bits 0x%x",
                   options & ~kUserOptions);
  ctx->options = options;
  return GPD_OK;
}

int gpd_ctx_set_decoders(gpd_ctx *ctx, uint32_t decoders) {
  if (!ctx) return set_err(GPD_ERR_INVALID, "gpd_ctx_set_decoders: ctx is NULL");
  if (decoders & ~GPD_DEC_ALL)
    return set_err(GPD_ERR_INVALID, "gpd_ctx_set_decoders: unknown decoder bits 0x%x", decoders);
  if (decoders == ctx->decoders) return GPD_OK;
  const int rc = build_image(ctx, decoders, ctx->t_eth, ctx->t_proto, ctx->t_tcp, ctx->t_udp);
  if (rc == GPD_OK) ctx->decoders = decoders;  // a failed rebuild keeps the old mask and image
  return rc;
}

int gpd_ctx_add_decoders(gpd_ctx *ctx, uint32_t decoders) {
  if (!ctx) return set_err(GPD_ERR_INVALID, "gpd_ctx_add_decoders: ctx is NULL");
  if (decoders & ~GPD_DEC_ALL)
    return set_err(GPD_ERR_INVALID, "gpd_ctx_add_decoders: unknown decoder bits 0x%x", decoders);
  if ((ctx->decoders | decoders) == ctx->decoders) return GPD_OK;
  const uint32_t next = ctx->decoders | decoders;
  const int rc = build_image(ctx, next, ctx->t_eth, ctx->t_proto, ctx->t_tcp, ctx->t_udp);
  if (rc == GPD_OK) ctx->decoders = next;
  return rc;
}

int gpd_ctx_create(int device, const gpd_config *cfg, gpd_ctx **out) {
  if (!out) return set_err(GPD_ERR_INVALID, "gpd_ctx_create: out is NULL");
  *out = nullptr;
  int ndev = 0;
  const hipError_t dc = hipGetDeviceCount(&ndev);
  if (dc != hipSuccess || ndev == 0)
    return set_err(GPD_ERR_NODEVICE, "gpd_ctx_create: no HIP device available (%s, %d devices)",
                   hipGetErrorString(dc), ndev);
  if (device < 0 || device >= ndev)
    return set_err(GPD_ERR_INVALID, "gpd_ctx_create: device %d out of range [0,%d)", device, ndev);
  gpd_config defaults{};
  defaults.first_layer = GPD_LT_ETHERNET;
  defaults.decoders = GPD_DEC_ALL;
  if (!cfg) cfg = &defaults;
  if (cfg->decoders & ~GPD_DEC_ALL)
    return set_err(GPD_ERR_INVALID, "gpd_ctx_create: unknown decoder bits 0x%x", cfg->decoders);
  gpd_ctx *ctx = new gpd_ctx;
  ctx->device = device;
  ctx->first = cfg->first_layer;
  ctx->decoders = cfg->decoders;
  if (cfg->options & ~kUserOptions) {
    delete ctx;
    return set_err(GPD_ERR_INVALID, "gpd_ctx_create: unknown option bits 0x%x",
                   cfg->options & ~kUserOptions);
  }
  ctx->options = cfg->options;
  hipDeviceProp_t prop;
  gpd::DeviceScope dscope_;
  if (dscope_.set(device) != hipSuccess || hipGetDeviceProperties(&prop, device) != hipSuccess) {
    delete ctx;
    return set_err(GPD_ERR_HIP, "gpd_ctx_create: cannot query device %d", device);
  }
  ctx->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  int rc = gpd_ctx_reload_tables(ctx, cfg);
  if (rc) {
    delete ctx;
    return rc;
  }
  *out = ctx;
  return GPD_OK;
}

static void free_slots(gpd_ctx *ctx) {
  if (ctx->tw_in) (void)hipStreamSynchronize(ctx->tw_in);
  for (auto &s : ctx->slot) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.stream_out) (void)hipStreamSynchronize(s.stream_out);
    for (void *p : {(void *)s.h_data, (void *)s.h_off, (void *)s.h_len, (void *)s.h_status,
                    (void *)s.h_csum, (void *)s.h_layers, (void *)s.h_nh, (void *)s.h_th,
                    (void *)s.h_hoff, (void *)s.h_ext, (void *)s.h_det, (void *)s.h_tw})
      if (p) (void)hipHostFree(p);
    for (void *p : {(void *)s.d_data, (void *)s.d_off, (void *)s.d_len, (void *)s.d_status,
                    (void *)s.d_csum, (void *)s.d_layers, (void *)s.d_nh, (void *)s.d_th,
                    (void *)s.d_hoff, (void *)s.d_ext, (void *)s.d_det, (void *)s.d_pw, (void *)s.d_tw})
      if (p) (void)hipFree(p);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    if (s.stream_out) (void)hipStreamDestroy(s.stream_out);
    for (hipEvent_t e : {s.ev_in, s.ev_dec, s.ev_out})
      if (e) (void)hipEventDestroy(e);
    s = gpd_ctx::Slot{};
  }
  if (ctx->d_pw_ctl) (void)hipFree(ctx->d_pw_ctl);
  if (ctx->h_pw_ctl) (void)hipHostFree(ctx->h_pw_ctl);
  for (auto &e : ctx->ev_pw)
    if (e) (void)hipEventDestroy(e);
  if (ctx->tw_in) (void)hipStreamDestroy(ctx->tw_in);
  ctx->tw_in = nullptr;
  for (auto &e : ctx->ev_tw)
    if (e) (void)hipEventDestroy(e), e = nullptr;
  for (auto &e : ctx->ev_twdec)
    if (e) (void)hipEventDestroy(e), e = nullptr;
  for (auto &e : ctx->ev_twin)
    if (e) (void)hipEventDestroy(e), e = nullptr;
  ctx->d_pw_ctl = ctx->h_pw_ctl = nullptr;
  ctx->ev_pw[0] = ctx->ev_pw[1] = nullptr;
  ctx->slot_bytes = ctx->slot_pkts = 0;
}

int gpd_ctx_destroy(gpd_ctx *ctx) {
  if (!ctx) return GPD_OK;
  gpd::DeviceScope dscope_;
  (void)dscope_.set(ctx->device);
  free_slots(ctx);
  if (ctx->d_image) (void)hipFree(ctx->d_image);
  if (ctx->d_pages) (void)hipFree(ctx->d_pages);
  for (auto &kv : ctx->fallback) {
    if (kv.second.d) (void)hipFree(kv.second.d);
    if (kv.second.wc) (void)hipFree(kv.second.wc);
  }
  for (auto &sc : ctx->scratch)
    if (sc.d) (void)hipFree(sc.d);
  for (const auto &r : ctx->registered) (void)hipHostUnregister((void *)r.first);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->evm) (void)hipEventDestroy(ctx->evm);
  delete ctx;
  return GPD_OK;
}

int gpd_last_launch_split(gpd_ctx *ctx, uint64_t *fallback, float *fast_ms, float *list_ms) {
  if (!ctx || !fallback || !fast_ms || !list_ms)
    return set_err(GPD_ERR_INVALID, "gpd_last_launch_split: null argument");
  if (!ctx->timed || !ctx->timed_split)
    return set_err(GPD_ERR_INVALID, "gpd_last_launch_split: no timed fast-path launch "
                                    "(gpd_ctx_set_timing(1), then one gpd_decode of <= 2^30 packets)");
  gpd::DeviceScope dscope_;
  HIP_TRY(dscope_.set(ctx->device));
  HIP_TRY(hipEventSynchronize(ctx->ev1));
  HIP_TRY(hipEventElapsedTime(fast_ms, ctx->ev0, ctx->evm));
  HIP_TRY(hipEventElapsedTime(list_ms, ctx->evm, ctx->ev1));
  // the launch's per-wave counts stay until the launch after next on the stream rewrites them
  std::vector<uint32_t> wc(ctx->timed_fb_waves);
  if (!wc.empty())
    HIP_TRY(hipMemcpy(wc.data(), ctx->timed_fb_wc, wc.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
  uint64_t c = 0;
  for (uint32_t v : wc) c += v;
  *fallback = c;
  return GPD_OK;
}

int gpd_ctx_set_tuning(gpd_ctx *ctx, const gpd_tuning *t) {
  if (!ctx) return set_err(GPD_ERR_INVALID, "gpd_ctx_set_tuning: null ctx");
  const gpd_tuning automatic{0, -1, -1, 0, -1, -1, 0, -1};  // (waves_per_simd 0: automatic)
  if (!t) t = &automatic;
  if (t->window_bytes != 0 && t->window_bytes != 4096 && t->window_bytes != 8192)
    return set_err(GPD_ERR_INVALID, "gpd_ctx_set_tuning: window_bytes %u (0, 4096 or 8192)", t->window_bytes);
  if (t->shift < -1 || t->shift > 1 || t->reg_prefix < -1 || t->reg_prefix > 1 || t->header_once < -1 ||
      t->header_once > 2 || t->device_walk < -1 || t->device_walk > 1)
    return set_err(GPD_ERR_INVALID,
                   "gpd_ctx_set_tuning: shift / reg_prefix / device_walk outside {-1, 0, 1}, header_once "
                   "outside {-1, 0, 1, 2}");
  if (t->waves_per_simd != 0 && (t->waves_per_simd < 2 || t->waves_per_simd > 4))
    return set_err(GPD_ERR_INVALID, "gpd_ctx_set_tuning: waves_per_simd %d (0, 2, 3 or 4)", t->waves_per_simd);
  if (t->grid_rounds < 0 || t->grid_rounds > 8)
    return set_err(GPD_ERR_INVALID, "gpd_ctx_set_tuning: grid_rounds %d (0 .. 8)", t->grid_rounds);
  if (t->split < -1 || t->split > 1)
    return set_err(GPD_ERR_INVALID, "gpd_ctx_set_tuning: split %d (-1, 0 or 1)", t->split);
  ctx->tune = *t;
  return GPD_OK;
}

int gpd_ctx_set_timing(gpd_ctx *ctx, int enable) {
  if (!ctx) return set_err(GPD_ERR_INVALID, "gpd_ctx_set_timing: null ctx");
  gpd::DeviceScope dscope_;
  HIP_TRY(dscope_.set(ctx->device));
  if (enable && !ctx->ev0) {
    HIP_TRY(hipEventCreate(&ctx->ev0));
    HIP_TRY(hipEventCreate(&ctx->ev1));
    HIP_TRY(hipEventCreate(&ctx->evm));
  }
  ctx->timing = enable != 0;
  ctx->timed = false;
  return GPD_OK;
}

float gpd_last_kernel_ms(gpd_ctx *ctx) {
  if (!ctx || !ctx->timed) return -1.0f;
  float ms = -1.0f;
  if (hipEventSynchronize(ctx->ev1) != hipSuccess) return -1.0f;
  if (hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1) != hipSuccess) return -1.0f;
  return ms;
}

// Largest batch of one call: packet indices and (n + 63) / 64 stay 32-bit (gpd.h gpd_batch).
constexpr uint64_t kMaxBatchPackets = 0xFFFFFF00ull;

static int check_batch(const gpd_batch *in, const gpd_result *out) {
  if (!in || !out) return set_err(GPD_ERR_INVALID, "gpd_decode: null batch or result");
  if (in->n == 0) return GPD_OK;
  if (!in->data || !in->offset || !in->caplen)
    return set_err(GPD_ERR_INVALID, "gpd_decode: batch data/offset/caplen must be non-NULL");
  if (out->records) {
    if (out->status || out->layers || out->net_hash || out->tp_hash || out->csum)
      return set_err(GPD_ERR_INVALID, "gpd_decode: records excludes the status/layers/net_hash/tp_hash/csum arrays");
  } else if (!out->status || !out->layers) {
    return set_err(GPD_ERR_INVALID, "gpd_decode: result status/layers must be non-NULL");
  }
  if ((reinterpret_cast<uintptr_t>(in->data) & 15) != 0)
    return set_err(GPD_ERR_INVALID, "gpd_decode: data pointer must be 16-byte aligned");
  if (in->data_len > 0xFFFFFFF0ull)
    return set_err(GPD_ERR_INVALID, "gpd_decode: data_len %llu exceeds the 32-bit offset range",
                   (unsigned long long)in->data_len);
  if (in->n > kMaxBatchPackets)  // (packet and tile counts stay 32-bit in every kernel)
    return set_err(GPD_ERR_INVALID, "gpd_decode: batch of %llu packets (max 2^32 - 256)",
                   (unsigned long long)in->n);
  return GPD_OK;
}

// n_dev: the packet count is read on the device (at most in->n); geom_n: the packet count the
// staging choices assume (0: in->n) — both for batches whose records the device walk found.
static int launch(gpd_ctx *ctx, const gpd_batch *in, const gpd_result *out, hipStream_t stream,
                  bool record, const uint32_t *n_dev = nullptr, uint64_t geom_n = 0, uint64_t geom_bytes = 0) {
  gpd::KParams P{};
  P.data = in->data;
  P.data_len = in->data_len;
  P.offset = in->offset;
  P.caplen = in->caplen;
  P.n = in->n;
  P.n_dev = n_dev;
  P.status = out->status;
  P.layers = out->layers;
  P.net_hash = out->net_hash;
  P.tp_hash = out->tp_hash;
  P.csum = out->csum;
  P.ext = out->ext;
  P.hdr_off = out->hdr_off;
  P.rec = out->records;
  P.detail = out->detail;
  P.image = ctx->d_image;
  P.pages = ctx->d_pages;
  P.image_words = ctx->image_words;
  P.use_pages = ctx->use_pages;
  P.eth_base = ctx->eth_base; P.tcp_base = ctx->tcp_base; P.udp_base = ctx->udp_base;
  P.eth_bits = ctx->eth_bits; P.tcp_bits = ctx->tcp_bits; P.udp_bits = ctx->udp_bits;
  P.eth_mult = ctx->eth_mult; P.tcp_mult = ctx->tcp_mult; P.udp_mult = ctx->udp_mult;
  P.fixed = ctx->fixed;
  // LDS window per buffer: the smallest of 4/8 KiB that holds a typical 64-packet tile
  const uint64_t gn = geom_n ? geom_n : in->n;
  const uint64_t mean_slot = ((geom_bytes ? geom_bytes : in->data_len) + gn - 1) / gn;
  P.stage = mean_slot * 64 <= 4096 ? 4096u : 8192u;
  if (ctx->tune.window_bytes) P.stage = ctx->tune.window_bytes;
  P.first = ctx->first;
  P.decoders = ctx->decoders;
  P.options = ctx->options;
  // streamed bytes and results use the nt cache policy (read once / written once)
  P.options |= 3u << 28;
  // Window copies shifted so that network headers sit 16-byte aligned in LDS, for batches of
  // small frames (mean slot <= 96 B: a window holds 40+ packets and the saved misaligned reads
  // outweigh the shifted copy; with IMIX-sized frames they do not).  gpd_ctx_set_tuning can
  // force either copy (the parity tests cover both).
  const bool shift = ctx->tune.shift >= 0 ? ctx->tune.shift != 0 : mean_slot <= 96;
  if (shift) P.options |= 1u << 27;
  // long frames (mean slot > 160 B): 8 KiB windows whose chunk prefix sums are computed from
  // the registers at commit
  if (ctx->tune.reg_prefix >= 0 ? ctx->tune.reg_prefix != 0 : (mean_slot > 160 && !shift))
    P.options |= 1u << 26;
  // ... whose 64-packet tiles span several windows: decoded once per tile from the headers the
  // windows stage (seg_pass), not once per window with the lanes each window holds — by default
  // over 8 KiB rounds of each tile's contiguous run (ro_kernel) rather than windows cut at packet
  // boundaries (IMIX 0.319 -> 0.296 ms, same box, profiles/r04/ro_ab/)
  const int ho = ctx->tune.header_once >= 0 ? ctx->tune.header_once : (mean_slot > 160 && !shift ? 2 : 0);
  if (P.stage == 8192 && ho == 1) P.options |= 1u << 25;
  if (ho == 2) P.options |= 1u << 24;
  P.waves = (uint32_t)ctx->tune.waves_per_simd;
  P.rounds = (uint32_t)ctx->tune.grid_rounds;
  // 4 KiB windows of small frames by the loader / decoder split kernel (automatic: on; config 2
  // 0.319 -> 0.297 ms, tcp64 0.321 -> 0.304, same box)
  P.split = ctx->tune.split >= 0 ? (uint32_t)ctx->tune.split : 1u;
  P.nstores = out->records ? 2u + (out->hdr_off != nullptr)
                           : 2u + (out->net_hash != nullptr) + (out->tp_hash != nullptr) +
                                 (out->csum != nullptr) + (out->hdr_off != nullptr);
  if (gpd::fast_eligible(P)) {  // fallback list scratch for this stream, sized for one launch
    const uint64_t need = std::min<uint64_t>(in->n, gpd::kMaxLaunchPackets);
    auto &fb = ctx->fallback[stream];
    if (fb.cap < need) {
      if (fb.d) {
        HIP_TRY(hipStreamSynchronize(stream));
        HIP_TRY(hipFree(fb.d));
        HIP_TRY(hipFree(fb.wc));
        fb.d = fb.wc = nullptr;
        fb.cap = 0;
      }
      // the list: 64 entries per tile (each wave's region spans its tiles), after the flags
      HIP_TRY(hipMalloc(&fb.d, 128 * sizeof(uint32_t) + (need + 64) * sizeof(uint64_t)));
      HIP_TRY(hipMemset(fb.d, 0, 128 * sizeof(uint32_t)));  // both flags start at zero
      HIP_TRY(hipMalloc(&fb.wc, 2ull * ctx->num_cus * gpd::kMaxFastWavesPerCU * sizeof(uint32_t)));
      fb.cap = need;
      fb.parity = 0;
    }
    P.fb_list = reinterpret_cast<uint64_t *>(fb.d + 128);
  }
  if (record) HIP_TRY(hipEventRecord(ctx->ev0, stream));
  const bool split = record && in->n <= gpd::kMaxLaunchPackets && gpd::fast_eligible(P);
  ctx->timed_split = false;
  // launches of <= kMaxLaunchPackets packets keep every packet/tile index 32-bit in the kernel
  for (uint64_t lo = 0; lo < in->n; lo += gpd::kMaxLaunchPackets) {
    gpd::KParams Q = P;
    Q.n = std::min<uint64_t>(gpd::kMaxLaunchPackets, in->n - lo);
    Q.offset = in->offset + lo;
    Q.caplen = in->caplen + lo;
    Q.status = out->status ? out->status + lo : nullptr;
    Q.layers = out->layers ? out->layers + lo : nullptr;
    Q.rec = out->records ? out->records + lo : nullptr;
    Q.net_hash = out->net_hash ? out->net_hash + lo : nullptr;
    Q.tp_hash = out->tp_hash ? out->tp_hash + lo : nullptr;
    Q.csum = out->csum ? out->csum + lo : nullptr;
    Q.ext = out->ext ? out->ext + lo : nullptr;
    Q.hdr_off = out->hdr_off ? out->hdr_off + lo : nullptr;
    Q.detail = out->detail ? out->detail + lo : nullptr;
    if (gpd::fast_eligible(P)) {  // per-wave counts, two arrays used alternately (a timed
      auto &fb = ctx->fallback[stream];  // launch's counts survive the next launch for the split)
      Q.fb_wcount = fb.wc + (size_t)ctx->num_cus * gpd::kMaxFastWavesPerCU * fb.parity;
      fb.parity ^= 1u;
    }
    uint32_t fbw = 0;
    hipError_t e = gpd::launch_decode(Q, stream, ctx->num_cus, split ? ctx->evm : nullptr, &fbw);
    if (e != hipSuccess) return set_err(GPD_ERR_HIP, "decode kernel launch: %s", hipGetErrorString(e));
    if (split) {
      ctx->timed_fb_wc = Q.fb_wcount;
      ctx->timed_fb_waves = fbw;
    }
  }
  if (record) {
    HIP_TRY(hipEventRecord(ctx->ev1, stream));
    ctx->timed = true;
    ctx->timed_split = split;
  }
  return GPD_OK;
}

int gpd_decode(gpd_ctx *ctx, const gpd_batch *in, const gpd_result *out, void *stream) {
  if (!ctx) return set_err(GPD_ERR_INVALID, "gpd_decode: null ctx");
  int rc = check_batch(in, out);
  if (rc || in->n == 0) return rc;
  gpd::DeviceScope dscope_;
  HIP_TRY(dscope_.set(ctx->device));
  return launch(ctx, in, out, (hipStream_t)stream, ctx->timing);
}

int gpd_sync(gpd_ctx *ctx, void *stream) {
  if (!ctx) return set_err(GPD_ERR_INVALID, "gpd_sync: null ctx");
  gpd::DeviceScope dscope_;
  HIP_TRY(dscope_.set(ctx->device));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return GPD_OK;
}

// ---- IPv4 fragment hand-off (include/gpd_defrag.h) ----
int gpd_ip4_fragments(gpd_ctx *ctx, const gpd_batch *in, const gpd_result *res, gpd_ip4_frag *out,
                      uint64_t max_out, uint64_t *count, void *stream) {
  if (!ctx || !in || !res || !count) return set_err(GPD_ERR_INVALID, "gpd_ip4_fragments: null argument");
  *count = 0;
  if (in->n == 0) return GPD_OK;
  if (in->n > 0xFFFFFF00ull) return set_err(GPD_ERR_INVALID, "gpd_ip4_fragments: batch of %llu packets (max 2^32 - 256)",
                                            (unsigned long long)in->n);
  if (!in->data || !in->offset || !in->caplen)
    return set_err(GPD_ERR_INVALID, "gpd_ip4_fragments: batch data/offset/caplen must be non-NULL");
  if (!res->hdr_off || (!res->records && (!res->status || !res->layers)))
    return set_err(GPD_ERR_INVALID, "gpd_ip4_fragments: needs hdr_off and status + layers (or records)");
  if (max_out && !out) return set_err(GPD_ERR_INVALID, "gpd_ip4_fragments: null out with max_out > 0");
  gpd::DeviceScope dscope_;
  HIP_TRY(dscope_.set(ctx->device));
  gpd::FragArgs A{};
  gpd::KParams &P = A.P;
  P.data = in->data;
  P.data_len = in->data_len;
  P.offset = in->offset;
  P.caplen = in->caplen;
  P.n = in->n;
  P.status = res->status;
  P.layers = res->layers;
  P.rec = res->records;
  P.hdr_off = res->hdr_off;
  P.image = ctx->d_image;
  P.pages = ctx->d_pages;
  P.image_words = ctx->image_words;
  P.use_pages = ctx->use_pages;
  P.eth_base = ctx->eth_base; P.tcp_base = ctx->tcp_base; P.udp_base = ctx->udp_base;
  P.eth_bits = ctx->eth_bits; P.tcp_bits = ctx->tcp_bits; P.udp_bits = ctx->udp_bits;
  P.eth_mult = ctx->eth_mult; P.tcp_mult = ctx->tcp_mult; P.udp_mult = ctx->udp_mult;
  P.fixed = ctx->fixed;
  P.first = ctx->first;
  P.decoders = ctx->decoders;
  P.options = ctx->options;
  A.out = out;
  A.max_out = (uint32_t)std::min<uint64_t>(max_out, in->n);
  A.nblk = (uint32_t)((in->n + 2047) / 2048);
  A.blk = static_cast<uint32_t *>(gpd::ctx_scratch(ctx, 12, ((size_t)A.nblk + 1) * 4));
  A.idx = static_cast<uint32_t *>(gpd::ctx_scratch(ctx, 13, (size_t)in->n * 4));
  A.mask = static_cast<uint64_t *>(gpd::ctx_scratch(ctx, 14, ((size_t)in->n + 63) / 64 * 8));
  if (!A.blk || !A.idx || !A.mask) return set_err(GPD_ERR_NOMEM, "gpd_ip4_fragments: scratch allocation failed");
  const hipStream_t s = (hipStream_t)stream;
  hipError_t e = gpd::launch_ip4_frag(A, s, ctx->num_cus);
  if (e != hipSuccess) return set_err(GPD_ERR_HIP, "gpd_ip4_fragments launch: %s", hipGetErrorString(e));
  uint32_t total = 0;
  HIP_TRY(hipMemcpyAsync(&total, A.blk + A.nblk, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  *count = total;
  return GPD_OK;
}

// ---- host-memory path: chunked, double-buffered pinned H2D -> decode -> D2H ----
static int alloc_slots(gpd_ctx *ctx, uint64_t bytes, uint64_t pkts, bool ext, bool det) {
  if (ctx->slot_bytes >= bytes && ctx->slot_pkts >= pkts && (!ext || ctx->slot[0].d_ext) &&
      (!det || ctx->slot[0].d_det))
    return GPD_OK;
  ext = ext || ctx->slot[0].d_ext;  // (a re-allocation keeps what earlier calls asked for)
  det = det || ctx->slot[0].d_det;
  free_slots(ctx);
  for (auto &s : ctx->slot) {
    HIP_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    HIP_TRY(hipHostMalloc(&s.h_data, bytes + 64, hipHostMallocDefault));
    HIP_TRY(hipMalloc(&s.d_data, bytes + 64));
    HIP_TRY(hipHostMalloc(&s.h_off, pkts * 4, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&s.h_len, pkts * 4, hipHostMallocDefault));
    HIP_TRY(hipMalloc(&s.d_off, pkts * 4));
    HIP_TRY(hipMalloc(&s.d_len, pkts * 4));
    HIP_TRY(hipHostMalloc(&s.h_status, pkts * 4, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&s.h_csum, pkts * 4, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&s.h_layers, pkts * 8, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&s.h_nh, pkts * 8, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&s.h_th, pkts * 8, hipHostMallocDefault));
    HIP_TRY(hipMalloc(&s.d_status, pkts * 4));
    HIP_TRY(hipMalloc(&s.d_csum, pkts * 4));
    HIP_TRY(hipMalloc(&s.d_layers, pkts * 8));
    HIP_TRY(hipMalloc(&s.d_nh, pkts * 8));
    HIP_TRY(hipMalloc(&s.d_th, pkts * 8));
    HIP_TRY(hipHostMalloc(&s.h_hoff, pkts * 4, hipHostMallocDefault));
    HIP_TRY(hipMalloc(&s.d_hoff, pkts * 4));
    if (ext) {
      HIP_TRY(hipHostMalloc(&s.h_ext, pkts * sizeof(gpd_ext_rec), hipHostMallocDefault));
      HIP_TRY(hipMalloc(&s.d_ext, pkts * sizeof(gpd_ext_rec)));
    }
    if (det) {
      HIP_TRY(hipHostMalloc(&s.h_det, pkts * sizeof(gpd_detail), hipHostMallocDefault));
      HIP_TRY(hipMalloc(&s.d_det, pkts * sizeof(gpd_detail)));
    }
    HIP_TRY(hipMalloc(&s.d_pw, 5ull * gpd::kPwMaxSeg * 4));
  }
  HIP_TRY(hipMalloc(&ctx->d_pw_ctl, 2 * sizeof(gpd::PwCtl)));
  HIP_TRY(hipHostMalloc(&ctx->h_pw_ctl, 2 * sizeof(gpd::PwCtl), hipHostMallocDefault));
  for (auto &e : ctx->ev_pw) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  ctx->slot_bytes = bytes;
  ctx->slot_pkts = pkts;
  return GPD_OK;
}

// Error exits of the staged paths leave no slot in flight: every busy slot is waited for and
// dropped (its results belong to the failed call and are not drained anywhere), so the next
// call on the context starts from idle slots.  On success every slot was drained already.
struct SlotGuard {
  gpd_ctx *ctx;
  ~SlotGuard() {
    for (auto &s : ctx->slot)
      if (s.busy) {
        if (ctx->tw_in) (void)hipStreamSynchronize(ctx->tw_in);
        (void)hipStreamSynchronize(s.stream);
        if (s.stream_out) (void)hipStreamSynchronize(s.stream_out);
        s.busy = false;
      }
  }
};

static void drain_slot(gpd_ctx::Slot &s, const gpd_result *out) {
  const uint64_t m = s.hi - s.lo;
  if (!s.direct) {
    par_for(m, 1u << 16, [&](uint64_t a, uint64_t b) {
      const uint64_t c = b - a;
      std::memcpy(out->status + s.lo + a, s.h_status + a, c * 4);
      std::memcpy(out->layers + s.lo + a, s.h_layers + a, c * 8);
      if (out->csum) std::memcpy(out->csum + s.lo + a, s.h_csum + a, c * 4);
      if (out->net_hash) std::memcpy(out->net_hash + s.lo + a, s.h_nh + a, c * 8);
      if (out->tp_hash) std::memcpy(out->tp_hash + s.lo + a, s.h_th + a, c * 8);
      if (out->hdr_off) std::memcpy(out->hdr_off + s.lo + a, s.h_hoff + a, c * 4);
      if (out->ext) std::memcpy(out->ext + s.lo + a, s.h_ext + a, c * sizeof(gpd_ext_rec));
      if (out->detail) std::memcpy(out->detail + s.lo + a, s.h_det + a, c * sizeof(gpd_detail));
    });
  }
  s.busy = false;
}

// Results of packets [lo, lo + m) device -> host on the slot's stream: straight into the
// caller's arrays when every one of them lies in registered memory (gpd_host_register; then
// the drain copies nothing), else into the slot's pinned arrays for drain_slot to copy.
static hipError_t results_d2h(gpd_ctx *ctx, gpd_ctx::Slot &s, const gpd_result *out, uint64_t lo,
                              uint64_t m, hipStream_t stream) {
  auto reg = [&](const void *p, uint64_t bytes) {
    return p == nullptr || ctx->is_registered(static_cast<const uint8_t *>(p), bytes);
  };
  s.direct = !out->ext && reg(out->status + lo, m * 4) && reg(out->layers + lo, m * 8) &&
             reg(out->csum ? out->csum + lo : nullptr, m * 4) &&
             reg(out->net_hash ? out->net_hash + lo : nullptr, m * 8) &&
             reg(out->tp_hash ? out->tp_hash + lo : nullptr, m * 8) &&
             reg(out->hdr_off ? out->hdr_off + lo : nullptr, m * 4) &&
             reg(out->detail ? out->detail + lo : nullptr, m * sizeof(gpd_detail));
  auto cp = [&](void *host, const void *dev, uint64_t bytes) {
    return hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, stream);
  };
  hipError_t e = cp(s.direct ? (void *)(out->status + lo) : (void *)s.h_status, s.d_status, m * 4);
  if (e == hipSuccess) e = cp(s.direct ? (void *)(out->layers + lo) : (void *)s.h_layers, s.d_layers, m * 8);
  if (e == hipSuccess && out->csum) e = cp(s.direct ? (void *)(out->csum + lo) : (void *)s.h_csum, s.d_csum, m * 4);
  if (e == hipSuccess && out->net_hash)
    e = cp(s.direct ? (void *)(out->net_hash + lo) : (void *)s.h_nh, s.d_nh, m * 8);
  if (e == hipSuccess && out->tp_hash)
    e = cp(s.direct ? (void *)(out->tp_hash + lo) : (void *)s.h_th, s.d_th, m * 8);
  if (e == hipSuccess && out->hdr_off)
    e = cp(s.direct ? (void *)(out->hdr_off + lo) : (void *)s.h_hoff, s.d_hoff, m * 4);
  if (e == hipSuccess && out->ext) e = cp(s.h_ext, s.d_ext, m * sizeof(gpd_ext_rec));
  if (e == hipSuccess && out->detail)
    e = cp(s.direct ? (void *)(out->detail + lo) : (void *)s.h_det, s.d_det, m * sizeof(gpd_detail));
  return e;
}

int gpd_decode_host(gpd_ctx *ctx, const gpd_batch *in, const gpd_result *out) {
  if (!ctx) return set_err(GPD_ERR_INVALID, "gpd_decode_host: null ctx");
  if (!in || !out || !out->status || !out->layers)
    return set_err(GPD_ERR_INVALID, "gpd_decode_host: null batch/result");
  if (in->n == 0) return GPD_OK;
  if (in->n > kMaxBatchPackets)
    return set_err(GPD_ERR_INVALID, "gpd_decode_host: batch of %llu packets (max 2^32 - 256)",
                   (unsigned long long)in->n);
  gpd::DeviceScope dscope_;
  HIP_TRY(dscope_.set(ctx->device));
  const uint64_t kPkts = 1u << 20, kBytes = 256ull << 20;
  int rc = alloc_slots(ctx, kBytes, kPkts, out->ext != nullptr, out->detail != nullptr);
  if (rc) return rc;
  // Each slot's chunk: H2D and decode on its stream, the results D2H on its stream_out, so the
  // next chunks' H2D never waits behind a D2H (the link carries both directions at once)
  for (auto &s : ctx->slot) {
    if (!s.stream_out) HIP_TRY(hipStreamCreateWithFlags(&s.stream_out, hipStreamNonBlocking));
    for (hipEvent_t *e : {&s.ev_in, &s.ev_dec, &s.ev_out})
      if (!*e) HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  SlotGuard guard{ctx};
  uint64_t i = 0;
  int k = 0;
  while (i < in->n) {
    auto &s = ctx->slot[k];
    if (s.busy) HIP_TRY(hipEventSynchronize(s.ev_in));  // chunk k-2's H2D read the host staging
    // Span mode: packets [i, j) lie inside one window of the source buffer of at most kBytes
    // with few gaps (the usual back-to-back batch): that window travels as it is (straight
    // from the caller's buffer when it is registered) and the offsets are rebased.
    // Otherwise the packets are repacked 16-byte aligned into the slot.
    uint64_t j = i, used = 0;
    const uint64_t lo16 = std::min<uint64_t>(in->offset[i], in->data_len) & ~15ull;
    uint64_t span_hi = lo16;
    while (j < in->n && j - i < kPkts) {
      const uint64_t o = in->offset[j], e = o + in->caplen[j];
      if (o < lo16 || e > in->data_len || e - lo16 > kBytes) break;
      span_hi = std::max(span_hi, e);
      used += in->caplen[j];
      j++;
    }
    // (a registered window travels by DMA alone, so it may carry more gap — e.g. an AF_PACKET
    // ring's frame headers — before a 16-thread host repack of the packets would be cheaper)
    const bool reg = j > i && ctx->is_registered(in->data + lo16, span_hi - lo16);
    const bool span = j > i && (span_hi - lo16) <= (reg ? 4 : 2) * used + 4096;
    uint64_t pos = 0;
    // a span whose descriptors are registered too (a capture loop pins its arrays once): they
    // travel by DMA as they are, and the kernel reads the window through a base pointer moved
    // back by lo16, so the caller's absolute offsets index it — no host pass over the chunk
    bool dreg = false;
    if (span) {
      pos = span_hi - lo16;
      const uint64_t m = j - i;
      // (the kernel's buffer end lo16 + pos must stay in the 32-bit offset range; past 4 GiB the
      // offsets are rebased instead)
      dreg = lo16 + pos <= 0xFFFFFFF0ull && ctx->is_registered((const uint8_t *)(in->offset + i), m * 4) &&
             ctx->is_registered((const uint8_t *)(in->caplen + i), m * 4);
      if (!dreg)
        par_for(m, 1u << 16, [&](uint64_t a, uint64_t b) {
          for (uint64_t p = a; p < b; p++) s.h_off[p] = (uint32_t)(in->offset[i + p] - lo16);
          std::memcpy(s.h_len + a, in->caplen + i + a, (b - a) * 4);
        });
      const uint64_t bytes = std::min<uint64_t>((pos + 15) & ~15ull, ((in->data_len + 15) & ~15ull) - lo16);
      if (ctx->is_registered(in->data + lo16, bytes)) {
        HIP_TRY(hipMemcpyAsync(s.d_data, in->data + lo16, bytes, hipMemcpyHostToDevice, s.stream));
      } else {
        par_memcpy(s.h_data, in->data + lo16, bytes);
        HIP_TRY(hipMemcpyAsync(s.d_data, s.h_data, bytes, hipMemcpyHostToDevice, s.stream));
      }
    } else {
      j = i;
      used = 0;
      while (j < in->n && j - i < kPkts) {
        const uint32_t len = in->caplen[j];
        const uint64_t need = ((used + 15) & ~15ull) + len;
        if (need > kBytes) break;
        used = need;
        j++;
      }
      if (j == i) return set_err(GPD_ERR_INVALID, "gpd_decode_host: packet %llu larger than %llu bytes",
                                 (unsigned long long)i, (unsigned long long)kBytes);
      for (uint64_t p = i; p < j; p++) {  // positions (cheap), then the copies in parallel
        pos = (pos + 15) & ~15ull;
        s.h_off[p - i] = (uint32_t)pos;
        s.h_len[p - i] = in->caplen[p];
        pos += in->caplen[p];
      }
      par_for(j - i, 1u << 14, [&](uint64_t a, uint64_t b) {
        for (uint64_t p = a; p < b; p++)
          std::memcpy(s.h_data + s.h_off[p], in->data + in->offset[i + p], s.h_len[p]);
      });
      HIP_TRY(hipMemcpyAsync(s.d_data, s.h_data, (pos + 15) & ~15ull, hipMemcpyHostToDevice, s.stream));
    }
    const uint64_t m = j - i;
    HIP_TRY(hipMemcpyAsync(s.d_off, dreg ? in->offset + i : s.h_off, m * 4, hipMemcpyHostToDevice, s.stream));
    HIP_TRY(hipMemcpyAsync(s.d_len, dreg ? in->caplen + i : s.h_len, m * 4, hipMemcpyHostToDevice, s.stream));
    HIP_TRY(hipEventRecord(s.ev_in, s.stream));
    if (s.busy) {  // chunk k-2's results are back (and drained) before this decode rewrites them
      HIP_TRY(hipEventSynchronize(s.ev_out));
      drain_slot(s, out);
    }
    gpd_batch b{s.d_data, pos, s.d_off, s.d_len, m};
    if (dreg) {
      b.data = s.d_data - lo16;  // 16-aligned (lo16 is); the kernel never reads below lo16
      b.data_len = lo16 + pos;
    }
    gpd_result r{s.d_status, s.d_layers, s.d_nh, s.d_th, s.d_csum, out->ext ? s.d_ext : nullptr,
                 out->hdr_off ? s.d_hoff : nullptr, nullptr, out->detail ? s.d_det : nullptr};
    rc = launch(ctx, &b, &r, s.stream, false, nullptr, 0, pos);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(s.ev_dec, s.stream));
    HIP_TRY(hipStreamWaitEvent(s.stream_out, s.ev_dec, 0));
    HIP_TRY(results_d2h(ctx, s, out, i, m, s.stream_out));
    HIP_TRY(hipEventRecord(s.ev_out, s.stream_out));
    s.lo = i;
    s.hi = j;
    s.busy = true;
    i = j;
    k ^= 1;
  }
  for (auto &s : ctx->slot) {
    if (s.busy) {
      HIP_TRY(hipStreamSynchronize(s.stream));
      HIP_TRY(hipStreamSynchronize(s.stream_out));
      drain_slot(s, out);
    }
  }
  return GPD_OK;
}

// ---- pcap capture in host memory: index, then raw-byte chunks H2D -> decode -> D2H ----
int gpd_host_register(gpd_ctx *ctx, const void *ptr, uint64_t len) {
  if (!ctx || !ptr || !len) return set_err(GPD_ERR_INVALID, "gpd_host_register: bad argument");
  gpd::DeviceScope dscope_;
  HIP_TRY(dscope_.set(ctx->device));
  HIP_TRY(hipHostRegister(const_cast<void *>(ptr), len, hipHostRegisterDefault));
  ctx->registered.emplace_back((const uint8_t *)ptr, len);
  return GPD_OK;
}

// The NUMA node of a device's PCI function (sysfs), -1 when unknown.
static int device_numa_node(int device) {
  char bus[64] = {0};
  int count = 0;
  // (a failed HIP call would stay the thread's last error, and the caller's next launch check,
  // torch's included, would report it: clear it)
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count ||
      hipDeviceGetPCIBusId(bus, (int)sizeof bus - 1, device) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  for (char *c = bus; *c; c++) *c = (char)tolower((unsigned char)*c);
  char path[160];
  std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE *f = std::fopen(path, "r");
  if (!f) return -1;
  int node = -1;
  if (std::fscanf(f, "%d", &node) != 1) node = -1;
  std::fclose(f);
  return node;
}

int gpd_host_bind_local(int device, void *ptr, uint64_t len, int *node_out) {
  if (node_out) *node_out = -1;
  if (!ptr || !len) return set_err(GPD_ERR_INVALID, "gpd_host_bind_local: bad argument");
  const int node = device_numa_node(device);
  if (node_out) *node_out = node;
  if (node < 0) return GPD_OK;  // one node, or the platform does not say
  if (node >= 1024) return set_err(GPD_ERR_INVALID, "gpd_host_bind_local: node %d", node);
  const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE);
  const uint64_t lo = ((uint64_t)ptr + page - 1) & ~(page - 1), hi = ((uint64_t)ptr + len) & ~(page - 1);
  if (hi <= lo) return GPD_OK;
  unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {0};
  mask[node / (8 * sizeof(unsigned long))] = 1ul << (node % (8 * sizeof(unsigned long)));
  // MPOL_PREFERRED (1): the node while it has free pages; MPOL_MF_MOVE (2): migrate pages
  // already placed elsewhere
  if (syscall(SYS_mbind, (void *)lo, hi - lo, 1, mask, (unsigned long)(8 * sizeof mask), 2u) != 0)
    return set_err(GPD_ERR_INVALID, "gpd_host_bind_local: mbind: %s", std::strerror(errno));
  return GPD_OK;
}

int gpd_host_unregister(gpd_ctx *ctx, const void *ptr) {
  if (!ctx) return set_err(GPD_ERR_INVALID, "gpd_host_unregister: null ctx");
  for (size_t k = 0; k < ctx->registered.size(); k++) {
    if (ctx->registered[k].first == ptr) {
      gpd::DeviceScope dscope_;
      HIP_TRY(dscope_.set(ctx->device));
      for (auto &s : ctx->slot)
        if (s.stream) HIP_TRY(hipStreamSynchronize(s.stream));
      HIP_TRY(hipHostUnregister(const_cast<void *>(ptr)));
      ctx->registered.erase(ctx->registered.begin() + (long)k);
      return GPD_OK;
    }
  }
  return set_err(GPD_ERR_INVALID, "gpd_host_unregister: pointer not registered");
}

// memcpy split over threads (the staging copy of an unregistered capture)
static void par_memcpy(uint8_t *dst, const uint8_t *src, uint64_t n, int nthreads) {
  const uint64_t kMin = 8ull << 20;
  int T = (int)std::min<uint64_t>((uint64_t)std::max(1, nthreads), std::max<uint64_t>(1, n / kMin));
  if (T <= 1) {
    std::memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> th;
  for (int k = 0; k < T; k++) {
    const uint64_t lo = n * (uint64_t)k / (uint64_t)T, hi = n * (uint64_t)(k + 1) / (uint64_t)T;
    th.emplace_back([=] { std::memcpy(dst + lo, src + lo, hi - lo); });
  }
  for (auto &t : th) t.join();
}

// Host-clock phases of this thread's last gpd_decode_pcap(_at) call (gpd_decode_pcap_last_times).
static thread_local double g_pt_walk = 0, g_pt_walkwait = 0, g_pt_stage = 0, g_pt_sync = 0, g_pt_drain = 0,
                           g_pt_total = 0;
// ... and its device-walk chunks: walked, handed to the host, and the reasons (PwCtl::status bits)
static thread_local uint32_t g_pw_counts[7];
static thread_local uint64_t g_pw_miss[2] = {~0ull, ~0ull};  // the last refuted speculation: start, segment
static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int gpd_decode_pcap(gpd_ctx *ctx, const uint8_t *buf, uint64_t len, uint64_t max_n,
                    const gpd_result *out, uint64_t *n_out, uint64_t *next_pos, int *stop,
                    int nthreads) {
  if (!ctx || !buf) return set_err(GPD_ERR_INVALID, "gpd_decode_pcap: null argument");
  gpd_pcap_info info;
  const int rc = gpd_pcap_header(buf, len, &info);
  if (rc) return rc;
  return gpd_decode_pcap_at(ctx, buf, len, &info, GPD_PCAP_HEADER_BYTES, max_n, out, n_out, next_pos, stop,
                            nthreads);
}

// The pcap path with the record walk on the host (gpd_pcap.cpp), one part ahead of the chunks.
static int decode_pcap_host_walk(gpd_ctx *ctx, const uint8_t *buf, uint64_t len, const gpd_pcap_info *info,
                                 uint64_t pos, uint64_t max_n, const gpd_result *out, uint64_t *n_out,
                                 uint64_t *next_pos, int *stop, int nthreads) {
  *n_out = 0;
  if (next_pos) *next_pos = pos;
  if (stop) *stop = GPD_PCAP_STOP_LIMIT;
  if (max_n == 0) return GPD_OK;
  const uint64_t kPkts = 1u << 20;
  // staging chunks of up to 256 MiB; slots of 64 MiB or more that the device walk already holds
  // serve as they are when a record fits them (a stretch the device walk hands over: pinned
  // slots re-allocated in the middle of a replay cost ~130 ms, r04)
  const uint64_t kBytes = ctx->slot_bytes >= (64ull << 20) && ctx->slot_bytes >= 64ull + info->snaplen
                              ? std::min<uint64_t>(ctx->slot_bytes, 256ull << 20) : 256ull << 20;
  const uint64_t kPart = 1u << 21;  // records per walked part (the first, walked before any
  const uint64_t kPart0 = 1u << 19; // transfer can start, is smaller)
  int rc = alloc_slots(ctx, kBytes, kPkts, false, out->detail != nullptr);
  if (rc) return rc;
  SlotGuard guard{ctx};
  // The record walk runs one part (kPart records) ahead of the transfers, on a helper thread:
  // while part q's chunks travel and decode, part q+1 is walked.  Two parts' record positions
  // and capture lengths are kept per calling thread across calls (a replay or capture loop
  // calls again and again; fresh pages for 12 B per record would cost more than the walk).
  struct Part {
    gpd::PcapResult W;
    std::vector<uint64_t> rp;
    std::vector<uint32_t> rcap;
    int rc = 0;
    std::string err;
  };
  static thread_local Part part[2];
  double walk_ms = 0;  // (written by the walking thread, read after its join)
  auto walk_part = [&](Part &P, uint64_t at, uint64_t m) {
    const double t0 = now_ms();
    if (P.rp.size() < m) {
      P.rp.resize(m);
      P.rcap.resize(m);
    }
    gpd::PcapOut o;  // positions and capture lengths only (what a decode needs)
    o.pos64 = P.rp.data();
    o.cap = P.rcap.data();
    P.rc = gpd::pcap_index_flat(buf, len, *info, at, m, nthreads, o, P.W);
    P.err = P.rc ? std::string(gpd_last_error_string()) : std::string();  // (the walker's thread)
    walk_ms += now_ms() - t0;
  };
  uint64_t done = 0;  // records decoded (the output index of the next one)
  int q = 0;
  walk_part(part[0], pos, std::min(kPart0, max_n));
  struct Joiner {  // every exit, errors included, waits for the walk running ahead
    std::thread t;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  } ahead;
  int k = 0;
  for (;;) {
    Part &cur = part[q];
    const uint64_t n = cur.W.n;
    const bool more = cur.rc == GPD_OK && cur.W.stop == GPD_PCAP_STOP_LIMIT && n > 0 && done + n < max_n;
    if (more)  // walk the next part while this one is staged
      ahead.t = std::thread(walk_part, std::ref(part[q ^ 1]), cur.W.next_pos, std::min(kPart, max_n - done - n));
    uint64_t i = 0;
    while (i < n) {
      auto &s = ctx->slot[k];
      if (s.busy) {
        const double t0 = now_ms();
        HIP_TRY(hipStreamSynchronize(s.stream));
        const double t1 = now_ms();
        drain_slot(s, out);
        g_pt_sync += t1 - t0;
        g_pt_drain += now_ms() - t1;
      }
      const double t_stage = now_ms();
      // records [i, j) whose bytes (from the first one's data, rounded down to 16) fit the slot
      const uint64_t base = (cur.rp[i] + GPD_PCAP_RECORD_BYTES) & ~15ull;
      uint64_t j = i;
      while (j < n && j - i < kPkts && cur.rp[j] + GPD_PCAP_RECORD_BYTES + cur.rcap[j] - base <= kBytes) j++;
      if (j == i) {
        return set_err(GPD_ERR_INVALID, "gpd_decode_pcap: record %llu larger than %llu bytes",
                       (unsigned long long)(done + i), (unsigned long long)kBytes);
      }
      const uint64_t m = j - i;
      const uint64_t end = cur.rp[j - 1] + GPD_PCAP_RECORD_BYTES + cur.rcap[j - 1];
      const uint64_t span = end - base;
      // (plain pointers: the worker threads would see their own thread_local vectors)
      const uint64_t *RP = cur.rp.data() + i;
      const uint32_t *RC = cur.rcap.data() + i;
      par_for(m, 1u << 16, [&](uint64_t a, uint64_t b) {
        for (uint64_t p = a; p < b; p++) s.h_off[p] = (uint32_t)(RP[p] + GPD_PCAP_RECORD_BYTES - base);
        std::memcpy(s.h_len + a, RC + a, (b - a) * 4);
      });
      const uint8_t *src = buf + base;
      if (!ctx->is_registered(src, span)) {  // (a shard registers only its own bytes)
        par_memcpy(s.h_data, src, span, nthreads);
        src = s.h_data;
      }
      hipError_t e = hipMemcpyAsync(s.d_data, src, span, hipMemcpyHostToDevice, s.stream);
      if (e == hipSuccess) e = hipMemcpyAsync(s.d_off, s.h_off, m * 4, hipMemcpyHostToDevice, s.stream);
      if (e == hipSuccess) e = hipMemcpyAsync(s.d_len, s.h_len, m * 4, hipMemcpyHostToDevice, s.stream);
      if (e != hipSuccess) {
        return set_err(GPD_ERR_HIP, "gpd_decode_pcap: H2D: %s", hipGetErrorString(e));
      }
      gpd_batch b{s.d_data, span, s.d_off, s.d_len, m};
      gpd_result r{s.d_status, s.d_layers, s.d_nh, s.d_th, s.d_csum, nullptr,
                   out->hdr_off ? s.d_hoff : nullptr, nullptr, out->detail ? s.d_det : nullptr};
      rc = launch(ctx, &b, &r, s.stream, false);
      if (rc) return rc;
      e = results_d2h(ctx, s, out, done + i, m, s.stream);
      if (e != hipSuccess) {
        return set_err(GPD_ERR_HIP, "gpd_decode_pcap: D2H: %s", hipGetErrorString(e));
      }
      g_pt_stage += now_ms() - t_stage;
      s.lo = done + i;
      s.hi = done + j;
      s.busy = true;
      i = j;
      k ^= 1;
    }
    done += n;
    *n_out = done;
    if (next_pos) *next_pos = cur.W.next_pos;
    if (stop) *stop = cur.W.stop;
    if (!more) {
      if (cur.rc) {  // the walk stopped at a record the reference rejects: decode what preceded it
        for (auto &s : ctx->slot)
          if (s.busy) {
            HIP_TRY(hipStreamSynchronize(s.stream));
            drain_slot(s, out);
          }
        return set_err(cur.rc, "%s", cur.err.c_str());
      }
      break;
    }
    const double tj = now_ms();
    ahead.t.join();
    g_pt_walkwait += now_ms() - tj;
    q ^= 1;
  }
  for (auto &s : ctx->slot) {
    if (s.busy) {
      const double t0 = now_ms();
      HIP_TRY(hipStreamSynchronize(s.stream));
      const double t1 = now_ms();
      drain_slot(s, out);
      g_pt_sync += t1 - t0;
      g_pt_drain += now_ms() - t1;
    }
  }
  g_pt_walk += walk_ms;
  return GPD_OK;
}

// The pcap path with the record walk on the device (gpd_pcapwalk.hip): the capture travels
// in fixed chunks of 64 MiB (plus the longest record past them) on two slots, each chunk's
// records are found in HBM (the walk of chunk k waits for chunk k-1's, which hands it its
// first record header), decoded there, and their results copied back.  The host reads one
// 16-byte control block per chunk: how many records it held and whether the device walk
// stood (status 0).  *handled records were decoded; *resume is the record header where the
// host walk must take over (a chunk with status 1: a rejected record, a partial record at
// the end, a speculation the walk missed), UINT64_MAX when the call is complete.
static int decode_device_walk(gpd_ctx *ctx, const uint8_t *buf, uint64_t len, const gpd_pcap_info &I,
                                   uint64_t pos, uint64_t max_n, const gpd_result *out, int nthreads,
                                   uint64_t *handled, uint64_t *resume, uint64_t *next_pos, int *stop,
                                   bool *ineligible) {
  constexpr uint64_t kChunk = (uint64_t)gpd::kPwSeg * gpd::kPwMaxSeg;
  const uint64_t margin = (16ull + I.snaplen + 31ull) & ~15ull;  // the longest record past a chunk
  const uint64_t cap_pkts = kChunk / GPD_PCAP_RECORD_BYTES;       // records a chunk can hold
  *handled = 0;
  *resume = pos;
  // (records that long, or a capture whose first records cannot be indexed: the host walk,
  // for the rest of the call — *ineligible)
  *ineligible = true;
  if (I.snaplen > (16u << 20)) return GPD_OK;
  // the mean record size (the decode's staging choices): the first records, walked here
  uint64_t mean = 96;
  {
    uint64_t sp[64];
    uint32_t sc[64];
    gpd::PcapOut o;
    o.pos64 = sp;
    o.cap = sc;
    gpd::PcapResult R;
    if (gpd::pcap_index_flat(buf, len, I, pos, 64, 1, o, R) != GPD_OK || R.n == 0) return GPD_OK;
    mean = std::max<uint64_t>(16, (R.next_pos - pos) / R.n);
  }
  *ineligible = false;
  int rc = alloc_slots(ctx, std::max<uint64_t>(ctx->slot_bytes, kChunk + margin + 64),
                       std::max<uint64_t>(ctx->slot_pkts, cap_pkts), false, out->detail != nullptr);
  if (rc) return rc;
  SlotGuard guard{ctx};
  // Chunk k's work on slot k & 1: its bytes H2D, then (after chunk k-1's walk) its walk, its
  // control block back to the host, its fill and its decode.  The next chunk is queued before
  // the host waits for this one's count, so the copy engine never waits for a walk.
  auto issue = [&](int k, uint64_t B, uint64_t entry0) -> int {
    auto &s = ctx->slot[k & 1];
    if (s.busy) {
      HIP_TRY(hipStreamSynchronize(s.stream));
      drain_slot(s, out);
      s.busy = false;
    }
    const uint64_t own = std::min<uint64_t>(kChunk, len - B);
    const uint64_t T = std::min<uint64_t>(own + margin, len - B);
    const bool last = B + own >= len;
    const uint8_t *src = buf + B;
    if (!ctx->is_registered(src, T)) {
      HIP_TRY(hipStreamSynchronize(s.stream));  // (its staging buffer may still be read)
      par_memcpy(s.h_data, src, T, nthreads);
      src = s.h_data;
    }
    gpd::PwCtl *dc = ctx->d_pw_ctl + (k & 1), *hc = ctx->h_pw_ctl + (k & 1);
    HIP_TRY(hipMemcpyAsync(s.d_data, src, T, hipMemcpyHostToDevice, s.stream));
    if (k == 0) {
      hc->entry = (uint32_t)entry0;
      HIP_TRY(hipMemcpyAsync(&dc->entry, &hc->entry, 4, hipMemcpyHostToDevice, s.stream));
    } else {
      HIP_TRY(hipStreamWaitEvent(s.stream, ctx->ev_pw[(k - 1) & 1], 0));
    }
    gpd::PwArgs A{};
    A.d = s.d_data;
    A.T = (uint32_t)T;
    A.own_end = (uint32_t)own;
    A.nseg = (uint32_t)((own + gpd::kPwSeg - 1) / gpd::kPwSeg);
    A.snaplen = I.snaplen;
    A.be = I.big_endian != 0;
    A.nano = I.nano != 0;
    A.last = last;
    A.ctl = dc;
    A.ctl_next = last ? nullptr : ctx->d_pw_ctl + ((k + 1) & 1);
    A.st = s.d_pw;
    A.ex = s.d_pw + gpd::kPwMaxSeg;
    A.ct = s.d_pw + 2 * gpd::kPwMaxSeg;
    A.bad = s.d_pw + 3 * gpd::kPwMaxSeg;
    A.base = s.d_pw + 4 * gpd::kPwMaxSeg;
    A.off = s.d_off;
    A.len = s.d_len;
    hipError_t e = gpd::launch_pcap_walk(A, s.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(hc, dc, sizeof(gpd::PwCtl), hipMemcpyDeviceToHost, s.stream);
    if (e == hipSuccess) e = hipEventRecord(ctx->ev_pw[k & 1], s.stream);
    if (e == hipSuccess) e = gpd::launch_pcap_fill(A, s.stream);
    if (e != hipSuccess) return set_err(GPD_ERR_HIP, "gpd_decode_pcap: device walk: %s", hipGetErrorString(e));
    gpd_batch b{s.d_data, T, s.d_off, s.d_len, cap_pkts};
    gpd_result r{s.d_status, s.d_layers, s.d_nh, s.d_th, s.d_csum, nullptr, out->hdr_off ? s.d_hoff : nullptr,
                 nullptr, out->detail ? s.d_det : nullptr};
    return launch(ctx, &b, &r, s.stream, false, &dc->n, std::max<uint64_t>(1, own / mean));
  };
  uint64_t B = pos & ~15ull;  // chunk base (16-byte aligned: the decoder's batch buffer)
  uint64_t entry = pos - B;   // its first record header
  uint64_t done = 0;
  *resume = UINT64_MAX;
  rc = issue(0, B, entry);
  if (rc) return rc;
  for (int k = 0;; k++) {
    auto &s = ctx->slot[k & 1];
    const uint64_t own = std::min<uint64_t>(kChunk, len - B);
    const bool last = B + own >= len;
    // queue the next chunk now unless this one should end the call (its records, estimated
    // from the mean record size, cover what is left)
    const bool ahead = !last && done + own / mean < max_n;
    if (ahead && (rc = issue(k + 1, B + own, 0))) return rc;
    HIP_TRY(hipEventSynchronize(ctx->ev_pw[k & 1]));  // chunk k walked: its count
    const gpd::PwCtl c = ctx->h_pw_ctl[k & 1];
    g_pw_counts[0]++;
    g_pw_counts[6] += c.pad[0];
    if (c.miss_at != 0xFFFFFFFFu) {
      g_pw_miss[0] = B + c.miss_st;
      g_pw_miss[1] = B + (uint64_t)c.miss_at * gpd::kPwSeg;
    }
    if (c.status != 0) {
      g_pw_counts[1]++;
      for (int b = 0; b < 4; b++) g_pw_counts[2 + b] += (c.status >> (b + 1)) & 1u;  // the host walks from this chunk's entry (its decode saw 0 records)
      *resume = B + entry;
      break;
    }
    const uint64_t take = std::min<uint64_t>(c.n, max_n - done);
    hipError_t e = results_d2h(ctx, s, out, done, take, s.stream);
    if (e != hipSuccess) return set_err(GPD_ERR_HIP, "gpd_decode_pcap: D2H: %s", hipGetErrorString(e));
    s.lo = done;
    s.hi = done + take;
    s.busy = take > 0;
    done += take;
    if (take < c.n) {  // the bound falls inside this chunk: the header of the record after it
      HIP_TRY(hipMemcpyAsync(s.h_off, s.d_off + take, 4, hipMemcpyDeviceToHost, s.stream));
      HIP_TRY(hipStreamSynchronize(s.stream));
      if (next_pos) *next_pos = B + s.h_off[0] - GPD_PCAP_RECORD_BYTES;
      if (stop) *stop = GPD_PCAP_STOP_LIMIT;
      break;
    }
    if (done == max_n) {
      if (next_pos) *next_pos = B + c.next;
      if (stop) *stop = GPD_PCAP_STOP_LIMIT;
      break;
    }
    if (last) {  // status 0 on the last chunk: the walk ended exactly at the capture's end
      if (next_pos) *next_pos = len;
      if (stop) *stop = GPD_PCAP_STOP_EOF;
      break;
    }
    entry = c.next - own;
    B += own;
    if (!ahead && (rc = issue(k + 1, B, 0))) return rc;
  }
  for (auto &s : ctx->slot) {  // (a chunk queued ahead and not needed is waited for and dropped)
    HIP_TRY(hipStreamSynchronize(s.stream));
    if (s.busy) {
      drain_slot(s, out);
      s.busy = false;
    }
  }
  *handled = done;
  return GPD_OK;
}

// Records whose header starts in [pos, pos + span), as the ReadPacketData loop finds them, up to
// the first one it would reject (the host walk then stops there with the reference's error).
static uint64_t count_records(const uint8_t *buf, uint64_t len, const gpd_pcap_info &I, uint64_t pos,
                              uint64_t span, uint64_t max_n) {
  auto rd = [&](uint64_t p) {
    uint32_t v;
    std::memcpy(&v, buf + p, 4);
    return I.big_endian ? __builtin_bswap32(v) : v;
  };
  uint64_t n = 0, p = pos;
  while (n < max_n && p < pos + span && p + GPD_PCAP_RECORD_BYTES <= len) {
    const uint32_t cap = rd(p + 8), wire = rd(p + 12);
    if (cap > I.snaplen || cap > wire || p + GPD_PCAP_RECORD_BYTES + cap > len) break;
    p += GPD_PCAP_RECORD_BYTES + cap;
    n++;
  }
  return n;
}

int gpd_decode_pcap_at(gpd_ctx *ctx, const uint8_t *buf, uint64_t len, const gpd_pcap_info *info,
                       uint64_t pos, uint64_t max_n, const gpd_result *out, uint64_t *n_out,
                       uint64_t *next_pos, int *stop, int nthreads) {
  if (!ctx || !buf || !info || !out || !out->status || !out->layers || !n_out)
    return set_err(GPD_ERR_INVALID, "gpd_decode_pcap: null argument");
  if (out->ext) return set_err(GPD_ERR_INVALID, "gpd_decode_pcap: ext records not supported");
  if (out->records) return set_err(GPD_ERR_INVALID, "gpd_decode_pcap: results as SoA arrays only");
  if (pos > len) return set_err(GPD_ERR_INVALID, "gpd_decode_pcap_at: pos beyond the buffer");
  if (nthreads <= 0) nthreads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  // this call's diagnostics (gpd_decode_pcap_last_*), reset before any early return
  const double t_call = now_ms();
  g_pt_walk = g_pt_walkwait = g_pt_stage = g_pt_sync = g_pt_drain = 0;
  for (auto &c : g_pw_counts) c = 0;
  g_pw_miss[0] = g_pw_miss[1] = ~0ull;
  struct Total {
    double t;
    ~Total() { g_pt_total = now_ms() - t; }
  } total{t_call};
  *n_out = 0;
  if (next_pos) *next_pos = pos;
  if (stop) *stop = GPD_PCAP_STOP_LIMIT;
  if (max_n == 0) return GPD_OK;
  gpd::DeviceScope dscope_;
  HIP_TRY(dscope_.set(ctx->device));
  bool dw = ctx->tune.device_walk != 0;
  uint64_t done = 0, at = pos;
  auto shifted = [&](uint64_t d) {
    gpd_result r = *out;
    auto sh = [&](auto *p) { return p ? p + d : p; };
    r.status = sh(out->status);
    r.layers = sh(out->layers);
    r.net_hash = sh(out->net_hash);
    r.tp_hash = sh(out->tp_hash);
    r.csum = sh(out->csum);
    r.hdr_off = sh(out->hdr_off);
    r.detail = sh(out->detail);
    return r;
  };
  for (;;) {
    if (dw) {
      uint64_t resume, handled = 0;
      bool ineligible = false;
      const gpd_result r = shifted(done);
      const int rc = decode_device_walk(ctx, buf, len, *info, at, max_n - done, &r, nthreads, &handled,
                                        &resume, next_pos, stop, &ineligible);
      done += handled;
      *n_out = done;
      if (rc) return rc;
      if (resume == UINT64_MAX) return GPD_OK;
      at = resume;
      if (ineligible) dw = false;  // one unbounded (pipelined) host walk does the rest
    }
    // The host walk from `at`: all of the call without the device walk; else only the chunk
    // the device walk could not vouch for (a record the reference rejects, a capture ending
    // inside a record, a speculation its stitch refuted), and then the device walk again
    // (one refuted speculation used to send the rest of the call to the host walk: r04, a
    // 2^24-record replay call 28 -> 200 ms)
    uint64_t lim = max_n - done;
    if (dw) {
      constexpr uint64_t kSpan = (uint64_t)gpd::kPwSeg * gpd::kPwMaxSeg;  // the device walk's chunk
      lim = std::min(lim, count_records(buf, len, *info, at, kSpan, lim) + 1u);
    }
    const gpd_result r = shifted(done);
    uint64_t k = 0, nxt = at;
    int st = GPD_PCAP_STOP_LIMIT;
    const int rc = decode_pcap_host_walk(ctx, buf, len, info, at, lim, &r, &k, &nxt, &st, nthreads);
    done += k;
    *n_out = done;
    if (next_pos) *next_pos = nxt;
    if (stop) *stop = st;
    if (rc || !dw || st != GPD_PCAP_STOP_LIMIT || done == max_n) return rc;
    at = nxt;
  }
}

void gpd_decode_pcap_last_walk_miss(uint64_t *pos2) {
  if (!pos2) return;
  pos2[0] = g_pw_miss[0];
  pos2[1] = g_pw_miss[1];
}

void gpd_decode_pcap_last_walk_counts(uint32_t *c7) {
  if (!c7) return;
  for (int k = 0; k < 7; k++) c7[k] = g_pw_counts[k];
}

void gpd_decode_pcap_last_times(double *ms6) {
  if (!ms6) return;
  ms6[0] = g_pt_total;     // the whole call
  ms6[1] = g_pt_walk;      // record walks (the first on the caller, the rest ahead on a helper)
  ms6[2] = g_pt_walkwait;  // waiting for a walk running ahead
  ms6[3] = g_pt_stage;     // descriptor rebase, staging copies, issuing transfers and launches
  ms6[4] = g_pt_sync;      // waiting for a slot's transfers and decode
  ms6[5] = g_pt_drain;     // copying a slot's results out (none with registered result arrays)
}

}  // extern "C"

// ---- TPACKET_V3 ring: the blocks H2D in groups, walked and decoded on the device ----
namespace {
constexpr uint64_t kTwPkts = 1u << 19;       // packets per group
constexpr uint64_t kTwMaxBlocks = 16384;     // blocks per group
constexpr uint64_t kTwTab = kTwMaxBlocks * sizeof(gpd::TwBlock), kTwSt = kTwMaxBlocks * 4;
// A group's per-packet arrays packed into one region, so one D2H brings them back: decode
// results, caplen (the walk's, the decode's input), then the capture info, each array
// 256-byte aligned.  The region is laid out for the group's packet count m.
// The detail records come last: they travel (in a copy of their own) only when asked for.
enum TwArr { kLayers, kNh, kTh, kStatus, kCsum, kHoff, kCap, kCiOff, kCiTs, kCiWire, kCiIfx, kCiVlan, kCiTci, kDet,
             kTwN };
constexpr uint64_t kTwW[kTwN] = {8, 8, 8, 4, 4, 4, 4, 8, 8, 4, 4, 4, 4, sizeof(gpd_detail)};
struct TwLay {
  uint64_t off[kTwN + 1];  // off[kCiOff]: the end of the results; off[kDet]: of the capture info
  explicit TwLay(uint64_t m) {
    uint64_t o = 0;
    for (int a = 0; a < kTwN; a++) {
      off[a] = o;
      o += (kTwW[a] * m + 255) & ~255ull;
    }
    off[kTwN] = o;
  }
};
const uint64_t kTwRegion = TwLay(kTwPkts).off[kTwN];
// a slot's d_tw: the group's block table, its status words, its region.  Its h_tw: two of
// each (a slot holds groups k and k + 2 at once: k + 2 is queued before the host copies k out).
constexpr uint64_t kTwDevSt = kTwTab;
inline uint64_t tw_dreg() { return kTwTab + kTwSt; }
inline uint64_t tw_htab(uint32_t set) { return set * kTwTab; }
inline uint64_t tw_hst(uint32_t set) { return 2 * kTwTab + set * kTwSt; }
inline uint64_t tw_hreg(uint32_t set) { return 2 * kTwTab + 2 * kTwSt + set * kTwRegion; }
}  // namespace

int gpd::decode_tpv3_device(gpd_ctx *ctx, const gpd_tpv3_ring &R, const std::vector<TwPlan> &plan,
                            uint64_t n, bool add_vlan, const gpd_tpv3_pkts *pk, const gpd_result *out,
                            int nthreads, bool *fallback) {
  *fallback = true;
  const uint64_t B = R.block_size;
  if (ctx->tune.device_walk == 0 || out->ext || out->records || (B & 15u) || B > kTwGroup || plan.empty())
    return GPD_OK;
  for (const auto &p : plan)
    if (p.emit > kTwPkts || (p.emit && (p.entry + 48 > B || (p.entry & 15u)))) return GPD_OK;
  if (nthreads <= 0) nthreads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  gpd::DeviceScope dscope_;
  HIP_TRY(dscope_.set(ctx->device));
  int rc = alloc_slots(ctx, std::max<uint64_t>(ctx->slot_bytes, kTwGroup),
                       std::max<uint64_t>(ctx->slot_pkts, kTwPkts), false, false);
  if (rc) return rc;
  for (auto &s : ctx->slot) {
    if (!s.d_tw) HIP_TRY(hipMalloc(&s.d_tw, tw_dreg() + kTwRegion));
    if (!s.h_tw) HIP_TRY(hipHostMalloc(&s.h_tw, tw_hreg(2), hipHostMallocDefault));
    if (!s.stream_out) HIP_TRY(hipStreamCreateWithFlags(&s.stream_out, hipStreamNonBlocking));
  }
  if (!ctx->tw_in) HIP_TRY(hipStreamCreateWithFlags(&ctx->tw_in, hipStreamNonBlocking));
  for (auto *ev : {ctx->ev_tw, ctx->ev_twdec})
    for (int q = 0; q < 4; q++)
      if (!ev[q]) HIP_TRY(hipEventCreateWithFlags(&ev[q], hipEventDisableTiming));
  for (auto &e : ctx->ev_twin)
    if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  SlotGuard guard{ctx};
  const bool ci = pk != nullptr;
  struct Group {
    uint64_t lo = 0, m = 0;
    uint32_t nb = 0, set = 0;
    bool direct = false;
  };
  std::vector<Group> grp;
  // the caller's array for each region array (NULL: not asked for)
  void *dst[kTwN] = {out->layers, out->net_hash, out->tp_hash, out->status, out->csum, out->hdr_off,
                     ci ? pk->caplen : nullptr, ci ? pk->offset : nullptr, ci ? pk->ts_ns : nullptr,
                     ci ? pk->wire_len : nullptr, ci ? pk->ifindex : nullptr, ci ? pk->vlan : nullptr,
                     ci ? pk->vlan_tci : nullptr, out->detail};
  // group k done: every block walked as the host would, then its results copied out
  auto complete = [&](size_t k) -> int {
    HIP_TRY(hipEventSynchronize(ctx->ev_tw[k & 3]));
    const Group &G = grp[k];
    const auto &s = ctx->slot[k & 1];
    const uint32_t *st = reinterpret_cast<const uint32_t *>(s.h_tw + tw_hst(G.set));
    uint32_t any = 0;
    for (uint32_t b = 0; b < G.nb; b++) any |= st[b];
    if ((any & 1u) || (add_vlan && (any & 2u))) return 1;
    if (!G.direct && G.m) {
      const TwLay L(G.m);
      const uint8_t *reg = s.h_tw + tw_hreg(G.set);
      par_for(G.m, 1u << 15, [&](uint64_t a, uint64_t b) {
        for (int q = 0; q < kTwN; q++)
          if (dst[q])
            std::memcpy(static_cast<uint8_t *>(dst[q]) + (G.lo + a) * kTwW[q], reg + L.off[q] + a * kTwW[q],
                        (b - a) * kTwW[q]);
      });
    }
    return GPD_OK;
  };
  // Group k goes to slot k & 1 and host buffers (k >> 1) & 1.  Its bytes go on the copy
  // stream (all groups in order), its walk and decode on the slot's stream, its D2H on the
  // slot's second stream, so no transfer queues behind a kernel.  Group k is queued before the
  // host waits for group k - 2 and copies it out, so no stream waits for the host.
  size_t a = 0;
  while (a < plan.size()) {
    // the group: consecutive ring blocks (no wrap) within the byte, block and packet bounds
    size_t b = a + 1;
    uint64_t m = plan[a].emit;
    while (b < plan.size() && plan[b].ring_block == plan[b - 1].ring_block + 1 && (b - a + 1) * B <= kTwGroup &&
           b - a < kTwMaxBlocks && m + plan[b].emit <= kTwPkts)
      m += plan[b++].emit;
    const size_t k = grp.size();
    auto &s = ctx->slot[k & 1];
    Group G;
    G.lo = plan[a].out;
    G.m = m;
    G.nb = (uint32_t)(b - a);
    G.set = (uint32_t)((k >> 1) & 1);
    const uint64_t bytes = (uint64_t)G.nb * B;
    const TwLay L(std::max<uint64_t>(m, 1));
    auto *tb = reinterpret_cast<gpd::TwBlock *>(s.h_tw + tw_htab(G.set));  // (group k - 4's: done)
    for (uint32_t q = 0; q < G.nb; q++)
      tb[q] = gpd::TwBlock{(uint32_t)plan[a + q].entry, plan[a + q].emit, (uint32_t)(plan[a + q].out - G.lo), 0};
    const uint8_t *src = R.base + (uint64_t)plan[a].ring_block * B;
    if (!ctx->is_registered(src, bytes)) {
      if (k >= 2) HIP_TRY(hipEventSynchronize(ctx->ev_twin[k & 1]));  // group k - 2's bytes are in HBM
      par_memcpy(s.h_data, src, bytes, nthreads);
      src = s.h_data;
    }
    s.busy = true;  // (work in flight from here: an error exit waits for it)
    // the bytes on the copy stream, right behind the previous group's (the link stays busy
    // while groups are walked), once group k - 2's decode has read the slot's buffer
    if (k >= 2) HIP_TRY(hipStreamWaitEvent(ctx->tw_in, ctx->ev_twdec[(k - 2) & 3], 0));
    HIP_TRY(hipMemcpyAsync(s.d_data, src, bytes, hipMemcpyHostToDevice, ctx->tw_in));
    HIP_TRY(hipEventRecord(ctx->ev_twin[k & 1], ctx->tw_in));
    HIP_TRY(hipStreamWaitEvent(s.stream, ctx->ev_twin[k & 1], 0));
    HIP_TRY(hipMemcpyAsync(s.d_tw, tb, G.nb * sizeof(gpd::TwBlock), hipMemcpyHostToDevice, s.stream));
    // the region and status words are group k - 2's until its D2H is done
    if (k >= 2) HIP_TRY(hipStreamWaitEvent(s.stream, ctx->ev_tw[(k - 2) & 3], 0));
    uint8_t *dr = s.d_tw + tw_dreg();
    auto dev = [&](int q) { return dr + L.off[q]; };
    gpd::TwArgs A{};
    A.d = s.d_data;
    A.block_size = (uint32_t)B;
    A.nblk = G.nb;
    A.ring_off0 = (uint64_t)plan[a].ring_block * B;
    A.blk = reinterpret_cast<const gpd::TwBlock *>(s.d_tw);
    A.st = reinterpret_cast<uint32_t *>(s.d_tw + kTwDevSt);
    A.off = s.d_off;
    A.len = reinterpret_cast<uint32_t *>(dev(kCap));
    if (ci) {
      A.ci_off = reinterpret_cast<uint64_t *>(dev(kCiOff));
      A.ci_ts = reinterpret_cast<uint64_t *>(dev(kCiTs));
      A.ci_wire = reinterpret_cast<uint32_t *>(dev(kCiWire));
      A.ci_ifx = reinterpret_cast<int32_t *>(dev(kCiIfx));
      A.ci_vlan = reinterpret_cast<int32_t *>(dev(kCiVlan));
      A.ci_tci = reinterpret_cast<uint32_t *>(dev(kCiTci));
    }
    hipError_t e = gpd::launch_tpv3_walk(A, s.stream);
    if (e != hipSuccess) return set_err(GPD_ERR_HIP, "gpd_decode_tpv3: device walk: %s", hipGetErrorString(e));
    if (m) {
      gpd_batch bt{s.d_data, bytes, s.d_off, A.len, m};
      gpd_result r{reinterpret_cast<uint32_t *>(dev(kStatus)), reinterpret_cast<uint64_t *>(dev(kLayers)),
                   reinterpret_cast<uint64_t *>(dev(kNh)), reinterpret_cast<uint64_t *>(dev(kTh)),
                   reinterpret_cast<uint32_t *>(dev(kCsum)), nullptr,
                   out->hdr_off ? reinterpret_cast<uint32_t *>(dev(kHoff)) : nullptr, nullptr,
                   out->detail ? reinterpret_cast<gpd_detail *>(dev(kDet)) : nullptr};
      if ((rc = launch(ctx, &bt, &r, s.stream, false))) return rc;
    }
    HIP_TRY(hipEventRecord(ctx->ev_twdec[k & 3], s.stream));
    HIP_TRY(hipStreamWaitEvent(s.stream_out, ctx->ev_twdec[k & 3], 0));
    HIP_TRY(hipMemcpyAsync(s.h_tw + tw_hst(G.set), A.st, G.nb * 4, hipMemcpyDeviceToHost, s.stream_out));
    if (m) {
      G.direct = true;
      for (int q = 0; q < kTwN; q++)
        G.direct = G.direct && (!dst[q] || ctx->is_registered(static_cast<uint8_t *>(dst[q]) + G.lo * kTwW[q],
                                                               m * kTwW[q]));
      if (G.direct) {
        for (int q = 0; q < kTwN; q++)
          if (dst[q])
            HIP_TRY(hipMemcpyAsync(static_cast<uint8_t *>(dst[q]) + G.lo * kTwW[q], dev(q), m * kTwW[q],
                                   hipMemcpyDeviceToHost, s.stream_out));
      } else {
        HIP_TRY(hipMemcpyAsync(s.h_tw + tw_hreg(G.set), dr, L.off[ci ? kDet : kCiOff], hipMemcpyDeviceToHost,
                               s.stream_out));
        if (out->detail)
          HIP_TRY(hipMemcpyAsync(s.h_tw + tw_hreg(G.set) + L.off[kDet], dr + L.off[kDet], m * kTwW[kDet],
                                 hipMemcpyDeviceToHost, s.stream_out));
      }
    }
    HIP_TRY(hipEventRecord(ctx->ev_tw[k & 3], s.stream_out));
    grp.push_back(G);
    if (k >= 2 && (rc = complete(k - 2))) return rc == 1 ? GPD_OK : rc;  // (the guard waits)
    a = b;
  }
  for (size_t k = grp.size() >= 2 ? grp.size() - 2 : 0; k < grp.size(); k++)
    if ((rc = complete(k))) return rc == 1 ? GPD_OK : rc;
  for (auto &s : ctx->slot) s.busy = false;
  *fallback = false;
  return GPD_OK;
}
