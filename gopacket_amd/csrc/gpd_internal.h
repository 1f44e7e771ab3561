// gpd_internal.h — shared between the HIP kernels and the host runtime (not public ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpd.h"

namespace gpd {

// Every C-ABI entry point that selects its context's device restores the caller's current
// device on return: a Go thread or a torch process calling in with another device
// current keeps it.  `set` switches only when needed; the destructor switches back.
struct DeviceScope {
  int prev = -1;
  DeviceScope() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  hipError_t set(int device) { return device == prev ? hipSuccess : hipSetDevice(device); }
  ~DeviceScope() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope &) = delete;
  DeviceScope &operator=(const DeviceScope &) = delete;
};

// ---- device dispatch tables ---------------------------------------------------------
// Two encodings of the same four reference tables (ethertype[65536], ipproto[256],
// tcp_port[65536], udp_port[65536]; layers/enums.go:304-345, layers/ports.go:62-122):
//
// (a) HASH (default, copied into LDS by every workgroup): the tables are sparse (the
//     reference defaults hold 18 + 11 + 16 nonzero 16-bit entries), so each 64K table
//     is a two-way bucketed hash of its nonzero entries: 2^bits buckets of two u32 slots
//     {key << 16 | LayerType << 8 | LUT entry of that LayerType}, with a per-table
//     multiplier chosen by the host so that no bucket overflows.  One ds_read_b64 yields
//     both candidates, and the matching slot gives the next LayerType and its decoder
//     (needs every mapped LayerType < 256).
//     Layout in u32 words:
//       [0,32)                     type LUT: byte t = decoder id | code << 4 for t < 128
//                                  (decoder id 15 = not registered)
//       [32,288)                   ipproto -> LayerType | LUT entry << 16
//       [eth_base, +2^(eth_bits+1))  ethertype hash (8-byte aligned)
//       [tcp_base, +2^(tcp_bits+1))  tcp port hash
//       [udp_base, +2^(udp_bits+1))  udp port hash
// (b) PAGES (fallback when a table is too dense for the LDS budget): the image holds only
//     the LUT and ipproto; the 64K tables are two-level pages in global memory, u16 words:
//     [256,512) eth dir, [512,768) tcp dir, [768,1024) udp dir, then 256-entry pages
//     (page 0 = zeros).
constexpr uint32_t kHashLutWords = 32;
constexpr uint32_t kHashProtoWords = 256;
constexpr uint32_t kHashMaxWords = 4096;  // 16 KB cap for the LDS image
// Fixed layout (when the three tables fit it with one shared multiplier): compiled into the
// fast kernel, so its lookups need no per-table base/size registers.
constexpr uint32_t kFixBits = 6;
constexpr uint32_t kFixEthBase = kHashLutWords + kHashProtoWords;  // 288
constexpr uint32_t kFixTcpBase = kFixEthBase + (2u << kFixBits);     // 416
constexpr uint32_t kFixUdpBase = kFixTcpBase + (2u << kFixBits);     // 544
constexpr uint32_t kFixWords = kFixUdpBase + (2u << kFixBits);       // 672
constexpr uint32_t kTabIpProto = 0;
constexpr uint32_t kTabEthDir = 256;
constexpr uint32_t kTabTcpDir = 512;
constexpr uint32_t kTabUdpDir = 768;
constexpr uint32_t kTabPages = 1024;

struct KParams {
  const uint8_t *data;
  uint64_t data_len;
  const uint32_t *offset;
  const uint32_t *caplen;
  uint64_t n;
  const uint32_t *n_dev;       // when set, the packet count is min(n, *n_dev), read on the device
  uint32_t *status;
  uint64_t *layers;
  uint64_t *net_hash;
  uint64_t *tp_hash;
  uint32_t *csum;
  gpd_ext_rec *ext;
  uint32_t *hdr_off;
  gpd_record *rec;             // AoS results (status .. csum NULL)
  gpd_detail *detail;          // error arguments / deep stacks (generic decoder only; may be NULL)
  const uint32_t *image;       // LUT + ipproto (+ hash tables in HASH mode); staged into LDS
  const uint16_t *pages;       // PAGES mode: two-level page tables in global memory
  uint32_t image_words;
  uint32_t use_pages;          // 1 => 64K lookups go to `pages`
  uint32_t eth_base, tcp_base, udp_base;  // word offsets of the hashes inside `image`
  uint32_t eth_bits, tcp_bits, udp_bits;  // log2 of each hash's bucket count
  uint32_t eth_mult, tcp_mult, udp_mult;  // each hash's multiplier (odd, < 2^16)
  uint32_t first;
  uint32_t decoders;
  uint32_t options;
  uint32_t stage;              // LDS window bytes per buffer (chosen by the runtime)
  uint32_t nstores;            // store instructions per tile (non-NULL result arrays)
  uint32_t fixed;              // tables in the kFix* layout (eth_mult shared by all three)
  uint32_t waves;              // fast kernel waves per SIMD (0: the default for the window)
  uint32_t rounds;             // fast kernel grid rounds of resident workgroups (0: the default)
  uint32_t split;              // 4 KiB windows by the loader / decoder split kernel (sp_kernel)
  uint64_t *fb_list;           // fast kernel: packets left to the generic decoder (offset << 32 |
                               // index: the decode's loads skip the descriptor), in one private
                               // region per wave (64 x its tiles), which that wave decodes after
                               // its tiles (see rs_kernel)
  uint32_t *fb_wcount;         // per fast-kernel wave: entries in its region
  uint32_t fb_waves;           // waves of the fast launch (set by launch_decode)
};
// Upper bound of the fast kernel's waves per launch, per compute unit (workgroups per CU x
// grid rounds x 4 waves): sizes fb_wcount.
constexpr uint32_t kMaxFastWavesPerCU = 4 * 8 * 4;

// True when launch_decode takes the fast kernel (needs fb_list with room for P.n entries and
// fb_wcount).
bool fast_eligible(const KParams &P);

// The pcap record walk on the GPU (gpd_pcapwalk.hip): one chunk of capture bytes in HBM.
constexpr uint32_t kPwSeg = 2048;        // bytes per walking lane
constexpr uint32_t kPwMaxSeg = 1u << 15; // segments per chunk (64 MiB)
struct PwCtl {       // a chunk's control block (device; copied back to the host)
  uint32_t entry;    // in: its first record header (relative to the chunk)
  uint32_t n;        // out: records whose headers start in [entry, own_end)
  uint32_t next;     // out: the first record header at or past own_end
  uint32_t status;   // out: 0, or 1 | reasons (2 speculation refuted, 4 rejected record, 8 header
                     // not covered, 16 walk ends short) = the host walks from `entry` (gpd_pcapwalk.hip)
  uint32_t miss_st;  // out (diagnostic): the first refuted speculation's start ...
  uint32_t miss_at;  // ... and its segment (kNone: none)
  uint32_t pad[2];   // [0]: segments the stitch re-walked from the true walk's position
};
struct PwArgs {
  const uint8_t *d;        // the chunk's bytes in HBM
  uint32_t T;              // bytes there
  uint32_t own_end;        // records whose headers start before this are the chunk's
  uint32_t nseg;           // ceil(own_end / kPwSeg)
  uint32_t snaplen;
  bool be, nano, last;     // header byte order, ns timestamps; the chunk ends the capture (T = its end)
  PwCtl *ctl, *ctl_next;   // this chunk's block; the next chunk's (its entry is written)
  uint32_t *st, *ex, *ct, *bad, *base;  // per segment
  uint32_t *off, *len;     // per record: data offset, capture length
};
hipError_t launch_pcap_walk(const PwArgs &A, hipStream_t stream);
hipError_t launch_pcap_fill(const PwArgs &A, hipStream_t stream);

// The TPACKET_V3 block walk on the GPU (gpd_tpv3walk.hip): one group of consecutive ring
// blocks in HBM, one workgroup per block.
constexpr uint32_t kTwWin = 32768;           // LDS window of a block's bytes
#ifndef GPD_TW_GROUP_MIB
#define GPD_TW_GROUP_MIB 64  // (A/B builds override it)
#endif
constexpr uint64_t kTwGroup = (uint64_t)GPD_TW_GROUP_MIB << 20;  // bytes of ring blocks per group
struct TwBlock {      // one walked block (host plan, afpacket.go:303-316 + header.go:144-149)
  uint32_t entry;     // its first emitted packet header (relative to the block; 16-aligned)
  uint32_t emit;      // packets the read loop returns from it
  uint32_t out;       // index of its first packet in the group's output
  uint32_t pad;
};
struct TwArgs {
  const uint8_t *d;        // the group's blocks, in ring order
  uint32_t block_size;
  uint32_t nblk;
  uint64_t ring_off0;      // the group's first block's offset in the ring
  const TwBlock *blk;
  uint32_t *st;            // per block: bit 0 a header or frame outside the block, or a step
                           // the device walk does not take (0, or not a multiple of 16);
                           // bit 1 a frame with a nonzero vlan_tci
  uint32_t *off, *len;     // per packet: frame offset in the group, tp_snaplen
  uint64_t *ci_off;        // optional capture info (NULL: not written): frame offset in the ring,
  uint32_t *ci_wire;       //   tp_len,
  uint64_t *ci_ts;         //   tp_sec * 1e9 + tp_nsec,
  int32_t *ci_ifx;         //   sockaddr_ll.sll_ifindex,
  int32_t *ci_vlan;        //   AncillaryVLAN or -1,
  uint32_t *ci_tci;        //   tp_vlan_tci
};
hipError_t launch_tpv3_walk(const TwArgs &A, hipStream_t stream);

// The IPv4 fragment hand-off (include/gpd_defrag.h): the decoded batch and tables in P (its
// status/layers or rec, and hdr_off, are the decode's results), scratch and the records.
}  // namespace gpd
#include "../../include/gpd_defrag.h"
namespace gpd {
struct FragArgs {
  KParams P;
  gpd_ip4_frag *out;
  uint32_t max_out;   // records written: min(candidates, max_out)
  uint32_t nblk;      // ceil(n / 2048)
  uint32_t *blk;      // nblk + 1: per-block candidate counts -> exclusive prefix; [nblk] = total
  uint64_t *mask;     // ceil(n / 64): bit l of word w = packet 64w + l is a candidate
  uint32_t *idx;      // n: the candidates' packet indices in order
};
hipError_t launch_ip4_frag(const FragArgs &A, hipStream_t stream, int num_cus);

// One launch covers at most this many packets, so packet and tile indices are 32-bit.
constexpr uint64_t kMaxLaunchPackets = 1ull << 30;

// Launch the decode kernel over P (asynchronous on `stream`).  `mid` (may be null) is
// recorded between the fast kernel and the list kernel of the fallback packets.
// *fb_waves (may be null) receives the fast kernel's wave count (0 for the generic kernel).
hipError_t launch_decode(const KParams &P, hipStream_t stream, int num_cus, hipEvent_t mid = nullptr,
                         uint32_t *fb_waves = nullptr);

// Host side: set the thread's gpd_last_error_string() text and return `code` (gpd_runtime.cpp).
int set_error(int code, const char *fmt, ...);

// Host side: the device and compute-unit count of a context (gpd_runtime.cpp).
int ctx_device(const gpd_ctx *ctx);
int ctx_num_cus(const gpd_ctx *ctx);
// Host side: device scratch buffer `slot` (0..15) of at least `bytes`, kept with the context
// and grown on demand; nullptr when out of memory.  Callers synchronise before reuse.
void *ctx_scratch(gpd_ctx *ctx, int slot, size_t bytes);

// Host side: the sequential pcap record walk over buf[pos:len), built in parallel
// (gpd_pcap.cpp; semantics in include/gpd_pcap.h).  Positions are record-header offsets.
}  // namespace gpd
#include "../../include/gpd_pcap.h"
#include <vector>
namespace gpd {
// Where a walk writes its records (any pointer may be NULL): record i's header position
// pos64[i], its data offset off32[i] = pos + 16 - base, cap / wire / ts as ReadPacketData
// returns them.
struct PcapOut {
  uint64_t base = 0;
  uint32_t *off32 = nullptr;
  uint64_t *pos64 = nullptr;
  uint32_t *cap = nullptr, *wire = nullptr;
  uint64_t *ts = nullptr;
};
struct PcapResult {
  uint64_t n = 0, next_pos = 0;  // records written; where the next record header starts
  int stop = 0;                  // GPD_PCAP_STOP_*
  uint32_t a0 = 0, a1 = 0;       // the stop's error arguments
  bool off32_overflow = false;   // an off32 did not fit 32 bits
};
// The sequential ReadPacketData loop from pos, at most max_n records, into `out`; returns
// GPD_OK or GPD_ERR_PCAP with the reference's error text (the records before the stop are
// written and counted).
int pcap_index_flat(const uint8_t *buf, uint64_t len, const gpd_pcap_info &I, uint64_t pos, uint64_t max_n,
                    int nthreads, const PcapOut &out, PcapResult &R);
int pcap_locate(const uint8_t *buf, uint64_t len, const gpd_pcap_info &I, uint64_t pos,
                const uint64_t *targets, uint64_t k, uint64_t *pos_out, uint64_t *n_total, int *stop,
                int nthreads);
}  // namespace gpd
#include "../../include/gpd_afpacket.h"
namespace gpd {
// One user-owned block of a gpd_decode_tpv3 call, as the host planned it (gpd_afpacket.cpp).
struct TwPlan {
  uint32_t ring_block;  // index in the ring
  uint32_t emit;        // packets the read loop returns from it
  uint64_t out;         // index of its first packet in the call's output
  uint64_t entry;       // its first emitted packet header (relative to the block)
};
// gpd_decode_tpv3 with the block walk on the device (gpd_runtime.cpp): the planned blocks
// travel to HBM in groups of consecutive ring blocks, are walked there (gpd_tpv3walk.hip)
// and decoded, and results and capture info come back.  *fallback: the device path does not
// apply (tuning, geometry, a block the walk rejects, a tagged frame with add_vlan) and the
// caller runs the host path for the whole call (nothing returned so far counts).
int decode_tpv3_device(gpd_ctx *ctx, const gpd_tpv3_ring &R, const std::vector<TwPlan> &plan, uint64_t n,
                       bool add_vlan, const gpd_tpv3_pkts *pk, const gpd_result *out, int nthreads,
                       bool *fallback);

// Multiplicative hash of a 16-bit key into 2^bits buckets (host and device must agree).
__host__ __device__ inline uint32_t key_hash(uint32_t key, uint32_t mult, uint32_t bits) {
  return ((key * mult) & 0xFFFFu) >> (16 - bits);
}

}  // namespace gpd
