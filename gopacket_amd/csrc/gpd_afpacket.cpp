// gpd_afpacket.cpp — TPACKET_V3 ring walk and decode (include/gpd_afpacket.h).
//
// Restates the reference's per-packet read loop over an AF_PACKET v3 ring (paths relative to
// google/gopacket) for every block user space owns at the time of the call:
//   block at offset k ........ afpacket/afpacket.go:445-453 (getTPacketHeader, v3 case:
//                              rawring + frameSize*offset*framesPerBlock = k * blockSize)
//   owned by user space ...... afpacket.go:459 (block_status & TP_STATUS_USER)
//   first packet, empty block  afpacket.go:303-316 + header.go:144-149 (initV3Wrapper; a
//                              first packet with tp_len 0 sends the loop to next())
//   packet fields ............ header.go:151-180 (getVLAN, getTime, getData, getLength,
//                              getIfaceIndex), afpacket.go:318-326 (CaptureInfo)
//   next packet .............. header.go:181-195 (tp_next_offset, else tpAlign(snaplen+mac))
//   hand the block back ...... afpacket.go:282-287, header.go:162-164 (block_status = 0)
//   VLAN tag insertion ....... header.go:74-82 (OptAddVLANHeader, tci != 0)
// The walk models a read loop that is already running (headerNextNeeded set, afpacket.go:303):
// the first-ever read of a handle differs only for a block whose first packet reports
// tp_len 0, which the kernel does not produce for a delivered frame.
// Deviation (safety): a header or frame reaching outside its block, which the reference would
// read as raw memory, stops the walk with GPD_ERR_INVALID instead.
#include <hip/hip_runtime.h>
#include <linux/if_packet.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "gpd_internal.h"
#include "../../include/gpd_afpacket.h"

namespace {

constexpr uint32_t kAlign = TPACKET_ALIGNMENT;  // afpacket/header.go:56-60 tpAlign
inline uint64_t tp_align(uint64_t x) { return (x + kAlign - 1) & ~(uint64_t)(kAlign - 1); }

struct BlockPlan {
  uint32_t ring_block;  // index in the ring
  uint32_t emit;        // packets the read loop returns from it
  uint64_t out;         // index of its first packet in the output
};

// Packets ZeroCopyReadPacketData returns from one user-owned block (see the file comment):
// the first packet, unless its tp_len is 0 (then next() decides), then next() while
// used < num_pkts.  An empty block whose stale first tp_len is nonzero still yields that one
// packet, as the reference's loop does.
inline uint32_t block_emits(const tpacket_hdr_v1 &bh, const tpacket3_hdr &p0) {
  if (p0.tp_len == 0) return bh.num_pkts >= 2 ? bh.num_pkts - 1 : 0;
  return bh.num_pkts >= 1 ? bh.num_pkts : 1;
}

int walk_block(const gpd_tpv3_ring &R, const BlockPlan &B, const gpd_tpv3_pkts &pk, uint32_t *off32) {
  const uint8_t *blk = R.base + (uint64_t)B.ring_block * R.block_size;
  const auto *desc = reinterpret_cast<const tpacket_block_desc *>(blk);
  const tpacket_hdr_v1 &bh = desc->hdr.bh1;
  uint64_t pos = bh.offset_to_first_pkt;  // initV3Wrapper, header.go:144-149
  uint32_t used = 0;
  auto advance = [&](const tpacket3_hdr &h) -> bool {  // v3wrapper.next, header.go:181-195
    used++;
    if (used >= bh.num_pkts) return false;
    pos += h.tp_next_offset != 0 ? (uint64_t)h.tp_next_offset : tp_align((uint64_t)h.tp_snaplen + h.tp_mac);
    return true;
  };
  auto header_at = [&](uint64_t p) -> const tpacket3_hdr * {
    if (p + sizeof(tpacket3_hdr) > R.block_size) return nullptr;
    return reinterpret_cast<const tpacket3_hdr *>(blk + p);
  };
  const tpacket3_hdr *h = header_at(pos);
  if (!h) return gpd::set_error(GPD_ERR_INVALID, "tpv3 block %u: first packet header outside the block", B.ring_block);
  if (h->tp_len == 0) {  // afpacket.go:313-316: retry -> next()
    if (!advance(*h)) return GPD_OK;
    h = header_at(pos);
    if (!h) return gpd::set_error(GPD_ERR_INVALID, "tpv3 block %u: packet header outside the block", B.ring_block);
  }
  for (uint64_t j = B.out;; j++) {
    const uint64_t data = pos + h->tp_mac;
    if (data + h->tp_snaplen > R.block_size)
      return gpd::set_error(GPD_ERR_INVALID, "tpv3 block %u: frame outside the block", B.ring_block);
    pk.offset[j] = (uint64_t)B.ring_block * R.block_size + data;
    if (off32) off32[j] = (uint32_t)pk.offset[j];  // rings below 4 GiB: a gpd_batch offset
    pk.caplen[j] = h->tp_snaplen;
    if (pk.wire_len) pk.wire_len[j] = h->tp_len;
    if (pk.ts_ns) pk.ts_ns[j] = (uint64_t)h->tp_sec * 1000000000ull + h->tp_nsec;
    if (pk.ifindex) {  // getIfaceIndex: sockaddr_ll after the aligned header (header.go:177-180)
      const uint64_t ll = pos + tp_align(sizeof(tpacket3_hdr));
      int32_t idx = 0;
      if (ll + sizeof(sockaddr_ll) <= R.block_size)
        memcpy(&idx, blk + ll + offsetof(sockaddr_ll, sll_ifindex), sizeof idx);
      pk.ifindex[j] = idx;
    }
    if (pk.vlan)  // getVLAN, header.go:151-157
      pk.vlan[j] = (h->tp_status & TP_STATUS_VLAN_VALID) ? (int32_t)(h->hv1.tp_vlan_tci & 0xfff) : -1;
    if (pk.vlan_tci) pk.vlan_tci[j] = h->hv1.tp_vlan_tci;
    if (!advance(*h)) break;
    h = header_at(pos);
    if (!h) return gpd::set_error(GPD_ERR_INVALID, "tpv3 block %u: packet header outside the block", B.ring_block);
  }
  return GPD_OK;
}

int plan_walk(const gpd_tpv3_ring *R, uint32_t first, uint32_t max_blocks, uint64_t max_n,
              std::vector<BlockPlan> &plan, uint64_t &n) {
  n = 0;
  if (!R || !R->base || R->block_size < sizeof(tpacket_block_desc) || R->num_blocks == 0)
    return gpd::set_error(GPD_ERR_INVALID, "tpv3: bad ring geometry");
  const uint32_t limit = std::min(max_blocks, R->num_blocks);
  for (uint32_t b = 0; b < limit; b++) {
    const uint32_t k = (uint32_t)(((uint64_t)first + b) % R->num_blocks);
    uint8_t *blk = R->base + (uint64_t)k * R->block_size;
    auto *desc = reinterpret_cast<tpacket_block_desc *>(blk);
    const uint32_t status = __atomic_load_n(&desc->hdr.bh1.block_status, __ATOMIC_ACQUIRE);
    if (!(status & TP_STATUS_USER)) break;  // the kernel still owns it: the loop would poll
    const tpacket_hdr_v1 &bh = desc->hdr.bh1;
    if ((uint64_t)bh.offset_to_first_pkt + sizeof(tpacket3_hdr) > R->block_size)
      return gpd::set_error(GPD_ERR_INVALID, "tpv3 block %u: first packet header outside the block", k);
    const auto *p0 = reinterpret_cast<const tpacket3_hdr *>(blk + bh.offset_to_first_pkt);
    const uint32_t e = block_emits(bh, *p0);
    if (n + e > max_n) {
      if (plan.empty())
        return gpd::set_error(GPD_ERR_INVALID, "tpv3: max_n %llu is smaller than block %u's %u packets",
                              (unsigned long long)max_n, k, e);
      break;
    }
    plan.push_back(BlockPlan{k, e, n});
    n += e;
  }
  return GPD_OK;
}

thread_local int g_last_path = 0;  // gpd_decode_tpv3_last_path

int run_walk(const gpd_tpv3_ring *R, const std::vector<BlockPlan> &plan, const gpd_tpv3_pkts &pk,
             int nthreads, uint32_t *off32 = nullptr) {
  // nthreads <= 0: the machine's cores, at most 16 (blocks are few and cheap to walk)
  int T = nthreads > 0 ? nthreads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  T = (int)std::min<size_t>((size_t)T, plan.size());
  if (plan.size() < 8) T = 1;  // a thread per block costs more than walking a few blocks
  if (T <= 1) {
    for (const auto &b : plan) {
      int rc = walk_block(*R, b, pk, off32);
      if (rc) return rc;
    }
    return GPD_OK;
  }
  std::vector<int> rc(T, GPD_OK);
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)
    th.emplace_back([&, t] {
      for (size_t b = t; b < plan.size() && rc[t] == GPD_OK; b += T) rc[t] = walk_block(*R, plan[b], pk, off32);
    });
  for (auto &x : th) x.join();
  for (int r : rc)
    if (r) return gpd::set_error(r, "tpv3: corrupt block (see the walk)");
  return GPD_OK;
}

}  // namespace

extern "C" {

int gpd_tpv3_walk(const gpd_tpv3_ring *ring, uint32_t first_block, uint32_t max_blocks,
                  uint64_t max_n, const gpd_tpv3_pkts *pk, uint64_t *n_out, uint32_t *blocks_out,
                  int nthreads) {
  if (!pk || !pk->offset || !pk->caplen || !n_out || !blocks_out)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_tpv3_walk: null argument");
  *n_out = 0;
  *blocks_out = 0;
  std::vector<BlockPlan> plan;
  uint64_t n = 0;
  int rc = plan_walk(ring, first_block, max_blocks, max_n, plan, n);
  if (rc) return rc;
  rc = run_walk(ring, plan, *pk, nthreads);
  if (rc) return rc;
  *n_out = n;
  *blocks_out = (uint32_t)plan.size();
  return GPD_OK;
}

int gpd_decode_tpv3_last_path(void) { return g_last_path; }

int gpd_tpv3_release(const gpd_tpv3_ring *ring, uint32_t first_block, uint32_t count) {
  if (!ring || !ring->base || ring->num_blocks == 0)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_tpv3_release: bad ring");
  for (uint32_t b = 0; b < count && b < ring->num_blocks; b++) {
    const uint32_t k = (uint32_t)(((uint64_t)first_block + b) % ring->num_blocks);
    auto *desc = reinterpret_cast<tpacket_block_desc *>(ring->base + (uint64_t)k * ring->block_size);
    __atomic_store_n(&desc->hdr.bh1.block_status, (uint32_t)TP_STATUS_KERNEL, __ATOMIC_RELEASE);
  }
  return GPD_OK;
}

int gpd_decode_tpv3(gpd_ctx *ctx, const gpd_tpv3_ring *ring, uint32_t first_block,
                    uint32_t max_blocks, int add_vlan_header, uint64_t max_n,
                    const gpd_result *out, const gpd_tpv3_pkts *pk_out, uint64_t *n_out,
                    uint32_t *blocks_out, int nthreads) {
  if (!ctx || !out || !out->status || !out->layers || !n_out || !blocks_out)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_decode_tpv3: null argument");
  if (out->ext || out->records)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_decode_tpv3: SoA results only (no ext records; detail is fine)");
  *n_out = 0;
  *blocks_out = 0;
  std::vector<BlockPlan> plan;
  uint64_t n = 0;
  int rc = plan_walk(ring, first_block, max_blocks, max_n, plan, n);
  if (rc || plan.empty()) return rc;
  {
    // The walk on the device (gpd_tpv3walk.hip): each block's first emitted packet from its
    // descriptor here, every other step there.  It declines (tuning, geometry, a walk leaving
    // its block, a tag to insert) before anything it returned counts; the host path follows.
    std::vector<gpd::TwPlan> tp(plan.size());
    for (size_t j = 0; j < plan.size(); j++) {
      const BlockPlan &bp = plan[j];
      uint64_t entry = 0;
      if (bp.emit) {
        const uint8_t *blk = ring->base + (uint64_t)bp.ring_block * ring->block_size;
        const tpacket_hdr_v1 &bh = reinterpret_cast<const tpacket_block_desc *>(blk)->hdr.bh1;
        entry = bh.offset_to_first_pkt;
        const auto *p0 = reinterpret_cast<const tpacket3_hdr *>(blk + entry);
        if (p0->tp_len == 0)  // afpacket.go:313-316: the retry's next() (header.go:181-195)
          entry += p0->tp_next_offset != 0 ? (uint64_t)p0->tp_next_offset
                                           : tp_align((uint64_t)p0->tp_snaplen + p0->tp_mac);
      }
      tp[j] = gpd::TwPlan{bp.ring_block, bp.emit, bp.out, entry};
    }
    bool fallback = true;
    rc = gpd::decode_tpv3_device(ctx, *ring, tp, n, add_vlan_header != 0, pk_out, out, nthreads, &fallback);
    if (rc) return rc;
    if (!fallback) {
      g_last_path = 1;
      *n_out = n;
      *blocks_out = (uint32_t)plan.size();
      return GPD_OK;
    }
  }
  // the walk writes straight into the caller's arrays where it has them
  std::vector<uint64_t> off_own;
  std::vector<uint32_t> cap_own, tci_own;
  gpd_tpv3_pkts pk = pk_out ? *pk_out : gpd_tpv3_pkts{};
  if (!pk.offset) {
    off_own.resize(n);
    pk.offset = off_own.data();
  }
  if (!pk.caplen) {
    cap_own.resize(n);
    pk.caplen = cap_own.data();
  }
  if (add_vlan_header && !pk.vlan_tci) {
    tci_own.resize(n);
    pk.vlan_tci = tci_own.data();
  }
  const uint64_t ring_bytes = (uint64_t)ring->block_size * ring->num_blocks;
  // batch offsets for the ring as the buffer (kept per thread across calls: a capture loop
  // calls again and again, and fresh pages cost more than the walk)
  static thread_local std::vector<uint32_t> off32;
  const bool direct = ring_bytes <= 0xFFFFFFF0ull;
  if (direct && off32.size() < n) off32.resize(n);
  rc = run_walk(ring, plan, pk, nthreads, direct ? off32.data() : nullptr);
  if (rc) return rc;
  const uint64_t *off = pk.offset;
  const uint32_t *cap = pk.caplen, *tci = pk.vlan_tci;
  bool tagging = false;
  if (add_vlan_header)
    for (uint64_t i = 0; i < n && !tagging; i++) tagging = tci[i] != 0;
  if (!tagging && direct) {
    // No frame needs a tag inserted: the ring itself is the batch buffer (offsets relative to
    // its base) and the pipelined host path moves it — whole runs of frames straight from a
    // registered ring, or the frames repacked in parallel — with two chunks in flight.
    const gpd_batch hb{ring->base, ring_bytes, off32.data(), cap, n};
    rc = gpd_decode_host(ctx, &hb, out);
    if (rc) return rc;
    g_last_path = 0;
    *n_out = n;
    *blocks_out = (uint32_t)plan.size();
    return GPD_OK;
  }
  // device image: the walked blocks in walk order, then the VLAN-tagged copies
  const uint64_t B = ring->block_size, nb = plan.size();
  std::vector<uint32_t> doff(n), dcap(n);
  std::vector<uint8_t> tagged;
  for (uint64_t j = 0; j < nb; j++) {
    const BlockPlan &bp = plan[j];
    for (uint64_t i = bp.out; i < bp.out + bp.emit; i++) {
      doff[i] = (uint32_t)(j * B + (off[i] - (uint64_t)bp.ring_block * B));
      dcap[i] = cap[i];
      if (add_vlan_header && tci[i] != 0) {  // insertVlanHeader, header.go:74-82
        if (cap[i] < 12)
          return gpd::set_error(GPD_ERR_INVALID, "gpd_decode_tpv3: packet %llu: %u bytes cannot take a "
                                "VLAN tag (the reference's data[0:12] panics)", (unsigned long long)i, cap[i]);
        while (tagged.size() % 16) tagged.push_back(0);
        const uint8_t *d = ring->base + off[i];
        doff[i] = (uint32_t)(nb * B + tagged.size());
        tagged.insert(tagged.end(), d, d + 12);
        const uint8_t tag[4] = {0x81, 0x00, (uint8_t)((tci[i] >> 8) & 0xff), (uint8_t)(tci[i] & 0xff)};
        tagged.insert(tagged.end(), tag, tag + 4);
        tagged.insert(tagged.end(), d + 12, d + cap[i]);
        dcap[i] = cap[i] + 4;
      }
    }
  }
  const uint64_t data_len = nb * B + tagged.size();
  if (data_len > 0xFFFFFFF0ull)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_decode_tpv3: %llu walked bytes exceed one batch",
                          (unsigned long long)data_len);
  gpd::DeviceScope dscope_;
  if (dscope_.set(gpd::ctx_device(ctx)) != hipSuccess)
    return gpd::set_error(GPD_ERR_HIP, "gpd_decode_tpv3: hipSetDevice");
  // context scratch slots 0-8 (kept across calls: a ring is walked again and again)
  auto *d_data = static_cast<uint8_t *>(gpd::ctx_scratch(ctx, 0, ((data_len + 15) & ~15ull) + 64));
  uint32_t *d_off = static_cast<uint32_t *>(gpd::ctx_scratch(ctx, 1, n * 4));
  uint32_t *d_cap = static_cast<uint32_t *>(gpd::ctx_scratch(ctx, 2, n * 4));
  uint32_t *d_st = static_cast<uint32_t *>(gpd::ctx_scratch(ctx, 3, n * 4));
  uint32_t *d_cs = static_cast<uint32_t *>(gpd::ctx_scratch(ctx, 4, n * 4));
  uint32_t *d_ho = static_cast<uint32_t *>(gpd::ctx_scratch(ctx, 5, n * 4));
  uint64_t *d_ly = static_cast<uint64_t *>(gpd::ctx_scratch(ctx, 6, n * 8));
  uint64_t *d_nh = static_cast<uint64_t *>(gpd::ctx_scratch(ctx, 7, n * 8));
  uint64_t *d_th = static_cast<uint64_t *>(gpd::ctx_scratch(ctx, 8, n * 8));
  gpd_detail *d_dt = out->detail ? static_cast<gpd_detail *>(gpd::ctx_scratch(ctx, 9, n * sizeof(gpd_detail)))
                                 : nullptr;
  hipError_t e = hipSuccess;
  for (void *p : {(void *)d_data, (void *)d_off, (void *)d_cap, (void *)d_st, (void *)d_cs,
                  (void *)d_ho, (void *)d_ly, (void *)d_nh, (void *)d_th})
    if (!p) e = hipErrorOutOfMemory;
  if (out->detail && !d_dt) e = hipErrorOutOfMemory;
  // the walked blocks, ring order from first_block (one copy per contiguous run)
  for (uint64_t j = 0; j < nb && e == hipSuccess;) {
    uint64_t k = j + 1;
    while (k < nb && plan[k].ring_block == plan[k - 1].ring_block + 1) k++;
    e = hipMemcpy(d_data + j * B, ring->base + (uint64_t)plan[j].ring_block * B, (k - j) * B,
                  hipMemcpyHostToDevice);
    j = k;
  }
  if (e == hipSuccess && !tagged.empty())
    e = hipMemcpy(d_data + nb * B, tagged.data(), tagged.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_off, doff.data(), n * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_cap, dcap.data(), n * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    gpd_batch b{d_data, data_len, d_off, d_cap, n};
    gpd_result r{d_st, d_ly, d_nh, d_th, d_cs, nullptr, d_ho, nullptr, d_dt};
    rc = gpd_decode(ctx, &b, &r, nullptr);
    if (rc == GPD_OK) e = hipDeviceSynchronize();
  }
  if (e == hipSuccess && rc == GPD_OK) {
    e = hipMemcpy(out->status, d_st, n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out->layers, d_ly, n * 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess && out->net_hash) e = hipMemcpy(out->net_hash, d_nh, n * 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess && out->tp_hash) e = hipMemcpy(out->tp_hash, d_th, n * 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess && out->csum) e = hipMemcpy(out->csum, d_cs, n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess && out->hdr_off) e = hipMemcpy(out->hdr_off, d_ho, n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess && out->detail)
      e = hipMemcpy(out->detail, d_dt, n * sizeof(gpd_detail), hipMemcpyDeviceToHost);
  }
  if (rc) return rc;
  if (e != hipSuccess) return gpd::set_error(GPD_ERR_HIP, "gpd_decode_tpv3: %s", hipGetErrorString(e));
  g_last_path = 0;
  *n_out = n;
  *blocks_out = (uint32_t)nb;
  return GPD_OK;
}

}  // extern "C"
