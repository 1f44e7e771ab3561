// gpd_tpv3walk.hip — the TPACKET_V3 block walk on the GPU, for gpd_decode_tpv3
// (include/gpd_afpacket.h).
//
// The host walk (gpd_afpacket.cpp walk_block) follows each user-owned block's packet list —
// tp_next_offset, else tpAlign(tp_snaplen + tp_mac) (afpacket/header.go:181-195) — and on a GPU
// box's share of host cores that walk, not PCIe, bounds the ring's decode.
// Here the blocks travel to HBM whole, in groups of consecutive ring blocks, and each block is
// walked by one workgroup:
//
//   the block's bytes pass through a 32 KiB LDS window; the workgroup finds the packet
//   list's headers inside the window by pointer doubling over its 16-byte granules (below),
//   then every lane reads its packets' headers from LDS, checks that each frame lies inside
//   the block, and writes the decode's offset / length and the capture info
//   (afpacket.go:318-326, header.go:151-180) at the packets' indices, coalesced; the window
//   moves to the next header.  (One lane following the list — one dependent LDS read and
//   ~40 instructions per packet — took 1.2 ms per 6,500-packet block.)
//
// The host plans the blocks (status word, num_pkts, first packet: afpacket.go:303-316,
// header.go:144-149) and knows every block's packet count and output index beforehand, so
// nothing is stitched.  A block whose walk leaves the block (which the host walk reports as an
// error, with its text) or meets a frame carrying a VLAN tag when OptAddVLANHeader is on (the
// host path inserts the tag) sets its status word, and the host redoes the call.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gpd_internal.h"

namespace gpd {

namespace {

constexpr uint32_t kHdr = 48;              // sizeof(struct tpacket3_hdr)
constexpr uint32_t kHdrLl = kHdr + 20;     // + sizeof(struct sockaddr_ll) (header.go:177-180)
constexpr uint32_t kVlanValid = 1u << 4;   // TP_STATUS_VLAN_VALID (linux/if_packet.h)

}  // namespace

// tpacket3_hdr words (linux/if_packet.h): 0 tp_next_offset, 1 tp_sec, 2 tp_nsec,
// 3 tp_snaplen, 4 tp_len, 5 tp_status, 6 tp_mac | tp_net << 16, 7 tp_rxhash, 8 tp_vlan_tci.
//
// One window pass.  Headers sit on 16-byte granules (TPACKET_ALIGNMENT: the kernel's
// tp_next_offset and tpAlign steps are multiples of 16), so the window's 2048 granules are the
// candidate headers and the pass entry is granule 0.  Every candidate c whose header lies in
// the window gets its successor J(c) = c + step / 16 (step = tp_next_offset, else
// tpAlign(tp_snaplen + tp_mac): header.go:181-195), or EXIT when that leaves the window, or BAD
// for a step that is 0 or not a multiple of 16.  Then rounds k = 0, 1, ... mark J(c) for every
// marked c and square J (J <- J o J): after round k the first 2^(k+1) packets of the chain from
// the entry are marked (and only packets of that chain ever are), and a round that marks
// nothing new ends it.  Packets are in chain order exactly in granule order (steps are
// positive), so a packet's index is the count of marked granules before it.  A pass costs
// about log2(packets in the window) rounds of 8 LDS reads per lane instead of one dependent
// LDS read per packet on one lane.
namespace {
constexpr uint32_t kGran = kTwWin / 16u;   // candidate headers per window
constexpr uint32_t kPer = kGran / 256u;    // per lane
constexpr uint16_t kExit = 0xFFFFu, kBad = 0xFFFEu;
}  // namespace

__global__ __launch_bounds__(256) void tw_walk(TwArgs A) {
  __shared__ uint4 win[kGran];
  __shared__ uint16_t s_j[kGran];
  __shared__ uint8_t s_m[kGran];
  __shared__ uint32_t s_cnt[kPer * 4];
  __shared__ uint32_t s_last;
  const uint32_t j = blockIdx.x, t = threadIdx.x, wv = t >> 6, ln = t & 63u;
  const TwBlock b = A.blk[j];
  const uint32_t B = A.block_size;
  const uint8_t *blk = A.d + (uint64_t)j * B;
  const uint32_t *w32 = reinterpret_cast<const uint32_t *>(win);
  auto step = [&](uint32_t c) -> uint32_t {  // v3wrapper.next from the header at granule c
    const uint32_t nx = w32[4u * c];
    return nx ? nx : ((w32[4u * c + 3u] + (w32[4u * c + 6u] & 0xFFFFu) + 15u) & ~15u);
  };
  uint32_t pos = b.entry;  // (16-byte aligned and pos + 48 <= B: the host checked the entry)
  uint32_t done = 0, err = 0, tag = 0, bad = 0;
  while (done < b.emit && !err) {
    const uint32_t w0 = pos, w1 = min(w0 + kTwWin, B), wlen = w1 - w0;
    {  // all of a lane's loads in flight before the first LDS write
      const uint32_t nq = wlen >> 4;
      uint4 v[kPer];
#pragma unroll
      for (uint32_t u = 0; u < kPer; u++) {
        const uint32_t q = min(t + 256u * u, nq - 1u);  // (unconditional: no wait per load)
        v[u] = *reinterpret_cast<const uint4 *>(blk + w0 + 16u * q);
      }
#pragma unroll
      for (uint32_t u = 0; u < kPer; u++)  // (lanes past the end rewrite the last granule's bytes)
        win[min(t + 256u * u, nq - 1u)] = v[u];
    }
    // candidates whose header (and sockaddr_ll, for the interface index) lies in the window;
    // in the block's last window, every header inside the block
    const uint32_t n_in = w1 == B ? (wlen - kHdr) / 16u + 1u : (wlen - kHdrLl) / 16u + 1u;
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < kPer; u++) {
      const uint32_t c = t + 256u * u;
      uint16_t jv = kExit;
      if (c < n_in) {
        const uint32_t st = step(c);
        if (st == 0u || (st & 15u)) {
          jv = kBad;
        } else {
          const uint32_t sc = st >> 4;
          jv = sc < n_in - c ? (uint16_t)(c + sc) : kExit;
        }
      }
      s_j[c] = jv;
      s_m[c] = c == 0u;
    }
    __syncthreads();
    for (;;) {
      uint32_t changed = 0;
#pragma unroll
      for (uint32_t u = 0; u < kPer; u++) {
        const uint32_t c = t + 256u * u;
        if (s_m[c]) {
          const uint32_t jv = s_j[c];
          if (jv < kGran && !s_m[jv]) {
            s_m[jv] = 1;
            changed = 1;
          }
        }
      }
      if (!__syncthreads_or(changed)) break;
      uint16_t jn[kPer];
#pragma unroll
      for (uint32_t u = 0; u < kPer; u++) {
        const uint32_t jv = s_j[t + 256u * u];
        jn[u] = jv < kGran ? s_j[jv] : (uint16_t)jv;
      }
      __syncthreads();
#pragma unroll
      for (uint32_t u = 0; u < kPer; u++) s_j[t + 256u * u] = jn[u];
      __syncthreads();
    }
    // packet index of every marked granule: ballots per wave and row, then their prefix
    uint32_t fl = 0, rk[kPer];
#pragma unroll
    for (uint32_t u = 0; u < kPer; u++) {
      const bool m = s_m[t + 256u * u] != 0;
      const uint64_t bal = __ballot(m);
      fl |= (uint32_t)m << u;
      rk[u] = (uint32_t)__popcll(bal & ((1ull << ln) - 1ull));
      if (ln == 0) s_cnt[u * 4u + wv] = (uint32_t)__popcll(bal);
    }
    __syncthreads();
    uint32_t total = 0;
#pragma unroll
    for (uint32_t u = 0; u < kPer; u++) {
      const uint32_t before = total;
      for (uint32_t w = 0; w < 4u; w++) total += s_cnt[u * 4u + w];
      for (uint32_t w = 0; w < wv; w++) rk[u] += s_cnt[u * 4u + w];
      rk[u] += before;
    }
    const uint32_t take = min(total, b.emit - done);  // v3wrapper.next: used >= num_pkts
#pragma unroll
    for (uint32_t u = 0; u < kPer; u++) {
      if (!((fl >> u) & 1u)) continue;
      const uint32_t c = t + 256u * u, h = 4u * c;
      if (rk[u] == total - 1u) s_last = c;
      if (rk[u] >= take) continue;
      const uint32_t p = w0 + 16u * c;  // header position in the block
      const uint32_t snap = w32[h + 3], mac = w32[h + 6] & 0xFFFFu, tci = w32[h + 8];
      const uint32_t data = p + mac;
      bad |= (uint64_t)data + snap > B;  // walk_block: frame outside the block
      const uint32_t q = b.out + done + rk[u];
      A.off[q] = j * B + data;
      A.len[q] = snap;
      tag |= tci;
      if (A.ci_off) {
        A.ci_off[q] = A.ring_off0 + (uint64_t)j * B + data;
        A.ci_wire[q] = w32[h + 4];
        A.ci_ts[q] = (uint64_t)w32[h + 1] * 1000000000ull + w32[h + 2];
        A.ci_ifx[q] = p + kHdrLl <= B ? (int32_t)w32[h + 13] : 0;
        A.ci_vlan[q] = (w32[h + 5] & kVlanValid) ? (int32_t)(tci & 0xFFFu) : -1;
        A.ci_tci[q] = tci;
      }
    }
    __syncthreads();
    done += take;
    if (done < b.emit) {  // the chain left the window (or stopped at a BAD step) after its last packet
      const uint32_t st = step(s_last);
      const uint64_t nxt = (uint64_t)w0 + 16u * s_last + st;
      if (st == 0u || (st & 15u) || nxt + kHdr > B) err = 1;  // (the host walk decides those)
      pos = (uint32_t)nxt;
    }
    if (__syncthreads_or(bad)) err = 1;  // (also: the next pass overwrites the window)
  }
  const int tagged = __syncthreads_or(tag != 0u);
  if (t == 0) A.st[j] = err | (tagged ? 2u : 0u);
}

hipError_t launch_tpv3_walk(const TwArgs &A, hipStream_t stream) {
  if (A.nblk == 0) return hipSuccess;
  if ((A.block_size & 15u) || (uint64_t)A.block_size * A.nblk > kTwGroup) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tw_walk, dim3(A.nblk), dim3(256), 0, stream, A);
  return hipGetLastError();
}

}  // namespace gpd
