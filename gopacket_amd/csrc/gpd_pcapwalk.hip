// gpd_pcapwalk.hip — the pcap record walk on the GPU, for gpd_decode_pcap_at (include/gpd_pcap.h).
//
// The host walk (gpd_pcap.cpp) reads every record header of the capture in host memory, and on
// a GPU box's share of host cores that walk, not PCIe, bounds a replay.  Here the
// capture's bytes travel to HBM in fixed byte chunks first, and the records are found there:
//
//   pw_walk    one lane per 2 KiB segment of the chunk.  The segment holding the chunk's entry
//              (the first record header, handed on by the previous chunk) walks from it; every
//              later segment starts speculatively at its first position whose 8-header chain
//              passes every ReadPacketData check (pcapgo/read.go:120-137) and walks while its
//              headers start inside the segment: start, exit (first header at or past the
//              segment's end), record count, and whether a header failed a check;
//   pw_stitch  one workgroup: the true walk runs through the segments exactly when every
//              segment that found a start begins where the previous such segment's walk left
//              off, and every segment that found none is jumped by it.  Then the counts' prefix
//              sums are the records' indices, the last exit is where the next chunk's walk
//              starts, and the chunk's record count goes to the control block (for the decode
//              launch and the host).  Anything else — a speculation that the true walk does
//              not meet, a rejected record, a capture that ends in a partial record — sets
//              status 1 and count 0: the host walks from this chunk's entry on instead, with
//              the reference's exact stop and error text;
//   pw_fill    one lane per segment again: its records' data offsets (relative to the chunk)
//              and capture lengths, at their indices.
//
// The decode kernel then reads the record count from the control block (KParams::n_dev).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gpd_internal.h"

namespace gpd {

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;

struct PwHdr {
  uint32_t cap, wire;
};

__device__ __forceinline__ uint32_t rd32(const uint8_t *p, bool be) {
  const uint32_t v = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
  return be ? __builtin_bswap32(v) : v;
}

// One ReadPacketData step at p of the chunk's T bytes: true when the record passes every check
// and its data lies inside the bytes (a record the host would reject, or one cut by the end of
// the capture, is false: the host decides those).
__device__ __forceinline__ bool pw_step(const PwArgs &A, uint32_t p, uint32_t &cap) {
  if (p + 16u > A.T) return false;
  const uint8_t *h = A.d + p;
  cap = rd32(h + 8, A.be);
  const uint32_t wire = rd32(h + 12, A.be);
  if (cap > A.snaplen || cap > wire) return false;  // read.go:125-131
  return (uint64_t)p + 16u + cap <= A.T;            // read.go:133-134
}

// A header at x whose chain of 8 passes every check (or reaches the capture's end exactly, or
// the end of the bytes this chunk holds, after at least one).  Three things the reader accepts
// are not taken as evidence here: an all-zero header (zero-filled payload is a chain of valid
// empty records), a fraction-of-second field of a second or more (bytes that merely pass the
// length checks rarely hold one below 10^6, resp. 10^9), and timestamps that run backwards.
// A wrong speculation is caught by the stitch, at the cost of the host walk; these keep it rare.
__device__ __forceinline__ bool pw_plausible(const PwArgs &A, uint32_t x) {
  uint32_t psec = 0, pfrac = 0;
  for (int k = 0; k < 8; k++) {
    if (x >= A.T) return k > 0 && (A.last ? x == A.T : true);
    uint32_t cap;
    if (!pw_step(A, x, cap)) return false;
    const uint8_t *h = A.d + x;
    if ((rd32(h, false) | rd32(h + 4, false) | rd32(h + 8, false) | rd32(h + 12, false)) == 0u) return false;
    const uint32_t sec = rd32(h, A.be), frac = rd32(h + 4, A.be);
    if (frac >= (A.nano ? 1000000000u : 1000000u)) return false;  // not a sub-second count
    if (sec < psec || (sec == psec && frac < pfrac)) return false;  // time runs backwards
    psec = sec;
    pfrac = frac;
    x += 16u + cap;
  }
  return true;
}

}  // namespace

__global__ __launch_bounds__(256) void pw_walk(PwArgs A) {
  const uint32_t s = blockIdx.x * 256u + threadIdx.x;
  if (s >= A.nseg) return;
  const uint32_t lo = s * kPwSeg, hi = min(lo + kPwSeg, A.own_end);
  const uint32_t e = A.ctl->entry;
  uint32_t start = kNone;
  if (e >= lo && e < hi) {
    start = e;
  } else if (e < lo) {  // speculation: the first plausible header of the segment
    // (when a record's original length equals its capture length, the view 4 bytes on —
    // seconds := fraction, fraction := length, length := original length — passes the same
    // checks and advances by the same steps as the true walk, forever)
    // Views of a true header shifted by a few bytes can chain in parallel with it too (64-B
    // records: the view one byte early reads length 64 << 8, a step of 205 records): of the
    // plausible positions within 8 bytes, the one with the shortest record is taken, and one
    // that is the 4-byte shift of a plausible header just before it is passed over.
    const uint32_t lim = min(hi, lo + 16u + A.snaplen + 1u);
    uint32_t x = lo;
    while (x < lim) {
      if (!pw_plausible(A, x)) {
        x++;
        continue;
      }
      uint32_t best = x, bc = rd32(A.d + x + 8, A.be);
      for (uint32_t y = x + 1; y < min(x + 8u, lim); y++)
        if (pw_plausible(A, y)) {
          const uint32_t c = rd32(A.d + y + 8, A.be);
          if (c < bc) {
            best = y;
            bc = c;
          }
        }
      if (best >= 4u && pw_plausible(A, best - 4u) && rd32(A.d + best + 4u, A.be) <= bc) {
        x = best + 1u;
        continue;
      }
      start = best;
      break;
    }
  }
  uint32_t p = start, cnt = 0, bad = 0;
  if (start != kNone) {
    while (p < hi) {
      uint32_t cap;
      if (!pw_step(A, p, cap)) {
        bad = 1;
        break;
      }
      cnt++;
      p += 16u + cap;
    }
  }
  A.st[s] = start;
  A.ex[s] = p;
  A.ct[s] = cnt;
  A.bad[s] = bad;
}

// One workgroup of 1024 lanes; lane t owns segments [t*R, t*R + R).  Where the true walk
// disagrees with a segment's speculation (it enters the segment elsewhere, or enters one whose
// scan found no start), the owning lane re-walks that segment from where the true walk stands,
// and the check runs again (a fix can move where the next lane's first segment is entered):
// up to kFixRounds rounds, after which the chunk is the host's.  Payload bytes that read as a
// chain of plausible headers (config 5's 64-B records: a view 3 bytes into each record chains
// 16,400-byte "records" forever) then cost a few microseconds of this workgroup instead of a
// host walk of the chunk.
constexpr int kFixRounds = 4;

__device__ __forceinline__ void pw_rewalk(const PwArgs &A, uint32_t s, uint32_t at, uint32_t hi) {
  if (at >= hi) {  // a longer record covers the whole segment: no header starts in it
    A.st[s] = kNone;
    A.ct[s] = 0;
    A.bad[s] = 0;
    return;
  }
  uint32_t p = at, cnt = 0, bad = 0;
  while (p < hi) {
    uint32_t cap;
    if (!pw_step(A, p, cap)) {
      bad = 1;
      break;
    }
    cnt++;
    p += 16u + cap;
  }
  A.st[s] = at;
  A.ex[s] = p;
  A.ct[s] = cnt;
  A.bad[s] = bad;
}

__global__ __launch_bounds__(1024) void pw_stitch(PwArgs A) {
  __shared__ uint32_t s_cnt[1024], s_last[1024], s_ok[1024], s_fixed, s_nfix;
  __shared__ unsigned long long s_miss;  // the first refuted segment << 32 | its speculated start
  const uint32_t t = threadIdx.x;
  const uint32_t R = (A.nseg + 1023u) / 1024u;
  const uint32_t a = min(t * R, A.nseg), b = min(a + R, A.nseg);
  const uint32_t e = A.ctl->entry;
  if (t == 0) {
    s_miss = ~0ull;
    s_nfix = 0;
  }
  uint32_t why = 0;  // the host's reasons (PwCtl::status bits), 0 = the walk stands
  for (int round = 0;; round++) {
    uint32_t cnt = 0, last = kNone;  // this lane's record count and last segment that found a start
    for (uint32_t s = a; s < b; s++) {
      if (A.st[s] != kNone) {
        cnt += A.ct[s];
        last = s;
      }
    }
    s_cnt[t] = cnt;
    s_last[t] = last;
    if (t == 0) s_fixed = 0;
    __syncthreads();
    // inclusive scans across lanes (Hillis-Steele; 1024 entries): + of counts, max of last
    for (uint32_t d = 1; d < 1024u; d <<= 1) {
      const uint32_t c = t >= d ? s_cnt[t - d] : 0u;
      const uint32_t l = t >= d ? s_last[t - d] : kNone;
      __syncthreads();
      s_cnt[t] += c;
      if (l != kNone && (s_last[t] == kNone || l > s_last[t])) s_last[t] = l;
      __syncthreads();
    }
    uint32_t base = t ? s_cnt[t - 1] : 0u;
    uint32_t prev = t ? s_last[t - 1] : kNone;  // the last segment with a start before a
    uint32_t fixed = 0;
    why = 0;
    for (uint32_t s = a; s < b; s++) {
      const uint32_t lo = s * kPwSeg, hi = min(lo + kPwSeg, A.own_end);
      // where the true walk stands when it reaches this segment
      const uint32_t at = prev == kNone ? e : A.ex[prev];
      uint32_t st = A.st[s];
      const bool refuted = st != kNone && st != at;             // a speculation the true walk misses
      const bool uncovered = st == kNone && at >= lo && at < hi;  // a header of the true walk, unwalked
      if (refuted || uncovered) {
        if (round < kFixRounds) {
          if (refuted) atomicMin(&s_miss, ((unsigned long long)s << 32) | st);
          // (`at` below the segment: the previous lane is fixing a segment of its own in this
          // round, and the next round sees where the walk really enters this one)
          if (at >= lo) {
            pw_rewalk(A, s, at, hi);
            st = A.st[s];
          }
          fixed++;
        } else {
          why |= refuted ? 2u : 8u;
        }
      }
      if (st != kNone) {
        if (A.bad[s]) why |= 4u;  // a record the reference rejects (or cut by the bytes)
        A.base[s] = base;
        base += A.ct[s];
        prev = s;
      }
    }
    if (fixed) {
      s_fixed = 1u;
      atomicAdd(&s_nfix, fixed);
    }
    __threadfence_block();  // (the re-walked segments' words, for the other lanes' next round)
    __syncthreads();
    const bool again = s_fixed != 0u;
    __syncthreads();
    if (!again) break;
  }
  s_ok[t] = why;
  __syncthreads();
  for (uint32_t d = 512; d > 0; d >>= 1) {
    if (t < d) s_ok[t] |= s_ok[t + d];
    __syncthreads();
  }
  if (t == 1023u) {
    const uint32_t total = s_cnt[1023];
    const uint32_t lastseg = s_last[1023];
    const uint32_t next = lastseg == kNone ? e : A.ex[lastseg];
    // a capture that does not end exactly after a record (or a chunk whose walk stopped short
    // of its end) is the host's to walk
    const bool done = A.last ? next == A.T : next >= A.own_end;
    const uint32_t why_all = s_ok[0] | (done ? 0u : 16u);  // 16: the walk ends short of the bytes
    A.ctl->miss_st = s_miss == ~0ull ? kNone : (uint32_t)s_miss;
    A.ctl->miss_at = s_miss == ~0ull ? kNone : (uint32_t)(s_miss >> 32);
    A.ctl->pad[0] = s_nfix;  // segments re-walked here
    const bool good = why_all == 0u;
    A.ctl->n = good ? total : 0u;
    A.ctl->next = next;
    A.ctl->status = good ? 0u : 1u | why_all;
    if (good && A.ctl_next) A.ctl_next->entry = next - A.own_end;
  }
}

__global__ __launch_bounds__(256) void pw_fill(PwArgs A) {
  const uint32_t s = blockIdx.x * 256u + threadIdx.x;
  if (s >= A.nseg || A.ctl->status != 0u) return;
  const uint32_t start = A.st[s];
  if (start == kNone) return;
  uint32_t p = start, k = A.base[s];
  const uint32_t c = A.ct[s];
  for (uint32_t j = 0; j < c; j++) {
    const uint32_t cap = rd32(A.d + p + 8, A.be);
    A.off[k + j] = p + 16u;
    A.len[k + j] = cap;
    p += 16u + cap;
  }
}

hipError_t launch_pcap_walk(const PwArgs &A, hipStream_t stream) {
  const unsigned g = (A.nseg + 255u) / 256u;
  if (A.nseg > kPwMaxSeg) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pw_walk, dim3(g ? g : 1), dim3(256), 0, stream, A);
  hipLaunchKernelGGL(pw_stitch, dim3(1), dim3(1024), 0, stream, A);
  return hipGetLastError();
}

hipError_t launch_pcap_fill(const PwArgs &A, hipStream_t stream) {
  const unsigned g = (A.nseg + 255u) / 256u;
  hipLaunchKernelGGL(pw_fill, dim3(g ? g : 1), dim3(256), 0, stream, A);
  return hipGetLastError();
}

}  // namespace gpd
