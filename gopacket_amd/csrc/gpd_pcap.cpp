// gpd_pcap.cpp — pcap record walk, host side of include/gpd_pcap.h.
//
// Restates pcapgo's reader on an in-memory capture (paths relative to google/gopacket):
//   readHeader ........ pcapgo/read.go:78-117   (magics read.go:47-49, write.go:32; v2.4)
//   ReadPacketData .... pcapgo/read.go:120-137  (snaplen / original-length checks)
//   readPacketHeader .. pcapgo/read.go:165-177  (timestamp = time.Unix(sec, uint32(frac*factor)))
// Instead of copying each record out, the walk returns where each record's bytes lie in the
// capture, so the capture buffer itself is the decoder's batch buffer.
//
// The walk is a linked list (each record header gives the next record's position).  With
// several threads the buffer is cut into segments; every segment but the first is walked
// speculatively from the first position whose header chain looks like pcap records, and the
// segments are stitched in order: the true walk (segment 0, exact) ends at its first record
// header at or past the next segment's start, and if the speculative walk of that segment
// visited the same position, both walks coincide from there on (the list is deterministic),
// so the speculative records from that position on are the true ones.  A segment whose
// speculation the true walk never meets is re-walked sequentially.  The result is therefore
// the sequential walk's for every input; speculation only decides how much of it runs in
// parallel.  Records are produced in two parallel passes over a window: the speculative
// count (no stores), then — once the stitch has fixed where the true walk enters each segment
// and how many of its records come before — a fill that writes every segment's records
// straight into the caller's flat arrays at their final index.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "gpd_internal.h"
#include "../../include/gpd_pcap.h"

namespace gpd {

namespace {

inline uint32_t rd32(const uint8_t *p, bool be) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return be ? __builtin_bswap32(v) : v;
}
inline uint16_t rd16(const uint8_t *p, bool be) {
  uint16_t v;
  std::memcpy(&v, p, 2);
  return be ? (uint16_t)__builtin_bswap16(v) : v;
}

struct End {
  uint64_t pos = 0;  // next record header position (the exit of a segment walk, or the stop)
  int stop = GPD_PCAP_STOP_LIMIT;
  uint32_t a0 = 0, a1 = 0;  // error arguments
  bool stopped = false;     // the walk ended for good (EOF or a rejected record)
};

// One ReadPacketData step at position p: 1 = a record (fields set), 0 = the walk stops (e set).
inline int step(const uint8_t *buf, uint64_t len, const gpd_pcap_info &I, uint64_t p, uint32_t &cap,
                uint32_t &wire, uint64_t &ts, End &e) {
  const uint64_t avail = len - p;
  const bool be = I.big_endian != 0;
  if (avail == 0) {  // io.ReadFull of the header reads nothing: io.EOF, the normal end
    e.stop = GPD_PCAP_STOP_EOF;
    return 0;
  }
  if (avail < GPD_PCAP_RECORD_BYTES) {  // read.go:166-168, io.ErrUnexpectedEOF
    e.stop = GPD_PCAP_STOP_SHORT_HDR;
    return 0;
  }
  const uint8_t *h = buf + p;
  cap = rd32(h + 8, be);
  wire = rd32(h + 12, be);
  if (cap > I.snaplen) {  // read.go:125-127
    e.stop = GPD_PCAP_STOP_SNAPLEN;
    e.a0 = cap;
    e.a1 = I.snaplen;
    return 0;
  }
  if (cap > wire) {  // read.go:129-131
    e.stop = GPD_PCAP_STOP_ORIGLEN;
    e.a0 = cap;
    e.a1 = wire;
    return 0;
  }
  if (avail - GPD_PCAP_RECORD_BYTES < cap) {  // read.go:133-134, io.ReadFull of the data
    e.stop = GPD_PCAP_STOP_SHORT_DATA;
    e.a0 = (uint32_t)(avail - GPD_PCAP_RECORD_BYTES);  // 0 => io.EOF, else ErrUnexpectedEOF
    return 0;
  }
  const uint32_t factor = I.nano ? 1u : 1000u;
  ts = (uint64_t)rd32(h, be) * 1000000000ull + (uint32_t)(rd32(h + 4, be) * factor);  // read.go:172
  return 1;
}

// Walk from p while record headers start before `limit`, at most max_n records, writing
// record k of this walk at index at + k of `out`; returns the records written.
uint64_t walk_store(const uint8_t *buf, uint64_t len, const gpd_pcap_info &I, uint64_t p, uint64_t limit,
                uint64_t max_n, const PcapOut &out, uint64_t at, End &e, bool &overflow) {
  uint64_t n = 0;
  const uint64_t d = GPD_PCAP_RECORD_BYTES - out.base;  // off32 = pos + 16 - base (mod 2^64)
  while (p < limit) {
    if (n == max_n) {
      e.stop = GPD_PCAP_STOP_LIMIT;
      e.pos = p;
      e.stopped = true;
      return n;
    }
    uint32_t cap, wire;
    uint64_t ts;
    if (!step(buf, len, I, p, cap, wire, ts, e)) {
      e.pos = p;
      e.stopped = true;
      return n;
    }
    const uint64_t k = at + n;
    if (out.off32) {
      const uint64_t o = p + d;
      overflow |= o >= (1ull << 32);
      out.off32[k] = (uint32_t)o;
    }
    if (out.pos64) out.pos64[k] = p;
    if (out.cap) out.cap[k] = cap;
    if (out.wire) out.wire[k] = wire;
    if (out.ts) out.ts[k] = ts;
    n++;
    p += GPD_PCAP_RECORD_BYTES + (uint64_t)cap;
    // the chain only moves forward through contiguous records: stream the bytes ahead of it
    // so each dependent header read hits the cache instead of paying DRAM latency
    __builtin_prefetch(buf + std::min(p + 2048, len), 0, 0);
    __builtin_prefetch(buf + std::min(p + 4096, len), 0, 0);
  }
  e.pos = p;  // exit: the first record header at or past `limit`
  e.stopped = false;
  return n;
}

// A header at x that, with the `depth` headers after it, passes every check of a record.
bool plausible_chain(const uint8_t *buf, uint64_t len, const gpd_pcap_info &I, uint64_t x, int depth) {
  End e;
  for (int k = 0; k < depth; k++) {
    if (x == len) return k > 0;  // the chain reaches the end of the capture exactly
    uint32_t cap, wire;
    uint64_t ts;
    if (!step(buf, len, I, x, cap, wire, ts, e)) return false;
    x += GPD_PCAP_RECORD_BYTES + (uint64_t)cap;
  }
  return true;
}

thread_local int g_last_threads = 0, g_last_rewalks = 0, g_last_met = 0;

// nthreads <= 0: the machine's cores, at most 16 (a GPU's share of a shared host)
int default_threads() { return (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency())); }

// Counting walk (gpd_pcap_locate): the same steps as walk() without storing the records; the
// first `keep` positions are remembered so that a speculative segment can be met.
struct Count {
  uint64_t n = 0;
  std::vector<uint64_t> first;
  End e;
};
void count_walk(const uint8_t *buf, uint64_t len, const gpd_pcap_info &I, uint64_t p, uint64_t limit,
                uint64_t max_n, size_t keep, Count &c) {
  c.n = 0;
  c.first.clear();
  while (p < limit) {
    if (c.n == max_n) {
      c.e.stop = GPD_PCAP_STOP_LIMIT;
      c.e.pos = p;
      c.e.stopped = true;
      return;
    }
    uint32_t cap, wire;
    uint64_t ts;
    if (!step(buf, len, I, p, cap, wire, ts, c.e)) {
      c.e.pos = p;
      c.e.stopped = true;
      return;
    }
    if (c.first.size() < keep) c.first.push_back(p);
    c.n++;
    p += GPD_PCAP_RECORD_BYTES + (uint64_t)cap;
    __builtin_prefetch(buf + std::min(p + 2048, len), 0, 0);
    __builtin_prefetch(buf + std::min(p + 4096, len), 0, 0);
  }
  c.e.pos = p;
  c.e.stopped = false;
}

}  // namespace

// gpd_pcap_locate (see gpd_pcap.h): one parallel counting pass over buf[pos:len) gives every
// segment's record count on the true walk (speculation + stitching as in pcap_walk); each
// target is then reached by a sequential walk inside the one segment that holds it.
int pcap_locate(const uint8_t *buf, uint64_t len, const gpd_pcap_info &I, uint64_t pos,
                const uint64_t *targets, uint64_t k, uint64_t *pos_out, uint64_t *n_total, int *stop_out,
                int nthreads) {
  if (nthreads <= 0) nthreads = default_threads();
  const uint64_t span = len > pos ? len - pos : 0;
  const uint64_t kMinSeg = 4ull << 20;
  const int T = (int)std::min<uint64_t>((uint64_t)nthreads, std::max<uint64_t>(1, span / kMinSeg));
  std::vector<uint64_t> seg(T + 1);
  for (int s = 0; s <= T; s++) seg[s] = pos + span * (uint64_t)s / (uint64_t)T;
  const size_t kKeep = 4096;  // a speculation that syncs later than this is re-walked
  std::vector<Count> C(T);
  auto run = [&](int s) {
    if (s == 0) {
      count_walk(buf, len, I, pos, seg[1], UINT64_MAX, 0, C[0]);
      return;
    }
    const uint64_t hi = std::min<uint64_t>(seg[s + 1], seg[s] + GPD_PCAP_RECORD_BYTES + (uint64_t)I.snaplen + 1);
    for (uint64_t x = seg[s]; x < hi; x++) {
      if (plausible_chain(buf, len, I, x, 8)) {
        count_walk(buf, len, I, x, seg[s + 1], UINT64_MAX, kKeep, C[s]);
        return;
      }
    }
    C[s].e.stopped = false;
    C[s].e.pos = UINT64_MAX;
  };
  if (T == 1) {
    run(0);
  } else {
    std::vector<std::thread> th;
    for (int s = 1; s < T; s++) th.emplace_back(run, s);
    run(0);
    for (auto &t : th) t.join();
  }
  // stitch: the true walk's entry position and record count before each segment
  std::vector<uint64_t> entry(T + 1, UINT64_MAX), before(T + 1, 0);
  entry[0] = pos;
  End cur = C[0].e;
  uint64_t n = C[0].n;
  int last = 0;  // the last segment the true walk enters
  for (int s = 1; s < T && !cur.stopped; s++) {
    entry[s] = cur.pos;
    before[s] = n;
    last = s;
    if (cur.pos >= seg[s + 1]) continue;  // no true record starts in segment s
    const auto &F = C[s].first;
    auto it = std::lower_bound(F.begin(), F.end(), cur.pos);
    if (it != F.end() && *it == cur.pos) {
      n += C[s].n - (uint64_t)(it - F.begin());
      cur = C[s].e;
    } else {
      Count c;
      count_walk(buf, len, I, cur.pos, seg[s + 1], UINT64_MAX, 0, c);
      n += c.n;
      cur = c.e;
    }
  }
  if (!cur.stopped) cur.stop = GPD_PCAP_STOP_EOF;
  if (n_total) *n_total = n;
  if (stop_out) *stop_out = cur.stop;
  uint64_t at_pos = pos, at_n = 0;  // the last position resolved (targets ascend)
  for (uint64_t t = 0; t < k; t++) {
    const uint64_t want = targets[t];
    if (t && want < targets[t - 1]) return set_error(GPD_ERR_INVALID, "gpd_pcap_locate: targets must ascend");
    if (want > n) return set_error(GPD_ERR_INVALID, "gpd_pcap_locate: target %llu beyond the %llu records of the walk",
                                   (unsigned long long)want, (unsigned long long)n);
    if (want == n) {
      pos_out[t] = cur.pos;
      continue;
    }
    int s = last;  // start from the nearest known point before the target
    while (s > 0 && before[s] > want) s--;
    if (before[s] > at_n) {
      at_n = before[s];
      at_pos = entry[s];
    }
    Count c;
    count_walk(buf, len, I, at_pos, len, want - at_n, 0, c);
    pos_out[t] = at_pos = c.e.pos;
    at_n = want;
  }
  return GPD_OK;
}

// Run f(k) for k in [0, T): k >= 1 on threads of their own, k = 0 on the caller's.
template <class F>
void par_segments(int T, F f) {
  if (T == 1) {
    f(0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve((size_t)T - 1);
  for (int k = 1; k < T; k++) th.emplace_back(f, k);
  f(0);
  for (auto &t : th) t.join();
}

// The sequential walk's result over buf[pos:len) (see gpd_pcap.h), built in parallel.
//
// Window by window: the window is cut into segments; the count pass walks every segment
// (segment 0 from the true position, bounded by the records still wanted; the others
// speculatively) without storing; the stitch follows the true walk through the segments'
// counts (re-counting a segment its speculation missed) and so knows, per segment, where the
// true walk enters it and how many records precede it; the fill pass then walks each
// segment's true records again and writes them at their final index.  An unbounded walk is
// one window over the whole buffer.  A bounded one must not read the whole buffer: its first
// 256 records are walked sequentially (learning the mean record size), and each later window
// spans the bytes the records still missing would take at 1.1x that mean.  Windows only
// bound how far each pass reads ahead: the records and the stop are the sequential walk's.
int pcap_index_flat(const uint8_t *buf, uint64_t len, const gpd_pcap_info &I, uint64_t pos, uint64_t max_n,
                    int nthreads, const PcapOut &out, PcapResult &R) {
  R = PcapResult{};
  if (nthreads <= 0) nthreads = default_threads();
  const uint64_t kMinSeg = 4ull << 20;
  const size_t kKeep = 4096;  // a speculation that syncs later than this is re-counted
  auto threads_for = [&](uint64_t span) {
    return (int)std::min<uint64_t>((uint64_t)nthreads, std::max<uint64_t>(1, span / kMinSeg));
  };
  int threads = 1, met = 0, rewalks = 0;
  bool overflow = false;
  End cur;
  cur.pos = pos;
  uint64_t have = 0;
  const bool bounded = max_n < (len > pos ? len - pos : 0) / GPD_PCAP_RECORD_BYTES;
  if (bounded) {  // learn the record sizes
    have = walk_store(buf, len, I, pos, len, std::min<uint64_t>(256, max_n), out, 0, cur, overflow);
    if (cur.stopped && cur.stop == GPD_PCAP_STOP_LIMIT) cur.stopped = false;
  }
  while (!cur.stopped && cur.pos < len && have < max_n) {
    const uint64_t rem = max_n - have;
    uint64_t end = len;
    if (bounded) {
      const double mean = have ? (double)(cur.pos - pos) / (double)have : 96.0;
      end = std::min<uint64_t>(len, cur.pos + (uint64_t)((double)rem * mean * 1.1) + 65536);
    }
    const int T = threads_for(end - cur.pos);
    threads = std::max(threads, T);
    if (T == 1) {  // one segment: a single storing pass
      End e;
      have += walk_store(buf, len, I, cur.pos, end, rem, out, have, e, overflow);
      cur = e;
      if (cur.stopped && cur.stop == GPD_PCAP_STOP_LIMIT && have < max_n) cur.stopped = false;
      continue;
    }
    std::vector<uint64_t> seg(T + 1);
    for (int k = 0; k <= T; k++) seg[k] = cur.pos + (end - cur.pos) * (uint64_t)k / (uint64_t)T;
    // count pass
    std::vector<Count> C(T);
    par_segments(T, [&](int k) {
      if (k == 0) {
        count_walk(buf, len, I, cur.pos, seg[1], rem, 0, C[0]);
        return;
      }
      const uint64_t hi = std::min<uint64_t>(seg[k + 1], seg[k] + GPD_PCAP_RECORD_BYTES + (uint64_t)I.snaplen + 1);
      for (uint64_t x = seg[k]; x < hi; x++) {
        if (plausible_chain(buf, len, I, x, 8)) {
          count_walk(buf, len, I, x, seg[k + 1], UINT64_MAX, kKeep, C[k]);
          return;
        }
      }
      C[k].e.stopped = false;
      C[k].e.pos = UINT64_MAX;  // no speculation
    });
    // stitch: where the true walk enters each segment, and its records there
    std::vector<uint64_t> entry(T, 0), cnt(T, 0);
    End e = C[0].e;
    entry[0] = cur.pos;
    cnt[0] = C[0].n;
    uint64_t tot = cnt[0];
    int used = 1;
    for (int k = 1; k < T && !e.stopped && tot < rem; k++) {
      entry[k] = e.pos;
      used = k + 1;
      if (e.pos >= seg[k + 1]) continue;  // no true record starts in segment k
      const auto &F = C[k].first;
      auto it = std::lower_bound(F.begin(), F.end(), e.pos);
      if (it != F.end() && *it == e.pos) {  // the true walk meets the speculation
        cnt[k] = C[k].n - (uint64_t)(it - F.begin());
        e = C[k].e;
        met++;
      } else {  // it never does: count this segment from the true position
        Count c;
        count_walk(buf, len, I, e.pos, seg[k + 1], UINT64_MAX, 0, c);
        cnt[k] = c.n;
        e = c.e;
        rewalks++;
      }
      tot += cnt[k];
    }
    bool trimmed = false;
    if (tot > rem) {  // the bound falls inside segment used-1
      cnt[used - 1] -= tot - rem;
      tot = rem;
      trimmed = true;
    }
    // fill pass: each segment's true records at their final index
    std::vector<uint64_t> at(used + 1, have);
    for (int k = 0; k < used; k++) at[k + 1] = at[k] + cnt[k];
    std::vector<End> F(used);
    std::vector<char> ovf(used, 0);
    par_segments(used, [&](int k) {
      bool o = false;
      if (cnt[k]) walk_store(buf, len, I, entry[k], len, cnt[k], out, at[k], F[k], o);
      ovf[k] = o;
    });
    for (int k = 0; k < used; k++) overflow |= ovf[k] != 0;
    if (trimmed) {  // the walk continues right after the last record written
      e = F[used - 1];
      e.stop = GPD_PCAP_STOP_LIMIT;
      e.stopped = true;
    }
    have += tot;
    cur = e;
    if (cur.stopped && cur.stop == GPD_PCAP_STOP_LIMIT && have < max_n) cur.stopped = false;
  }
  if (!cur.stopped && cur.pos >= len) {  // the walk reached the end: the next header starts exactly there
    cur.stop = GPD_PCAP_STOP_EOF;
    cur.stopped = true;
  }
  if (have == max_n) {  // as the sequential loop: the limit first
    cur.stop = GPD_PCAP_STOP_LIMIT;
    cur.a0 = cur.a1 = 0;
  }
  R.n = have;
  R.next_pos = cur.pos;
  R.stop = cur.stop;
  R.a0 = cur.a0;
  R.a1 = cur.a1;
  R.off32_overflow = overflow;
  g_last_threads = threads;
  g_last_met = met;
  g_last_rewalks = rewalks;
  switch (R.stop) {
    case GPD_PCAP_STOP_SHORT_HDR:
      return set_error(GPD_ERR_PCAP, "unexpected EOF");
    case GPD_PCAP_STOP_SNAPLEN:
      return set_error(GPD_ERR_PCAP, "capture length exceeds snap length: %u > %u", R.a0, R.a1);
    case GPD_PCAP_STOP_ORIGLEN:
      return set_error(GPD_ERR_PCAP, "capture length exceeds original packet length: %u > %u", R.a0, R.a1);
    case GPD_PCAP_STOP_SHORT_DATA:
      return set_error(GPD_ERR_PCAP, R.a0 == 0 ? "EOF" : "unexpected EOF");
    default:
      return GPD_OK;
  }
}

}  // namespace gpd

extern "C" {

int gpd_pcap_header(const uint8_t *buf, uint64_t len, gpd_pcap_info *info) {
  if (!info || (!buf && len)) return gpd::set_error(GPD_ERR_INVALID, "gpd_pcap_header: null argument");
  std::memset(info, 0, sizeof *info);
  // bufio Peek(2) then io.ReadFull(24) (read.go:79-92)
  if (len < 2) return gpd::set_error(GPD_ERR_PCAP, "EOF");
  if (buf[0] == 0x1f && buf[1] == 0x8b)
    return gpd::set_error(GPD_ERR_INVALID, "gzip-compressed capture: inflate it before indexing");
  if (len < GPD_PCAP_HEADER_BYTES) return gpd::set_error(GPD_ERR_PCAP, "unexpected EOF");
  uint32_t magic;
  std::memcpy(&magic, buf, 4);  // binary.LittleEndian.Uint32(buf[0:4])
  info->magic = magic;
  if (magic == GPD_PCAP_MAGIC_NANO) {
    info->big_endian = 0, info->nano = 1;
  } else if (magic == GPD_PCAP_MAGIC_NANO_BE) {
    info->big_endian = 1, info->nano = 1;
  } else if (magic == GPD_PCAP_MAGIC_MICRO) {
    info->big_endian = 0, info->nano = 0;
  } else if (magic == GPD_PCAP_MAGIC_MICRO_BE) {
    info->big_endian = 1, info->nano = 0;
  } else {
    return gpd::set_error(GPD_ERR_PCAP, "Unknown magic %x", magic);
  }
  const bool be = info->big_endian != 0;
  info->version_major = gpd::rd16(buf + 4, be);
  if (info->version_major != 2)
    return gpd::set_error(GPD_ERR_PCAP, "Unknown major version %u", info->version_major);
  info->version_minor = gpd::rd16(buf + 6, be);
  if (info->version_minor != 4)
    return gpd::set_error(GPD_ERR_PCAP, "Unknown minor version %u", info->version_minor);
  info->snaplen = gpd::rd32(buf + 16, be);
  info->linktype = gpd::rd32(buf + 20, be);
  return GPD_OK;
}

int gpd_pcap_index(const uint8_t *buf, uint64_t len, const gpd_pcap_info *info, uint64_t pos,
                   uint64_t max_n, uint32_t *offset, uint32_t *caplen, uint32_t *wirelen,
                   uint64_t *ts_ns, uint64_t *n_out, uint64_t *next_pos, int *stop, int nthreads) {
  if (!info || !n_out || (!buf && len) || (max_n && (!offset || !caplen)))
    return gpd::set_error(GPD_ERR_INVALID, "gpd_pcap_index: null argument");
  if (pos > len) return gpd::set_error(GPD_ERR_INVALID, "gpd_pcap_index: pos beyond the buffer");
  gpd::PcapOut o;
  o.off32 = offset;
  o.cap = caplen;
  o.wire = wirelen;
  o.ts = ts_ns;
  gpd::PcapResult R;
  const int rc = gpd::pcap_index_flat(buf, len, *info, pos, max_n, nthreads, o, R);
  if (R.off32_overflow)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_pcap_index: record offsets beyond 4 GiB; index the capture in windows");
  *n_out = R.n;
  if (next_pos) *next_pos = R.next_pos;
  if (stop) *stop = R.stop;
  return rc;
}

int gpd_pcap_locate(const uint8_t *buf, uint64_t len, const gpd_pcap_info *info, uint64_t pos,
                    const uint64_t *targets, uint64_t k, uint64_t *pos_out, uint64_t *n_total, int *stop,
                    int nthreads) {
  if (!info || (!buf && len) || (k && (!targets || !pos_out)))
    return gpd::set_error(GPD_ERR_INVALID, "gpd_pcap_locate: null argument");
  if (pos > len) return gpd::set_error(GPD_ERR_INVALID, "gpd_pcap_locate: pos beyond the buffer");
  return gpd::pcap_locate(buf, len, *info, pos, targets, k, pos_out, n_total, stop, nthreads);
}

void gpd_pcap_last_stats(int *threads, int *met, int *rewalks) {
  if (threads) *threads = gpd::g_last_threads;
  if (met) *met = gpd::g_last_met;
  if (rewalks) *rewalks = gpd::g_last_rewalks;
}

}  // extern "C"
