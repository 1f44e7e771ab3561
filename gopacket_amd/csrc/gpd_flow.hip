// gpd_flow.hip — MI355X flow table (include/gpd_flow.h): find-or-create the connection
// record of every decoded packet, keyed by its [2]Flow{NetworkFlow(), TransportFlow()}.
//
// Reference (paths relative to google/gopacket):
//   key ............... tcpassembly/assembly.go:289,543 (key{netFlow, t.TransportFlow()}),
//                       reassembly/tcpassembly.go:389,644
//   Flow equality ..... flows.go:140-146 (struct fields; NewFlow zero-pads to 16, :214-224)
//   find-or-create .... tcpassembly/assembly.go:495-511 (StreamPool.getConnection)
//   endpoints ......... layers/ip4.go:63-65, layers/ip6.go:49-51, layers/tcp.go:331-333,
//                       layers/udp.go:123-125, layers/endpoints.go:20-32
//
// One lane per packet.  The decoder already left, per packet, the EndpointTypes of both
// flows (status bits 20-27) and where their layers sit (hdr_off), so the key is gathered
// straight from the packet bytes in HBM: 16+16 address bytes, 4 port bytes, the types.
// Records live in an open-addressing table of 2^k slots, each split in two: a 64-byte hot
// record on a line of its own (fingerprint, key, packed counter word, last) — everything a
// packet of an existing flow reads or updates — and a 16-byte cold record (first, counter
// spills).  A record is claimed by one 64-bit compare-and-swap of the key's fingerprint; the
// claimer then stores the key.
// The per-flow counters are device atomics, folded first over runs of neighbouring lanes on
// one record (fold_run).  A second launch compares every packet's key with its record's
// stored key (visible after the launch boundary), so a fingerprint collision is caught and
// reported instead of silently merging two flows; packets that claimed their record wrote
// its key themselves and are skipped (the insert's claim bits, FlowParams::made).
// Sharding over GPUs (gpd_flow_keys / gpd_flow_insert_keys): the same key, gathered once,
// travels as a 64-byte record to the rank its FastHash pair names; two passes (count per
// owner, then scatter with wave-aggregated cursors) group the records by owner without a
// sort, and the owner inserts records exactly as packets.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "gpd_internal.h"
#include "../../include/gpd_flow.h"

namespace gpd {

constexpr int kFlowThreads = 256;
static_assert(sizeof(gpd_flow_rec) == 80, "gpd_flow_rec layout (include/gpd_flow.h)");

enum : uint32_t { FS_FLOWS = 0, FS_PACKETS, FS_NOKEY, FS_FULL, FS_COLL, FS_EXPORT, FS_WORDS = 8 };
// The stats words lie 128 B apart: every wave adds its tallies when it ends, and device-scope
// atomics on one line serialise at the memory side (~12 ns each), the words of a line together.
constexpr uint32_t kStatStride = 16;
__host__ __device__ constexpr uint32_t stat_at(uint32_t w) { return w * kStatStride; }

// A slot of the table, as two records (gpd_flow_export assembles the public gpd_flow_rec).
// The hot record is one 64-byte line: a packet of a flow that already exists reads its
// fingerprint and key and updates `cnt` and `last` there, and touches no other line when its
// sequence number is above every earlier call's (then `first` cannot fall: FlowParams::seen).
struct alignas(64) FlowHot {
  uint64_t fp;       // fingerprint | epoch << 56; 0 = empty
  uint32_t key[10];  // src[16], dst[16], ports, types (flow_key's words)
  uint64_t cnt;      // packed counter word: packets << B | bytes mod 2^B (add_run)
  uint64_t last;
};
struct FlowCold {
  uint64_t first;
  uint64_t spill;  // (byte-field carries) << 32 + (packet-field wraps), see add_run
};
static_assert(sizeof(FlowHot) == 64 && sizeof(FlowCold) == 16, "flow table slot layout");

static_assert(sizeof(gpd_flow_key) == 64, "gpd_flow_key layout (include/gpd_flow.h)");

// A record's counters inside the table (gpd_flow_export unpacks them into the public
// gpd_flow_rec fields): `bytes` holds one packed word, packets << B | bytes mod 2^B (B =
// kCountBits), so one 64-bit atomicAdd updates both; `packets` holds the spills, (carries
// out of the byte field) << 32 + (wraps of the 64-bit word), each in units of 2^B bytes and
// 2^(64-B) packets.  See add_run.
constexpr uint32_t kCountBits = 40;
// A record's fingerprint word: the key's 56-bit fingerprint, and in the top byte the epoch
// (1..255, the insert launch's number mod 255) of the launch that claimed it.  The claim's CAS
// writes both, so every lane that finds the record reads the epoch with the fingerprint: a
// record claimed by an earlier launch has its key and counters published (the launch
// boundary), and the insert updates and checks it at once; one claimed in this launch (or
// 255 launches ago: deferring is always correct) is left to the verify launch.
constexpr uint64_t kFpBits = (1ull << 56) - 1ull;

struct FlowParams {
  const uint8_t *data;
  uint64_t data_len;
  const uint32_t *offset, *caplen, *status, *hdr_off;
  uint32_t *flow_id;
  uint64_t n, base;
  FlowHot *tab;
  uint64_t mask;  // capacity - 1
  unsigned long long *stats;
  // sharding (gpd_flow_keys / gpd_flow_insert_keys)
  const gpd_flow_key *keys;  // key records to insert (KEYS kernels)
  const uint64_t *net_hash, *tp_hash;
  gpd_flow_key *kout;         // partitioned key records (gpd_flow_keys)
  unsigned long long *parts;  // [0, nparts): counts; [nparts, 2 nparts): scatter cursors
  uint32_t nparts;
  // insert -> verify: bit l of word w set when packet 64w+l claimed its record (and so wrote
  // the key the verify would compare against); one word per wave iteration
  uint64_t *made = nullptr;
  uint64_t fp_mask = kFpBits;  // gpd_flow_test_fingerprint_bits (kFpBits in production)
  uint32_t cbits = kCountBits;  // gpd_flow_test_counter_bits (kCountBits in production)
  const gpd_record *rec = nullptr;  // results in the gpd_record form (status and hashes there)
  uint64_t tag = 1ull << 56;    // this launch's epoch (1..255) in the fingerprint word's top byte
  FlowCold *cold = nullptr;     // the slots' cold records, beside tab
  // 1 + the highest sequence number of every earlier insert call into this table (the host's
  // count of index_base + n); ~0 when unknown (key records inserted: their sequence numbers
  // are the senders')
  uint64_t seen = ~0ull;
};

// The key of packet i as 10 words: src[16], dst[16], ports (raw wire bytes), types.  Returns
// false when the packet has no network + transport pair (gpd.h status / hdr_off words).
__device__ __forceinline__ bool flow_key(const FlowParams &P, uint64_t i, uint32_t (&k)[10]) {
  const uint32_t st = P.rec ? P.rec[i].status : P.status[i], ho = P.hdr_off[i];
  const uint32_t nt = (st >> 20) & 15u, tt = (st >> 24) & 15u;
  const uint32_t no = ho & 0xFFFFu, to = ho >> 16;
  if (nt == 0 || tt == 0 || no == 0xFFFFu || to == 0xFFFFu) return false;
  const uint64_t off = min((uint64_t)P.offset[i], P.data_len);
  const uint8_t *pkt = P.data + off;
  const uint32_t alen = nt == 1u ? 4u : 16u;
  const uint8_t *src = pkt + no + (nt == 1u ? 12u : 8u);  // ip4.go:63-65 / ip6.go:49-51
  const uint8_t *dst = src + alen;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    uint32_t a = 0, b = 0;
    if ((uint32_t)w * 4u < alen) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        a |= (uint32_t)src[4 * w + j] << (8 * j);
        b |= (uint32_t)dst[4 * w + j] << (8 * j);
      }
    }
    k[w] = a;  // NewFlow zero-pads the unused address bytes (flows.go:214-224)
    k[4 + w] = b;
  }
  const uint8_t *tp = pkt + to;  // tcp.go:331-333 / udp.go:123-125: ports as raw bytes
  k[8] = (uint32_t)tp[0] | ((uint32_t)tp[1] << 8) | ((uint32_t)tp[2] << 16) | ((uint32_t)tp[3] << 24);
  k[9] = nt | (tt << 8) | (alen << 16);
  return true;
}

__device__ __forceinline__ uint64_t fingerprint(const uint32_t (&k)[10], uint64_t mask) {
  uint64_t h = 0x9E3779B97F4A7C15ull;
#pragma unroll
  for (int w = 0; w < 10; w += 2) {
    h ^= ((uint64_t)k[w + 1] << 32) | k[w];
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 32;
  }
  h ^= h >> 33;
  h *= 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 33;
  h &= mask;
  return h ? h : 1ull;
}

// Run counters: every lane tallies its wave's count (the ballot is wave-uniform) across the
// grid-stride loop, and lane 0 adds the tally once when the wave ends.  One atomic per wave
// iteration on these few shared words serialised at the memory side and cost most of the
// insert (7.6 ms of 2^24 packets); one per wave per launch costs nothing.
__device__ __forceinline__ void wave_tally(unsigned long long &t, bool pred) {
  t += (unsigned long long)__popcll(__ballot(pred));
}
__device__ __forceinline__ void wave_flush(unsigned long long *ctr, unsigned long long t) {
  if (t && (threadIdx.x & 63u) == 0u) atomicAdd(ctr, t);
}

// Consecutive lanes of a wave that update the same record (a burst of one flow: capture
// order keeps a flow's packets together, and key records stay in packet order) fold their
// updates before the atomics.  A segmented inclusive scan over runs of equal slots leaves the
// run's min/max seq and its packet and byte sums in the run's last lane, which alone issues
// the four atomics.  min, max and + are associative and commutative, so every record ends
// bit-identical to one atomic per packet.  A wave with no runs (every lane a different
// record, e.g. all new flows) skips the scan.  Called by all 64 lanes.
// pb packs packets (bits 57-63, at most 64) and bytes (at most 64 x 2^32 < 2^57).
constexpr int kPktShift = 57;
__device__ __forceinline__ bool fold_run(bool counted, uint64_t s, uint64_t &mn, uint64_t &mx,
                                         uint64_t &pb, uint32_t &start) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t key = counted ? s : ~(uint64_t)lane;  // uncounted lanes never join a run
  const uint64_t prev = __shfl_up(key, 1u, 64);
  const uint64_t heads = __ballot(lane == 0u || prev != key);
  const bool tail = lane == 63u || ((heads >> (lane + 1u)) & 1ull);
  start = lane;
  if (heads == ~0ull) return tail;  // no two neighbours share a record
  start = 63u - (uint32_t)__builtin_clzll(heads & ((2ull << lane) - 1ull));
#pragma unroll
  for (uint32_t d = 1; d < 64u; d <<= 1) {
    const uint64_t omn = __shfl_up(mn, d, 64), omx = __shfl_up(mx, d, 64), opb = __shfl_up(pb, d, 64);
    if (lane >= start + d) {
      mn = min(mn, omn);
      mx = max(mx, omx);
      pb += opb;
    }
  }
  return tail;
}

// The counter updates of one run (fold_run's totals, in its last lane).  A run whose first
// lane claimed the record in this launch is the record's first writer, so the insert stores
// its totals plainly; every other run adds them with atomics in the verify launch, after
// those stores (the launch boundary orders them).  So a new flow costs its claim CAS and
// plain stores, and the atomics are left to packets of flows that already existed.
__device__ __forceinline__ void store_run(FlowHot &r, FlowCold &c, uint64_t mn, uint64_t mx, uint64_t pb,
                                          uint32_t B) {
  const uint64_t pk = pb >> kPktShift, by = pb & ((1ull << kPktShift) - 1ull);
  r.last = mx;
  r.cnt = (pk << B) | (by & ((1ull << B) - 1ull));  // (pk <= 64 < 2^(64-B))
  c.first = mn;
  c.spill = (by >> B) << 32;
}
// The packed add.  x = pk << B + by goes in with one atomicAdd that returns the old word; the
// lane whose add carried out of the byte field (c carries: ((old mod 2^B) + by) >> B) takes
// c << B back out of the packet field and books c carries, and the lane whose add or
// take-back wrapped the 64-bit word books +1 / -1 wraps.  Each carry and wrap is seen by
// exactly the lane that caused it, so at the end of the launch
//   packets = (word >> B) + wraps << (64-B),   bytes = (word mod 2^B) + carries << B
// exactly, in any order of the adds.  Carries need 2^40 bytes and wraps 2^24 packets of one
// flow in production, so the spill atomics are rare; the add's return is the price.
// `later`: mn is above every sequence number of earlier calls (seen) and the record was
// claimed by one of them, so its `first` is below mn and the cold record is not touched.
__device__ __forceinline__ void add_run(FlowHot &r, FlowCold &cr, uint64_t mn, uint64_t mx, uint64_t pb,
                                        uint32_t B, bool later) {
  // `first` only falls: a read at or below mn (a flow seen in an earlier batch) proves the
  // min a no-op; a stale read is only ever larger, and then the atomic runs
  if (!later) {
    const uint64_t f = *reinterpret_cast<volatile uint64_t *>(&cr.first);
    if (mn < f) atomicMin(reinterpret_cast<unsigned long long *>(&cr.first), (unsigned long long)mn);
  }
  atomicMax(reinterpret_cast<unsigned long long *>(&r.last), (unsigned long long)mx);
  const uint64_t pk = pb >> kPktShift, by = pb & ((1ull << kPktShift) - 1ull), M = (1ull << B) - 1ull;
  const uint64_t x = (pk << B) + by;
  auto *w = reinterpret_cast<unsigned long long *>(&r.cnt);
  const uint64_t old = atomicAdd(w, (unsigned long long)x);
  const uint64_t c = ((old & M) + by) >> B;
  uint64_t spill = (c << 32) + (old + x < old ? 1ull : 0ull);
  if (c) {
    const uint64_t back = c << B;
    const uint64_t old2 = atomicAdd(w, (unsigned long long)(0ull - back));
    if (old2 < back) spill -= 1ull;
  }
  if (spill) atomicAdd(reinterpret_cast<unsigned long long *>(&cr.spill), (unsigned long long)spill);
}

// Is the record's stored key the packet's key?  The key's 40 bytes (record bytes 8..47) as one
// 8-byte and two 16-byte loads issued together, compared branch-free: a short-circuit `&&`
// compiled to eight dependent load-wait-compare steps per packet of an existing flow
// (round 6: 0.9 ms of the 2.43-ms existing-flow insert, tools/flow_prof.sh).
struct StoredKey {
  uint2 a;
  uint4 b, c;
};
__device__ __forceinline__ StoredKey load_key(const FlowHot &r) {
  return StoredKey{*reinterpret_cast<const uint2 *>(&r.key[0]), *reinterpret_cast<const uint4 *>(&r.key[2]),
                   *reinterpret_cast<const uint4 *>(&r.key[6])};
}
__device__ __forceinline__ bool key_eq(const StoredKey &r, const uint32_t (&k)[10]) {
  const uint32_t d = (r.a.x ^ k[0]) | (r.a.y ^ k[1]) | (r.b.x ^ k[2]) | (r.b.y ^ k[3]) | (r.b.z ^ k[4]) |
                     (r.b.w ^ k[5]) | (r.c.x ^ k[6]) | (r.c.y ^ k[7]) | (r.c.z ^ k[8]) | (r.c.w ^ k[9]);
  return d == 0u;
}
__device__ __forceinline__ bool same_key(const FlowHot &r, const uint32_t (&k)[10]) {
  return key_eq(load_key(r), k);
}

// Sequence number and captured length of item i.
template <bool KEYS>
__device__ __forceinline__ void item_seq(const FlowParams &P, uint64_t i, uint64_t &seq,
                                         uint32_t &caplen) {
  if constexpr (KEYS) {
    seq = P.keys[i].seq;
    caplen = P.keys[i].caplen;
  } else {
    seq = P.base + i;
    caplen = P.caplen[i];
  }
}

// Key of item i: gathered from the packet bytes, or read from a key record (KEYS).
template <bool KEYS>
__device__ __forceinline__ bool item_key(const FlowParams &P, uint64_t i, uint32_t (&k)[10],
                                         uint64_t &seq, uint32_t &caplen) {
  if constexpr (KEYS) {
    const gpd_flow_key &r = P.keys[i];
#pragma unroll
    for (int j = 0; j < 10; j++) k[j] = r.key[j];
    seq = r.seq;
    caplen = r.caplen;
    return true;
  } else {
    seq = P.base + i;
    caplen = P.caplen[i];
    return flow_key(P, i, k);
  }
}

template <bool KEYS>
__global__ __launch_bounds__(kFlowThreads) void flow_insert_kernel(FlowParams P) {
  unsigned long long t_flows = 0, t_packets = 0, t_nokey = 0, t_full = 0, t_coll = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)kFlowThreads + threadIdx.x; i - threadIdx.x < P.n;
       i += (uint64_t)gridDim.x * kFlowThreads) {
    const bool live = i < P.n;
    uint32_t k[10];
    uint64_t seq = 0;
    uint32_t caplen = 0;
    const bool keyed = live && item_key<KEYS>(P, i, k, seq, caplen);
    bool created = false, full = false, pre = false;
    uint64_t s = 0;
    // A lane whose left neighbour holds the same fingerprint (a burst) follows the same
    // probe sequence to the same record: only the first lane of each such run probes, and
    // the others take its slot afterwards.
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t fp = keyed ? fingerprint(k, P.fp_mask) : 0ull;  // fingerprints are never 0
    const uint64_t fp_prev = __shfl_up(fp, 1u, 64);
    const uint64_t lead = __ballot(!keyed || lane == 0u || fp_prev != fp);
    const bool probes = keyed && ((lead >> lane) & 1ull);
    if (probes) {
      s = fp & P.mask;
      uint64_t probe = 0;
      for (; probe <= P.mask; probe++) {  // every lane leaves after at most capacity probes
        // a record's fingerprint only goes 0 -> fp within a launch, so a plain read that sees
        // a fingerprint is final; only an empty slot needs the compare-and-swap
        unsigned long long old = *reinterpret_cast<volatile unsigned long long *>(&P.tab[s].fp);
        if (old == 0ull)
          old = atomicCAS(reinterpret_cast<unsigned long long *>(&P.tab[s].fp), 0ull,
                          (unsigned long long)(fp | P.tag));
        if (old == 0ull) {  // claimed: store the key (read by the verify launch)
          FlowHot &r = P.tab[s];
#pragma unroll
          for (int j = 0; j < 10; j++) r.key[j] = k[j];
          created = true;
          break;
        }
        if ((old & kFpBits) == fp) {
          pre = (old & ~kFpBits) != P.tag;  // claimed by an earlier launch
          break;
        }
        s = (s + 1) & P.mask;
      }
      if (probe > P.mask) full = true;
    }
    if (lead != ~0ull) {  // run members take the slot their run's first lane found
      const uint32_t start = 63u - (uint32_t)__builtin_clzll(lead & ((2ull << lane) - 1ull));
      const uint64_t hs = __shfl(s, (int)start, 64);
      const int hflags = __shfl((int)full | ((int)pre << 1), (int)start, 64);
      if (keyed && !probes) {
        s = hs;
        full = (hflags & 1) != 0;
        pre = (hflags & 2) != 0;
      }
    }
    const uint64_t made = __ballot(created);
    // done: the packet's update and key check happen here (its record is its own, or was
    // published before this launch); the verify launch skips these packets
    const uint64_t done = __ballot(created || (pre && keyed && !full));
    if (lane == 0u && i < P.n) P.made[i >> 6] = done;  // i = the wave's first packet
    const bool counted = keyed && !full;
    // the key check of a record an earlier launch published: its loads issued ahead of the
    // counter atomics (in flight together), the compare after them
    const bool chk = counted && pre;
    StoredKey rk{};
    if (chk) rk = load_key(P.tab[s]);
    uint64_t mn = seq, mx = seq, pb = (1ull << kPktShift) | caplen;
    uint32_t start;
    const bool tail = fold_run(counted, s, mn, mx, pb, start);
    if (counted && tail) {
      if ((made >> start) & 1ull) store_run(P.tab[s], P.cold[s], mn, mx, pb, P.cbits);
      else if (pre) add_run(P.tab[s], P.cold[s], mn, mx, pb, P.cbits, mn >= P.seen);
    }
    const bool bad = chk && !key_eq(rk, k);
    if (bad) P.flow_id[i] = (uint32_t)s | GPD_FLOW_COLLISION;
    if (live && !bad) P.flow_id[i] = !keyed ? GPD_FLOW_NONE : full ? GPD_FLOW_FULL : (uint32_t)s;
    wave_tally(t_coll, bad);
    wave_tally(t_flows, created);
    wave_tally(t_packets, counted);
    wave_tally(t_nokey, live && !keyed);
    wave_tally(t_full, full);
  }
  wave_flush(P.stats + stat_at(FS_FLOWS), t_flows);
  wave_flush(P.stats + stat_at(FS_PACKETS), t_packets);
  wave_flush(P.stats + stat_at(FS_NOKEY), t_nokey);
  wave_flush(P.stats + stat_at(FS_FULL), t_full);
  wave_flush(P.stats + stat_at(FS_COLL), t_coll);
}

// Second pass: the counter updates of runs that found an existing record, and every item's
// key against its record's stored key.
template <bool KEYS>
__global__ __launch_bounds__(kFlowThreads) void flow_verify_kernel(FlowParams P) {
  unsigned long long t_coll = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)kFlowThreads + threadIdx.x; i - threadIdx.x < P.n;
       i += (uint64_t)gridDim.x * kFlowThreads) {
    bool bad = false;
    // the insert's runs again (same lanes, same slots); a run whose first lane claimed the
    // record has stored its totals already
    const uint32_t id = i < P.n ? P.flow_id[i] : GPD_FLOW_NONE;
    const uint64_t made = i - (threadIdx.x & 63u) < P.n ? P.made[i >> 6] : 0ull;
    const bool counted = id < GPD_FLOW_FULL;
    uint64_t mn = 0, mx = 0, pb = 0;
    uint32_t caplen = 0, start;
    if (counted && !((made >> (threadIdx.x & 63u)) & 1ull)) {
      item_seq<KEYS>(P, i, mn, caplen);
      mx = mn;
      pb = (1ull << kPktShift) | caplen;
    }
    const bool tail = fold_run(counted, id, mn, mx, pb, start);
    if (counted && tail && !((made >> start) & 1ull)) add_run(P.tab[id], P.cold[id], mn, mx, pb, P.cbits, false);
    if (i < P.n) {
      uint32_t k[10];
      uint64_t seq;
      // a packet that claimed its record wrote that record's key itself
      const bool mine = (made >> (threadIdx.x & 63u)) & 1ull;
      if (counted && !mine && item_key<KEYS>(P, i, k, seq, caplen)) {
        if (!same_key(P.tab[id], k)) {
          P.flow_id[i] = id | GPD_FLOW_COLLISION;
          bad = true;
        }
      }
    }
    wave_tally(t_coll, bad);
  }
  wave_flush(P.stats + stat_at(FS_COLL), t_coll);
}

// Owner rank of a keyed packet: the high half of the two direction-symmetric FastHashes'
// xor, scaled to [0, nparts) (doc.go:216-228 picks a worker by flow.FastHash()).
__device__ __forceinline__ uint32_t flow_owner(const FlowParams &P, uint64_t i) {
  const uint64_t h = P.rec ? P.rec[i].net_hash ^ P.rec[i].tp_hash : P.net_hash[i] ^ P.tp_hash[i];
  return (uint32_t)(((h >> 32) * (uint64_t)P.nparts) >> 32);
}

// Wave-aggregated claim of one slot of counter ctr[owner] (LDS) for every lane with `has`:
// one LDS atomic per distinct owner in the wave; returns the lane's slot.
__device__ __forceinline__ uint32_t wave_claim(uint32_t *ctr, bool has, uint32_t owner) {
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t todo = __ballot(has);
  uint32_t slot = 0;
  while (todo) {
    const uint32_t o = __builtin_amdgcn_readlane(owner, (int)__builtin_ctzll(todo));
    const uint64_t m = __ballot(has && owner == o);
    const int leader = (int)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == (uint32_t)leader) base = atomicAdd(ctr + o, (uint32_t)__popcll(m));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
    if (has && owner == o)
      slot = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    todo &= ~m;
  }
  return slot;
}

// gpd_flow_keys, pass 1: each workgroup counts its packets per owner in LDS and writes the
// counts owner-major (parts[p * G + b]), so that one exclusive scan of the whole array gives
// every (owner, workgroup) its output range.  No global atomics.
__global__ __launch_bounds__(kFlowThreads) void flow_part_count_kernel(FlowParams P) {
  __shared__ uint32_t cnt[GPD_FLOW_MAX_PARTS];
  for (uint32_t p = threadIdx.x; p < P.nparts; p += kFlowThreads) cnt[p] = 0;
  __syncthreads();
  for (uint64_t i = blockIdx.x * (uint64_t)kFlowThreads + threadIdx.x; i - threadIdx.x < P.n;
       i += (uint64_t)gridDim.x * kFlowThreads) {
    uint32_t k[10];
    const bool keyed = i < P.n && flow_key(P, i, k);
    (void)wave_claim(cnt, keyed, keyed ? flow_owner(P, i) : 0u);
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < P.nparts; p += kFlowThreads)
    P.parts[(uint64_t)p * gridDim.x + blockIdx.x] = cnt[p];
}

// Pass 2 (one workgroup): exclusive scan of the L = nparts * G counts in place; parts[L] =
// the total, and parts[L + 1 + p] = owner p's total.
__global__ __launch_bounds__(1024) void flow_part_scan_kernel(unsigned long long *parts, uint64_t L,
                                                              uint32_t nparts, uint32_t G) {
  __shared__ unsigned long long sums[1024];
  const uint64_t per = (L + 1023) / 1024, lo = threadIdx.x * per, hi = min(L, lo + per);
  unsigned long long s = 0;
  for (uint64_t j = lo; j < hi; j++) s += parts[j];
  sums[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long run = 0;
    for (int t = 0; t < 1024; t++) {
      const unsigned long long v = sums[t];
      sums[t] = run;
      run += v;
    }
    parts[L] = run;
  }
  __syncthreads();
  unsigned long long run = sums[threadIdx.x];
  for (uint64_t j = lo; j < hi; j++) {
    const unsigned long long v = parts[j];
    parts[j] = run;
    run += v;
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < nparts; p += 1024)
    parts[L + 1 + p] = parts[(uint64_t)(p + 1) * G < L ? (uint64_t)(p + 1) * G : L] - parts[(uint64_t)p * G];
}

// Pass 3: each keyed packet's record at its (owner, workgroup) range start + an LDS slot.
// Same grid and packet-to-workgroup mapping as pass 1.
__global__ __launch_bounds__(kFlowThreads) void flow_part_scatter_kernel(FlowParams P) {
  __shared__ uint32_t cur[GPD_FLOW_MAX_PARTS];
  __shared__ unsigned long long start[GPD_FLOW_MAX_PARTS];
  for (uint32_t p = threadIdx.x; p < P.nparts; p += kFlowThreads) {
    cur[p] = 0;
    start[p] = P.parts[(uint64_t)p * gridDim.x + blockIdx.x];
  }
  __syncthreads();
  for (uint64_t i = blockIdx.x * (uint64_t)kFlowThreads + threadIdx.x; i - threadIdx.x < P.n;
       i += (uint64_t)gridDim.x * kFlowThreads) {
    uint32_t k[10];
    const bool keyed = i < P.n && flow_key(P, i, k);
    const uint32_t o = keyed ? flow_owner(P, i) : 0u;
    const uint32_t slot = wave_claim(cur, keyed, o);
    if (keyed) {
      gpd_flow_key r;
#pragma unroll
      for (int j = 0; j < 10; j++) r.key[j] = k[j];
      r.caplen = P.caplen[i];
      r.owner = o;
      r.seq = P.base + i;
      r.fp = fingerprint(k, P.fp_mask);
      P.kout[start[o] + slot] = r;
    }
  }
}

// gpd_flow_key_ids: every packet's (owner, flow id) from the key records it sent and the ids
// their owners returned (sent record j <-> ids[j]).
__global__ __launch_bounds__(kFlowThreads) void flow_ids_fill_kernel(int32_t *owner, uint32_t *flow_id,
                                                                     uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)kFlowThreads + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kFlowThreads) {
    owner[i] = -1;
    flow_id[i] = GPD_FLOW_NONE;
  }
}
__global__ __launch_bounds__(kFlowThreads) void flow_ids_scatter_kernel(const gpd_flow_key *keys, uint64_t m,
                                                                        const uint32_t *ids, uint64_t base,
                                                                        uint64_t n, int32_t *owner,
                                                                        uint32_t *flow_id) {
  for (uint64_t j = blockIdx.x * (uint64_t)kFlowThreads + threadIdx.x; j < m;
       j += (uint64_t)gridDim.x * kFlowThreads) {
    const uint64_t i = keys[j].seq - base;
    if (i < n) {
      owner[i] = (int32_t)keys[j].owner;
      flow_id[i] = ids[j];
    }
  }
}

__global__ __launch_bounds__(kFlowThreads) void flow_reset_kernel(FlowHot *tab, FlowCold *cold, uint64_t cap) {
  for (uint64_t s = blockIdx.x * (uint64_t)kFlowThreads + threadIdx.x; s < cap;
       s += (uint64_t)gridDim.x * kFlowThreads) {
    tab[s] = FlowHot{};
    cold[s] = FlowCold{~0ull, 0ull};
  }
}

// A slot's two records as the public gpd_flow_rec, counters unpacked:
//   packets = (cnt >> B) + wraps << (64-B),   bytes = (cnt mod 2^B) + carries << B
__global__ __launch_bounds__(kFlowThreads) void flow_export_kernel(const FlowHot *tab, const FlowCold *cold,
                                                                  uint64_t cap, gpd_flow_rec *out,
                                                                  uint32_t *idx, uint64_t max,
                                                                  unsigned long long *stats, uint32_t B) {
  for (uint64_t s = blockIdx.x * (uint64_t)kFlowThreads + threadIdx.x; s < cap;
       s += (uint64_t)gridDim.x * kFlowThreads) {
    const FlowHot h = tab[s];
    if (h.fp != 0) {
      const unsigned long long j = atomicAdd(stats + stat_at(FS_EXPORT), 1ull);
      if (j < max) {
        const FlowCold c = cold[s];
        gpd_flow_rec r{};
        r.fp = h.fp & kFpBits;  // the fingerprint without its epoch
        uint32_t *w = reinterpret_cast<uint32_t *>(r.src);
#pragma unroll
        for (int k = 0; k < 9; k++) w[k] = h.key[k];  // src, dst, ports
        r.net_type = (uint8_t)(h.key[9] & 0xFFu);
        r.tp_type = (uint8_t)((h.key[9] >> 8) & 0xFFu);
        r.addr_len = (uint8_t)(h.key[9] >> 16);
        r.first = c.first;
        r.last = h.last;
        r.packets = (h.cnt >> B) + ((c.spill & 0xFFFFFFFFull) << (64u - B));
        r.bytes = (h.cnt & ((1ull << B) - 1ull)) + ((c.spill >> 32) << B);
        out[j] = r;
        idx[j] = (uint32_t)s;
      }
    }
  }
}

}  // namespace gpd

struct gpd_flowtable {
  int device = 0;
  int num_cus = 256;
  gpd::FlowHot *tab = nullptr;   // hot records, 64 B each
  gpd::FlowCold *cold = nullptr;  // cold records, 16 B each
  uint64_t cap = 0;
  unsigned long long *stats = nullptr;  // FS_WORDS counters
  unsigned long long *parts = nullptr;  // gpd_flow_keys: nparts x grid counts (+ totals), grown on use
  uint64_t parts_words = 0;
  uint64_t *made = nullptr;  // insert -> verify claim bits, one word per 64 packets, grown on use
  uint64_t made_words = 0;
  uint64_t fp_mask = gpd::kFpBits;  // gpd_flow_test_fingerprint_bits
  uint32_t cbits = gpd::kCountBits;  // gpd_flow_test_counter_bits
  uint32_t epoch = 0;                 // insert launches so far, mod 255
  uint64_t seen = 0;                  // FlowParams::seen, while seen_known
  bool seen_known = true;             // false after key records went in (until a reset)
};

// The next insert launch's epoch tag (1..255 in the fingerprint word's top byte).
static uint64_t next_tag(gpd_flowtable *ft) {
  ft->epoch = ft->epoch % 255u + 1u;
  return (uint64_t)ft->epoch << 56;
}

#define FLOW_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return gpd::set_error(GPD_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_));          \
  } while (0)

static unsigned grid_for(uint64_t work, int num_cus) {
  const uint64_t blocks = (work + gpd::kFlowThreads - 1) / gpd::kFlowThreads;
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)num_cus * 8));
}

static hipError_t grow_made(gpd_flowtable *ft, uint64_t n) {
  const uint64_t words = (n + 63) / 64;
  if (ft->made_words >= words) return hipSuccess;
  if (ft->made) {
    const hipError_t e = hipFree(ft->made);
    if (e != hipSuccess) return e;
  }
  ft->made = nullptr;
  ft->made_words = 0;
  const hipError_t e = hipMalloc(&ft->made, words * sizeof(uint64_t));
  if (e == hipSuccess) ft->made_words = words;
  return e;
}

// Endpoint / Flow FastHash of caller-built keys (gpd_fast_hash): one lane per key.
__device__ __forceinline__ uint64_t fnv_raw16(uint4 raw, uint32_t len) {  // flows.go:60-67
  const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
  uint64_t h = 14695981039346656037ull;
#pragma unroll
  for (uint32_t k = 0; k < 16; k++)
    if (k < len) h = (h ^ ((w[k >> 2] >> (8 * (k & 3))) & 0xFFu)) * 1099511628211ull;
  return h;
}
__global__ __launch_bounds__(256) void fast_hash_kernel(uint64_t n, const int64_t *typ, const uint4 *src,
                                                        const uint8_t *src_len, const uint4 *dst,
                                                        const uint8_t *dst_len, uint64_t *out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h = fnv_raw16(src[i], src_len[i]);
    if (dst) h += fnv_raw16(dst[i], dst_len[i]);  // flows.go:170: commutative in src and dst
    out[i] = (h ^ (uint64_t)typ[i]) * 1099511628211ull;
  }
}

extern "C" {

int gpd_fast_hash(int device, uint64_t n, const int64_t *typ, const uint8_t *src, const uint8_t *src_len,
                  const uint8_t *dst, const uint8_t *dst_len, uint64_t *out, void *stream) {
  if (n == 0) return GPD_OK;
  if (!typ || !src || !src_len || !out || (dst && !dst_len))
    return gpd::set_error(GPD_ERR_INVALID, "gpd_fast_hash: null argument");
  if (((uintptr_t)src | (uintptr_t)(dst ? dst : src)) & 15u)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_fast_hash: raw arrays must be 16-byte aligned");
  gpd::DeviceScope dscope_;
  FLOW_TRY(dscope_.set(device));
  int cus = 0;
  FLOW_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, (uint64_t)std::max(cus, 1) * 8);
  hipLaunchKernelGGL(fast_hash_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n, typ,
                     reinterpret_cast<const uint4 *>(src), src_len, reinterpret_cast<const uint4 *>(dst),
                     dst_len, out);
  FLOW_TRY(hipGetLastError());
  return GPD_OK;
}

int gpd_flow_create(gpd_ctx *ctx, uint64_t capacity, gpd_flowtable **out) {
  if (!ctx || !out) return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_create: null argument");
  *out = nullptr;
  if (capacity == 0 || capacity > (1ull << 31))
    return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_create: capacity %llu outside [1, 2^31]",
                          (unsigned long long)capacity);
  uint64_t cap = 1;
  while (cap < capacity) cap <<= 1;
  gpd_flowtable *ft = new gpd_flowtable;
  ft->device = gpd::ctx_device(ctx);
  ft->num_cus = gpd::ctx_num_cus(ctx);
  ft->cap = cap;
  gpd::DeviceScope dscope_;
  hipError_t e = dscope_.set(ft->device);
  if (e == hipSuccess) e = hipMalloc(&ft->tab, cap * sizeof(gpd::FlowHot));
  if (e == hipSuccess) e = hipMalloc(&ft->cold, cap * sizeof(gpd::FlowCold));
  if (e == hipSuccess) e = hipMalloc(&ft->stats, gpd::stat_at(gpd::FS_WORDS) * sizeof(unsigned long long));
  if (e != hipSuccess) {
    gpd_flow_destroy(ft);
    return gpd::set_error(e == hipErrorOutOfMemory ? GPD_ERR_NOMEM : GPD_ERR_HIP,
                          "gpd_flow_create: %s", hipGetErrorString(e));
  }
  int rc = gpd_flow_reset(ft, nullptr);
  if (rc == GPD_OK) rc = hipDeviceSynchronize() == hipSuccess ? GPD_OK : GPD_ERR_HIP;
  if (rc != GPD_OK) {
    gpd_flow_destroy(ft);
    return rc;
  }
  *out = ft;
  return GPD_OK;
}

int gpd_flow_reset(gpd_flowtable *ft, void *stream) {
  if (!ft) return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_reset: null table");
  gpd::DeviceScope dscope_;
  FLOW_TRY(dscope_.set(ft->device));
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(gpd::flow_reset_kernel, dim3(grid_for(ft->cap, ft->num_cus)),
                     dim3(gpd::kFlowThreads), 0, s, ft->tab, ft->cold, ft->cap);
  FLOW_TRY(hipGetLastError());
  FLOW_TRY(hipMemsetAsync(ft->stats, 0, gpd::stat_at(gpd::FS_WORDS) * sizeof(unsigned long long), s));
  ft->seen = 0;
  ft->seen_known = true;
  return GPD_OK;
}

int gpd_flow_insert(gpd_flowtable *ft, const gpd_batch *in, const gpd_result *res,
                    uint32_t *flow_id, uint64_t index_base, void *stream) {
  if (!ft || !in || !res || !flow_id)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_insert: null argument");
  if (!(res->status || res->records) || !res->hdr_off)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_insert: the results need status (or records) and hdr_off");
  if (in->n == 0) return GPD_OK;
  if (!in->data || !in->offset || !in->caplen)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_insert: null batch array");
  gpd::DeviceScope dscope_;
  FLOW_TRY(dscope_.set(ft->device));
  gpd::FlowParams P{in->data, in->data_len, in->offset, in->caplen, res->status, res->hdr_off,
                    flow_id, in->n, index_base, ft->tab, ft->cap - 1, ft->stats,
                    nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  FLOW_TRY(grow_made(ft, in->n));
  P.made = ft->made;
  P.fp_mask = ft->fp_mask;
  P.rec = res->records;
  P.cbits = ft->cbits;
  P.tag = next_tag(ft);
  P.cold = ft->cold;
  P.seen = ft->seen_known ? ft->seen : ~0ull;
  const uint64_t top = index_base + in->n < index_base ? ~0ull : index_base + in->n;  // (saturating)
  ft->seen = std::max(ft->seen, top);
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(grid_for(in->n, ft->num_cus)), block(gpd::kFlowThreads);
  hipLaunchKernelGGL(gpd::flow_insert_kernel<false>, grid, block, 0, s, P);
  FLOW_TRY(hipGetLastError());
  hipLaunchKernelGGL(gpd::flow_verify_kernel<false>, grid, block, 0, s, P);
  FLOW_TRY(hipGetLastError());
  return GPD_OK;
}

int gpd_flow_keys(gpd_flowtable *ft, const gpd_batch *in, const gpd_result *res, uint32_t nparts,
                  uint64_t index_base, gpd_flow_key *keys, uint64_t *part_count, void *stream) {
  if (!ft || !in || !res || !part_count || (in->n && !keys))
    return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_keys: null argument");
  if (nparts == 0 || nparts > GPD_FLOW_MAX_PARTS)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_keys: nparts %u outside [1, %d]", nparts,
                          GPD_FLOW_MAX_PARTS);
  if (!res->hdr_off || !(res->records || (res->status && res->net_hash && res->tp_hash)))
    return gpd::set_error(GPD_ERR_INVALID,
                          "gpd_flow_keys: the results need hdr_off and records, or status, net_hash and tp_hash");
  for (uint32_t p = 0; p < nparts; p++) part_count[p] = 0;
  if (in->n == 0) return GPD_OK;
  if (!in->data || !in->offset || !in->caplen)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_keys: null batch array");
  gpd::DeviceScope dscope_;
  FLOW_TRY(dscope_.set(ft->device));
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(grid_for(in->n, ft->num_cus)), block(gpd::kFlowThreads);
  const uint64_t L = (uint64_t)nparts * grid.x, words = L + 1 + nparts;
  if (ft->parts_words < words) {
    if (ft->parts) FLOW_TRY(hipFree(ft->parts));
    ft->parts = nullptr;
    ft->parts_words = 0;
    FLOW_TRY(hipMalloc(&ft->parts, words * sizeof(unsigned long long)));
    ft->parts_words = words;
  }
  gpd::FlowParams P{in->data, in->data_len, in->offset, in->caplen, res->status, res->hdr_off,
                    nullptr, in->n, index_base, ft->tab, ft->cap - 1, ft->stats,
                    nullptr, res->net_hash, res->tp_hash, keys, ft->parts, nparts};
  P.fp_mask = ft->fp_mask;
  P.rec = res->records;
  hipLaunchKernelGGL(gpd::flow_part_count_kernel, grid, block, 0, s, P);
  FLOW_TRY(hipGetLastError());
  hipLaunchKernelGGL(gpd::flow_part_scan_kernel, dim3(1), dim3(1024), 0, s, ft->parts, L, nparts, grid.x);
  FLOW_TRY(hipGetLastError());
  hipLaunchKernelGGL(gpd::flow_part_scatter_kernel, grid, block, 0, s, P);
  FLOW_TRY(hipGetLastError());
  std::vector<unsigned long long> h(nparts);
  FLOW_TRY(hipMemcpyAsync(h.data(), ft->parts + L + 1, nparts * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, s));
  FLOW_TRY(hipStreamSynchronize(s));
  for (uint32_t p = 0; p < nparts; p++) part_count[p] = h[p];
  return GPD_OK;
}

int gpd_flow_key_ids(gpd_flowtable *ft, const gpd_flow_key *keys, uint64_t m, const uint32_t *ids,
                     uint64_t index_base, uint64_t n, int32_t *owner, uint32_t *flow_id, void *stream) {
  if (!ft || (m && (!keys || !ids)) || (n && (!owner || !flow_id)))
    return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_key_ids: null argument");
  if (n == 0) return GPD_OK;
  gpd::DeviceScope dscope_;
  FLOW_TRY(dscope_.set(ft->device));
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(gpd::flow_ids_fill_kernel, dim3(grid_for(n, ft->num_cus)), dim3(gpd::kFlowThreads),
                     0, s, owner, flow_id, n);
  FLOW_TRY(hipGetLastError());
  if (m) {
    hipLaunchKernelGGL(gpd::flow_ids_scatter_kernel, dim3(grid_for(m, ft->num_cus)),
                       dim3(gpd::kFlowThreads), 0, s, keys, m, ids, index_base, n, owner, flow_id);
    FLOW_TRY(hipGetLastError());
  }
  return GPD_OK;
}

int gpd_flow_insert_keys(gpd_flowtable *ft, const gpd_flow_key *keys, uint64_t n,
                         uint32_t *flow_id, void *stream) {
  if (!ft || (n && (!keys || !flow_id)))
    return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_insert_keys: null argument");
  if (n == 0) return GPD_OK;
  gpd::DeviceScope dscope_;
  FLOW_TRY(dscope_.set(ft->device));
  gpd::FlowParams P{nullptr, 0, nullptr, nullptr, nullptr, nullptr, flow_id, n, 0, ft->tab,
                    ft->cap - 1, ft->stats, keys, nullptr, nullptr, nullptr, nullptr, 0};
  FLOW_TRY(grow_made(ft, n));
  P.made = ft->made;
  P.fp_mask = ft->fp_mask;  // (key records carry their sender's fingerprint; recomputed here)
  P.cbits = ft->cbits;
  P.tag = next_tag(ft);
  P.cold = ft->cold;
  ft->seen_known = false;  // (P.seen stays ~0: the key records' sequence numbers are unknown here)
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(grid_for(n, ft->num_cus)), block(gpd::kFlowThreads);
  hipLaunchKernelGGL(gpd::flow_insert_kernel<true>, grid, block, 0, s, P);
  FLOW_TRY(hipGetLastError());
  hipLaunchKernelGGL(gpd::flow_verify_kernel<true>, grid, block, 0, s, P);
  FLOW_TRY(hipGetLastError());
  return GPD_OK;
}

int gpd_flow_stats_get(gpd_flowtable *ft, gpd_flow_stats *out, void *stream) {
  if (!ft || !out) return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_stats_get: null argument");
  gpd::DeviceScope dscope_;
  FLOW_TRY(dscope_.set(ft->device));
  unsigned long long hs[gpd::stat_at(gpd::FS_WORDS)], h[gpd::FS_WORDS];
  FLOW_TRY(hipMemcpyAsync(hs, ft->stats, sizeof hs, hipMemcpyDeviceToHost, (hipStream_t)stream));
  FLOW_TRY(hipStreamSynchronize((hipStream_t)stream));
  for (uint32_t w = 0; w < gpd::FS_WORDS; w++) h[w] = hs[gpd::stat_at(w)];
  out->flows = h[gpd::FS_FLOWS];
  out->packets = h[gpd::FS_PACKETS];
  out->no_key = h[gpd::FS_NOKEY];
  out->full = h[gpd::FS_FULL];
  out->collisions = h[gpd::FS_COLL];
  out->capacity = ft->cap;
  return GPD_OK;
}

int gpd_flow_export(gpd_flowtable *ft, gpd_flow_rec *out, uint32_t *rec_index, uint64_t max,
                    uint64_t *n, void *stream) {
  if (!ft || !out || !n) return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_export: null argument");
  *n = 0;
  gpd::DeviceScope dscope_;
  FLOW_TRY(dscope_.set(ft->device));
  hipStream_t s = (hipStream_t)stream;
  gpd_flow_stats st;
  int rc = gpd_flow_stats_get(ft, &st, stream);
  if (rc) return rc;
  const uint64_t m = std::min<uint64_t>(max, st.flows);
  if (m == 0) return GPD_OK;
  gpd_flow_rec *d_out = nullptr;
  uint32_t *d_idx = nullptr;
  FLOW_TRY(hipMalloc(&d_out, m * sizeof(gpd_flow_rec)));
  hipError_t e = hipMalloc(&d_idx, m * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemsetAsync(ft->stats + gpd::stat_at(gpd::FS_EXPORT), 0, sizeof(unsigned long long), s);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(gpd::flow_export_kernel, dim3(grid_for(ft->cap, ft->num_cus)),
                       dim3(gpd::kFlowThreads), 0, s, ft->tab, ft->cold, ft->cap, d_out, d_idx, m, ft->stats,
                       ft->cbits);
    e = hipGetLastError();
  }
  std::vector<gpd_flow_rec> recs(m);
  std::vector<uint32_t> idx(m);
  if (e == hipSuccess) e = hipMemcpyAsync(recs.data(), d_out, m * sizeof(gpd_flow_rec), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(idx.data(), d_idx, m * sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(d_out);
  (void)hipFree(d_idx);
  if (e != hipSuccess) return gpd::set_error(GPD_ERR_HIP, "gpd_flow_export: %s", hipGetErrorString(e));
  std::vector<uint64_t> order(m);
  for (uint64_t j = 0; j < m; j++) order[j] = j;
  std::sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) {
    return recs[a].first != recs[b].first ? recs[a].first < recs[b].first : idx[a] < idx[b];
  });
  for (uint64_t j = 0; j < m; j++) {
    out[j] = recs[order[j]];
    if (rec_index) rec_index[j] = idx[order[j]];
  }
  *n = m;
  return GPD_OK;
}

int gpd_flow_test_fingerprint_bits(gpd_flowtable *ft, uint32_t bits) {
  if (!ft || bits == 0 || bits > 64)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_test_fingerprint_bits: bits %u outside [1, 64]", bits);
  ft->fp_mask = bits >= 56 ? gpd::kFpBits : (1ull << bits) - 1ull;
  return GPD_OK;
}

int gpd_flow_test_counter_bits(gpd_flowtable *ft, uint32_t bits) {
  if (!ft || bits == 0 || bits > 57)
    return gpd::set_error(GPD_ERR_INVALID, "gpd_flow_test_counter_bits: bits %u outside [1, 57]", bits);
  ft->cbits = bits;
  return GPD_OK;
}

int gpd_flow_destroy(gpd_flowtable *ft) {
  if (!ft) return GPD_OK;
  gpd::DeviceScope dscope_;
  (void)dscope_.set(ft->device);
  if (ft->tab) (void)hipFree(ft->tab);
  if (ft->cold) (void)hipFree(ft->cold);
  if (ft->stats) (void)hipFree(ft->stats);
  if (ft->parts) (void)hipFree(ft->parts);
  if (ft->made) (void)hipFree(ft->made);
  delete ft;
  return GPD_OK;
}

}  // extern "C"
