/*
 * gpd_flow.h — C-ABI of the GPU flow table behind the batched decoder.
 *
 * The reference's immediate consumer of decoded packets is the stream assembler, which keys
 * every TCP packet by the pair [2]gopacket.Flow{NetworkFlow(), TransportFlow()} and finds or
 * creates the connection for that key in a Go map (tcpassembly/assembly.go:289 `type key
 * [2]gopacket.Flow`, :311 `conns map[key]*connection`, :495-511 getConnection, :543 the key
 * built from a packet; reassembly/tcpassembly.go:389,644).  Flow equality is struct
 * equality: EndpointType, both lengths, and the raw bytes zero-padded to 16 (flows.go:140-146,
 * NewFlow :214-224).
 * Here the same find-or-create runs for a whole decoded batch in HBM: every packet whose
 * decode left both a network and a transport layer (TCP or UDP) is looked up by its exact
 * key; a new key creates a flow record; each packet gets the index of its flow record.
 *
 * Reference interfaces each entry point replaces (paths relative to google/gopacket):
 *   gpd_flow_create   tcpassembly.NewStreamPool and the `conns map[key]*connection` it holds
 *                                                        tcpassembly/assembly.go:305-343
 *   gpd_flow_insert   StreamPool.getConnection(k, ...) for every packet of a batch, with
 *                     k = key{netFlow, t.TransportFlow()} as AssembleWithTimestamp builds it
 *                                                        tcpassembly/assembly.go:495-511,533-543;
 *                                                        reassembly/tcpassembly.go:644
 *   gpd_flow_export   iterating the pool's connections (StreamPool.connections,
 *                     tcpassembly/assembly.go:193-200)
 *   gpd_flow_reset / gpd_flow_destroy                    (pool lifetime)
 *
 * The table is open addressing in HBM: 2^k slots of 80 bytes (a 64-byte line of what every
 * packet of the flow reads and updates, and 16 bytes of `first` and counter spills); a record is claimed by a
 * 56-bit fingerprint of its key (tagged with the claiming call's epoch) with one
 * compare-and-swap, and every packet's full key is compared with the record's stored key — at
 * once for records of earlier calls, in a second pass for records claimed in the same call —
 * so a fingerprint collision is detected (counted in gpd_flow_stats.collisions, the packet's
 * flow id flagged) rather than merging two flows silently.
 */
#ifndef GPD_FLOW_H_
#define GPD_FLOW_H_
#include "gpd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One flow record as gpd_flow_export copies it out (80 B; the table keeps the same fields as
 * a 64-byte and a 16-byte record per slot). */
typedef struct gpd_flow_rec {
  uint64_t fp;          /* key fingerprint (56 bits); 0 = empty record */
  uint8_t  src[16];     /* NetworkFlow().Src() raw bytes (4 used for IPv4) */
  uint8_t  dst[16];     /* NetworkFlow().Dst() raw bytes */
  uint8_t  sport[2];    /* TransportFlow().Src() raw bytes (big-endian port) */
  uint8_t  dport[2];    /* TransportFlow().Dst() raw bytes */
  uint8_t  net_type;    /* EndpointType of the network flow: 1 IPv4, 2 IPv6 */
  uint8_t  tp_type;     /* EndpointType of the transport flow: 4 TCP, 5 UDP */
  uint8_t  addr_len;    /* 4 or 16 */
  uint8_t  reserved;
  uint64_t first;       /* lowest packet sequence number (index_base + i) of the flow */
  uint64_t packets;     /* packets of the flow */
  uint64_t bytes;       /* sum of their captured lengths */
  uint64_t last;        /* highest packet sequence number */
} gpd_flow_rec;

/* flow_id[i] values besides a record index */
#define GPD_FLOW_NONE       0xFFFFFFFFu  /* packet has no network + transport layer pair */
#define GPD_FLOW_FULL       0xFFFFFFFEu  /* no free record found (table full) */
#define GPD_FLOW_COLLISION  0x80000000u  /* OR-ed into the id: fingerprint matched, key did not */

typedef struct gpd_flow_stats {
  uint64_t flows;        /* records in use */
  uint64_t packets;      /* packets assigned to a flow (all inserts since the last reset) */
  uint64_t no_key;       /* packets without a network + transport pair */
  uint64_t full;         /* packets that found no free record */
  uint64_t collisions;   /* packets whose fingerprint matched another key (should stay 0) */
  uint64_t capacity;     /* records in the table */
} gpd_flow_stats;

typedef struct gpd_flowtable gpd_flowtable;

/* A table of at least `capacity` records (rounded up to a power of two) on ctx's device.
 * Like the reference's StreamPool under its mutex (tcpassembly/assembly.go:313), a table
 * takes one call at a time: its inserts share per-table scratch (claim bits, partition
 * counts), so calls on a table must be ordered on one stream (or synchronised between
 * streams). */
int gpd_flow_create(gpd_ctx *ctx, uint64_t capacity, gpd_flowtable **out);
/* Empty the table (asynchronous on `stream`). */
int gpd_flow_reset(gpd_flowtable *ft, void *stream);
/* Find-or-create the flow of every packet of a decoded batch (device pointers): `in` is the
 * batch gpd_decode read, `res` its results (hdr_off, and status or the gpd_record form), flow_id[n] receives
 * each packet's record index (or a GPD_FLOW_* value).  Packet i counts as sequence number
 * index_base + i.  Asynchronous on `stream`; the batch must be decoded on that stream first. */
int gpd_flow_insert(gpd_flowtable *ft, const gpd_batch *in, const gpd_result *res,
                    uint32_t *flow_id, uint64_t index_base, void *stream);
/* Counters since the last reset (synchronises `stream`). */
int gpd_flow_stats_get(gpd_flowtable *ft, gpd_flow_stats *out, void *stream);
/* Copy up to max occupied records to host memory, ordered by `first` (synchronises
 * `stream`); *n = number copied.  rec_index (may be NULL) receives each one's index. */
int gpd_flow_export(gpd_flowtable *ft, gpd_flow_rec *out, uint32_t *rec_index, uint64_t max,
                    uint64_t *n, void *stream);
int gpd_flow_destroy(gpd_flowtable *ft);

/* Endpoint.FastHash / Flow.FastHash (flows.go:60-83,167-174) of n endpoints or flows held in
 * device memory on `device` as gopacket lays them out (flows.go:32-36,142-146): typ[i] (the
 * EndpointType, int64), the raw bytes zero-padded to MaxEndpointSize = 16 (src, dst: n x 16
 * bytes, 16-byte aligned) and their lengths (src_len, dst_len: n bytes, at most 16, as
 * NewEndpoint / NewFlow guarantee; larger values hash 16 bytes).  A flow (dst != NULL):
 * out[i] = ((fnvHash(src) + fnvHash(dst)) ^ typ) * fnvPrime, the same for a flow and its
 * Reverse(); an endpoint (dst == NULL, dst_len ignored): out[i] = (fnvHash(src) ^ typ) *
 * fnvPrime.  Replaces the per-object methods for keys a caller builds itself (e.g. the
 * [2]Flow keys of tcpassembly/assembly.go:289 from stored records). */
int gpd_fast_hash(int device, uint64_t n, const int64_t *typ, const uint8_t *src, const uint8_t *src_len,
                  const uint8_t *dst, const uint8_t *dst_len, uint64_t *out, void *stream);

/* Testing hook: keep only the low `bits` (1..64) bits of every key fingerprint (56 or more =
 * all 56, the default) from the next insert on, so that distinct keys share fingerprints and the
 * collision path (GPD_FLOW_COLLISION, gpd_flow_stats.collisions) runs.  Call it on an empty
 * table (after create or reset); a production table never calls it. */
int gpd_flow_test_fingerprint_bits(gpd_flowtable *ft, uint32_t bits);
/* Testing hook: split each record's packed counter word at `bits` (1..57; 40 = the default)
 * instead, so that its byte field carries and its packet field wraps within a test's
 * packets and the exact spill accounting runs.  Call it on an empty table. */
int gpd_flow_test_counter_bits(gpd_flowtable *ft, uint32_t bits);

/* ---- flow-affine sharding over several GPUs ----
 * The reference's fan-out idiom sends every packet of a flow to one worker picked by the
 * flow's FastHash (doc.go:216-228: "flow.FastHash() % numWorkers").  With one table per GPU,
 * each rank turns its decoded packets into 64-byte key records grouped by owning rank
 * (gpd_flow_keys), the ranks exchange them with one all-to-all, and each rank inserts the
 * records it received into its own table (gpd_flow_insert_keys): every flow lives on exactly
 * one rank and both directions of a conversation on the same one.
 * owner = ((NetworkFlow().FastHash() ^ TransportFlow().FastHash()) >> 32) * nparts >> 32
 * (both hashes are direction-symmetric, flows.go:167-174). */
typedef struct gpd_flow_key {
  uint32_t key[10];  /* src[16], dst[16], ports[4] as raw bytes; net_type | tp_type << 8 | addr_len << 16 */
  uint32_t caplen;   /* the packet's captured length */
  uint32_t owner;    /* the rank that owns the flow */
  uint64_t seq;      /* packet sequence number: index_base + the packet's index in its batch */
  uint64_t fp;       /* the key's fingerprint (the table's slot hash) */
} gpd_flow_key;      /* 64 B */

#define GPD_FLOW_MAX_PARTS 1024

/* Key records of every packet of a decoded device batch that has a network + transport pair,
 * grouped by owner: partition p occupies keys[start_p, start_p + part_count[p]) with start_p
 * the sum of the counts below p.  `res` needs hdr_off and either the gpd_record form or status,
 * net_hash and tp_hash (decode without GPD_OPT_NO_FLOW_HASH); `keys` (device) holds in->n records; part_count (host,
 * nparts entries) is filled when the call returns (it synchronises `stream`: the counts size
 * the exchange).  Order within a partition is unspecified.  1 <= nparts <= GPD_FLOW_MAX_PARTS. */
int gpd_flow_keys(gpd_flowtable *ft, const gpd_batch *in, const gpd_result *res, uint32_t nparts,
                  uint64_t index_base, gpd_flow_key *keys, uint64_t *part_count, void *stream);
/* Find-or-create the flow of every key record (device array of n), as gpd_flow_insert does for
 * packets; flow_id[n] receives each record's index in this table (or a GPD_FLOW_* value).
 * Asynchronous on `stream`. */
int gpd_flow_insert_keys(gpd_flowtable *ft, const gpd_flow_key *keys, uint64_t n,
                         uint32_t *flow_id, void *stream);
/* Back on the sending rank: given the m key records it sent (gpd_flow_keys' order) and the flow
 * ids their owners returned for them (ids[j] for keys[j]), fill owner[n] (the owning rank, -1
 * for a packet without a key) and flow_id[n] (the record index on the owner, GPD_FLOW_NONE
 * without a key) for the n packets of the batch.  Device arrays; asynchronous on `stream`. */
int gpd_flow_key_ids(gpd_flowtable *ft, const gpd_flow_key *keys, uint64_t m, const uint32_t *ids,
                     uint64_t index_base, uint64_t n, int32_t *owner, uint32_t *flow_id, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GPD_FLOW_H_ */
