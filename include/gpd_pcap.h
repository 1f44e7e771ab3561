/*
 * gpd_pcap.h — C-ABI of the pcap ingest in front of the batched decoder.
 *
 * The reference reads a capture file one record at a time: pcapgo.NewReader parses the
 * 24-byte file header and every ReadPacketData call parses one 16-byte record header and
 * copies the record's bytes out (pcapgo/read.go:65-177).  Here a capture that is already in
 * memory (a read or mmap'ed file) is indexed in one call — the record walk fills offset /
 * caplen arrays that point INTO the capture buffer — and those arrays are exactly a
 * gpd_batch over the capture bytes: nothing is repacked, and the raw capture bytes are what
 * travel to HBM.
 *
 * Reference interfaces each entry point replaces (paths relative to google/gopacket):
 *   gpd_pcap_header       pcapgo.NewReader / readHeader             pcapgo/read.go:65-117
 *                         (Snaplen(), LinkType(), Resolution()       pcapgo/read.go:183-227)
 *   gpd_pcap_index        the loop `for { data, ci, err := r.ReadPacketData() ... }` over a
 *                         whole capture: ReadPacketData + readPacketHeader
 *                                                                  pcapgo/read.go:120-177
 *   gpd_decode_pcap       that loop feeding DecodingLayerParser.DecodeLayers
 *                         (examples/statsassembly/main.go:171-177, pcap/gopacket_benchmark/
 *                         benchmark.go:226-236): index + H2D of the raw capture bytes +
 *                         gpd_decode + D2H, double-buffered
 *   gpd_host_register     (no reference counterpart) pin a caller buffer so the H2D of
 *                         gpd_decode_pcap reads it in place
 *   gpd_host_bind_local   (no reference counterpart) put a caller buffer's pages on the GPU's
 *                         NUMA node
 *
 * gzip-compressed captures (pcapgo/read.go:79-86) are inflated by the caller (the Python
 * layer does it transparently); the walker sees uncompressed bytes.
 */
#ifndef GPD_PCAP_H_
#define GPD_PCAP_H_
#include "gpd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* pcapgo magics (pcapgo/read.go:47-49, pcapgo/write.go:32) and version (write.go:33-34) */
#define GPD_PCAP_MAGIC_MICRO     0xA1B2C3D4u
#define GPD_PCAP_MAGIC_NANO      0xA1B23C4Du
#define GPD_PCAP_MAGIC_MICRO_BE  0xD4C3B2A1u
#define GPD_PCAP_MAGIC_NANO_BE   0x4D3CB2A1u
#define GPD_PCAP_HEADER_BYTES    24
#define GPD_PCAP_RECORD_BYTES    16

/* Error returned when the walk stops at a record the reference would reject; the reference's
 * error text is in gpd_last_error_string(). */
#define GPD_ERR_PCAP (-5)

/* Why a walk ended (gpd_pcap_index *stop). */
#define GPD_PCAP_STOP_LIMIT     0  /* max_n records were returned; more may follow at *next_pos */
#define GPD_PCAP_STOP_EOF       1  /* clean end: no bytes left where a record header would start (io.EOF) */
#define GPD_PCAP_STOP_SHORT_HDR 2  /* 1..15 bytes left for a record header: "unexpected EOF" */
#define GPD_PCAP_STOP_SNAPLEN   3  /* "capture length exceeds snap length: %d > %d" (read.go:125-127) */
#define GPD_PCAP_STOP_ORIGLEN   4  /* "capture length exceeds original packet length: %d > %d" (read.go:129-131) */
#define GPD_PCAP_STOP_SHORT_DATA 5 /* record data cut short: "unexpected EOF" ("EOF" when no byte is left) */

typedef struct gpd_pcap_info {
  uint32_t magic;          /* as read little-endian from bytes 0..3 */
  uint32_t big_endian;     /* byte order of every header field */
  uint32_t nano;           /* 1: nanosecond timestamps (nanoSecsFactor 1), 0: microseconds (1000) */
  uint32_t version_major;  /* 2 */
  uint32_t version_minor;  /* 4 */
  uint32_t snaplen;        /* Snaplen() */
  uint32_t linktype;       /* LinkType() (1 = Ethernet) */
  uint32_t reserved;
} gpd_pcap_info;

/* readHeader (pcapgo/read.go:78-117) on buf[0:len): GPD_OK, or GPD_ERR_PCAP with the reference's
 * text ("EOF", "unexpected EOF", "Unknown magic %x", "Unknown major version %d", "Unknown minor
 * version %d").  A gzip magic (1f 8b) is reported as GPD_ERR_INVALID: inflate it first. */
int gpd_pcap_header(const uint8_t *buf, uint64_t len, gpd_pcap_info *info);

/* Walk the records of buf[pos:len) as successive ReadPacketData calls would (pcapgo/read.go:
 * 120-137,165-177; pos = 24 for a whole file).  Record i of the walk is returned as
 *   offset[i]  byte offset of its data in buf (record header + 16); < 2^32, so index captures
 *              of more than 4 GiB in windows (pass buf = file + window base)
 *   caplen[i]  CaptureInfo.CaptureLength, wirelen[i] CaptureInfo.Length (may be NULL)
 *   ts_ns[i]   CaptureInfo.Timestamp as Unix nanoseconds, with the reference's uint32
 *              product usec * nanoSecsFactor (read.go:172) (may be NULL)
 * The walk stops after max_n records (*stop = LIMIT, *next_pos = where the next record header
 * starts), at the clean end of the data (EOF), or at the first record the reference rejects:
 * then *n_out counts the records before it, *next_pos is its header position and the call
 * returns GPD_ERR_PCAP with the reference's error text.  nthreads > 1 walks segments of the
 * buffer speculatively in parallel and stitches them where the true walk meets them; the
 * result is identical to the sequential walk for every input (a segment whose speculation
 * never meets the true walk is re-walked sequentially).  nthreads <= 0: the machine's cores,
 * at most 16. */
int gpd_pcap_index(const uint8_t *buf, uint64_t len, const gpd_pcap_info *info, uint64_t pos,
                   uint64_t max_n, uint32_t *offset, uint32_t *caplen, uint32_t *wirelen,
                   uint64_t *ts_ns, uint64_t *n_out, uint64_t *next_pos, int *stop, int nthreads);

/* Index + decode a whole in-memory capture with the context's parser: the raw capture bytes
 * are copied host -> device in 64 MiB chunks as they lie in the capture (through pinned
 * staging, or directly when buf lies in memory registered with gpd_host_register), the
 * records are found in HBM by a parallel walk on the device (gpd_pcapwalk.hip), decoded where
 * they lie, and the results copied back, with two chunks in flight.  Wherever the device walk
 * cannot vouch for the records (a record the reference rejects, a capture ending inside a
 * record, a speculation its stitch refutes), the host walk (as gpd_pcap_index, nthreads as
 * there) takes over from that chunk, so results, counts, stops and error texts are always the
 * sequential reader's (gpd_tuning.device_walk = 0 selects the host walk throughout).
 * `out` holds host arrays of max_n entries (status and layers required, the rest optional;
 * ext and records not supported).  Returns like gpd_pcap_index: the records before a
 * rejected one are decoded and counted in *n_out.  The host walk's record index (12 B per
 * record) is kept per calling thread and reused by the next call, so that a replay or
 * capture loop touches no fresh pages. */
int gpd_decode_pcap(gpd_ctx *ctx, const uint8_t *buf, uint64_t len, uint64_t max_n,
                    const gpd_result *out, uint64_t *n_out, uint64_t *next_pos, int *stop,
                    int nthreads);

/* gpd_decode_pcap continued from record header position `pos` of a capture whose file header
 * `info` was already parsed (gpd_pcap_header): the next max_n ReadPacketData records of the
 * loop are decoded exactly as gpd_decode_pcap decodes them, and *next_pos tells where the
 * following call continues.  This is the loop over a capture too large for one call (a
 * replay streamed in chunks of records), and the loop over one shard of a capture: a shard's
 * first record position comes from gpd_pcap_locate.  buf may exceed 4 GiB. */
int gpd_decode_pcap_at(gpd_ctx *ctx, const uint8_t *buf, uint64_t len, const gpd_pcap_info *info,
                       uint64_t pos, uint64_t max_n, const gpd_result *out, uint64_t *n_out,
                       uint64_t *next_pos, int *stop, int nthreads);

/* Record positions without indexing: the ReadPacketData loop from `pos` with every record
 * read and dropped.  targets[0..k) are record numbers of that walk (0 = the record at pos),
 * ascending; pos_out[t] is the header position of record targets[t] (a target equal to the
 * walk's record count gives the position where the walk ends).  *n_total (may be NULL) is
 * the number of records the walk reads before its end (EOF or the first rejected record,
 * whose kind goes to *stop, may be NULL).  A target beyond *n_total is GPD_ERR_INVALID.
 * This is how a capture is cut by packet index into shards [g*N/G, (g+1)*N/G) (one shard
 * per GPU) with one parallel counting pass (nthreads as gpd_pcap_index) and no
 * per-record arrays. */
int gpd_pcap_locate(const uint8_t *buf, uint64_t len, const gpd_pcap_info *info, uint64_t pos,
                    const uint64_t *targets, uint64_t k, uint64_t *pos_out, uint64_t *n_total, int *stop,
                    int nthreads);

/* Diagnostics: host-clock phases (ms) of this thread's last gpd_decode_pcap(_at) call: total,
 * record walks, waiting for a walk running ahead, staging and issuing, waiting for slots,
 * copying results out. */
void gpd_decode_pcap_last_times(double *ms6);

/* Diagnostics: this thread's last gpd_decode_pcap(_at) call's device-walk chunks — [0] walked,
 * [1] handed to the host walk, and of those [2] a speculation the stitch could not correct,
 * [3] a record the reader rejects (or one cut by the chunk's bytes), [4] a true record header
 * no segment's walk covered, [5] a walk that ends short of the chunk; [6] 2-KiB segments the
 * stitch re-walked from the true walk's position (a refuted speculation, corrected there). */
void gpd_decode_pcap_last_walk_counts(uint32_t *c7);
/* ... and where its last refuted speculation started and the 2-KiB segment it walked (buffer
 * positions; UINT64_MAX when none). */
void gpd_decode_pcap_last_walk_miss(uint64_t *pos2);

/* Diagnostics of this thread's last walk: segments walked in parallel, segments whose
 * speculation the true walk met, segments re-walked sequentially. */
void gpd_pcap_last_stats(int *threads, int *met, int *rewalks);

/* Pin / unpin host memory for in-place H2D (hipHostRegister on the context's device). */
int gpd_host_register(gpd_ctx *ctx, const void *ptr, uint64_t len);
int gpd_host_unregister(gpd_ctx *ctx, const void *ptr);

/* Place host memory on the NUMA node of device `device`'s PCI function (mbind, preferred
 * policy, over the whole pages of [ptr, ptr + len); pages already placed elsewhere move).  A
 * capture buffer there reaches the GPU without crossing the link between sockets; bound before
 * its pages are first written, nothing moves.  *node (may be NULL): the node, or -1 when the
 * platform names none (then nothing is done and GPD_OK is returned). */
int gpd_host_bind_local(int device, void *ptr, uint64_t len, int *node);

#ifdef __cplusplus
}
#endif
#endif /* GPD_PCAP_H_ */
