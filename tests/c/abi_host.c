/*
 * abi_host.c — TEST DRIVER: a plain C host program on the C-ABI (what the cgo binding in
 * go/gpdecode does), with no Python or PyTorch in the process, so libgpd.so runs on
 * /opt/rocm's HIP runtime exactly as it would under Go.
 *
 *   abi_host BATCH_FILE [ERR_OUT PROTO_NAMES]
 *
 * BATCH_FILE: u64 data_len, u64 n, u32 decoders, u32 options, data[data_len], u32 offset[n],
 * u32 caplen[n].  The batch is decoded three ways and every output word is compared:
 *   1. gpd_decode on device buffers (hipMalloc + hipMemcpy, the caller's own stream),
 *   2. gpd_decode_host (host arrays, pinned double-buffered staging inside the library),
 *   3. the CPU oracle (oracle/libgpd_oracle.so, test infrastructure) as the checker,
 *   4. gpd_decode_pcap over an in-memory pcap file holding the same packets (records at
 *      unaligned offsets, raw capture bytes sent to HBM),
 * and then the device results feed the flow table (gpd_flow_insert on the caller's stream):
 * every packet's flow record must hold exactly the key bytes at the packet's hdr_off
 * positions, the per-record packet/byte/first/last counters must match a recount, records
 * must have pairwise distinct keys, and gpd_flow_stats must add up.  Last, the fragment
 * hand-off (gpd_ip4_fragments) over the same device results: its records must be exactly the
 * packets whose last network layer is an IPv4 header with MoreFragments or an offset and no
 * DF, in packet order, with the key and fields of those header bytes and the securityChecks
 * verdict (ip4defrag/defrag.go:162-198) recomputed here.
 * Every path also fills the gpd_detail array (gpd.h): for each packet with a decode error or
 * more than 12 layers it must equal the oracle's ext prefix (decoded list, error arguments) in
 * all three paths.  With ERR_OUT, the error value DecodeLayers returns (parser.go:302-326) is
 * rebuilt from the device's status + detail words alone — the reference's format strings, with
 * IPProtocol.String() names read from PROTO_NAMES (256 lines) — and written as "i<TAB>text"
 * lines, one per failing packet, for the Python test to compare with the oracle's texts.
 * Prints "abi_host ok N F R" (F = flows, R = fragments) and exits 0 when everything agrees.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "../../include/gpd.h"
#include "../../include/gpd_defrag.h"
#include "../../include/gpd_flow.h"
#include "../../include/gpd_pcap.h"
#include "../../oracle/gpd_oracle.h"

#define CHECK(x)                                                                    \
  do {                                                                              \
    int rc_ = (x);                                                                  \
    if (rc_ != 0) {                                                                 \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_,         \
              gpd_last_error_string());                                             \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)
#define HCHECK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)

typedef struct {
  uint32_t *status, *csum, *hdr_off;
  uint64_t *layers, *net_hash, *tp_hash;
  gpd_detail *detail;
} res_t;

static res_t res_alloc(uint64_t n) {
  res_t r;
  r.status = calloc(n, 4);
  r.csum = calloc(n, 4);
  r.hdr_off = calloc(n, 4);
  r.layers = calloc(n, 8);
  r.net_hash = calloc(n, 8);
  r.tp_hash = calloc(n, 8);
  r.detail = calloc(n + 1, sizeof(gpd_detail));
  return r;
}

/* gpd.h gpd_detail: written for decode errors and stacks deeper than the core word */
static int has_detail(uint32_t st) {
  return GPD_STATUS_CLASS(st) == GPD_ST_DECODE_ERROR || GPD_STATUS_NLAYERS(st) > GPD_CORE_MAX_LAYERS ||
         GPD_STATUS_SATURATED(st);
}

/* the detail records of `a` vs the oracle's ext records (their first 24 bytes: same layout) */
static int detail_cmp(const char *what, const res_t *a, const gpd_ext_rec *ext, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) {
    if (!has_detail(a->status[i])) continue;
    const gpd_detail *d = &a->detail[i];
    if (d->layer_codes[0] != ext[i].layer_codes[0] || d->layer_codes[1] != ext[i].layer_codes[1] ||
        d->err_arg0 != ext[i].err_arg0 || d->err_arg1 != ext[i].err_arg1) {
      fprintf(stderr, "%s: packet %llu detail differs: codes %016llx %016llx/%016llx %016llx args %u %u/%u %u\n",
              what, (unsigned long long)i, (unsigned long long)d->layer_codes[0],
              (unsigned long long)d->layer_codes[1], (unsigned long long)ext[i].layer_codes[0],
              (unsigned long long)ext[i].layer_codes[1], d->err_arg0, d->err_arg1, ext[i].err_arg0,
              ext[i].err_arg1);
      return 1;
    }
  }
  return 0;
}

/* The error text of enum gpd_err `code` with the detail record's arguments: the format string
 * at each `return ...error` site of the reference (the file:line list is in gpd.h). */
static void error_text(char *out, size_t cap, uint32_t code, uint32_t a0, uint32_t a1, char names[256][64]) {
  switch (code) {
    case 1: snprintf(out, cap, "Ethernet packet too small"); break;
    case 2: snprintf(out, cap, "802.1Q tag length %u too short", a0); break;
    case 3: snprintf(out, cap, "Invalid ip4 header. Length %u less than 20", a0); break;
    case 4: snprintf(out, cap, "Invalid (too small) IP length (%u < 20)", a0); break;
    case 5: snprintf(out, cap, "Invalid (too small) IP header length (%u < 5)", a0); break;
    case 6: snprintf(out, cap, "Invalid IP header length > IP length (%u > %u)", a0, a1); break;
    case 7: snprintf(out, cap, "Not all IP header bytes available"); break;
    case 8: snprintf(out, cap, "Invalid ip4 option length. Length %u less than 2", a0); break;
    case 9: snprintf(out, cap, "IP option length exceeds remaining IP header size, option type %u length %u", a0, a1); break;
    case 10: snprintf(out, cap, "Invalid IP option type %u length %u. Must be greater than 2", a0, a1); break;
    case 11: snprintf(out, cap, "Invalid ip6 header. Length %u less than 40", a0); break;
    case 12: snprintf(out, cap, "Invalid ip6-extension header. Length %u less than 2", a0); break;
    case 13: snprintf(out, cap, "Invalid ip6-extension header. Length %u less than specified length %u", a0, a1); break;
    case 14: snprintf(out, cap, "IPv6 header option too small"); break;
    case 15: snprintf(out, cap, "IPv6 header TLV option too small"); break;
    case 16: snprintf(out, cap, "Jumbo length TLV data must have length 4"); break;
    case 17: snprintf(out, cap, "Jumbo length cannot be less than 65536"); break;
    case 18: snprintf(out, cap, "IPv6 has jumbo length and IPv6 length is not 0"); break;
    case 19: snprintf(out, cap, "IPv6 length 0, but HopByHop header does not have jumbogram option"); break;
    case 20: snprintf(out, cap, "IPv6 length 0, but next header is %s, not HopByHop", names[a0 & 255]); break;
    case 21: snprintf(out, cap, "Invalid TCP header. Length %u less than 20", a0); break;
    case 22: snprintf(out, cap, "Invalid TCP data offset %u < 5", a0); break;
    case 23: snprintf(out, cap, "TCP data offset greater than packet length"); break;
    case 24: snprintf(out, cap, "Invalid TCP option length. Length %u less than 2", a0); break;
    case 25: snprintf(out, cap, "Invalid TCP option length %u < 2", a0); break;
    case 26: snprintf(out, cap, "Invalid TCP option length %u exceeds remaining %u bytes", a0, a1); break;
    case 27: snprintf(out, cap, "Invalid UDP header. Length %u less than 8", a0); break;
    case 28: snprintf(out, cap, "UDP packet too small: %u bytes", a0); break;
    case 29: snprintf(out, cap, "vxlan packet too small"); break;
    case 30: snprintf(out, cap, "ICMP layer less then 8 bytes for ICMPv4 packet"); break;
    case 31: snprintf(out, cap, "LLC header too small"); break;
    default: snprintf(out, cap, "gpd: unknown error code %u", code); break;
  }
}

static int res_cmp(const char *what, const res_t *a, const res_t *b, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) {
    if (a->status[i] != b->status[i] || a->layers[i] != b->layers[i] ||
        a->net_hash[i] != b->net_hash[i] || a->tp_hash[i] != b->tp_hash[i] ||
        a->csum[i] != b->csum[i] || a->hdr_off[i] != b->hdr_off[i]) {
      fprintf(stderr,
              "%s: packet %llu differs: status %08x/%08x layers %016llx/%016llx net %016llx/%016llx "
              "tp %016llx/%016llx csum %08x/%08x\n",
              what, (unsigned long long)i, a->status[i], b->status[i],
              (unsigned long long)a->layers[i], (unsigned long long)b->layers[i],
              (unsigned long long)a->net_hash[i], (unsigned long long)b->net_hash[i],
              (unsigned long long)a->tp_hash[i], (unsigned long long)b->tp_hash[i], a->csum[i],
              b->csum[i]);
      return 1;
    }
  }
  return 0;
}

/* Key of packet i as the flow table stores it (gpd_flow.h): network endpoints at the
 * network-layer offset, ports at the transport offset. */
static int key_matches(const gpd_flow_rec *r, const uint8_t *pkt, uint32_t hoff) {
  const uint32_t no = GPD_HDR_NET(hoff), to = GPD_HDR_TP(hoff);
  if (no == GPD_HDR_NONE || to == GPD_HDR_NONE) return 0;
  const uint8_t *src = r->addr_len == 4 ? pkt + no + 12 : pkt + no + 8;
  const uint8_t *dst = src + r->addr_len;
  return memcmp(r->src, src, r->addr_len) == 0 && memcmp(r->dst, dst, r->addr_len) == 0 &&
         memcmp(r->sport, pkt + to, 2) == 0 && memcmp(r->dport, pkt + to + 2, 2) == 0;
}

static int rec_key_cmp(const void *a, const void *b) {
  const gpd_flow_rec *x = a, *y = b;
  /* compare every key field: types, length, addresses, ports (fields are contiguous) */
  return memcmp(x->src, y->src, offsetof(gpd_flow_rec, reserved) - offsetof(gpd_flow_rec, src));
}

static int check_flows(gpd_ctx *ctx, hipStream_t s, const gpd_batch *db, const gpd_result *dr,
                       const uint8_t *data, const uint32_t *off, const uint32_t *cap,
                       const uint32_t *hdr_off, uint64_t n, uint64_t *flows_out) {
  gpd_flowtable *ft = NULL;
  CHECK(gpd_flow_create(ctx, 2 * n + 64, &ft));
  uint32_t *d_id, *id = malloc(4 * n + 4);
  HCHECK(hipMalloc((void **)&d_id, 4 * n + 4));
  CHECK(gpd_flow_insert(ft, db, dr, d_id, 1000, s));
  gpd_flow_stats st;
  CHECK(gpd_flow_stats_get(ft, &st, s));
  HCHECK(hipMemcpy(id, d_id, 4 * n, hipMemcpyDeviceToHost));
  gpd_flow_rec *rec = calloc(st.flows + 1, sizeof *rec);
  uint32_t *ridx = calloc(st.flows + 1, 4);
  uint64_t nrec = 0;
  CHECK(gpd_flow_export(ft, rec, ridx, st.flows, &nrec, s));
  int bad = nrec != st.flows || st.full != 0 || st.collisions != 0;
  /* record index -> export slot */
  uint64_t *pk = calloc(nrec + 1, 8), *by = calloc(nrec + 1, 8), *lo = calloc(nrec + 1, 8),
           *hi = calloc(nrec + 1, 8);
  uint64_t assigned = 0, none = 0, *one = calloc(nrec + 1, 8);  /* a packet of each record */
  for (uint64_t i = 0; i < n && !bad; i++) {
    if (id[i] == GPD_FLOW_NONE) {
      none++;
      continue;
    }
    uint64_t k = 0;
    while (k < nrec && ridx[k] != id[i]) k++;
    if (k == nrec || !key_matches(&rec[k], data + off[i], hdr_off[i])) {
      fprintf(stderr, "flow: packet %llu id %u has no matching record\n", (unsigned long long)i, id[i]);
      bad = 1;
      break;
    }
    const uint64_t seq = 1000 + i;
    if (pk[k] == 0) one[k] = i;
    if (pk[k] == 0 || seq < lo[k]) lo[k] = seq;
    if (pk[k] == 0 || seq > hi[k]) hi[k] = seq;
    pk[k]++;
    by[k] += cap[i];
    assigned++;
  }
  for (uint64_t k = 0; k < nrec && !bad; k++)
    if (rec[k].packets != pk[k] || rec[k].bytes != by[k] || rec[k].first != lo[k] ||
        rec[k].last != hi[k]) {
      fprintf(stderr, "flow: record %u counters differ\n", ridx[k]);
      bad = 1;
    }
  /* gpd_fast_hash (ABI 9) of the records' network flows, rebuilt from their exported keys as
   * NewFlow would hold them: each must equal the decode's NetworkFlow FastHash of its packets */
  if (!bad && nrec > 0) {
    int64_t *typ = calloc(nrec, 8);
    uint8_t *raw = calloc(nrec, 32), *len = calloc(nrec, 2);
    uint64_t *fh = calloc(nrec, 8), *nh = malloc(8 * n);
    for (uint64_t k = 0; k < nrec; k++) {
      typ[k] = rec[k].net_type;
      memcpy(raw + 16 * k, rec[k].src, rec[k].addr_len);
      memcpy(raw + 16 * (nrec + k), rec[k].dst, rec[k].addr_len);
      len[k] = len[nrec + k] = rec[k].addr_len;
    }
    void *d_typ, *d_raw, *d_len, *d_fh;
    HCHECK(hipMalloc(&d_typ, 8 * nrec));
    HCHECK(hipMalloc(&d_raw, 32 * nrec));
    HCHECK(hipMalloc(&d_len, 2 * nrec));
    HCHECK(hipMalloc(&d_fh, 8 * nrec));
    HCHECK(hipMemcpy(d_typ, typ, 8 * nrec, hipMemcpyHostToDevice));
    HCHECK(hipMemcpy(d_raw, raw, 32 * nrec, hipMemcpyHostToDevice));
    HCHECK(hipMemcpy(d_len, len, 2 * nrec, hipMemcpyHostToDevice));
    int dev = 0;
    HCHECK(hipGetDevice(&dev));
    CHECK(gpd_fast_hash(dev, nrec, d_typ, d_raw, d_len, (uint8_t *)d_raw + 16 * nrec, (uint8_t *)d_len + nrec,
                        d_fh, s));
    HCHECK(hipStreamSynchronize(s));
    HCHECK(hipMemcpy(fh, d_fh, 8 * nrec, hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(nh, dr->net_hash, 8 * n, hipMemcpyDeviceToHost));
    for (uint64_t k = 0; k < nrec && !bad; k++)
      if (fh[k] != nh[one[k]]) {
        fprintf(stderr, "flow: gpd_fast_hash of record %u differs from its packets' net hash\n", ridx[k]);
        bad = 1;
      }
    HCHECK(hipFree(d_typ));
    HCHECK(hipFree(d_raw));
    HCHECK(hipFree(d_len));
    HCHECK(hipFree(d_fh));
    free(typ), free(raw), free(len), free(fh), free(nh);
  }
  if (!bad) {
    qsort(rec, nrec, sizeof *rec, rec_key_cmp);
    for (uint64_t k = 1; k < nrec; k++)
      if (rec_key_cmp(&rec[k - 1], &rec[k]) == 0) {
        fprintf(stderr, "flow: two records hold one key\n");
        bad = 1;
      }
  }
  if (!bad && (st.packets != assigned || st.no_key != none)) {
    fprintf(stderr, "flow: stats packets %llu/%llu no_key %llu/%llu\n",
            (unsigned long long)st.packets, (unsigned long long)assigned,
            (unsigned long long)st.no_key, (unsigned long long)none);
    bad = 1;
  }
  *flows_out = nrec;
  CHECK(gpd_flow_destroy(ft));
  HCHECK(hipFree(d_id));
  free(id), free(rec), free(ridx), free(pk), free(by), free(lo), free(hi), free(one);
  return bad;
}

/* The batch as a little-endian microsecond pcap file (pcapgo/write.go:32-34 header). */
static uint8_t *make_pcap(const uint8_t *data, const uint32_t *off, const uint32_t *cap,
                          uint64_t n, uint64_t *len) {
  uint64_t total = GPD_PCAP_HEADER_BYTES, snap = 0;
  for (uint64_t i = 0; i < n; i++) {
    total += GPD_PCAP_RECORD_BYTES + cap[i];
    if (cap[i] > snap) snap = cap[i];
  }
  uint8_t *b = calloc(total + 64, 1);
  const uint32_t h[6] = {GPD_PCAP_MAGIC_MICRO, 2 | (4u << 16), 0, 0, (uint32_t)snap + 1, 1};
  memcpy(b, h, 24);
  uint64_t p = GPD_PCAP_HEADER_BYTES;
  for (uint64_t i = 0; i < n; i++) {
    const uint32_t r[4] = {(uint32_t)i, 7, cap[i], cap[i]};
    memcpy(b + p, r, 16);
    memcpy(b + p + 16, data + off[i], cap[i]);
    p += 16 + cap[i];
  }
  *len = total;
  return b;
}

/* gpd_ip4_fragments vs a recount from the oracle's status / header-offset words and the bytes */
static int check_fragments(gpd_ctx *ctx, hipStream_t s, const gpd_batch *db, const gpd_result *dr,
                           const uint8_t *data, const uint32_t *off, const uint32_t *cap,
                           const uint32_t *status, const uint32_t *hdr_off, uint64_t n, uint64_t *nfrag) {
  gpd_ip4_frag *d_out = NULL;
  HCHECK(hipMalloc((void **)&d_out, sizeof(gpd_ip4_frag) * (n + 1)));
  uint64_t cnt = 0;
  CHECK(gpd_ip4_fragments(ctx, db, dr, d_out, n, &cnt, s));
  gpd_ip4_frag *fr = calloc(cnt + 1, sizeof(gpd_ip4_frag));
  HCHECK(hipMemcpy(fr, d_out, sizeof(gpd_ip4_frag) * cnt, hipMemcpyDeviceToHost));
  HCHECK(hipFree(d_out));
  uint64_t k = 0;
  int bad = 0;
  for (uint64_t i = 0; i < n && !bad; i++) {
    const uint32_t net = GPD_HDR_NET(hdr_off[i]);
    if (GPD_STATUS_NET_EPT(status[i]) != 1 || net == GPD_HDR_NONE) continue;
    const uint8_t *h = data + off[i] + net;
    const uint32_t ff = ((uint32_t)h[6] << 8) | h[7], flags = ff >> 13, fo = ff & 0x1FFF;
    if ((flags & 2) || (!(flags & 1) && fo == 0)) continue; /* dontDefrag */
    if (k >= cnt) { fprintf(stderr, "fragments: packet %llu missing\n", (unsigned long long)i); bad = 1; break; }
    const gpd_ip4_frag *r = &fr[k++];
    const uint32_t raw = ((uint32_t)h[2] << 8) | h[3], ihl = h[0] & 15u;
    const uint32_t id = ((uint32_t)h[4] << 8) | h[5];
    int ok = r->packet == i && r->net_off == net && memcmp(r->src, h + 12, 4) == 0 &&
             memcmp(r->dst, h + 16, 4) == 0 && r->id == id && r->frag_offset == fo && r->flags == flags &&
             r->ihl == ihl && net + 4 * ihl + r->payload_len <= cap[i];
    if (raw) {
      const uint16_t size = (uint16_t)(raw - 4 * ihl);
      const uint32_t v = size < 8 ? GPD_FRAG_TOO_SMALL : fo > 8183 ? GPD_FRAG_OFFSET : GPD_FRAG_INSERT;
      ok = ok && r->length == raw && r->verdict == v;
    }
    if (!ok) {
      fprintf(stderr, "fragments: record %llu (packet %llu) disagrees\n", (unsigned long long)(k - 1),
              (unsigned long long)i);
      bad = 1;
    }
  }
  if (!bad && k != cnt) {
    fprintf(stderr, "fragments: %llu records, %llu expected\n", (unsigned long long)cnt, (unsigned long long)k);
    bad = 1;
  }
  free(fr);
  *nfrag = cnt;
  return bad;
}

/* ABI 8: a context reconfigured in place keeps its tables and device, as the reference parser
 * keeps the global tables when IgnoreUnsupported is assigned (parser.go:182-195,336-350) and
 * AddDecodingLayer only adds a decoder (parser.go:197-202).  A UDP port is registered as VXLAN
 * (layers/ports.go:126-128) and the tables reloaded; VXLAN is added afterwards; then
 * IgnoreUnsupported is flipped both ways; every step decodes host and device batches against the
 * oracle on the same mutated tables.  Also: an all-empty batch, and unknown option bits. */
static int check_reconfig(const gpd_config *base, const uint8_t *data, uint64_t data_len,
                          const uint32_t *off, const uint32_t *cap, uint64_t n, const gpd_batch *db,
                          const gpd_result *dr, hipStream_t s, uint16_t vxlan_port, uint64_t *vx_out) {
  uint16_t *et = malloc(65536 * 2), *ip = malloc(256 * 2), *tp = malloc(65536 * 2),
           *up = malloc(65536 * 2);
  gpd_default_tables(et, ip, tp, up);
  up[vxlan_port] = GPD_LT_VXLAN;
  gpd_config cfg = *base;
  cfg.decoders = base->decoders & ~GPD_DEC_VXLAN;
  gpd_ctx *ctx = NULL;
  CHECK(gpd_ctx_create(0, &cfg, &ctx));
  cfg.ethertype = et, cfg.ipproto = ip, cfg.tcp_port = tp, cfg.udp_port = up;
  CHECK(gpd_ctx_reload_tables(ctx, &cfg));
  CHECK(gpd_ctx_add_decoders(ctx, base->decoders & GPD_DEC_VXLAN));
  int bad = 0;
  /* every bit outside the four GPD_OPT_* is refused: the runtime's launch flags (24-29) and the
   * diagnostic library's ablation bits (30: no DMA wait, 31: no decode) included */
  for (int b = 0; b < 32; b++) {
    const uint32_t bit = 1u << b;
    if (bit & (GPD_OPT_IGNORE_UNSUPPORTED | GPD_OPT_IGNORE_PANIC | GPD_OPT_NO_CHECKSUMS | GPD_OPT_NO_FLOW_HASH))
      continue;
    gpd_config bc = *base;
    gpd_ctx *bx = NULL;
    bc.options = base->options | bit;
    if (gpd_ctx_set_options(ctx, base->options | bit) != GPD_ERR_INVALID ||
        gpd_ctx_create(0, &bc, &bx) != GPD_ERR_INVALID || bx != NULL) {
      fprintf(stderr, "reconfig: option bit %d accepted\n", b);
      if (bx) gpd_ctx_destroy(bx);
      bad = 1;
    }
  }
  res_t hv = res_alloc(n), dv = res_alloc(n), ov = res_alloc(n);
  gpd_ext_rec *oext = calloc(n + 1, sizeof(gpd_ext_rec));
  gpo_tables t = {et, ip, tp, up};
  const uint32_t opts[3] = {base->options ^ GPD_OPT_IGNORE_UNSUPPORTED, base->options,
                            base->options ^ GPD_OPT_IGNORE_UNSUPPORTED};
  uint64_t vx = 0;
  for (int k = 0; k < 3 && !bad; k++) {
    CHECK(gpd_ctx_set_options(ctx, opts[k]));
    gpd_batch hb = {data, data_len, off, cap, n};
    gpd_result hr = {hv.status, hv.layers, hv.net_hash, hv.tp_hash, hv.csum, NULL, hv.hdr_off, NULL, hv.detail};
    CHECK(gpd_decode_host(ctx, &hb, &hr));
    CHECK(gpd_decode(ctx, db, dr, s));
    CHECK(gpd_sync(ctx, s));
    HCHECK(hipMemcpy(dv.status, dr->status, 4 * n, hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(dv.layers, dr->layers, 8 * n, hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(dv.net_hash, dr->net_hash, 8 * n, hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(dv.tp_hash, dr->tp_hash, 8 * n, hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(dv.csum, dr->csum, 4 * n, hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(dv.hdr_off, dr->hdr_off, 4 * n, hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(dv.detail, dr->detail, sizeof(gpd_detail) * n, hipMemcpyDeviceToHost));
    gpo_decode_batch(data, off, cap, n, GPD_LT_ETHERNET, base->decoders, opts[k], &t, ov.status,
                     ov.layers, ov.net_hash, ov.tp_hash, ov.csum, ov.hdr_off, oext, 8);
    bad |= res_cmp("reconfig host vs oracle", &hv, &ov, n) | res_cmp("reconfig device vs oracle", &dv, &ov, n);
    if (!bad) bad |= detail_cmp("reconfig detail", &hv, oext, n) | detail_cmp("reconfig detail", &dv, oext, n);
  }
  for (uint64_t i = 0; i < n; i++)  /* packets that reached the registered port's VXLAN decoder */
    for (uint32_t j = 0; j < GPD_STATUS_NLAYERS(ov.status[i]) && j < GPD_CORE_MAX_LAYERS; j++)
      if (GPD_LAYERS_CODE(ov.layers[i], j) == GPD_C_VXLAN) { vx++; break; }
  if (!bad && (base->decoders & GPD_DEC_VXLAN) && vx == 0) {
    fprintf(stderr, "reconfig: no packet decoded VXLAN on the registered port\n");
    bad = 1;
  }
  /* SetDecodingLayerContainer: the set replaced in place (VXLAN and Payload dropped) */
  if (!bad) {
    const uint32_t dec2 = base->decoders & ~(GPD_DEC_VXLAN | GPD_DEC_PAYLOAD);
    CHECK(gpd_ctx_set_decoders(ctx, dec2));
    gpd_batch hb = {data, data_len, off, cap, n};
    gpd_result hr = {hv.status, hv.layers, hv.net_hash, hv.tp_hash, hv.csum, NULL, hv.hdr_off, NULL, hv.detail};
    CHECK(gpd_decode_host(ctx, &hb, &hr));
    gpo_decode_batch(data, off, cap, n, GPD_LT_ETHERNET, dec2, opts[2], &t, ov.status, ov.layers,
                     ov.net_hash, ov.tp_hash, ov.csum, ov.hdr_off, oext, 8);
    bad |= res_cmp("set_decoders host vs oracle", &hv, &ov, n);
    if (!bad) bad |= detail_cmp("set_decoders detail", &hv, oext, n);
    CHECK(gpd_ctx_set_decoders(ctx, base->decoders));
  }
  /* a batch of empty packets (every CapLen 0, no data) */
  if (!bad) {
    const uint64_t m = 7;
    uint32_t z_off[7] = {0}, z_cap[7] = {0};
    uint8_t z_data[64] = {0};
    res_t zv = res_alloc(m), zo = res_alloc(m);
    gpd_batch zb = {z_data, 0, z_off, z_cap, m};
    gpd_result zr = {zv.status, zv.layers, zv.net_hash, zv.tp_hash, zv.csum, NULL, zv.hdr_off, NULL, zv.detail};
    CHECK(gpd_decode_host(ctx, &zb, &zr));
    gpo_decode_batch(z_data, z_off, z_cap, m, GPD_LT_ETHERNET, base->decoders, opts[2], &t,
                     zo.status, zo.layers, zo.net_hash, zo.tp_hash, zo.csum, zo.hdr_off, oext, 1);
    bad |= res_cmp("empty batch vs oracle", &zv, &zo, m);
  }
  CHECK(gpd_ctx_destroy(ctx));
  free(et), free(ip), free(tp), free(up), free(oext);
  *vx_out = vx;
  return bad;
}

int main(int argc, char **argv) {
  if (argc != 2 && argc != 4 && argc != 5) {
    fprintf(stderr, "usage: %s BATCH_FILE [ERR_OUT PROTO_NAMES [VXLAN_PORT]]\n", argv[0]);
    return 2;
  }
  FILE *f = fopen(argv[1], "rb");
  if (!f) { perror(argv[1]); return 2; }
  uint64_t hdr[2];
  uint32_t cfgw[2];
  if (fread(hdr, 8, 2, f) != 2 || fread(cfgw, 4, 2, f) != 2) return 2;
  const uint64_t data_len = hdr[0], n = hdr[1];
  const uint64_t alloc = ((data_len + 15) & ~15ull) + 64;  /* gpd.h: readable to round_up + pad */
  uint8_t *data = aligned_alloc(16, alloc);
  uint32_t *off = malloc(4 * n + 4), *cap = malloc(4 * n + 4);
  memset(data, 0, alloc);
  if (fread(data, 1, data_len, f) != data_len || fread(off, 4, n, f) != n ||
      fread(cap, 4, n, f) != n) {
    fprintf(stderr, "short batch file\n");
    return 2;
  }
  fclose(f);

  gpd_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.first_layer = GPD_LT_ETHERNET;
  cfg.decoders = cfgw[0];
  cfg.options = cfgw[1];
  gpd_ctx *ctx = NULL;
  CHECK(gpd_ctx_create(0, &cfg, &ctx));

  /* 1. device-resident batch on the caller's stream */
  res_t dv = res_alloc(n);
  void *d_data, *d_off, *d_cap, *d_st, *d_ly, *d_nh, *d_th, *d_cs, *d_ho, *d_dt;
  hipStream_t s;
  HCHECK(hipStreamCreate(&s));
  HCHECK(hipMalloc(&d_data, alloc));
  HCHECK(hipMalloc(&d_off, 4 * n + 4));
  HCHECK(hipMalloc(&d_cap, 4 * n + 4));
  HCHECK(hipMalloc(&d_st, 4 * n + 4));
  HCHECK(hipMalloc(&d_ly, 8 * n + 8));
  HCHECK(hipMalloc(&d_nh, 8 * n + 8));
  HCHECK(hipMalloc(&d_th, 8 * n + 8));
  HCHECK(hipMalloc(&d_cs, 4 * n + 4));
  HCHECK(hipMalloc(&d_ho, 4 * n + 4));
  HCHECK(hipMalloc(&d_dt, sizeof(gpd_detail) * (n + 1)));
  HCHECK(hipMemcpy(d_data, data, alloc, hipMemcpyHostToDevice));
  HCHECK(hipMemcpy(d_off, off, 4 * n, hipMemcpyHostToDevice));
  HCHECK(hipMemcpy(d_cap, cap, 4 * n, hipMemcpyHostToDevice));
  gpd_batch db = {(const uint8_t *)d_data, data_len, (const uint32_t *)d_off,
                  (const uint32_t *)d_cap, n};
  gpd_result dr = {(uint32_t *)d_st, (uint64_t *)d_ly, (uint64_t *)d_nh, (uint64_t *)d_th,
                   (uint32_t *)d_cs, NULL, (uint32_t *)d_ho, NULL, (gpd_detail *)d_dt};
  CHECK(gpd_decode(ctx, &db, &dr, s));
  CHECK(gpd_sync(ctx, s));
  HCHECK(hipMemcpy(dv.status, d_st, 4 * n, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(dv.layers, d_ly, 8 * n, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(dv.net_hash, d_nh, 8 * n, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(dv.tp_hash, d_th, 8 * n, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(dv.csum, d_cs, 4 * n, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(dv.hdr_off, d_ho, 4 * n, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(dv.detail, d_dt, sizeof(gpd_detail) * n, hipMemcpyDeviceToHost));

  /* 2. host batch through the library's pinned pipeline */
  res_t hv = res_alloc(n);
  gpd_batch hb = {data, data_len, off, cap, n};
  gpd_result hr = {hv.status, hv.layers, hv.net_hash, hv.tp_hash, hv.csum, NULL, hv.hdr_off, NULL, hv.detail};
  CHECK(gpd_decode_host(ctx, &hb, &hr));

  /* 3. the oracle */
  res_t ov = res_alloc(n);
  gpd_ext_rec *oext = calloc(n + 1, sizeof(gpd_ext_rec));
  uint16_t *et = malloc(65536 * 2), *ip = malloc(256 * 2), *tp = malloc(65536 * 2),
           *up = malloc(65536 * 2);
  gpd_default_tables(et, ip, tp, up);
  gpo_tables t = {et, ip, tp, up};
  gpo_decode_batch(data, off, cap, n, GPD_LT_ETHERNET, cfg.decoders, cfg.options, &t, ov.status,
                   ov.layers, ov.net_hash, ov.tp_hash, ov.csum, ov.hdr_off, oext, 8);

  /* 4. the same packets as a pcap capture */
  res_t pv = res_alloc(n);
  uint64_t plen = 0, pn = 0, pnext = 0;
  int pstop = -1;
  uint8_t *cap_file = make_pcap(data, off, cap, n, &plen);
  gpd_result pr = {pv.status, pv.layers, pv.net_hash, pv.tp_hash, pv.csum, NULL, pv.hdr_off, NULL, pv.detail};
  CHECK(gpd_decode_pcap(ctx, cap_file, plen, n, &pr, &pn, &pnext, &pstop, 4));
  int bad = res_cmp("gpd_decode vs oracle", &dv, &ov, n) | res_cmp("gpd_decode_host vs oracle", &hv, &ov, n);
  if (!bad) bad = detail_cmp("gpd_decode detail vs oracle", &dv, oext, n) |
                  detail_cmp("gpd_decode_host detail vs oracle", &hv, oext, n);
  if (pn != n || pnext != plen || (n > 0 && pstop != GPD_PCAP_STOP_LIMIT && pstop != GPD_PCAP_STOP_EOF)) {
    fprintf(stderr, "gpd_decode_pcap: n %llu/%llu next %llu/%llu stop %d\n", (unsigned long long)pn,
            (unsigned long long)n, (unsigned long long)pnext, (unsigned long long)plen, pstop);
    bad = 1;
  } else {
    bad |= res_cmp("gpd_decode_pcap vs oracle", &pv, &ov, n);
    if (!bad) bad |= detail_cmp("gpd_decode_pcap detail vs oracle", &pv, oext, n);
  }

  /* the error values, rebuilt from the device's status + detail words only */
  if (!bad && argc >= 4) {
    static char names[256][64];
    FILE *nf = fopen(argv[3], "r");
    if (!nf) { perror(argv[3]); return 2; }
    for (int p = 0; p < 256; p++) {
      if (!fgets(names[p], sizeof names[p], nf)) { fprintf(stderr, "short names file\n"); return 2; }
      names[p][strcspn(names[p], "\n")] = 0;
    }
    fclose(nf);
    FILE *ef = fopen(argv[2], "w");
    if (!ef) { perror(argv[2]); return 2; }
    char text[256];
    for (uint64_t i = 0; i < n; i++) {
      if (GPD_STATUS_CLASS(dv.status[i]) != GPD_ST_DECODE_ERROR) continue;
      error_text(text, sizeof text, GPD_STATUS_ERRCODE(dv.status[i]), dv.detail[i].err_arg0,
                 dv.detail[i].err_arg1, names);
      fprintf(ef, "%llu\t%s\n", (unsigned long long)i, text);
    }
    fclose(ef);
  }

  /* 5. the device results feed the flow table */
  uint64_t flows = 0;
  if (!bad && n > 0) bad |= check_flows(ctx, s, &db, &dr, data, off, cap, ov.hdr_off, n, &flows);

  /* 6. the fragment hand-off over the same device results */
  uint64_t frags = 0;
  if (!bad && n > 0) bad |= check_fragments(ctx, s, &db, &dr, data, off, cap, ov.status, ov.hdr_off, n, &frags);

  /* 7. in-place reconfiguration on a second context (ABI 8) */
  uint64_t vx = 0;
  if (!bad && argc >= 5) bad |= check_reconfig(&cfg, data, data_len, off, cap, n, &db, &dr, s,
                                               (uint16_t)atoi(argv[4]), &vx);

  CHECK(gpd_ctx_destroy(ctx));
  HCHECK(hipStreamDestroy(s));
  if (bad) return 1;
  printf("abi_host ok %llu %llu %llu %llu\n", (unsigned long long)n, (unsigned long long)flows,
         (unsigned long long)frags, (unsigned long long)vx);
  return 0;
}
