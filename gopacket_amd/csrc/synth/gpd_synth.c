/*
 * gpd_synth.c — WORKLOAD GENERATOR (bench and tests only; not part of libgpd.so).
 *
 * Native twin of gopacket_amd/synth.py make_udp64 (BASELINE config 2 packets) and of
 * gopacket_amd/pcap.py synth_capture's record framing, for captures too large to build with
 * numpy (config 5: 10^9 records, 80 GB).  Packet i depends only on (seed, i), so any range of
 * records can be generated on its own and by any number of threads; the bytes equal
 * make_udp64(n, seed).packet(i) exactly (tests/test_replay.py pins this).
 */
#include <pthread.h>
#include <stdint.h>
#include <string.h>

static inline uint64_t sm(uint64_t seed, uint64_t stream, uint64_t idx) {
  /* splitmix64 output idx of stream `stream` (synth.splitmix64: state seed + stream * 2^40) */
  uint64_t z = seed + (idx + (stream << 40)) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static inline uint32_t sum16(const uint8_t *a, int n) {
  uint32_t s = 0;
  for (int k = 0; k < n; k += 2) s += ((uint32_t)a[k] << 8) | a[k + 1];
  return s;
}

static inline uint16_t fold_not(uint64_t s) {
  s &= 0xFFFFFFFFull; /* the reference accumulates in uint32 */
  while (s > 0xFFFF) s = (s >> 16) + (s & 0xFFFF);
  return (uint16_t)~s;
}

static inline void be16(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)(v >> 8);
  p[1] = (uint8_t)v;
}

/* synth._udp64_rows for global row i */
static void udp64_packet(uint8_t *a, uint64_t seed, uint64_t i, const uint16_t *fp, uint32_t nfree) {
  const uint64_t r1 = sm(seed, 1, i + 1), r2 = sm(seed, 2, i + 1), r3 = sm(seed, 3, i + 1);
  const uint64_t m0 = sm(seed, 100, 2 * i + 1), m1 = sm(seed, 100, 2 * i + 2);
  for (int k = 0; k < 8; k++) a[k] = (uint8_t)(m0 >> (8 * k)) & 0xFE;
  for (int k = 0; k < 4; k++) a[8 + k] = (uint8_t)(m1 >> (8 * k)) & 0xFE;
  a[12] = 0x08, a[13] = 0x00;
  uint8_t *ip = a + 14;
  ip[0] = 0x45, ip[1] = 0;
  be16(ip + 2, 50);
  be16(ip + 4, (uint32_t)(r2 & 0xFFFF));
  ip[6] = 0x40, ip[7] = 0;
  ip[8] = (uint8_t)(((r2 >> 16) & 0xFF) | 1);
  ip[9] = 17;
  ip[10] = ip[11] = 0;
  const uint32_t src = (uint32_t)r1, dst = (uint32_t)(r1 >> 32);
  for (int k = 0; k < 4; k++) ip[12 + k] = (uint8_t)(src >> (24 - 8 * k)), ip[16 + k] = (uint8_t)(dst >> (24 - 8 * k));
  be16(ip + 10, fold_not(sum16(ip, 20)));
  uint8_t *u = a + 34;
  be16(u, fp[r3 % nfree]);
  be16(u + 2, fp[(r3 >> 32) % nfree]);
  be16(u + 4, 30);
  u[6] = u[7] = 0;
  for (int w = 0; w < 3; w++) {
    const uint64_t x = sm(seed, 101, 3 * i + 1 + (uint64_t)w);
    for (int k = 0; k < 8 && 8 * w + k < 22; k++) a[42 + 8 * w + k] = (uint8_t)(x >> (8 * k));
  }
  const uint64_t s = (uint64_t)sum16(ip + 12, 8) + 17 + 30 + sum16(u, 30);
  be16(u + 6, fold_not(s));
  if (i % 64 == 63) a[24] ^= 0x5A; /* 1 in 64: corrupted IPv4 header checksum */
}

struct job {
  uint8_t *dst;
  uint64_t lo, hi, first, seed;
  const uint16_t *fp;
  uint32_t nfree;
  int records;
};

static void *run(void *arg) {
  const struct job *j = (const struct job *)arg;
  const uint64_t stride = j->records ? 80 : 64;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    uint8_t *p = j->dst + (i - j->first) * stride;
    if (j->records) { /* pcap record header (LE micro): {i / 10^6, i % 10^6, 64, 64} */
      const uint32_t h[4] = {(uint32_t)(i / 1000000), (uint32_t)(i % 1000000), 64, 64};
      memcpy(p, h, 16);
      p += 16;
    }
    udp64_packet(p, j->seed, i, j->fp, j->nfree);
  }
  return 0;
}

/* Packets [lo, hi) of make_udp64(seed) written to dst: back to back (64 B each), or as pcap
 * records (16-B header + 64 B) when `records` is set.  free_ports: synth._free_ports of the
 * UDP port table.  nthreads <= 1 runs on the calling thread. */
void gpds_udp64(uint8_t *dst, uint64_t lo, uint64_t hi, uint64_t seed, const uint16_t *free_ports,
                uint32_t nfree, int records, int nthreads) {
  if (hi <= lo || !nfree) return;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  if ((uint64_t)nthreads > hi - lo) nthreads = (int)(hi - lo);
  struct job J[256];
  pthread_t th[256];
  for (int t = 0; t < nthreads; t++) {
    J[t] = (struct job){dst, lo + (hi - lo) * (uint64_t)t / (uint64_t)nthreads,
                        lo + (hi - lo) * (uint64_t)(t + 1) / (uint64_t)nthreads, lo, seed, free_ports, nfree,
                        records};
  }
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], 0, run, &J[t]);
  run(&J[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], 0);
}
