// gpd_internal.h — shared between the HIP kernels and the host runtime (not public ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpd.h"

namespace gpd {

// Device dispatch tables: a two-level page structure per 16-bit table.
//   words [0,256)      ipproto -> LayerType
//   words [256,512)    ethertype high byte -> page
//   words [512,768)    tcp port high byte  -> page
//   words [768,1024)   udp port high byte  -> page
//   words [1024, ...)  pages of 256 LayerTypes; page 0 is all zero
// The reference's tables are 3 x 64K + 256 entries (≈384 KB); with its defaults this
// structure is ≈9 KB, small enough for every lookup to hit L1/L2.
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
  uint32_t *status;
  uint64_t *layers;
  uint64_t *net_hash;
  uint64_t *tp_hash;
  uint32_t *csum;
  gpd_ext_rec *ext;
  const uint16_t *tables;
  uint32_t first;
  uint32_t decoders;
  uint32_t options;
  uint32_t pad;
};

// Launch the decode kernel over P (asynchronous on `stream`).
hipError_t launch_decode(const KParams &P, hipStream_t stream, int num_cus);

}  // namespace gpd
