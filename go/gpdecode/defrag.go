package gpdecode

// The IPv4 fragment hand-off (include/gpd_defrag.h) from Go.  Not compiled here (no Go
// toolchain); tests/test_defrag.py drives the same C entry point through ctypes on the GPU.

/*
#cgo CFLAGS: -I${SRCDIR}/../../include -I/opt/rocm/include -D__HIP_PLATFORM_AMD__
#cgo LDFLAGS: -L/opt/rocm/lib -lamdhip64
#include <hip/hip_runtime_api.h>
#include "gpd.h"
#include "gpd_defrag.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"unsafe"

	"github.com/google/gopacket"
	"github.com/google/gopacket/layers"
)

// Fragment verdicts (GPD_FRAG_*).
const (
	FragInsert   = 0 // hand the layer to DefragIPv4: it files it (defrag.go:98-135)
	FragTooSmall = 1 // DefragIPv4 returns securityChecks' "fragment too small" error
	FragOffset   = 2 // ... "fragment offset too big"
	FragOverrun  = 3 // ... "fragment will overrun" (never produced: uint16 sum, defrag.go:192)
	FragWhole    = 4 // DefragIPv4 returns the layer unchanged
)

// Fragment is one packet the defragmenter still has to see (C.gpd_ip4_frag).
type Fragment struct {
	Packet      uint32 // index in the batch
	NetOff      uint32 // the IPv4 header's offset in the packet
	Key         gopacket.Flow
	Id          uint16
	FragOffset  uint16
	Length      uint16
	Flags       layers.IPv4Flag
	IHL         uint8
	PayloadLen  uint32
	Verdict     uint8
}

// Layer rebuilds the DecodingLayerParser's IPv4 object for the fragment in a NEW layer over a
// COPY of its bytes: DecodeFromBytes over exactly the bytes the parser gave it (Contents +
// Payload), so Length, Payload and the truncation flag come out as the batch decode left them.
// A fresh object per fragment matters: IPv4Defragmenter keeps the *layers.IPv4 it is given in
// its pending list until the datagram completes (ip4defrag/defrag.go:221,245), and the copy
// keeps pending fragments valid when the batch buffer is reused for the next batch.
// (A packet whose IPv4 decode FAILED after assigning the header fields — the parser's object
// then holds that rejected header, ip4.go:195-210 — comes back with the same decode error.)
func (f *Fragment) Layer(b *PacketBatch) (*layers.IPv4, error) {
	pkt := b.Data[b.Offset[f.Packet] : b.Offset[f.Packet]+b.CapLen[f.Packet]]
	end := f.NetOff + 4*uint32(f.IHL) + f.PayloadLen
	buf := append([]byte(nil), pkt[f.NetOff:end]...)
	ip := new(layers.IPv4)
	return ip, ip.DecodeFromBytes(buf, gopacket.NilDecodeFeedback)
}

// Err is the error DefragIPv4 returns for the fragment without filing it (nil for FragInsert
// and FragWhole).
func (f *Fragment) Err() error {
	switch f.Verdict {
	case FragTooSmall:
		return fmt.Errorf("defrag: fragment too small (handcrafted? %d < %d)", f.Length-uint16(f.IHL)*4, 8)
	case FragOffset:
		return fmt.Errorf("defrag: fragment offset too big (handcrafted? %d > %d)", f.FragOffset, 8183)
	case FragOverrun:
		return fmt.Errorf("defrag: fragment will overrun (handcrafted? %d > %d)", f.FragOffset*8+f.Length, 65535)
	}
	return nil
}

// Fragments decodes the batch on the device and returns, in packet order, the packets for
// which IPv4Defragmenter.DefragIPv4 would not return the layer unchanged:
//
//	frags, _ := p.Fragments(&b)
//	for i := range frags {
//	    f := &frags[i]
//	    if err := f.Err(); err != nil { ...; continue }      // securityChecks
//	    ip4, err := f.Layer(&b)                               // its own object, its own bytes
//	    if err != nil { ...; continue }
//	    whole, _ := defragger.DefragIPv4WithTimestamp(ip4, ts[f.Packet])
//	}
//
// Every other packet skips the defragmenter.  A caller that already holds the batch's Result
// (DecodeBatch, DecodeCapture) uses FragmentsFrom instead: no second decode.
func (p *BatchDecodingLayerParser) Fragments(b *PacketBatch) ([]Fragment, error) {
	return p.fragments(b, nil)
}

// FragmentsFrom is Fragments over the results of a decode already run on b with this parser
// (r from DecodeBatch, or DecodeCapture of the same packets): the batch and r's status,
// layers and header-offset words go to the device, and only the hand-off runs there.
func (p *BatchDecodingLayerParser) FragmentsFrom(b *PacketBatch, r *Result) ([]Fragment, error) {
	if r == nil || len(r.Status) < len(b.Offset) || len(r.Layers) < len(b.Offset) || len(r.HdrOff) < len(b.Offset) {
		return nil, errors.New("gpdecode: FragmentsFrom needs the batch's Result (status, layers, header offsets)")
	}
	return p.fragments(b, r)
}

func (p *BatchDecodingLayerParser) fragments(b *PacketBatch, r *Result) ([]Fragment, error) {
	n := len(b.Offset)
	if n == 0 || len(b.Data) == 0 { // no packet bytes: no packet can be an IPv4 fragment
		return nil, nil
	}
	if err := p.configure(); err != nil {
		return nil, err
	}
	done, err := p.onDevice()
	if err != nil {
		return nil, err
	}
	defer done()
	sizes := []int{(len(b.Data)+15)&^15 + 64, 4 * n, 4 * n, 4 * n, 8 * n, 4 * n, 32 * n}
	bufs := make([]devBuf, len(sizes))
	for k, s := range sizes {
		d, err := devAlloc(s)
		if err != nil {
			return nil, err
		}
		bufs[k] = d
		defer d.free()
	}
	type upload struct {
		d devBuf
		p unsafe.Pointer
		n int
	}
	up := []upload{{bufs[0], unsafe.Pointer(&b.Data[0]), len(b.Data)}, {bufs[1], unsafe.Pointer(&b.Offset[0]), 4 * n},
		{bufs[2], unsafe.Pointer(&b.CapLen[0]), 4 * n}}
	if r != nil { // the decode's words, as gpd_ip4_fragments reads them
		up = append(up, upload{bufs[3], unsafe.Pointer(&r.Status[0]), 4 * n},
			upload{bufs[4], unsafe.Pointer(&r.Layers[0]), 8 * n}, upload{bufs[5], unsafe.Pointer(&r.HdrOff[0]), 4 * n})
	}
	for _, u := range up {
		if err := toDev(u.d, u.p, u.n); err != nil {
			return nil, err
		}
	}
	in := C.gpd_batch{data: (*C.uint8_t)(bufs[0].p), data_len: C.uint64_t(len(b.Data)),
		offset: (*C.uint32_t)(bufs[1].p), caplen: (*C.uint32_t)(bufs[2].p), n: C.uint64_t(n)}
	res := C.gpd_result{status: (*C.uint32_t)(bufs[3].p), layers: (*C.uint64_t)(bufs[4].p),
		hdr_off: (*C.uint32_t)(bufs[5].p)}
	if r == nil {
		if rc := C.gpd_decode(p.ctx, &in, &res, nil); rc != C.GPD_OK {
			return nil, lastError("gpd_decode", rc)
		}
	}
	var cnt C.uint64_t
	if rc := C.gpd_ip4_fragments(p.ctx, &in, &res, (*C.gpd_ip4_frag)(bufs[6].p), C.uint64_t(n), &cnt, nil); rc != C.GPD_OK {
		return nil, lastError("gpd_ip4_fragments", rc)
	}
	if cnt == 0 {
		return nil, nil
	}
	recs := make([]C.gpd_ip4_frag, int(cnt))
	if e := C.hipMemcpy(unsafe.Pointer(&recs[0]), bufs[6].p, C.size_t(32*int(cnt)), C.hipMemcpyDeviceToHost); e != C.hipSuccess {
		return nil, errors.New(C.GoString(C.hipGetErrorString(e)))
	}
	out := make([]Fragment, len(recs))
	for k := range recs {
		c := &recs[k]
		out[k] = Fragment{Packet: uint32(c.packet), NetOff: uint32(c.net_off),
			Key: gopacket.NewFlow(layers.EndpointIPv4, C.GoBytes(unsafe.Pointer(&c.src[0]), 4),
				C.GoBytes(unsafe.Pointer(&c.dst[0]), 4)),
			Id: uint16(c.id), FragOffset: uint16(c.frag_offset), Length: uint16(c.length),
			Flags: layers.IPv4Flag(c.flags), IHL: uint8(c.ihl), PayloadLen: uint32(c.payload_len),
			Verdict: uint8(c.verdict)}
	}
	runtime.KeepAlive(b)
	runtime.KeepAlive(r)
	return out, nil
}
