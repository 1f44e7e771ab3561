// Package gpdecode is the cgo binding a gopacket maintainer would add to run
// DecodingLayerParser batches on an MI355X through libgpd.so (include/gpd.h).
//
// It mirrors gopacket's parser surface (parser.go:182-350) with batch entry
// points: one DecodeBatch call decodes every packet of a PacketBatch in one
// kernel launch, then per-index accessors return what DecodeLayers, Truncated,
// NetworkFlow().FastHash(), TransportFlow().FastHash(), the IPv4 header checksum
// and TCP.ComputeChecksum() would have returned for that packet.
//
// NOTE: this image has no Go toolchain, so this file is not compiled or tested in
// this repository. The C-ABI it binds is exercised by the Python ctypes binding
// (gopacket_amd/_lib.py) and tests/test_parity_gpu.py.
package gpdecode

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../gopacket_amd -lgpd -Wl,-rpath,${SRCDIR}/../../gopacket_amd
#include <stdlib.h>
#include "gpd.h"
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

// Decoder bits: which DecodingLayers are registered (gpd.h GPD_DEC_*).
const (
	DecEthernet   = C.GPD_DEC_ETHERNET
	DecDot1Q      = C.GPD_DEC_DOT1Q
	DecIPv4       = C.GPD_DEC_IPV4
	DecIPv6       = C.GPD_DEC_IPV6
	DecIPv6Ext    = C.GPD_DEC_IPV6_EXT
	DecTCP        = C.GPD_DEC_TCP
	DecUDP        = C.GPD_DEC_UDP
	DecVXLAN      = C.GPD_DEC_VXLAN
	DecPayload    = C.GPD_DEC_PAYLOAD
	DecFragment   = C.GPD_DEC_FRAGMENT
	DecICMPv4     = C.GPD_DEC_ICMPV4
	DecLLC        = C.GPD_DEC_LLC
	DecAll        = C.GPD_DEC_ALL
	optIgnoreUnsp = C.GPD_OPT_IGNORE_UNSUPPORTED
	optIgnorePan  = C.GPD_OPT_IGNORE_PANIC
)

// decoderBit maps the DecodingLayer values a caller already builds for
// gopacket.NewDecodingLayerParser to the engine's decoder bits.
func decoderBit(d gopacket.DecodingLayer) (uint32, error) {
	switch d.(type) {
	case *layers.Ethernet:
		return DecEthernet, nil
	case *layers.Dot1Q:
		return DecDot1Q, nil
	case *layers.IPv4:
		return DecIPv4, nil
	case *layers.IPv6:
		return DecIPv6, nil
	case *layers.IPv6ExtensionSkipper:
		return DecIPv6Ext, nil
	case *layers.TCP:
		return DecTCP, nil
	case *layers.UDP:
		return DecUDP, nil
	case *layers.VXLAN:
		return DecVXLAN, nil
	case *gopacket.Payload:
		return DecPayload, nil
	case *gopacket.Fragment:
		return DecFragment, nil
	case *layers.ICMPv4:
		return DecICMPv4, nil
	case *layers.LLC:
		return DecLLC, nil
	}
	return 0, fmt.Errorf("gpdecode: %T has no MI355X decoder", d)
}

// BatchDecodingLayerParser is the batch form of gopacket.DecodingLayerParser.
// IgnoreUnsupported and IgnorePanic are plain fields, as in the reference
// (parser.go:182-195,336-350): assigning one changes the next call's options in
// place (gpd_ctx_set_options), and the context keeps its device, decoders and the
// tables ReloadTables gave it.
type BatchDecodingLayerParser struct {
	ctx               *C.gpd_ctx
	device            int
	first             gopacket.LayerType
	decoders          uint32
	IgnoreUnsupported bool // parser.go:336-350
	IgnorePanic       bool
	options           uint32 // the options the context holds
}

// NewBatchDecodingLayerParser mirrors gopacket.NewDecodingLayerParser
// (parser.go:222-233). The dispatch tables (EthernetTypeMetadata,
// IPProtocolMetadata, the TCP/UDP port maps) are snapshotted when the device
// context is created; call ReloadTables after layers.Register*PortLayerType.
func NewBatchDecodingLayerParser(device int, first gopacket.LayerType, decoders ...gopacket.DecodingLayer) (*BatchDecodingLayerParser, error) {
	p := &BatchDecodingLayerParser{device: device, first: first}
	for _, d := range decoders {
		bit, err := decoderBit(d)
		if err != nil {
			return nil, err
		}
		p.decoders |= bit
	}
	cfg := C.gpd_config{first_layer: C.uint32_t(first), decoders: C.uint32_t(p.decoders)}
	if rc := C.gpd_ctx_create(C.int(device), &cfg, &p.ctx); rc != C.GPD_OK {
		return nil, lastError("gpd_ctx_create", rc)
	}
	runtime.SetFinalizer(p, (*BatchDecodingLayerParser).Close)
	return p, nil
}

// AddDecodingLayer mirrors (*DecodingLayerParser).AddDecodingLayer (parser.go:197-202):
// the decoder joins the registered set of the existing context (gpd_ctx_add_decoders),
// whose device and reloaded tables stay.
func (p *BatchDecodingLayerParser) AddDecodingLayer(d gopacket.DecodingLayer) error {
	bit, err := decoderBit(d)
	if err != nil {
		return err
	}
	if rc := C.gpd_ctx_add_decoders(p.ctx, C.uint32_t(bit)); rc != C.GPD_OK {
		return lastError("gpd_ctx_add_decoders", rc)
	}
	p.decoders |= bit
	return nil
}

// kindTypes: each engine decoder kind and the CanDecode set it registers (gpd.h GPD_DEC_*).
var kindTypes = map[uint32][]gopacket.LayerType{
	DecEthernet: {layers.LayerTypeEthernet},
	DecDot1Q:    {layers.LayerTypeDot1Q},
	DecIPv4:     {layers.LayerTypeIPv4},
	DecIPv6:     {layers.LayerTypeIPv6},
	DecIPv6Ext: {layers.LayerTypeIPv6HopByHop, layers.LayerTypeIPv6Routing,
		layers.LayerTypeIPv6Fragment, layers.LayerTypeIPv6Destination},
	DecTCP:      {layers.LayerTypeTCP},
	DecUDP:      {layers.LayerTypeUDP},
	DecVXLAN:    {layers.LayerTypeVXLAN},
	DecPayload:  {gopacket.LayerTypePayload},
	DecFragment: {gopacket.LayerTypeFragment},
	DecICMPv4:   {layers.LayerTypeICMPv4},
	DecLLC:      {layers.LayerTypeLLC},
}

// SetDecodingLayerContainer mirrors (*DecodingLayerParser).SetDecodingLayerContainer
// (parser.go:236-242): the decoders dlc holds replace the registered set, in place
// (gpd_ctx_set_decoders; device and reloaded tables kept).  The engine registers decoder kinds
// whole: a container holding a kind for only part of its CanDecode set (IPv6ExtensionSkipper for
// some of 46..49) has no engine equivalent and is refused, and so is a container holding, for a
// layer type the engine decodes, a decoder it cannot run (decoderBit's error).  The parser keeps
// its previous set on any error.
func (p *BatchDecodingLayerParser) SetDecodingLayerContainer(dlc gopacket.DecodingLayerContainer) error {
	var mask uint32
	for bit, types := range kindTypes {
		held := 0
		for _, t := range types {
			if d, ok := dlc.Decoder(t); ok {
				b, err := decoderBit(d)
				if err != nil {
					// a decoder the engine cannot run (a caller's own DecodingLayer for a
					// type it takes): refused as NewBatchDecodingLayerParser refuses it, not
					// dropped (its packets would stop with UnsupportedLayerType later)
					return err
				}
				if b != bit {
					return fmt.Errorf("gpdecode: the container holds %T for layer type %v, which the engine decodes with another kind", d, t)
				}
				held++
			}
		}
		if held == len(types) {
			mask |= bit
		} else if held > 0 {
			return fmt.Errorf("gpdecode: the container holds decoder kind %#x for only %d of its %d layer types", bit, held, len(types))
		}
	}
	if rc := C.gpd_ctx_set_decoders(p.ctx, C.uint32_t(mask)); rc != C.GPD_OK {
		return lastError("gpd_ctx_set_decoders", rc)
	}
	p.decoders = mask
	return nil
}

// Device is the GPU the parser decodes on.
func (p *BatchDecodingLayerParser) Device() int { return p.device }

// Close releases the device context.
func (p *BatchDecodingLayerParser) Close() {
	if p.ctx != nil {
		C.gpd_ctx_destroy(p.ctx)
		p.ctx = nil
	}
}

// ReloadTables re-snapshots the reference's global dispatch tables
// (layers/ports.go:78-80,126-128) into the device context. The tables are
// passed as flat LayerType arrays; BuildTables shows how to fill them.
func (p *BatchDecodingLayerParser) ReloadTables(t *Tables) error {
	cfg := C.gpd_config{
		first_layer: C.uint32_t(p.first),
		decoders:    C.uint32_t(p.decoders),
		ethertype:   (*C.uint16_t)(unsafe.Pointer(&t.EtherType[0])),
		ipproto:     (*C.uint16_t)(unsafe.Pointer(&t.IPProtocol[0])),
		tcp_port:    (*C.uint16_t)(unsafe.Pointer(&t.TCPPort[0])),
		udp_port:    (*C.uint16_t)(unsafe.Pointer(&t.UDPPort[0])),
	}
	// cfg (Go memory) holds pointers into the four Go slices: cgo lets C see them only while
	// they are pinned (runtime.Pinner, Go 1.21+)
	var pn runtime.Pinner
	defer pn.Unpin()
	pinFirst(&pn, t.EtherType, t.IPProtocol, t.TCPPort, t.UDPPort)
	if rc := C.gpd_ctx_reload_tables(p.ctx, &cfg); rc != C.GPD_OK {
		return lastError("gpd_ctx_reload_tables", rc)
	}
	return nil
}

// Tables are the four reference tables as LayerType numbers.
type Tables struct {
	EtherType  [65536]uint16 // EthernetTypeMetadata[t].LayerType, layers/enums.go:304-321
	IPProtocol [256]uint16   // IPProtocolMetadata[p].LayerType, layers/enums.go:323-345
	TCPPort    [65536]uint16 // tcpPortLayerType, layers/ports.go:62-74 (0 => Payload)
	UDPPort    [65536]uint16 // udpPortLayerType, layers/ports.go:105-122
}

// BuildTables reads the live gopacket tables.
func BuildTables() *Tables {
	t := &Tables{}
	for i := 0; i < 65536; i++ {
		t.EtherType[i] = uint16(layers.EthernetTypeMetadata[i].LayerType)
		t.TCPPort[i] = uint16(layers.TCPPort(i).LayerType())
		t.UDPPort[i] = uint16(layers.UDPPort(i).LayerType())
		if t.TCPPort[i] == uint16(gopacket.LayerTypePayload) {
			t.TCPPort[i] = 0
		}
		if t.UDPPort[i] == uint16(gopacket.LayerTypePayload) {
			t.UDPPort[i] = 0
		}
	}
	for i := 0; i < 256; i++ {
		t.IPProtocol[i] = uint16(layers.IPProtocolMetadata[i].LayerType)
	}
	return t
}

// PacketBatch holds packets back to back: packet i is
// Data[Offset[i] : Offset[i]+CapLen[i]]. Data must stay valid until the call
// returns (gpd_decode_host copies it through pinned staging).
type PacketBatch struct {
	Data   []byte
	Offset []uint32
	CapLen []uint32
}

// Append adds one packet (e.g. the data from a pcap.Handle.ReadPacketData loop),
// 16-byte aligned, the layout the kernel's fast path expects.
func (b *PacketBatch) Append(pkt []byte) {
	for len(b.Data)%16 != 0 {
		b.Data = append(b.Data, 0)
	}
	b.Offset = append(b.Offset, uint32(len(b.Data)))
	b.CapLen = append(b.CapLen, uint32(len(pkt)))
	b.Data = append(b.Data, pkt...)
}

// Detail is gpd.h's gpd_detail (same 24-byte layout): the decoded list past the core word's
// 12 layers and the error's format arguments.  The kernel writes it only for packets with a
// decode error or more than 12 layers — exactly the packets its fast path leaves to the
// generic decoder, so asking for it never slows a batch down.
type Detail struct {
	Codes      [2]uint64 // decoded[0..31] as 4-bit codes, decoded[k] at bit 4*(k%16) of word k/16
	Arg0, Arg1 uint32    // the error text's arguments (enum gpd_err in gpd.h)
}

// Result is the per-packet SoA the kernel writes (include/gpd.h).
type Result struct {
	Status   []uint32
	Layers   []uint64
	NetHash  []uint64
	TpHash   []uint64
	Checksum []uint32
	HdrOff   []uint32 // gpd.h header offsets word: where the flows' layers sit
	Detail   []Detail // gpd.h gpd_detail: valid where hasDetail(i)
}

// DecodeBatch decodes every packet of b (host memory, pinned H2D -> kernel -> D2H).
func (p *BatchDecodingLayerParser) DecodeBatch(b *PacketBatch) (*Result, error) {
	n := len(b.Offset)
	r := newResult(n)
	if n == 0 {
		return r, nil
	}
	// the data buffer must be readable to round_up(len, 16) + 16; it is never empty here, so
	// a batch of empty packets (every CapLen 0, len(b.Data) == 0) still passes a valid pointer
	data := b.Data
	if cap(data) < len(data)+32 {
		data = append(make([]byte, 0, len(data)+32), data...)
	}
	data = data[:len(data)+1]
	in := C.gpd_batch{
		data:     (*C.uint8_t)(unsafe.Pointer(&data[0])),
		data_len: C.uint64_t(len(b.Data)),
		offset:   (*C.uint32_t)(unsafe.Pointer(&b.Offset[0])),
		caplen:   (*C.uint32_t)(unsafe.Pointer(&b.CapLen[0])),
		n:        C.uint64_t(n),
	}
	out := r.cResult()
	if err := p.configure(); err != nil {
		return nil, err
	}
	// in and out (Go memory) hold pointers into Go slices: pinned for the call
	var pn runtime.Pinner
	defer pn.Unpin()
	pinFirst(&pn, data, b.Offset, b.CapLen)
	r.pin(&pn)
	if rc := C.gpd_decode_host(p.ctx, &in, &out); rc != C.GPD_OK {
		return nil, lastError("gpd_decode_host", rc)
	}
	return r, nil
}

// pinFirst pins the backing array of every non-empty slice (its first element): a C struct
// in Go memory may hold pointers into Go memory only while they are pinned (cgo pointer
// rules; runtime.Pinner, Go 1.21+).  Slices over memory Go does not own (an mmap'ed ring or
// capture) must not be passed: Pin accepts Go pointers only.
func pinFirst(pn *runtime.Pinner, slices ...interface{}) {
	for _, s := range slices {
		switch v := s.(type) {
		case []byte:
			if len(v) > 0 {
				pn.Pin(&v[0])
			}
		case []uint16:
			if len(v) > 0 {
				pn.Pin(&v[0])
			}
		case []uint32:
			if len(v) > 0 {
				pn.Pin(&v[0])
			}
		case []uint64:
			if len(v) > 0 {
				pn.Pin(&v[0])
			}
		case []int32:
			if len(v) > 0 {
				pn.Pin(&v[0])
			}
		default:
			panic("gpdecode: pinFirst: unsupported slice type")
		}
	}
}

// configure hands changed IgnoreUnsupported / IgnorePanic fields to the context in place
// (gpd_ctx_set_options, ABI 8): the device, the decoder set and the reloaded tables stay.
func (p *BatchDecodingLayerParser) configure() error {
	var o uint32
	if p.IgnoreUnsupported {
		o |= optIgnoreUnsp
	}
	if p.IgnorePanic {
		o |= optIgnorePan
	}
	if o == p.options {
		return nil
	}
	if rc := C.gpd_ctx_set_options(p.ctx, C.uint32_t(o)); rc != C.GPD_OK {
		return lastError("gpd_ctx_set_options", rc)
	}
	p.options = o
	return nil
}

var codeLayerType = [16]gopacket.LayerType{0, layers.LayerTypeEthernet, layers.LayerTypeDot1Q,
	layers.LayerTypeIPv4, layers.LayerTypeIPv6, layers.LayerTypeIPv6HopByHop,
	layers.LayerTypeIPv6Routing, layers.LayerTypeIPv6Fragment, layers.LayerTypeIPv6Destination,
	layers.LayerTypeTCP, layers.LayerTypeUDP, layers.LayerTypeVXLAN,
	gopacket.LayerTypePayload, gopacket.LayerTypeFragment, layers.LayerTypeICMPv4, layers.LayerTypeLLC}

// hasDetail: the kernel wrote Detail[i] (a decode error, or more layers than the core word holds).
func (r *Result) hasDetail(i int) bool {
	s := r.Status[i]
	return s&3 == C.GPD_ST_DECODE_ERROR || (s>>4)&31 > C.GPD_CORE_MAX_LAYERS || s&8 != 0
}

// ErrStackTooDeep: len(decoded) of the packet exceeds what the result holds (more than 31
// layers: the status word saturates, and the detail record keeps the first 32).
var ErrStackTooDeep = errors.New("gpdecode: more than 31 layers decoded; the result keeps the first 32")

// nLayers is len(decoded) (31 when saturated) and code(i, k) the 4-bit code of decoded[k]:
// from the core word for the first 12, from the detail record past them.
func (r *Result) nLayers(i int) int { return int(r.Status[i]>>4) & 31 }

func (r *Result) code(i, k int) (uint64, bool) {
	if k < C.GPD_CORE_MAX_LAYERS {
		return (r.Layers[i] >> (16 + 4*uint(k))) & 15, true
	}
	if k >= 32 || len(r.Detail) <= i || !r.hasDetail(i) {
		return 0, false
	}
	return (r.Detail[i].Codes[k/16] >> (4 * uint(k%16))) & 15, true
}

// Decoded fills decoded exactly as DecodeLayers would (parser.go:302-316), any depth up to
// 31 layers (ErrStackTooDeep past that: the status word saturates).
func (r *Result) Decoded(i int, decoded *[]gopacket.LayerType) error {
	*decoded = (*decoded)[:0]
	n := r.nLayers(i)
	for k := 0; k < n; k++ {
		c, ok := r.code(i, k)
		if !ok {
			return fmt.Errorf("gpdecode: packet %d decoded %d layers; decode with a Detail array", i, n)
		}
		*decoded = append(*decoded, codeLayerType[c])
	}
	if r.Status[i]&8 != 0 {
		return ErrStackTooDeep
	}
	return nil
}

// Truncated is parser.Truncated after DecodeLayers on packet i.
func (r *Result) Truncated(i int) bool { return r.Status[i]&4 != 0 }

// Err is DecodeLayers' return value for packet i (parser.go:302-316): nil,
// gopacket.UnsupportedLayerType, or the failing layer's error with the reference's exact
// text — its format arguments come from the detail record.
func (r *Result) Err(i int) error {
	switch r.Status[i] & 3 {
	case C.GPD_ST_UNSUPPORTED:
		return gopacket.UnsupportedLayerType(gopacket.LayerType(r.Layers[i] & 0xFFFF))
	case C.GPD_ST_DECODE_ERROR:
		var a0, a1 uint32
		if len(r.Detail) > i {
			a0, a1 = r.Detail[i].Arg0, r.Detail[i].Arg1
		}
		return decodeError((r.Status[i]>>9)&63, a0, a1)
	}
	return nil
}

// lastCode is the kind of the last decoded layer with one of the two codes, over the whole
// decoded list (the detail record holds the layers past the core word's 12).
func (r *Result) lastCode(i int, a, b uint64) uint64 {
	n := r.nLayers(i)
	var last uint64
	for k := 0; k < n; k++ {
		c, ok := r.code(i, k)
		if !ok {
			break
		}
		if c == a || c == b {
			last = c
		}
	}
	return last
}

// Fill leaves the DecodingLayer objects exactly as DecodeLayers(packet i) leaves the parser's:
// it repeats the reference's loop (layers_decoder.go:60-79) over the decoded list the kernel
// reported — each layer's object (the one whose CanDecode holds its type) gets DecodeFromBytes
// over the previous layer's LayerPayload(), so a kind decoded twice (VXLAN's inner Ethernet and
// IPv4) ends holding the inner header — and, when the packet's decode failed, hands the failing
// layer's object its bytes as well (its DecodeFromBytes assigns fields before it returns the
// error, ip4.go:195-225, tcp.go:234-268, udp.go:35-53).  Pass the same objects the parser was
// built from.  Returns DecodeLayers' error value for the packet.
//
//	res, _ := p.DecodeBatch(&b)
//	var eth layers.Ethernet; var ip4 layers.IPv4; var tcp layers.TCP; var pl gopacket.Payload
//	for i := range b.Offset {
//	    err := p.Fill(res, &b, i, &eth, &ip4, &tcp, &pl)
//	    ... eth.SrcMAC, ip4.TTL, tcp.Options ...
//	}
func (p *BatchDecodingLayerParser) Fill(r *Result, b *PacketBatch, i int, decoders ...gopacket.DecodingLayer) error {
	var decoded []gopacket.LayerType
	if err := r.Decoded(i, &decoded); err != nil {
		return err
	}
	find := func(t gopacket.LayerType) gopacket.DecodingLayer {
		for _, d := range decoders {
			if d.CanDecode().Contains(t) {
				return d
			}
		}
		return nil
	}
	data := b.Data[b.Offset[i] : b.Offset[i]+b.CapLen[i]]
	next := p.first
	for k, t := range decoded {
		d := find(t)
		if d == nil {
			return fmt.Errorf("gpdecode: Fill: no object decodes %v (decoded[%d])", t, k)
		}
		if err := d.DecodeFromBytes(data, gopacket.NilDecodeFeedback); err != nil {
			return fmt.Errorf("gpdecode: Fill: %v failed on the host: %v", t, err)
		}
		data, next = d.LayerPayload(), d.NextLayerType()
	}
	derr := r.Err(i)
	if r.Status[i]&3 == C.GPD_ST_DECODE_ERROR && (len(decoded) == 0 || len(data) != 0) {
		if d := find(next); d != nil {
			_ = d.DecodeFromBytes(data, gopacket.NilDecodeFeedback) // returns derr again
		}
	}
	return derr
}

// NetworkFlow is ip4/ip6.NetworkFlow() after DecodeLayers on packet i (ip4.go:63-65,
// ip6.go:49-51): the endpoints are slices of the packet bytes at the offset the kernel
// reported, as the reference's layer structs slice them.
func (r *Result) NetworkFlow(b *PacketBatch, i int) (gopacket.Flow, bool) {
	off := r.HdrOff[i] & 0xFFFF
	pkt := b.Data[b.Offset[i] : b.Offset[i]+b.CapLen[i]]
	switch r.lastCode(i, C.GPD_C_IPV4, C.GPD_C_IPV6) {
	case C.GPD_C_IPV4:
		return gopacket.NewFlow(layers.EndpointIPv4, pkt[off+12:off+16], pkt[off+16:off+20]), true
	case C.GPD_C_IPV6:
		return gopacket.NewFlow(layers.EndpointIPv6, pkt[off+8:off+24], pkt[off+24:off+40]), true
	}
	return gopacket.Flow{}, false
}

// TransportFlow is tcp/udp.TransportFlow() after DecodeLayers on packet i (tcp.go:331-333,
// udp.go:123-125).  Together with NetworkFlow it is the [2]Flow key tcpassembly uses.
func (r *Result) TransportFlow(b *PacketBatch, i int) (gopacket.Flow, bool) {
	off := r.HdrOff[i] >> 16
	pkt := b.Data[b.Offset[i] : b.Offset[i]+b.CapLen[i]]
	switch r.lastCode(i, C.GPD_C_TCP, C.GPD_C_UDP) {
	case C.GPD_C_TCP:
		return gopacket.NewFlow(layers.EndpointTCPPort, pkt[off:off+2], pkt[off+2:off+4]), true
	case C.GPD_C_UDP:
		return gopacket.NewFlow(layers.EndpointUDPPort, pkt[off:off+2], pkt[off+2:off+4]), true
	}
	return gopacket.Flow{}, false
}

// NetworkFlowHash is ip4/ip6.NetworkFlow().FastHash() of the last network layer.
func (r *Result) NetworkFlowHash(i int) (uint64, bool) { return r.NetHash[i], r.Status[i]&(1<<16) != 0 }

// TransportFlowHash is tcp/udp.TransportFlow().FastHash() of the last transport.
func (r *Result) TransportFlowHash(i int) (uint64, bool) { return r.TpHash[i], r.Status[i]&(1<<17) != 0 }

// IPv4HeaderChecksum is layers/ip4.go:158 checksum(ip4.Contents): compare with ip4.Checksum.
func (r *Result) IPv4HeaderChecksum(i int) (uint16, bool) {
	return uint16(r.Checksum[i]), r.Status[i]&(1<<18) != 0
}

// TransportChecksum is TCP.ComputeChecksum() (or the same sum over UDP): 0 when valid.
func (r *Result) TransportChecksum(i int) (uint16, bool) {
	return uint16(r.Checksum[i] >> 16), r.Status[i]&(1<<19) != 0
}

// decodeError rebuilds the error one reference `return` site (enum gpd_err, file:line in gpd.h)
// gives, with its format string and its argument types, so err.Error() is the reference's text.
func decodeError(code, a0, a1 uint32) error {
	switch code {
	case 1:
		return errors.New("Ethernet packet too small") // ethernet.go:42-43
	case 2:
		return fmt.Errorf("802.1Q tag length %d too short", int(a0)) // dot1q.go:30-32
	case 3:
		return fmt.Errorf("Invalid ip4 header. Length %d less than 20", int(a0)) // ip4.go:189-191
	case 4:
		return fmt.Errorf("Invalid (too small) IP length (%d < 20)", uint16(a0)) // ip4.go:220-221
	case 5:
		return fmt.Errorf("Invalid (too small) IP header length (%d < 5)", uint8(a0)) // ip4.go:222-223
	case 6:
		return fmt.Errorf("Invalid IP header length > IP length (%d > %d)", uint8(a0), uint16(a1)) // :224-225
	case 7:
		return errors.New("Not all IP header bytes available") // ip4.go:231-232
	case 8:
		return fmt.Errorf("Invalid ip4 option length. Length %d less than 2", int(a0)) // ip4.go:257-259
	case 9:
		return fmt.Errorf("IP option length exceeds remaining IP header size, option type %v length %v",
			uint8(a0), uint8(a1)) // ip4.go:262-264
	case 10:
		return fmt.Errorf("Invalid IP option type %v length %d. Must be greater than 2", uint8(a0), uint8(a1)) // :266-267
	case 11:
		return fmt.Errorf("Invalid ip6 header. Length %d less than 40", int(a0)) // ip6.go:222-224
	case 12:
		return fmt.Errorf("Invalid ip6-extension header. Length %d less than 2", int(a0)) // ip6.go:419-421
	case 13:
		return fmt.Errorf("Invalid ip6-extension header. Length %d less than specified length %d",
			int(a0), int(a1)) // ip6.go:426-427
	case 14:
		return errors.New("IPv6 header option too small") // ip6.go:328-330
	case 15:
		return errors.New("IPv6 header TLV option too small") // ip6.go:340-342
	case 16:
		return errors.New("Jumbo length TLV data must have length 4") // ip6.go:67-68
	case 17:
		return fmt.Errorf("Jumbo length cannot be less than %d", 65536) // ip6.go:71-72
	case 18:
		return errors.New("IPv6 has jumbo length and IPv6 length is not 0") // ip6.go:257-258
	case 19:
		return errors.New("IPv6 length 0, but HopByHop header does not have jumbogram option") // ip6.go:259-260
	case 20:
		return fmt.Errorf("IPv6 length 0, but next header is %v, not HopByHop", layers.IPProtocol(a0)) // ip6.go:266-267
	case 21:
		return fmt.Errorf("Invalid TCP header. Length %d less than 20", int(a0)) // tcp.go:230-232
	case 22:
		return fmt.Errorf("Invalid TCP data offset %d < 5", uint8(a0)) // tcp.go:260-261
	case 23:
		return errors.New("TCP data offset greater than packet length") // tcp.go:264-268
	case 24:
		return fmt.Errorf("Invalid TCP option length. Length %d less than 2", int(a0)) // tcp.go:286-288
	case 25:
		return fmt.Errorf("Invalid TCP option length %d < 2", uint8(a0)) // tcp.go:291-292
	case 26:
		return fmt.Errorf("Invalid TCP option length %d exceeds remaining %d bytes", uint8(a0), int(a1)) // tcp.go:293-295
	case 27:
		return fmt.Errorf("Invalid UDP header. Length %d less than 8", int(a0)) // udp.go:31-33
	case 28:
		return fmt.Errorf("UDP packet too small: %d bytes", uint16(a0)) // udp.go:52-53
	case 29:
		return errors.New("vxlan packet too small") // vxlan.go:54-56
	case 30:
		return errors.New("ICMP layer less then 8 bytes for ICMPv4 packet") // icmp4.go:221-223
	case 31:
		return errors.New("LLC header too small") // llc.go:32-33,42-43
	}
	return fmt.Errorf("gpdecode: unknown error code %d", code)
}

func lastError(what string, rc C.int) error {
	return fmt.Errorf("%s: rc=%d: %s", what, int(rc), C.GoString(C.gpd_last_error_string()))
}
