package gpdecode

// Ingest and flow-table wrappers over include/gpd_pcap.h, include/gpd_afpacket.h and
// include/gpd_flow.h.  Like gpdecode.go this file is not compiled here (no Go toolchain);
// tests/c/abi_host.c drives the same C calls from a plain C host and checks them.

/*
#cgo CFLAGS: -I${SRCDIR}/../../include -I/opt/rocm/include -D__HIP_PLATFORM_AMD__
#cgo LDFLAGS: -L/opt/rocm/lib -lamdhip64
#include <stdlib.h>
#include <hip/hip_runtime_api.h>
#include "gpd.h"
#include "gpd_pcap.h"
#include "gpd_afpacket.h"
#include "gpd_flow.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"io"
	"runtime"
	"time"
	"unsafe"

	"github.com/google/gopacket"
	"github.com/google/gopacket/layers"
)

// CaptureHeader is what pcapgo.NewReader reads from the file header (pcapgo/read.go:78-117,
// 183-227).
type CaptureHeader struct {
	Snaplen   uint32
	LinkType  layers.LinkType
	Nanos     bool // Resolution() == time.Nanosecond
	BigEndian bool
}

// ReadCaptureHeader is pcapgo.NewReader on an in-memory capture; gzip captures must be
// inflated first.
func ReadCaptureHeader(capture []byte) (*CaptureHeader, error) {
	var info C.gpd_pcap_info
	if len(capture) == 0 {
		return nil, io.EOF
	}
	if rc := C.gpd_pcap_header((*C.uint8_t)(unsafe.Pointer(&capture[0])), C.uint64_t(len(capture)), &info); rc != C.GPD_OK {
		return nil, errors.New(C.GoString(C.gpd_last_error_string()))
	}
	return &CaptureHeader{Snaplen: uint32(info.snaplen), LinkType: layers.LinkType(info.linktype),
		Nanos: info.nano != 0, BigEndian: info.big_endian != 0}, nil
}

// DecodeCapture replaces
//
//	r, _ := pcapgo.NewReader(f)
//	for { data, _, err := r.ReadPacketData(); ...; parser.DecodeLayers(data, &decoded) }
//
// (pcapgo/read.go:120-177 feeding parser.go:277-317) for a capture already in memory (read
// or mmap'ed).  Records are indexed in place, the raw capture bytes go to HBM in chunks and
// every record is decoded; up to maxPackets records are returned.  The error is the one the
// read loop would have ended on: nil when the capture ended cleanly (io.EOF in the loop) or
// the limit was reached, else the reference's text for the rejected record (the records
// before it are decoded and counted in the Result).  next is where the next record header
// starts.
func (p *BatchDecodingLayerParser) DecodeCapture(capture []byte, maxPackets int) (r *Result, next int, err error) {
	if len(capture) < C.GPD_PCAP_HEADER_BYTES {
		return nil, 0, io.ErrUnexpectedEOF
	}
	if err := p.configure(); err != nil {
		return nil, 0, err
	}
	if maxPackets <= 0 {
		return newResult(0), C.GPD_PCAP_HEADER_BYTES, nil
	}
	r = newResult(maxPackets)
	out := r.cResult()
	var pn runtime.Pinner // out (Go memory) points into r's slices
	defer pn.Unpin()
	r.pin(&pn)
	var n, pos C.uint64_t
	var stop C.int
	rc := C.gpd_decode_pcap(p.ctx, (*C.uint8_t)(unsafe.Pointer(&capture[0])), C.uint64_t(len(capture)),
		C.uint64_t(maxPackets), &out, &n, &pos, &stop, 0)
	runtime.KeepAlive(capture)
	r.truncate(int(n))
	switch {
	case rc == C.GPD_ERR_PCAP:
		return r, int(pos), errors.New(C.GoString(C.gpd_last_error_string()))
	case rc != C.GPD_OK:
		return nil, 0, lastError("gpd_decode_pcap", rc)
	}
	return r, int(pos), nil
}

// Ring is a mapped TPACKET_V3 ring (afpacket options.go blockSize/numBlocks).  The Go side
// owns the mmap (golang.org/x/sys/unix.Mmap on the AF_PACKET socket, as afpacket.go:
// 155-240 sets it up); Ring only reads and releases its blocks.
type Ring struct {
	Mem       []byte
	BlockSize uint32
	NumBlocks uint32
	next      uint32 // afpacket.go:445 offset: the block the next read starts at
}

// RingPackets is the capture info of the packets a DecodeRing call decoded, in ring order
// (CaptureInfo, afpacket.go:318-326).
type RingPackets struct {
	Offset    []uint64 // frame start in Ring.Mem
	CapLen    []uint32
	Length    []uint32
	Timestamp []uint64 // Unix nanoseconds
	IfIndex   []int32
	VLAN      []int32 // AncillaryVLAN value, -1 when absent
}

// DecodeRing replaces the ZeroCopyReadPacketData + DecodeLayers loop over every block the
// kernel has already handed to user space (afpacket.go:300-330, header.go:137-195): the
// blocks are walked from the ring position, their bytes decoded where they lie, and the
// walked blocks handed back (releaseCurrentPacket, afpacket.go:282-287) once the results
// are in host memory.  addVLANHeader is OptAddVLANHeader (header.go:74-82,168-173).
// A call that finds the next block still owned by the kernel returns zero packets; the
// caller polls (afpacket.go:457-483) and calls again.
func (p *BatchDecodingLayerParser) DecodeRing(ring *Ring, maxPackets int, addVLANHeader bool) (*Result, *RingPackets, error) {
	if maxPackets <= 0 || len(ring.Mem) == 0 {
		return nil, nil, errors.New("gpdecode: DecodeRing needs a mapped ring and maxPackets > 0")
	}
	if err := p.configure(); err != nil {
		return nil, nil, err
	}
	cr := C.gpd_tpv3_ring{base: (*C.uint8_t)(unsafe.Pointer(&ring.Mem[0])),
		block_size: C.uint32_t(ring.BlockSize), num_blocks: C.uint32_t(ring.NumBlocks)}
	r := newResult(maxPackets)
	pk := &RingPackets{make([]uint64, maxPackets), make([]uint32, maxPackets), make([]uint32, maxPackets),
		make([]uint64, maxPackets), make([]int32, maxPackets), make([]int32, maxPackets)}
	cpk := C.gpd_tpv3_pkts{
		offset:   (*C.uint64_t)(unsafe.Pointer(&pk.Offset[0])),
		caplen:   (*C.uint32_t)(unsafe.Pointer(&pk.CapLen[0])),
		wire_len: (*C.uint32_t)(unsafe.Pointer(&pk.Length[0])),
		ts_ns:    (*C.uint64_t)(unsafe.Pointer(&pk.Timestamp[0])),
		ifindex:  (*C.int32_t)(unsafe.Pointer(&pk.IfIndex[0])),
		vlan:     (*C.int32_t)(unsafe.Pointer(&pk.VLAN[0])),
	}
	out := r.cResult()
	// out and cpk (Go memory) point into Go slices: pinned for the call; ring.Mem is the
	// mmap'ed ring (not Go memory), which cgo passes as it is
	var pn runtime.Pinner
	defer pn.Unpin()
	r.pin(&pn)
	pinFirst(&pn, pk.Offset, pk.CapLen, pk.Length, pk.Timestamp, pk.IfIndex, pk.VLAN)
	add := C.int(0)
	if addVLANHeader {
		add = 1
	}
	var n C.uint64_t
	var blocks C.uint32_t
	if rc := C.gpd_decode_tpv3(p.ctx, &cr, C.uint32_t(ring.next), C.uint32_t(ring.NumBlocks), add,
		C.uint64_t(maxPackets), &out, &cpk, &n, &blocks, 0); rc != C.GPD_OK {
		return nil, nil, lastError("gpd_decode_tpv3", rc)
	}
	if blocks > 0 {
		if rc := C.gpd_tpv3_release(&cr, C.uint32_t(ring.next), blocks); rc != C.GPD_OK {
			return nil, nil, lastError("gpd_tpv3_release", rc)
		}
		ring.next = (ring.next + uint32(blocks)) % ring.NumBlocks
	}
	runtime.KeepAlive(ring.Mem)
	r.truncate(int(n))
	k := int(n)
	pk.Offset, pk.CapLen, pk.Length = pk.Offset[:k], pk.CapLen[:k], pk.Length[:k]
	pk.Timestamp, pk.IfIndex, pk.VLAN = pk.Timestamp[:k], pk.IfIndex[:k], pk.VLAN[:k]
	return r, pk, nil
}

// CaptureInfo is packet i's gopacket.CaptureInfo.
func (pk *RingPackets) CaptureInfo(i int) gopacket.CaptureInfo {
	ci := gopacket.CaptureInfo{Timestamp: time.Unix(0, int64(pk.Timestamp[i])),
		CaptureLength: int(pk.CapLen[i]), Length: int(pk.Length[i]), InterfaceIndex: int(pk.IfIndex[i])}
	if pk.VLAN[i] >= 0 {
		ci.AncillaryData = append(ci.AncillaryData, layers.AncillaryVLAN{VLAN: int(pk.VLAN[i])})
	}
	return ci
}

// FlowTable is the batch form of tcpassembly's StreamPool connection map
// (tcpassembly/assembly.go:289-343,495-511): every decoded packet with a network and a
// TCP/UDP transport layer is looked up by its [2]gopacket.Flow key in an HBM hash table, a
// new key creates a record, and each packet gets its record's index.  The table lives on the
// parser's device; Insert takes the batch through HBM itself.
type FlowTable struct {
	ft     *C.gpd_flowtable
	parser *BatchDecodingLayerParser
	seq    uint64
}

// Flow-id values besides a record index (gpd_flow.h).
const (
	FlowNone      = C.GPD_FLOW_NONE
	FlowFull      = C.GPD_FLOW_FULL
	FlowCollision = C.GPD_FLOW_COLLISION
)

// NewFlowTable is tcpassembly.NewStreamPool with room for at least capacity connections.
func (p *BatchDecodingLayerParser) NewFlowTable(capacity int) (*FlowTable, error) {
	t := &FlowTable{parser: p}
	if rc := C.gpd_flow_create(p.ctx, C.uint64_t(capacity), &t.ft); rc != C.GPD_OK {
		return nil, lastError("gpd_flow_create", rc)
	}
	runtime.SetFinalizer(t, (*FlowTable).Close)
	return t, nil
}

// Close frees the table.
func (t *FlowTable) Close() {
	if t.ft != nil {
		C.gpd_flow_destroy(t.ft)
		t.ft = nil
	}
}

type devBuf struct{ p unsafe.Pointer }

// onDevice pins the goroutine to its OS thread and makes the parser's GPU current there, so
// the hipMalloc / hipMemcpy calls that follow land on the context's device (HIP's current
// device is per thread).  The returned func undoes the pin.
func (p *BatchDecodingLayerParser) onDevice() (func(), error) {
	runtime.LockOSThread()
	if e := C.hipSetDevice(C.int(p.device)); e != C.hipSuccess {
		runtime.UnlockOSThread()
		return nil, fmt.Errorf("hipSetDevice(%d): %s", p.device, C.GoString(C.hipGetErrorString(e)))
	}
	return runtime.UnlockOSThread, nil
}

// bytesPtr is &b[0], or nil for an empty slice (a batch of empty packets has no bytes).
func bytesPtr(b []byte) unsafe.Pointer {
	if len(b) == 0 {
		return nil
	}
	return unsafe.Pointer(&b[0])
}

func devAlloc(n int) (devBuf, error) {
	var p unsafe.Pointer
	if e := C.hipMalloc(&p, C.size_t(n+16)); e != C.hipSuccess {
		return devBuf{}, fmt.Errorf("hipMalloc(%d): %s", n, C.GoString(C.hipGetErrorString(e)))
	}
	return devBuf{p}, nil
}

func (d devBuf) free() { C.hipFree(d.p) }

func toDev(d devBuf, b unsafe.Pointer, n int) error {
	if n == 0 {
		return nil
	}
	if e := C.hipMemcpy(d.p, b, C.size_t(n), C.hipMemcpyHostToDevice); e != C.hipSuccess {
		return errors.New(C.GoString(C.hipGetErrorString(e)))
	}
	return nil
}

// Insert decodes b on the device and assigns every packet its flow (getConnection for each
// packet, assembly.go:533-543).  The returned ids index the records Flows returns; packets
// count as sequence numbers continuing from the previous Insert.
func (t *FlowTable) Insert(b *PacketBatch) (*Result, []uint32, error) {
	n := len(b.Offset)
	r := newResult(n)
	ids := make([]uint32, n)
	if n == 0 {
		return r, ids, nil
	}
	if err := t.parser.configure(); err != nil {
		return nil, nil, err
	}
	done, err := t.parser.onDevice()
	if err != nil {
		return nil, nil, err
	}
	defer done()
	sizes := []int{(len(b.Data)+15)&^15 + 64, 4 * n, 4 * n, 4 * n, 8 * n, 8 * n, 8 * n, 4 * n, 4 * n, 4 * n}
	bufs := make([]devBuf, len(sizes))
	for k, s := range sizes {
		d, err := devAlloc(s)
		if err != nil {
			return nil, nil, err
		}
		bufs[k] = d
		defer d.free()
	}
	if err := toDev(bufs[0], bytesPtr(b.Data), len(b.Data)); err != nil {
		return nil, nil, err
	}
	if err := toDev(bufs[1], unsafe.Pointer(&b.Offset[0]), 4*n); err != nil {
		return nil, nil, err
	}
	if err := toDev(bufs[2], unsafe.Pointer(&b.CapLen[0]), 4*n); err != nil {
		return nil, nil, err
	}
	in := C.gpd_batch{data: (*C.uint8_t)(bufs[0].p), data_len: C.uint64_t(len(b.Data)),
		offset: (*C.uint32_t)(bufs[1].p), caplen: (*C.uint32_t)(bufs[2].p), n: C.uint64_t(n)}
	res := C.gpd_result{status: (*C.uint32_t)(bufs[3].p), layers: (*C.uint64_t)(bufs[4].p),
		net_hash: (*C.uint64_t)(bufs[5].p), tp_hash: (*C.uint64_t)(bufs[6].p),
		csum: (*C.uint32_t)(bufs[7].p), hdr_off: (*C.uint32_t)(bufs[8].p)}
	if rc := C.gpd_decode(t.parser.ctx, &in, &res, nil); rc != C.GPD_OK {
		return nil, nil, lastError("gpd_decode", rc)
	}
	if rc := C.gpd_flow_insert(t.ft, &in, &res, (*C.uint32_t)(bufs[9].p), C.uint64_t(t.seq), nil); rc != C.GPD_OK {
		return nil, nil, lastError("gpd_flow_insert", rc)
	}
	if rc := C.gpd_sync(t.parser.ctx, nil); rc != C.GPD_OK {
		return nil, nil, lastError("gpd_sync", rc)
	}
	t.seq += uint64(n)
	back := []struct {
		dst unsafe.Pointer
		src devBuf
		n   int
	}{{unsafe.Pointer(&r.Status[0]), bufs[3], 4 * n}, {unsafe.Pointer(&r.Layers[0]), bufs[4], 8 * n},
		{unsafe.Pointer(&r.NetHash[0]), bufs[5], 8 * n}, {unsafe.Pointer(&r.TpHash[0]), bufs[6], 8 * n},
		{unsafe.Pointer(&r.Checksum[0]), bufs[7], 4 * n}, {unsafe.Pointer(&r.HdrOff[0]), bufs[8], 4 * n},
		{unsafe.Pointer(&ids[0]), bufs[9], 4 * n}}
	for _, c := range back {
		if e := C.hipMemcpy(c.dst, c.src.p, C.size_t(c.n), C.hipMemcpyDeviceToHost); e != C.hipSuccess {
			return nil, nil, errors.New(C.GoString(C.hipGetErrorString(e)))
		}
	}
	runtime.KeepAlive(b)
	return r, ids, nil
}

// FlowRecord is one connection of the table: its [2]gopacket.Flow key and counters.
type FlowRecord struct {
	Index          uint32
	Net, Transport gopacket.Flow
	First, Last    uint64 // packet sequence numbers
	Packets, Bytes uint64
}

// Flows lists the table's connections in order of first appearance (StreamPool.connections,
// assembly.go:193-200).
func (t *FlowTable) Flows() ([]FlowRecord, error) {
	var st C.gpd_flow_stats
	if rc := C.gpd_flow_stats_get(t.ft, &st, nil); rc != C.GPD_OK {
		return nil, lastError("gpd_flow_stats_get", rc)
	}
	if st.flows == 0 {
		return nil, nil
	}
	recs := make([]C.gpd_flow_rec, st.flows)
	idx := make([]uint32, st.flows)
	var n C.uint64_t
	if rc := C.gpd_flow_export(t.ft, &recs[0], (*C.uint32_t)(unsafe.Pointer(&idx[0])), st.flows, &n, nil); rc != C.GPD_OK {
		return nil, lastError("gpd_flow_export", rc)
	}
	out := make([]FlowRecord, int(n))
	for k := range out {
		c := &recs[k]
		al := int(c.addr_len)
		src := C.GoBytes(unsafe.Pointer(&c.src[0]), C.int(al))
		dst := C.GoBytes(unsafe.Pointer(&c.dst[0]), C.int(al))
		netType, tpType := layers.EndpointIPv4, layers.EndpointTCPPort
		if c.net_type == 2 {
			netType = layers.EndpointIPv6
		}
		if c.tp_type == 5 {
			tpType = layers.EndpointUDPPort
		}
		out[k] = FlowRecord{Index: idx[k], Net: gopacket.NewFlow(netType, src, dst),
			Transport: gopacket.NewFlow(tpType, C.GoBytes(unsafe.Pointer(&c.sport[0]), 2),
				C.GoBytes(unsafe.Pointer(&c.dport[0]), 2)),
			First: uint64(c.first), Last: uint64(c.last), Packets: uint64(c.packets), Bytes: uint64(c.bytes)}
	}
	return out, nil
}

func newResult(n int) *Result {
	return &Result{make([]uint32, n), make([]uint64, n), make([]uint64, n), make([]uint64, n),
		make([]uint32, n), make([]uint32, n), make([]Detail, n)}
}

// cResult points a gpd_result at r's arrays (r must hold at least one entry per packet).
func (r *Result) cResult() C.gpd_result {
	if len(r.Status) == 0 {
		return C.gpd_result{}
	}
	return C.gpd_result{
		status:   (*C.uint32_t)(unsafe.Pointer(&r.Status[0])),
		layers:   (*C.uint64_t)(unsafe.Pointer(&r.Layers[0])),
		net_hash: (*C.uint64_t)(unsafe.Pointer(&r.NetHash[0])),
		tp_hash:  (*C.uint64_t)(unsafe.Pointer(&r.TpHash[0])),
		csum:     (*C.uint32_t)(unsafe.Pointer(&r.Checksum[0])),
		hdr_off:  (*C.uint32_t)(unsafe.Pointer(&r.HdrOff[0])),
		detail:   (*C.gpd_detail)(unsafe.Pointer(&r.Detail[0])), // same 24-byte layout
	}
}

// pin pins r's arrays (the ones cResult points a gpd_result at) until pn.Unpin.
func (r *Result) pin(pn *runtime.Pinner) {
	pinFirst(pn, r.Status, r.Layers, r.NetHash, r.TpHash, r.Checksum, r.HdrOff)
	if len(r.Detail) > 0 {
		pn.Pin(&r.Detail[0])
	}
}

func (r *Result) truncate(n int) {
	r.Status, r.Layers, r.NetHash = r.Status[:n], r.Layers[:n], r.NetHash[:n]
	r.TpHash, r.Checksum, r.HdrOff = r.TpHash[:n], r.Checksum[:n], r.HdrOff[:n]
	r.Detail = r.Detail[:n]
}

// FastHashes is Flow.FastHash (flows.go:167-174) of many caller-built flows in one device
// launch (gpd_fast_hash): the EndpointType, both raw endpoints zero-padded to
// gopacket.MaxEndpointSize and their lengths go to HBM as gopacket lays a Flow out, and
// out[i] == flows[i].FastHash().  Use it for keys a program builds itself (tcpassembly's
// [2]gopacket.Flow from stored records); decoded packets carry theirs in Result.NetHash/TpHash.
func (p *BatchDecodingLayerParser) FastHashes(flows []gopacket.Flow) ([]uint64, error) {
	n := len(flows)
	out := make([]uint64, n)
	if n == 0 {
		return out, nil
	}
	typ := make([]int64, n)
	raw := make([]byte, 32*n) // src rows, then dst rows, 16 bytes each
	lens := make([]byte, 2*n) // src lengths, then dst lengths
	for i, f := range flows {
		src, dst := f.Endpoints()
		typ[i] = int64(f.EndpointType())
		lens[i] = byte(copy(raw[16*i:16*i+16], src.Raw()))
		lens[n+i] = byte(copy(raw[16*(n+i):16*(n+i)+16], dst.Raw()))
	}
	done, err := p.onDevice()
	if err != nil {
		return nil, err
	}
	defer done()
	sizes := []int{8 * n, 32 * n, 2 * n, 8 * n}
	bufs := make([]devBuf, len(sizes))
	for k, s := range sizes {
		d, err := devAlloc(s)
		if err != nil {
			return nil, err
		}
		bufs[k] = d
		defer d.free()
	}
	for k, h := range []unsafe.Pointer{unsafe.Pointer(&typ[0]), unsafe.Pointer(&raw[0]), unsafe.Pointer(&lens[0])} {
		if err := toDev(bufs[k], h, sizes[k]); err != nil {
			return nil, err
		}
	}
	src := (*C.uint8_t)(bufs[1].p)
	dst := (*C.uint8_t)(unsafe.Pointer(uintptr(bufs[1].p) + uintptr(16*n))) // (device memory: go 1.12's module)
	if rc := C.gpd_fast_hash(C.int(p.device), C.uint64_t(n), (*C.int64_t)(bufs[0].p), src, (*C.uint8_t)(bufs[2].p),
		dst, (*C.uint8_t)(unsafe.Pointer(uintptr(bufs[2].p) + uintptr(n))), (*C.uint64_t)(bufs[3].p), nil); rc != C.GPD_OK {
		return nil, lastError("gpd_fast_hash", rc)
	}
	if e := C.hipMemcpy(unsafe.Pointer(&out[0]), bufs[3].p, C.size_t(8*n), C.hipMemcpyDeviceToHost); e != C.hipSuccess {
		return nil, errors.New(C.GoString(C.hipGetErrorString(e)))
	}
	return out, nil
}
