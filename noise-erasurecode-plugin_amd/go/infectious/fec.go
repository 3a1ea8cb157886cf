// Package infectious is a drop-in replacement for the subset of
// github.com/vivint/infectious that da-moon/noise-erasurecode-plugin uses
// (main.go:24 import; NewFEC main.go:73,:248; (*FEC).Encode main.go:262;
// (*FEC).Decode main.go:77; Share / DeepCopy main.go:57-69,:254-258),
// implemented over the MI355X engine's C ABI (include/rsmi.h) with cgo.
//
// The plugin changes only its import path; every call site compiles as is.
// Requires Go >= 1.21 (runtime.Pinner, min/max builtins) and lib/librsmi.so built by
// `make -C noise-erasurecode-plugin_amd/csrc`.  Not compiled in this
// repository's CI (no Go toolchain in the build image); see INTEGRATION.md.
package infectious

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../lib -lrsmi -Wl,-rpath,${SRCDIR}/../../lib
#include <stdlib.h>
#include "rsmi.h"
#include "rsmi_wire.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"os"
	"runtime"
	"sort"
	"strconv"
	"strings"
	"sync"
	"unsafe"
)

// Share is infectious.Share: a numbered piece of an encoded input.
type Share struct {
	Number int
	Data   []byte
}

// DeepCopy returns a Share whose Data does not alias the receiver's.
func (s *Share) DeepCopy() (out Share) {
	out.Number = s.Number
	out.Data = append([]byte(nil), s.Data...)
	return out
}

type byNumber []Share

func (b byNumber) Len() int           { return len(b) }
func (b byNumber) Less(i, j int) bool { return b[i].Number < b[j].Number }
func (b byNumber) Swap(i, j int)      { b[i], b[j] = b[j], b[i] }

// NotEnoughShares mirrors infectious's error class of the same name.
var NotEnoughShares = errors.New("not enough shares")

func statusErr(st C.int) error {
	switch st {
	case C.RS_OK:
		return nil
	case C.RS_ENOT_ENOUGH:
		return NotEnoughShares
	default:
		return fmt.Errorf("infectious: %s", C.GoString(C.rs_strerror(st)))
	}
}

// FEC is a (k, n) code bound to one GPU context -- or to a device-set
// context over several GPUs (NewFECOnDevices, or NewFEC with RSMI_DEVICES
// set).  NewFEC's context is shared by every FEC with the same (k, n) in the
// process (the plugin calls NewFEC for every message, main.go:73/:248;
// building and uploading tables each time would dominate small messages).
type FEC struct {
	k, n  int
	ctx   *C.rs_ctx
	owned bool       // made by NewFECOnDevices: Close frees it
	mu    sync.Mutex // guards parity (reused between Encode calls like infectious)
	par   []byte
}

var (
	ctxMu    sync.Mutex
	ctxCache = map[[2]int]*C.rs_ctx{}
)

func checkKN(k, n int) error {
	if k <= 0 || n <= 0 || k > 256 || n > 256 || k > n {
		return errors.New("requires 1 <= k <= n <= 256")
	}
	return nil
}

// envDevices parses RSMI_DEVICES ("0,1,2,3,4,5,6,7"): the GPUs NewFEC's
// shared contexts span, so the unchanged plugin (main.go changes only its
// import) partitions its work over every GPU of the node.  Empty: one GPU.
func envDevices() ([]int, error) {
	v := strings.TrimSpace(os.Getenv("RSMI_DEVICES"))
	if v == "" {
		return nil, nil
	}
	var devs []int
	for _, f := range strings.Split(v, ",") {
		d, err := strconv.Atoi(strings.TrimSpace(f))
		if err != nil || d < 0 {
			return nil, fmt.Errorf("infectious: bad RSMI_DEVICES entry %q", f)
		}
		devs = append(devs, d)
	}
	return devs, nil
}

func newDeviceSet(k, n int, devices []int) (*C.rs_ctx, error) {
	cnt := len(devices)
	devs := (*[1 << 16]C.int)(C.malloc(C.size_t(cnt) * C.size_t(unsafe.Sizeof(C.int(0)))))[:cnt:cnt]
	defer C.free(unsafe.Pointer(&devs[0]))
	for i, d := range devices {
		devs[i] = C.int(d)
	}
	var ctx *C.rs_ctx
	if st := C.rs_new_devices(C.int(k), C.int(n), &devs[0], C.int(cnt), &ctx); st != C.RS_OK {
		return nil, statusErr(st)
	}
	return ctx, nil
}

// NewFEC mirrors infectious.NewFEC(k, n): error unless 1 <= k <= n <= 256.
// With RSMI_DEVICES set the shared context is a device set over those GPUs.
func NewFEC(k, n int) (*FEC, error) {
	if err := checkKN(k, n); err != nil {
		return nil, err
	}
	ctxMu.Lock()
	defer ctxMu.Unlock()
	ctx, ok := ctxCache[[2]int{k, n}]
	if !ok {
		devs, err := envDevices()
		if err != nil {
			return nil, err
		}
		if len(devs) > 0 {
			if ctx, err = newDeviceSet(k, n, devs); err != nil {
				return nil, err
			}
		} else if st := C.rs_new(C.int(k), C.int(n), &ctx); st != C.RS_OK {
			return nil, statusErr(st)
		}
		ctxCache[[2]int{k, n}] = ctx
	}
	return &FEC{k: k, n: n, ctx: ctx}, nil
}

// NewFECOnDevices is NewFEC over several GPUs (not in infectious): one
// device-set context (rs_new_devices) with a member per listed HIP device
// (north_star: stripes partitioned over the GPUs of one node).  Encode and
// Decode run on the least busy GPU; EncodeBatch and DecodeBatch split their
// messages into contiguous ranges, one per GPU, all at once.  The context is
// the caller's (not cached): Close frees it.
func NewFECOnDevices(k, n int, devices []int) (*FEC, error) {
	if err := checkKN(k, n); err != nil {
		return nil, err
	}
	if len(devices) == 0 {
		return nil, errors.New("infectious: no devices")
	}
	ctx, err := newDeviceSet(k, n, devices)
	if err != nil {
		return nil, err
	}
	return &FEC{k: k, n: n, ctx: ctx, owned: true}, nil
}

// Devices is the number of GPUs the FEC's context spans.
func (f *FEC) Devices() int { return int(C.rs_member_count(f.ctx)) }

// Close frees a context made by NewFECOnDevices; NewFEC's shared contexts
// live for the process.
func (f *FEC) Close() {
	if f.owned && f.ctx != nil {
		C.rs_free(f.ctx)
		f.ctx = nil
	}
}

// Required is the number of shares needed to reconstruct (k).
func (f *FEC) Required() int { return f.k }

// Total is the number of shares produced (n).
func (f *FEC) Total() int { return f.n }

// Encode calls output for shares 0..n-1.  Data shares alias input; parity
// shares alias a buffer reused by the next Encode (callers DeepCopy, as the
// plugin does at main.go:255-258).
func (f *FEC) Encode(input []byte, output func(Share)) error {
	size := len(input)
	if size%f.k != 0 {
		return fmt.Errorf("input length must be a multiple of %d", f.k)
	}
	bs := size / f.k
	m := f.n - f.k
	f.mu.Lock()
	defer f.mu.Unlock()
	if cap(f.par) < m*bs {
		f.par = make([]byte, m*bs)
	}
	par := f.par[:m*bs]
	if bs > 0 && m > 0 {
		// Go memory passed for the duration of the call only (cgo rules).
		st := C.rs_encode(f.ctx, (*C.uint8_t)(unsafe.Pointer(&input[0])), C.size_t(size),
			(*C.uint8_t)(unsafe.Pointer(&par[0])))
		if st != C.RS_OK {
			return statusErr(st)
		}
	}
	for i := 0; i < f.k; i++ {
		output(Share{Number: i, Data: input[i*bs : (i+1)*bs]})
	}
	for i := 0; i < m; i++ {
		output(Share{Number: f.k + i, Data: par[i*bs : (i+1)*bs]})
	}
	return nil
}

// Decode mirrors (*FEC).Decode(dst, shares): sorts shares by Number in
// place and returns the k*len(share) original bytes in dst (reallocated if
// too small).
func (f *FEC) Decode(dst []byte, shares []Share) ([]byte, error) {
	if len(shares) < f.k {
		return nil, NotEnoughShares
	}
	sort.Sort(byNumber(shares))
	pieceLen := len(shares[0].Data)
	for _, s := range shares {
		if len(s.Data) != pieceLen {
			return nil, errors.New("infectious: shares have different lengths")
		}
	}
	resultLen := pieceLen * f.k
	if cap(dst) < resultLen {
		dst = make([]byte, resultLen)
	} else {
		dst = dst[:resultLen]
	}
	// Zero-length shares still go through rs_decode, which validates the
	// share numbers (invalid id, duplicates) exactly like Rebuild does.
	cnt := len(shares)
	nums := (*[1 << 28]C.int)(C.malloc(C.size_t(cnt) * C.size_t(unsafe.Sizeof(C.int(0)))))[:cnt:cnt]
	ptrs := (*[1 << 28]*C.uint8_t)(C.malloc(C.size_t(cnt) * C.size_t(unsafe.Sizeof(uintptr(0)))))[:cnt:cnt]
	defer C.free(unsafe.Pointer(&nums[0]))
	defer C.free(unsafe.Pointer(&ptrs[0]))
	// Storing Go pointers in C memory requires pinning them (Go 1.21+).
	var pinner runtime.Pinner
	defer pinner.Unpin()
	for i := range shares {
		nums[i] = C.int(shares[i].Number)
		ptrs[i] = nil
		if pieceLen > 0 {
			pinner.Pin(&shares[i].Data[0])
			ptrs[i] = (*C.uint8_t)(unsafe.Pointer(&shares[i].Data[0]))
		}
	}
	var out *C.uint8_t
	if resultLen > 0 {
		out = (*C.uint8_t)(unsafe.Pointer(&dst[0]))
	}
	st := C.rs_decode(f.ctx, &nums[0], (**C.uint8_t)(unsafe.Pointer(&ptrs[0])), C.int(cnt),
		C.size_t(pieceLen), out)
	if st != C.RS_OK {
		return nil, statusErr(st)
	}
	return dst, nil
}

// DecodeBatch decodes many messages of this code in one GPU pass
// (rs_decode_batch; receive-side batching).  msgs[b] holds message b's
// shares, all of one length.  It returns each message's output or error;
// every message's shares are sorted in place like Decode sorts them.  When
// every survivor lies in engine-pinned memory (an Arena filled by
// UnmarshalShard), the GPU reads them there in place.
func (f *FEC) DecodeBatch(msgs [][]Share) ([][]byte, []error) {
	B := len(msgs)
	outs := make([][]byte, B)
	errs := make([]error, B)
	if B == 0 {
		return outs, errs
	}
	pieceLen := 0
	total := 0
	for _, m := range msgs {
		if len(m) > 0 {
			pieceLen = len(m[0].Data)
		}
		total += len(m)
	}
	for b, m := range msgs {
		sort.Sort(byNumber(m))
		for _, s := range m {
			if len(s.Data) != pieceLen {
				errs[b] = errors.New("infectious: shares have different lengths")
			}
		}
		outs[b] = make([]byte, pieceLen*f.k)
	}
	for _, e := range errs {
		if e != nil {
			return outs, errs
		}
	}
	cnt := max(total, 1)
	counts := (*[1 << 28]C.int)(C.malloc(C.size_t(B) * C.size_t(unsafe.Sizeof(C.int(0)))))[:B:B]
	nums := (*[1 << 28]C.int)(C.malloc(C.size_t(cnt) * C.size_t(unsafe.Sizeof(C.int(0)))))[:cnt:cnt]
	ptrs := (*[1 << 28]*C.uint8_t)(C.malloc(C.size_t(cnt) * C.size_t(unsafe.Sizeof(uintptr(0)))))[:cnt:cnt]
	dsts := (*[1 << 28]*C.uint8_t)(C.malloc(C.size_t(B) * C.size_t(unsafe.Sizeof(uintptr(0)))))[:B:B]
	codes := (*[1 << 28]C.int)(C.malloc(C.size_t(B) * C.size_t(unsafe.Sizeof(C.int(0)))))[:B:B]
	defer C.free(unsafe.Pointer(&counts[0]))
	defer C.free(unsafe.Pointer(&nums[0]))
	defer C.free(unsafe.Pointer(&ptrs[0]))
	defer C.free(unsafe.Pointer(&dsts[0]))
	defer C.free(unsafe.Pointer(&codes[0]))
	var pinner runtime.Pinner
	defer pinner.Unpin()
	j := 0
	for b, m := range msgs {
		counts[b] = C.int(len(m))
		for i := range m {
			nums[j] = C.int(m[i].Number)
			ptrs[j] = nil
			if pieceLen > 0 {
				pinner.Pin(&m[i].Data[0])
				ptrs[j] = (*C.uint8_t)(unsafe.Pointer(&m[i].Data[0]))
			}
			j++
		}
		dsts[b] = nil
		if len(outs[b]) > 0 {
			pinner.Pin(&outs[b][0])
			dsts[b] = (*C.uint8_t)(unsafe.Pointer(&outs[b][0]))
		}
	}
	C.rs_decode_batch(f.ctx, C.int(B), &counts[0], &nums[0], (**C.uint8_t)(unsafe.Pointer(&ptrs[0])),
		C.size_t(pieceLen), (**C.uint8_t)(unsafe.Pointer(&dsts[0])), &codes[0])
	for b := range msgs {
		if codes[b] != C.RS_OK {
			errs[b] = statusErr(codes[b])
			outs[b] = nil
		}
	}
	return outs, errs
}

// EncodeBatch is send-side batching (not in infectious): the parity of many
// equal-length messages in one GPU pass (rs_encode_batch).  parities[b] holds
// the n-k parity shares of inputs[b] back to back (share k+t at
// [t*S, (t+1)*S)); the data shares are inputs[b]'s own slices, as Encode
// emits them.
func (f *FEC) EncodeBatch(inputs [][]byte) (parities [][]byte, errs []error) {
	B := len(inputs)
	parities = make([][]byte, B)
	errs = make([]error, B)
	if B == 0 {
		return parities, errs
	}
	size := len(inputs[0])
	for b, in := range inputs {
		if len(in) != size {
			errs[b] = errors.New("infectious: messages have different lengths")
		}
	}
	for _, e := range errs {
		if e != nil {
			return parities, errs
		}
	}
	m := f.n - f.k
	plen := 0
	if size%f.k == 0 {
		plen = size / f.k * m
	}
	ins := (*[1 << 28]*C.uint8_t)(C.malloc(C.size_t(B) * C.size_t(unsafe.Sizeof(uintptr(0)))))[:B:B]
	outs := (*[1 << 28]*C.uint8_t)(C.malloc(C.size_t(B) * C.size_t(unsafe.Sizeof(uintptr(0)))))[:B:B]
	codes := (*[1 << 28]C.int)(C.malloc(C.size_t(B) * C.size_t(unsafe.Sizeof(C.int(0)))))[:B:B]
	defer C.free(unsafe.Pointer(&ins[0]))
	defer C.free(unsafe.Pointer(&outs[0]))
	defer C.free(unsafe.Pointer(&codes[0]))
	var pinner runtime.Pinner
	defer pinner.Unpin()
	for b, in := range inputs {
		parities[b] = make([]byte, plen)
		ins[b], outs[b] = nil, nil
		if size > 0 {
			pinner.Pin(&in[0])
			ins[b] = (*C.uint8_t)(unsafe.Pointer(&in[0]))
		}
		if plen > 0 {
			pinner.Pin(&parities[b][0])
			outs[b] = (*C.uint8_t)(unsafe.Pointer(&parities[b][0]))
		}
	}
	C.rs_encode_batch(f.ctx, C.int(B), (**C.uint8_t)(unsafe.Pointer(&ins[0])), C.size_t(size),
		(**C.uint8_t)(unsafe.Pointer(&outs[0])), &codes[0])
	for b := range inputs {
		if codes[b] != C.RS_OK {
			errs[b] = statusErr(codes[b])
			parities[b] = nil
		}
	}
	return parities, errs
}

// Arena is engine-pinned receive memory (rs_arena).  Shards unmarshalled
// into it are read in place by the GPU.  Not safe for concurrent use: one
// arena per receiving goroutine; Reset once its messages are decoded.
type Arena struct{ a *C.rs_arena }

// NewArena allocates an arena of the given size.
func NewArena(bytes int) (*Arena, error) {
	a := C.rs_arena_new(C.size_t(bytes))
	if a == nil {
		return nil, errors.New("infectious: pinned arena allocation failed")
	}
	return &Arena{a: a}, nil
}

// Reset recycles every slot of the arena.
func (a *Arena) Reset() { C.rs_arena_reset(a.a) }

// Free releases the arena's pinned memory.
func (a *Arena) Free() { C.rs_arena_free(a.a); a.a = nil }

// Put copies a share's bytes into a fresh slot (rs_arena_put: streaming
// stores, so the GPU's reads need not snoop the CPU's caches) and returns a
// Share whose Data aliases the arena (valid until Reset).
func (a *Arena) Put(number int, data []byte) (Share, error) {
	var p unsafe.Pointer
	if len(data) > 0 {
		p = unsafe.Pointer(&data[0])
	}
	slot := C.rs_arena_put(a.a, p, C.size_t(len(data)))
	if slot == nil {
		return Share{}, errors.New("infectious: arena full")
	}
	return Share{Number: number, Data: unsafe.Slice((*byte)(slot), len(data))}, nil
}

// UnmarshalShard parses a wire erasurecode.Shard (protobuf/shard.proto:21-27)
// and places ShardData in the arena -- the one copy gogo's Unmarshal makes
// anyway (shard.pb.go:468-503).  The returned Share's Data aliases the arena
// (valid until Reset); FileSignature is copied.
func (a *Arena) UnmarshalShard(wire []byte) (sig []byte, s Share, total, need uint64, err error) {
	var v C.rs_shard_view
	var p *C.uint8_t
	if len(wire) > 0 {
		p = (*C.uint8_t)(unsafe.Pointer(&wire[0]))
	}
	if st := C.rs_shard_unmarshal_arena(p, C.size_t(len(wire)), a.a, &v); st != 0 {
		return nil, Share{}, 0, 0, fmt.Errorf("proto: Shard unmarshal failed (%d)", int(st))
	}
	sig = C.GoBytes(unsafe.Pointer(v.file_signature), C.int(v.file_signature_len))
	s.Number = int(v.shard_number)
	if v.shard_data_len > 0 {
		s.Data = unsafe.Slice((*byte)(unsafe.Pointer(v.shard_data)), int(v.shard_data_len))
	}
	return sig, s, uint64(v.total_shards), uint64(v.minimum_needed_shards), nil
}

// HashBytes is the blake2b hash policy (main.go:38-41) for one or many
// messages through the engine's host/GPU crossover (rs_blake2b): a single
// message or a batch whose longest chain dominates is hashed on the host
// CPU, many messages in one GPU launch.  digestLen bytes each (noise's
// policy: 32).  Sign / Verify then run on the digests (main.go:219-223,
// :82-89).
func (f *FEC) HashBytes(msgs [][]byte, digestLen int) ([][]byte, error) {
	n := len(msgs)
	if n == 0 {
		return nil, nil
	}
	ptrs := (*[1 << 28]*C.uint8_t)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0)))))[:n:n]
	lens := (*[1 << 28]C.size_t)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.size_t(0)))))[:n:n]
	defer C.free(unsafe.Pointer(&ptrs[0]))
	defer C.free(unsafe.Pointer(&lens[0]))
	var pinner runtime.Pinner
	defer pinner.Unpin()
	for i, m := range msgs {
		ptrs[i] = nil
		lens[i] = C.size_t(len(m))
		if len(m) > 0 {
			pinner.Pin(&m[0])
			ptrs[i] = (*C.uint8_t)(unsafe.Pointer(&m[0]))
		}
	}
	out := make([]byte, n*digestLen)
	if st := C.rs_blake2b(f.ctx, C.int(n), (**C.uint8_t)(unsafe.Pointer(&ptrs[0])), &lens[0], C.int(digestLen),
		(*C.uint8_t)(unsafe.Pointer(&out[0])), nil); st != C.RS_OK {
		return nil, statusErr(st)
	}
	res := make([][]byte, n)
	for i := range res {
		res[i] = out[i*digestLen : (i+1)*digestLen]
	}
	return res, nil
}
