// Package infectious is a drop-in replacement for the subset of
// github.com/vivint/infectious that da-moon/noise-erasurecode-plugin uses
// (main.go:24 import; NewFEC main.go:73,:248; (*FEC).Encode main.go:262;
// (*FEC).Decode main.go:77; Share / DeepCopy main.go:57-69,:254-258),
// implemented over the MI355X engine's C ABI (include/rsmi.h) with cgo.
//
// The plugin changes only its import path; every call site compiles as is.
// Requires Go >= 1.21 (runtime.Pinner) and lib/librsmi.so built by
// `make -C noise-erasurecode-plugin_amd/csrc`.  Not compiled in this
// repository's CI (no Go toolchain in the build image); see INTEGRATION.md.
package infectious

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../lib -lrsmi -Wl,-rpath,${SRCDIR}/../../lib
#include <stdlib.h>
#include "rsmi.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"sort"
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

// FEC is a (k, n) code bound to one GPU context.  The context is shared by
// every FEC with the same (k, n) in the process (the plugin calls NewFEC for
// every message, main.go:73/:248; building and uploading tables each time
// would dominate small messages).
type FEC struct {
	k, n int
	ctx  *C.rs_ctx
	mu   sync.Mutex // guards parity (reused between Encode calls like infectious)
	par  []byte
}

var (
	ctxMu    sync.Mutex
	ctxCache = map[[2]int]*C.rs_ctx{}
)

// NewFEC mirrors infectious.NewFEC(k, n): error unless 1 <= k <= n <= 256.
func NewFEC(k, n int) (*FEC, error) {
	if k <= 0 || n <= 0 || k > 256 || n > 256 || k > n {
		return nil, errors.New("requires 1 <= k <= n <= 256")
	}
	ctxMu.Lock()
	defer ctxMu.Unlock()
	ctx, ok := ctxCache[[2]int{k, n}]
	if !ok {
		if st := C.rs_new(C.int(k), C.int(n), &ctx); st != C.RS_OK {
			return nil, statusErr(st)
		}
		ctxCache[[2]int{k, n}] = ctx
	}
	return &FEC{k: k, n: n, ctx: ctx}, nil
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
