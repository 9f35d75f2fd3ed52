package golhip

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../gol-distributed-final_amd/golhip -lgolhip -Wl,-rpath,${SRCDIR}/../../gol-distributed-final_amd/golhip
#include <stdlib.h>
#include "golhip.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"unsafe"
)

// Error is a nonzero status of a libgolhip call with its gol_last_error message.
type Error struct {
	Code    int
	Message string
}

func (e *Error) Error() string { return fmt.Sprintf("golhip %d: %s", e.Code, e.Message) }

func check(rc C.int) error {
	if rc == C.GOL_OK {
		return nil
	}
	return &Error{Code: int(rc), Message: C.GoString(C.gol_last_error())}
}

// flatten copies a [][]byte board into one contiguous buffer (the C ABI's row-major bytes).
func flatten(world [][]byte, h, w int) ([]byte, error) {
	if len(world) != h {
		return nil, fmt.Errorf("World has %d rows, ImageHeight is %d", len(world), h)
	}
	flat := make([]byte, h*w)
	for y, row := range world {
		if len(row) != w {
			return nil, fmt.Errorf("World row %d has %d bytes, ImageWidth is %d", y, len(row), w)
		}
		copy(flat[y*w:(y+1)*w], row)
	}
	return flat, nil
}

func rows(flat []byte, h, w int) [][]byte {
	out := make([][]byte, h)
	for y := range out {
		out[y] = flat[y*w : (y+1)*w]
	}
	return out
}

func bytePtr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// NextStateSlab is calculateNextState (worker.go:15-42) on the GPU: the next state of rows
// [startY, endY) of the h x w torus `world`.
func NextStateSlab(world [][]byte, startY, endY int) ([][]byte, error) {
	if len(world) == 0 {
		return nil, errors.New("empty World")
	}
	h, w := len(world), len(world[0])
	flat, err := flatten(world, h, w)
	if err != nil {
		return nil, err
	}
	out := make([]byte, (endY-startY)*w)
	if err := check(C.gol_next_state_slab(bytePtr(flat), C.int64_t(h), C.int64_t(w), C.int64_t(w),
		C.int64_t(startY), C.int64_t(endY), bytePtr(out), C.int64_t(w))); err != nil {
		return nil, err
	}
	return rows(out, endY-startY, w), nil
}

// PartitionRows is the broker's row split (broker.go:135-139, 172-206): rows of part i of n.
func PartitionRows(h, n, i int) (int, int, error) {
	var y0, y1 C.int64_t
	if err := check(C.gol_partition_rows(C.int64_t(h), C.int64_t(n), C.int64_t(i), &y0, &y1)); err != nil {
		return 0, 0, err
	}
	return int(y0), int(y1), nil
}

// LayoutBytes keeps a Run's board one byte per cell (GOL_LAYOUT_BYTES): one GPU, the byte pipeline.
const LayoutBytes = int(C.GOL_LAYOUT_BYTES)

// Config selects the broker's GPUs and kernel parameters (gol_config).
type Config struct {
	Device         int // first GPU; -1 = current
	Shards         int // GPUs the board of a Run is row-sharded over (<= 1: one GPU)
	TurnsPerLaunch int // 0 = library default
	Layout         int // 0 = automatic (bit board); LayoutBytes = one byte per cell, one GPU
}

// Broker is the C++ service behind the reference's Operations (broker.go:62-277): the board
// stays resident on the GPU(s) for the whole Run.
type Broker struct{ b *C.gol_broker }

// NewBroker creates the service object.
func NewBroker(cfg Config) (*Broker, error) {
	var b *C.gol_broker
	c := C.gol_config{device: C.int32_t(cfg.Device), turns_per_launch: C.int32_t(cfg.TurnsPerLaunch),
		shards: C.int32_t(cfg.Shards), layout: C.int32_t(cfg.Layout)}
	if err := check(C.gol_broker_create(&c, &b)); err != nil {
		return nil, err
	}
	return &Broker{b}, nil
}

// Close releases the GPU state.
func (s *Broker) Close() { C.gol_broker_destroy(s.b) }

// aliveBufPairs bounds the alive-list buffer handed to C per call (pairs of int32).
const aliveBufPairs = 1 << 20

type brokerCall func(*C.gol_broker, *C.gol_request, *C.gol_response) C.int

// call runs one broker method with Go-owned buffers, borrowed by C for the call only.  The
// request / response structs handed to C hold pointers to these buffers, so the buffers are
// pinned for the call (cgo pointer rules, runtime.Pinner).
func (s *Broker) call(f brokerCall, req Request, res *Response, wantWorld bool) error {
	var pin runtime.Pinner
	defer pin.Unpin()
	h, w := req.ImageHeight, req.ImageWidth
	creq := C.gol_request{Turns: C.int64_t(req.Turns), ImageHeight: C.int64_t(h), ImageWidth: C.int64_t(w),
		Threads: C.int64_t(req.Threads), EndY: C.int64_t(req.EndY), StartY: C.int64_t(req.StartY),
		Worker: C.int64_t(req.Worker)}
	if len(req.World) > 0 {
		flat, err := flatten(req.World, h, w)
		if err != nil {
			return err
		}
		pin.Pin(&flat[0])
		creq.World = bytePtr(flat)
		creq.world_stride = C.int64_t(w)
	}
	var world []byte
	cres := C.gol_response{}
	if wantWorld && h*w > 0 {
		world = make([]byte, h*w)
		pin.Pin(&world[0])
		cres.World = bytePtr(world)
		cres.world_stride = C.int64_t(w)
	}
	// The alive list (broker.go:47-58) comes back through a bounded buffer: a typical board's
	// list fits; a longer one is rebuilt here from the returned World (the same rule: every
	// byte != 0, row-major) instead of reserving 8 bytes per cell on every call.
	capPairs := h * w
	if capPairs > aliveBufPairs {
		capPairs = aliveBufPairs
	}
	alive := make([]C.int32_t, 2*capPairs+2)
	pin.Pin(&alive[0])
	cres.Alive = &alive[0]
	cres.alive_cap = C.int64_t(capPairs)
	if err := check(f(s.b, &creq, &cres)); err != nil {
		return err
	}
	res.TurnsCompleted, res.AliveCount = int(cres.TurnsCompleted), int(cres.AliveCount)
	if world != nil {
		res.World = rows(world, h, w)
	}
	n := int(cres.alive_len)
	if n <= capPairs {
		res.Alive = make([]Cell, n)
		for i := range res.Alive {
			res.Alive[i] = Cell{X: int(alive[2*i]), Y: int(alive[2*i+1])}
		}
	} else {
		res.Alive = make([]Cell, 0, n)
		for y := 0; y < h; y++ {
			for x, v := range world[y*w : (y+1)*w] {
				if v != 0 {
					res.Alive = append(res.Alive, Cell{X: x, Y: y})
				}
			}
		}
	}
	return nil
}

// Run is Operations.Run (broker.go:62-234).
func (s *Broker) Run(req Request, res *Response) error {
	return s.call(func(b *C.gol_broker, q *C.gol_request, r *C.gol_response) C.int { return C.gol_broker_run(b, q, r) },
		req, res, true)
}

// RetrieveCurrentData is Operations.RetrieveCurrentData (broker.go:256-277).
func (s *Broker) RetrieveCurrentData(req Request, res *Response) error {
	return s.call(func(b *C.gol_broker, q *C.gol_request, r *C.gol_response) C.int {
		return C.gol_broker_retrieve(b, q, r)
	}, req, res, true)
}

// Pause is Operations.Pause (broker.go:251-254).
func (s *Broker) Pause() error { return check(C.gol_broker_pause(s.b)) }

// Quit is Operations.Quit (broker.go:236-239).
func (s *Broker) Quit() error { return check(C.gol_broker_quit(s.b)) }

// SuperQuit is Operations.SuperQuit (broker.go:241-249).
func (s *Broker) SuperQuit() error { return check(C.gol_broker_superquit(s.b)) }
