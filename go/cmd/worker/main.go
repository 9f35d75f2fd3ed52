// Command worker is the drop-in for the reference's worker process (worker/worker.go): the
// same net/rpc service GameOfLifeOperations on the same -port flag, with the next-state of a
// row slab computed on the GPU by libgolhip.so instead of worker.go:15-70's per-cell loops.
package main

import (
	"flag"
	"fmt"
	"net"
	"net/rpc"
	"os"

	"golhip.local/gol/golhip"
)

// GameOfLifeOperations is the worker's RPC service (worker.go:73-86).
type GameOfLifeOperations struct{ quit chan bool }

// Update is worker.go:77-80: res.WorkSlice = next state of rows [StartY, EndY).
func (s *GameOfLifeOperations) Update(req golhip.Request, res *golhip.Response) (err error) {
	res.WorkSlice, err = golhip.NextStateSlab(req.World, req.StartY, req.EndY)
	res.Worker = req.Worker
	return
}

// WorkerQuit is worker.go:82-86: stop serving.
func (s *GameOfLifeOperations) WorkerQuit(req golhip.Request, res *golhip.Response) error {
	s.quit <- true
	return nil
}

func main() {
	port := flag.String("port", "8030", "port to listen on") // worker.go:91
	flag.Parse()
	ops := &GameOfLifeOperations{quit: make(chan bool, 1)}
	if err := rpc.RegisterName("GameOfLifeOperations", ops); err != nil {
		fmt.Fprintln(os.Stderr, err)
		os.Exit(1)
	}
	ln, err := net.Listen("tcp", ":"+*port)
	if err != nil {
		fmt.Fprintln(os.Stderr, err)
		os.Exit(1)
	}
	go func() {
		<-ops.quit
		ln.Close()
	}()
	rpc.Accept(ln)
}
