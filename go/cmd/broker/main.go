// Command broker is the drop-in for the reference's broker process (broker/broker.go): the same
// net/rpc service Operations on the same -port flag.  The board of a Run stays resident on the
// GPU(s) (libgolhip's engine, row-sharded over -gpus GPUs with RCCL halo exchange) instead of
// being shipped to every worker every turn (broker.go:143-157), so no worker list is dialled and
// Threads > number of workers no longer crashes (broker.go:146).
package main

import (
	"flag"
	"fmt"
	"net"
	"net/rpc"
	"os"

	"golhip.local/gol/golhip"
)

// Operations is the broker's RPC service (broker.go:60).
type Operations struct {
	b         *golhip.Broker
	superQuit chan bool
}

// Run is broker.go:62-234.
func (s *Operations) Run(req golhip.Request, res *golhip.Response) error { return s.b.Run(req, res) }

// RetrieveCurrentData is broker.go:256-277.
func (s *Operations) RetrieveCurrentData(req golhip.Request, res *golhip.Response) error {
	return s.b.RetrieveCurrentData(req, res)
}

// Pause is broker.go:251-254.
func (s *Operations) Pause(req golhip.Request, res *golhip.Response) error { return s.b.Pause() }

// Quit is broker.go:236-239.
func (s *Operations) Quit(req golhip.Request, res *golhip.Response) error { return s.b.Quit() }

// SuperQuit is broker.go:241-249: stop the run and the listener.
func (s *Operations) SuperQuit(req golhip.Request, res *golhip.Response) error {
	err := s.b.SuperQuit()
	s.superQuit <- true
	return err
}

func main() {
	port := flag.String("port", "8040", "port to listen on") // broker.go:281
	gpus := flag.Int("gpus", 1, "GPUs the board of a Run is row-sharded over")
	k := flag.Int("k", 0, "turns per kernel launch (0 = library default)")
	bytesBoard := flag.Bool("bytes", false, "keep the board one byte per cell on one GPU (GOL_LAYOUT_BYTES)")
	flag.Parse()
	layout := 0
	if *bytesBoard {
		layout = golhip.LayoutBytes
	}
	b, err := golhip.NewBroker(golhip.Config{Device: -1, Shards: *gpus, TurnsPerLaunch: *k, Layout: layout})
	if err != nil {
		fmt.Fprintln(os.Stderr, err)
		os.Exit(1)
	}
	defer b.Close()
	ops := &Operations{b: b, superQuit: make(chan bool, 1)}
	if err := rpc.RegisterName("Operations", ops); err != nil {
		fmt.Fprintln(os.Stderr, err)
		os.Exit(1)
	}
	ln, err := net.Listen("tcp", ":"+*port)
	if err != nil {
		fmt.Fprintln(os.Stderr, err)
		os.Exit(1)
	}
	go func() {
		<-ops.superQuit
		ln.Close()
	}()
	rpc.Accept(ln)
}
