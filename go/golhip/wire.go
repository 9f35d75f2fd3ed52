// Package golhip binds libgolhip.so (include/golhip.h) for the reference's net/rpc
// processes and declares their wire types.
//
// encoding/gob matches struct fields by name, so these types interoperate with the
// reference's stubs.Request / stubs.Response (stubs/stubs.go:20-38) and util.Cell
// (util/cell.go:4-5) although they live in another package.
package golhip

// RPC method names the reference's controller and broker call (stubs/stubs.go:5-11).
const (
	MethodUpdate     = "GameOfLifeOperations.Update"
	MethodWorkerQuit = "GameOfLifeOperations.WorkerQuit"
	MethodRun        = "Operations.Run"
	MethodRetrieve   = "Operations.RetrieveCurrentData"
	MethodPause      = "Operations.Pause"
	MethodQuit       = "Operations.Quit"
	MethodSuperQuit  = "Operations.SuperQuit"
)

// Cell is one alive cell, X the column and Y the row.
type Cell struct {
	X, Y int
}

// Request carries the board and the run parameters (gob field names of the reference).
type Request struct {
	World       [][]byte
	Turns       int
	ImageHeight int
	ImageWidth  int
	Threads     int
	EndY        int
	StartY      int
	Worker      int
}

// Response carries the results of a call (gob field names of the reference).
type Response struct {
	Alive          []Cell
	AliveCount     int
	TurnsCompleted int
	World          [][]byte
	WorkSlice      [][]byte
	Worker         int
}
