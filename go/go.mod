// Go drop-ins for the reference's broker and worker processes over libgolhip.so (cgo).
// No external requirements: the wire types are declared in package golhip with the
// reference's gob field names (stubs/stubs.go:13-38, util/cell.go:4-5).
module golhip.local/gol

go 1.21
