"""golhip -- MI355X-native Game-of-Life hot path behind the reference's broker/worker API.

* ``Engine``               one GPU, board resident in HBM (gol_engine_*)
* ``Operations``           broker RPC service mirror (broker.go:62-277)
* ``GameOfLifeOperations`` worker RPC service mirror (worker.go:73-86)
* ``ShardedBoard``         torch.distributed mirror of the sharded step (runs the library's plans)
* ``halo_plan`` / ``step_plan``  the sharded step's schedule as data (gol_halo_plan, gol_step_plan)
* ``distributor``          controller mirror (gol/gol.go + gol/distributor.go) over the broker API
* ``next_state_slab`` / ``partition_rows``  worker.go:15-70 / broker.go:135-206

Everything runs through libgolhip.so (hipcc, gfx950); there is no CPU fallback.
"""
from ._lib import GolError, device_count, halo_plan, lib, step_plan  # noqa: F401
from .broker import Operations  # noqa: F401
from .engine import Engine, next_state_slab, partition_rows  # noqa: F401
from .pgm import read_pgm, write_pgm_bytes  # noqa: F401
from .stubs import Cell, CellList, Parameters, Request, Response  # noqa: F401
from .worker import GameOfLifeOperations  # noqa: F401


def sharded_board(*args, **kwargs):
    """Construct a ShardedBoard (imports torch lazily)."""
    from .sharded import ShardedBoard
    return ShardedBoard(*args, **kwargs)
