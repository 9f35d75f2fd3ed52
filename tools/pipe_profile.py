"""Per-role wait profile of band_pipe_kernel (diagnostic build with -DGOL_PIPE_PROFILE=1,
loaded through GOLHIP_LIB): fractions of each pipeline role's cycles spent waiting for its
input block, for a free output slot and for its LDS row reads."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gol-distributed-final_amd")]
import torch  # noqa: E402

from golhip.sharded import ShardedBoard  # noqa: E402

H, W = 1 << 17, 1 << 20
b = ShardedBoard(H, W, turns_per_launch=12)
b.load_random(1)
b.step(12)  # to band layout + warm
torch.cuda.synchronize()
for rep in range(2):
    b.slots.zero_()
    top, bot = b.halo(12)
    b._exchange(12)
    b.kern.band_step(top, b.board, bot, b.buf[1 - b.cur], 0, b.R, 12, b.slots)
    torch.cuda.synchronize()
    s = b.slots.cpu().view(-1)
    for role in range(4):
        tot, w_in, w_free, w_lds, n = (int(s[role * 64 + 8 * i]) for i in range(5))
        print(f"role {role}: waves {n}  cycles/wave {tot / max(n, 1):.0f}  input wait {w_in / tot:.1%}  "
              f"free-slot wait {w_free / tot:.1%}  LDS row wait {w_lds / tot:.1%}", flush=True)
