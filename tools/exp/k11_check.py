"""Parity of a measurement build (argv[1]) against the oracle on band boards (strips, paired
one-round ranges, several launches with a short tail): exits 1 on any mismatch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gol-distributed-final_amd")]
import golhip  # noqa: E402
import golhip._lib as L  # noqa: E402
from oracle import oracle as O  # noqa: E402

lib = L.load(sys.argv[1])
bad = 0
for H, W, turns, seed in [(300, 1024, 45, 1), (97, 2048, 45, 2), (1000, 4096, 34, 3), (65536, 2048, 23, 4),
                          (33, 8192, 45, 5), (4100, 32768, 24, 6)]:
    ref, counts = O.bits_run(O.random_words(seed, 0, H, W // 64), turns, with_counts=True)
    with golhip.Engine(H, W, device=0, library=lib) as e:
        k = e.info()["turns_per_launch"]
        e.load_random(seed)
        got = e.step_counted(turns, k)
        ok = e.hash() == O.hash_words(ref) and list(got) == [int(counts[k * (i + 1) - 1]) for i in range(turns // k)]
    print(H, W, turns, "k", k, "ok" if ok else "MISMATCH", flush=True)
    bad += not ok
sys.exit(1 if bad else 0)
