#!/usr/bin/env python3
"""Time the CPU port's lego training iteration (bench.py's cpu_leg body, 4096 rays) at several thread
counts on this host, one iteration each after one warm-up, printing as it goes: how the §8(d) CPU leg
scales from the job's share to every physical core of the affinity mask. argv: thread counts."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    logical, share, physical = bench.cpu_threads()
    print(f"affinity {logical} logical, {physical} physical, share {share}, cpu {bench.cpu_model()}", flush=True)
    for n in [int(a) if a != "phys" else physical for a in sys.argv[1:]]:
        torch.set_num_threads(n)
        t0 = time.perf_counter()
        r = bench.cpu_leg(4096, 1024, 800, 1, 1)
        print(f"threads {n}: step {r['step_s']} s, {r['value']} rays/s (leg incl. warm-up {time.perf_counter() - t0:.1f} s)",
              flush=True)


if __name__ == "__main__":
    main()
