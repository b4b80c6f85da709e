#!/usr/bin/env python3
"""The C2 host-memory leg of bench.py alone (pageable and pinned host arrays), one line per
variant: python scripts/host_memory_ab.py [steps]  (env knobs such as OMP_NUM_THREADS apply)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from cwbl import synth  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
w = synth.make("c2")
for pinned in (False, True):
    r = bench.time_host_memory(w, 0, steps=steps, warmup=1, pinned=pinned)
    print(f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS')} {r['host_arrays']:22s} "
          f"{r['value'] / 1e6:6.2f} M pts/s {r['ms_per_step']:7.2f} ms/step "
          f"copy {r['ms_copy_per_step']:6.2f} ms", flush=True)
